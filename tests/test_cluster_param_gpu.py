"""GPU parity of the cluster parameter-flow token path:
DefaultTokenService.requestParamToken -> ClusterParamFlowChecker over ClusterParamMetric,
HIP engine (through the C-ABI) against the oracle's single-threaded replay on the same ordered
trace under a mocked clock.  Decisions (status, remaining) and ClusterParamMetric sums must be
bit-exact.  Each bucket map is a strict LRU of capacity 4000 (ClusterParamMetric.java:37-88): the
cparamlru_* vectors (tests/golden/make_cparam_lru_golden.py, an independent model; CLHM itself is not
vendored) and the small-capacity traces below evict."""
import ctypes as C

import numpy as np
import pytest

from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


@pytest.fixture(scope="module")
def cm():
    from sentinel_amd import cluster
    return cluster


def to_param_rules(cm, rules):
    out = []
    for r in rules:
        items = [cm.ParamFlowItem(object=v, count=c, class_type="long") for v, c in r.get("hot", {}).items()]
        out.append(cm.ParamFlowRule(resource=f"p{r['flow_id']}", count=r["count"], cluster_mode=True,
                                    param_flow_item_list=items,
                                    cluster_config=cm.ParamFlowClusterConfig(
                                        flow_id=r["flow_id"], threshold_type=r.get("threshold_type", 0),
                                        sample_count=r.get("sample_count", 10),
                                        window_interval_ms=r.get("window_interval_ms", 1000))))
    return out


class Pair:
    """Engine + oracle fed the same rule loads and requests."""

    def __init__(self, cm, max_batch=1 << 16, max_param_keys=1 << 16):
        self.cm = cm
        self.eng = cm.Engine(max_batch=max_batch, max_param_keys=max_param_keys)
        self.mgr = cm.ClusterParamFlowRuleManager(self.eng)
        self.svc = cm.DefaultTokenService(self.eng)
        self.L = H.lib()
        self.oh = self.L.orc_cluster_new(1.0, 1.0)
        self.keep = []

    def load(self, ns, rules):
        self.mgr.load_rules(ns, to_param_rules(self.cm, rules))
        arr = H.cluster_param_rules_array(rules, self.keep)
        self.L.orc_cluster_load_param_rules(self.oh, ns.encode(), arr, len(rules))

    def connected(self, ns, n):
        self.cm.ClusterFlowRuleManager(self.eng).set_connected_count(ns, n)
        self.L.orc_cluster_set_connected_count(self.oh, ns.encode(), n)

    def limit(self, ns, qps):
        self.cm.GlobalRequestLimiter(self.eng).init_if_absent(ns, qps)
        self.L.orc_cluster_set_namespace_limit(self.oh, ns.encode(), qps)

    def run(self, fid, acq, params, ts, ctx=""):
        got = self.svc.request_param_tokens(fid, acq, params, ts)
        n = len(fid)
        off = np.zeros(n + 1, dtype=np.uint32)
        for i, p in enumerate(params):
            off[i + 1] = off[i] + len(p)
        flat = np.ascontiguousarray([self.cm.param_value_key(v) for p in params for v in p] or [0], np.int64)
        out = (H.OrcTokenResult * n)()
        f = np.ascontiguousarray(fid, np.int64)
        a = np.ascontiguousarray(acq, np.int32)
        t = np.ascontiguousarray(ts, np.int64)
        self.L.orc_cluster_param_replay(self.oh, n, f.ctypes.data, a.ctypes.data, off.ctypes.data, flat.ctypes.data,
                                        t.ctypes.data, out)
        ref = np.frombuffer(out, dtype=np.int32).reshape(-1, 3)
        bad = np.nonzero((got["status"] != ref[:, 0]) | (got["remaining"] != ref[:, 1]))[0]
        if bad.size:
            i = int(bad[0])
            raise AssertionError(f"{ctx}: {bad.size} mismatches; first at {i}: flow={fid[i]} acq={acq[i]} "
                                 f"params={params[i]} ts={ts[i]} gpu=({got['status'][i]},{got['remaining'][i]}) "
                                 f"oracle=({ref[i, 0]},{ref[i, 1]})")
        return got

    def check_sums(self, flows_values, now):
        for f, v in flows_values:
            g = self.mgr.param_sum(f, v, now)
            o = self.L.orc_cluster_param_sum(self.oh, f, self.cm.param_value_key(v), now)
            assert g == o, (f, v, g, o)

    def check_top(self, flows, now, number=5):
        """ClusterParamMetric.getTopValues (the topParams of paramToMetricNode)."""
        for f in flows:
            got = self.mgr.top_values(f, now, number)
            vals = (C.c_int64 * number)()
            qps = (C.c_double * number)()
            k = self.L.orc_cluster_param_top_values(self.oh, f, now, number, vals, qps)
            assert got == [(vals[i], qps[i]) for i in range(k)], (f, now, got)

    def close(self):
        self.L.orc_cluster_free(self.oh)
        self.eng.close()


def test_basic_semantics(cm):
    """Validation, NO_RULE, count 5 per second per value, hot item override, remaining."""
    p = Pair(cm)
    p.load("default", [{"flow_id": 11, "count": 5, "threshold_type": 1, "hot": {7: 2}}])
    fid = [11, 11, 0, 11, 99, 11] + [11] * 12
    acq = [1, 1, 1, 0, 1, 1] + [1] * 12
    params = [[3], [3], [3], [3], [3], []] + [[3]] * 6 + [[7]] * 6
    ts = [T0 + i for i in range(len(fid))]
    got = p.run(fid, acq, params, ts, "basic")
    assert list(got["status"][:6]) == [0, 0, -4, -4, 3, -4]
    assert list(got["status"][6:12]) == [0, 0, 0, 1, 1, 1]      # 5 per second for value 3
    assert list(got["status"][12:18]) == [0, 0, 1, 1, 1, 1]     # hot item 7 -> 2
    p.check_sums([(11, 3), (11, 7), (11, 8)], ts[-1])
    p.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_single_value_traces(cm, seed):
    """Key-parallel path: single-valued requests, ascending time, Zipf-like values, several rules
    with hot items and AVG_LOCAL thresholds; several batches continue the same state."""
    rng = np.random.default_rng(seed)
    p = Pair(cm)
    p.connected("default", 3)
    rules = []
    for f in range(1, 41):
        r = {"flow_id": f, "count": float(rng.integers(1, 30)), "threshold_type": int(f % 2)}
        if f % 5 == 0:
            r["sample_count"], r["window_interval_ms"] = 5, 500
        if f % 3 == 0:
            r["hot"] = {int(v): int(rng.integers(0, 10)) for v in rng.integers(0, 50, size=3)}
        rules.append(r)
    p.load("default", rules)
    n = 40_000
    fid = rng.integers(1, 45, size=n)
    vals = np.minimum(rng.zipf(1.3, size=n), 200) - 1
    acq = np.where(rng.random(n) < 0.9, 1, rng.integers(1, 4, size=n))
    ts = T0 + np.cumsum(rng.integers(0, 2, size=n))
    params = [[int(v)] for v in vals]
    for lo in range(0, n, 10_000):
        sl = slice(lo, lo + 10_000)
        p.run(fid[sl], acq[sl], params[sl], ts[sl], f"seed={seed} batch@{lo}")
    p.check_sums([(int(f), int(v)) for f in range(1, 41) for v in (0, 1, 2, 5, 33)], int(ts[-1]))
    p.check_top(range(1, 46), int(ts[-1]))
    p.check_top(range(1, 41, 7), int(ts[-1]) + 450, number=12)
    p.check_top([3, 4], int(ts[-1]) + 5000)  # every bucket deprecated: empty
    p.close()


def test_multi_value_and_regression(cm):
    """Sequential path: collections of values (all must pass, every value is added, remaining -1),
    time going backwards inside a batch, acquire counts beyond the packed field."""
    rng = np.random.default_rng(7)
    p = Pair(cm)
    p.load("ns1", [{"flow_id": f, "count": float(rng.integers(2, 12)), "threshold_type": 1,
                    "sample_count": 2, "window_interval_ms": 1000} for f in range(1, 9)])
    n = 6000
    fid = rng.integers(1, 10, size=n)
    ts = T0 + np.cumsum(rng.integers(0, 3, size=n))
    back = rng.random(n) < 0.01
    ts[back] -= rng.integers(1, 900, size=back.sum())
    acq = np.where(rng.random(n) < 0.95, 1, rng.integers(100, 300, size=n))
    params = []
    for i in range(n):
        k = 1 if rng.random() < 0.6 else int(rng.integers(2, 4))
        params.append([int(v) for v in rng.integers(0, 12, size=k)])
    for lo in range(0, n, 2000):
        sl = slice(lo, lo + 2000)
        p.run(fid[sl], acq[sl], params[sl], ts[sl], f"batch@{lo}")
    p.check_sums([(f, v) for f in range(1, 9) for v in range(12)], int(ts.max()))
    p.check_top(range(1, 10), int(ts.max()), number=20)
    p.close()


def test_mixed_paths_limiter_and_reload(cm):
    """Some rules take the sequential path (multi-value requests) while others stay key-parallel in
    the same batch; a namespace QPS limiter shared with the flow path; rule reload keeps metrics of
    flowIds that stay and drops the others."""
    rng = np.random.default_rng(11)
    p = Pair(cm)
    p.limit("lim", 400.0)
    p.load("lim", [{"flow_id": f, "count": 20.0, "threshold_type": 1} for f in range(1, 6)])
    p.load("free", [{"flow_id": f, "count": 9.0, "threshold_type": 1, "sample_count": 4, "window_interval_ms": 200}
                    for f in range(10, 16)])
    n = 8000
    fid = np.where(rng.random(n) < 0.5, rng.integers(1, 6, size=n), rng.integers(10, 16, size=n))
    ts = T0 + np.cumsum(rng.integers(0, 2, size=n))
    params = [[int(rng.integers(0, 30))] if (f >= 10 or rng.random() < 0.7) else
              [int(x) for x in rng.integers(0, 30, size=2)] for f in fid]
    acq = np.ones(n, np.int64)
    p.run(fid[:4000], acq[:4000], params[:4000], ts[:4000], "before reload")
    # reload: flowIds 10..12 stay (metrics kept), 13..15 dropped, 16 new
    p.load("free", [{"flow_id": f, "count": 4.0, "threshold_type": 1, "sample_count": 4, "window_interval_ms": 200}
                    for f in (10, 11, 12, 16)])
    fid2 = np.where(fid[4000:] == 13, 16, fid[4000:])
    p.run(fid2, acq[4000:], params[4000:], ts[4000:], "after reload")
    p.check_sums([(f, v) for f in (1, 2, 10, 11, 16) for v in range(0, 30, 3)], int(ts[-1]))
    p.close()


@pytest.mark.parametrize("name", ["exhaust_then_evict", "exhaust_no_evict_at_capacity", "blocked_get_moves_to_mru",
                                  "two_buckets", "random_stream"])
def test_lru_golden_vectors(cm, name):
    """More than 4000 values a bucket at the default capacity: the engine against the vectors and the oracle.
    The first batches stay under 4000 keys (key-parallel path, access stamps only); the batch whose keys
    pass the capacity switches the rule to LRU mode from those stamps."""
    from tests.test_cluster_param_oracle import golden_rule, load_lru_golden
    doc = load_lru_golden(name)
    p = Pair(cm)
    p.load("default", [golden_rule(doc)])
    ev = doc["events"]
    n = len(ev)
    fid = np.full(n, doc["flow_id"], np.int64)
    acq = np.full(n, doc["acquire"], np.int64)
    ts = np.array([t for _, t in ev], np.int64)
    params = [[v] for v, _ in ev]
    exp = np.array(doc["expect"], np.int64)
    cuts = [0, n // 8, n // 3, n]
    for a, b in zip(cuts[:-1], cuts[1:]):
        got = p.run(fid[a:b], acq[a:b], params[a:b], ts[a:b], f"{name} batch@{a}")
        st = np.asarray(got["status"], np.int64)
        rem = np.asarray(got["remaining"], np.int64)
        bad = np.nonzero((st != exp[a:b, 0]) | (rem != exp[a:b, 1]))[0]
        assert bad.size == 0, (name, a + int(bad[0]), st[bad[0]], rem[bad[0]], exp[a + bad[0]])
    for v, t, sm in doc["sums"]:
        assert p.mgr.param_sum(doc["flow_id"], v, t) == sm, (v, t, sm)
    p.close()


def test_lru_small_capacity_mixed(cm):
    """Capacity 40 (the maxCapacity constructor argument): several rules and geometries, both paths, a
    rule switching mid-stream, collections, time going backwards, acquire counts beyond the packed field,
    getSum calls (accesses) and getTopValues between batches -- decisions, sums and top values bit-exact."""
    rng = np.random.default_rng(29)
    L = H.lib()
    p = Pair(cm)
    p.mgr.set_param_capacity(40)
    L.orc_cluster_set_param_capacity(40)
    try:
        p.load("default", [{"flow_id": f, "count": float(rng.integers(2, 6)), "threshold_type": 1,
                            "sample_count": [1, 2, 5, 10][f % 4], "window_interval_ms": 1000,
                            "hot": {1: 9} if f % 3 == 0 else {}} for f in range(1, 9)])
    finally:
        L.orc_cluster_set_param_capacity(0)
    p.mgr.set_param_capacity(0)
    n = 24000
    fid = rng.integers(1, 9, size=n)
    dom = np.where(fid <= 2, 30, np.where(fid <= 5, 120, 600))  # rules 1-2 never pass their capacity
    ts = T0 + np.cumsum(rng.integers(0, 2, size=n) * (rng.random(n) < 0.4))
    acq = np.where(rng.random(n) < 0.97, 1, rng.integers(2, 200, size=n))
    params = [[int(rng.integers(0, d))] for d in dom]
    for lo in range(0, n, 3000):
        sl = slice(lo, lo + 3000)
        f, a, t, pr = fid[sl].copy(), acq[sl].copy(), ts[sl].copy(), params[sl]
        if lo >= 12000:  # sequential path for everyone: collections and time going backwards
            pr = [q if rng.random() < 0.8 else q + [int(rng.integers(0, 50))] for q in pr]
            back = rng.random(len(t)) < 0.02
            t[back] -= rng.integers(1, 700, size=int(back.sum()))
        p.run(f, a, pr, t, f"batch@{lo}")
        now = int(t.max())
        p.check_sums([(ff, v) for ff in range(1, 9) for v in (0, 1, 7, 19)], now)
        p.check_top(range(1, 9), now, number=8)
    p.close()


def test_lru_area_of_dropped_rule_reused(cm):
    """A rule in LRU mode is dropped by a reload; a new rule of the same geometry then switches to LRU and
    gets the dropped rule's queue area from the pool. The dropped rule's keys stay in the key store: none
    of them may join the new rule's queues (its evictions, decisions and sums must equal the oracle's)."""
    rng = np.random.default_rng(41)
    L = H.lib()
    p = Pair(cm)
    p.mgr.set_param_capacity(40)
    L.orc_cluster_set_param_capacity(40)
    geo = {"count": 3.0, "threshold_type": 1, "sample_count": 2, "window_interval_ms": 1000}
    try:
        p.load("default", [dict(geo, flow_id=1), dict(geo, flow_id=2)])
        n = 3000
        ts = T0 + np.arange(n) // 4
        fid = np.where(rng.random(n) < 0.7, 1, 2)
        params = [[int(rng.integers(0, 200 if f == 1 else 20))] for f in fid]
        p.run(fid, np.ones(n, np.int64), params, ts, "rule 1 switches to LRU")
        p.load("default", [dict(geo, flow_id=2)])            # rule 1 and its metric dropped
        p.load("default", [dict(geo, flow_id=2), dict(geo, flow_id=3)])  # rule 3: same S and capacity
    finally:
        L.orc_cluster_set_param_capacity(0)
    p.mgr.set_param_capacity(0)
    t1 = int(ts[-1]) + 1
    for b in range(3):
        ts2 = t1 + b * 700 + np.arange(n) // 5
        fid2 = np.where(rng.random(n) < 0.8, 3, 2)
        params2 = [[int(rng.integers(0, 200 if f == 3 else 20))] for f in fid2]
        p.run(fid2, np.ones(n, np.int64), params2, ts2, f"rule 3 batch {b}")
        now = int(ts2[-1])
        p.check_sums([(3, v) for v in range(0, 200, 7)] + [(2, v) for v in range(20)], now)
        p.check_top([2, 3], now, number=10)
    p.close()
