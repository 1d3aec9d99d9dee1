"""GPU parity: the HIP cluster token-server path (through the C-ABI) against the
oracle's single-threaded replay of ClusterFlowChecker on the same ordered
trace under a mocked clock.  Decisions (status, remaining, waitInMs) and every
ClusterMetric counter must be bit-exact."""
import ctypes as C

import numpy as np
import pytest

from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def oracle_cluster(rules, namespace_conn=None, exceed=1.0, ratio=1.0):
    L = H.lib()
    h = L.orc_cluster_new(exceed, ratio)
    if namespace_conn:
        for ns, c in namespace_conn.items():
            L.orc_cluster_set_connected_count(h, ns.encode(), c)
    for ns, rs in rules.items():
        arr = H.cluster_rules_array(rs)
        L.orc_cluster_load_rules(h, ns.encode(), arr, len(rs))
    return h


def oracle_replay(h, fid, acq, prio, ts):
    L = H.lib()
    n = len(fid)
    out = (H.OrcTokenResult * n)()
    fid = np.ascontiguousarray(fid, np.int64)
    acq = np.ascontiguousarray(acq, np.int32)
    prio = np.ascontiguousarray(prio, np.uint8)
    ts = np.ascontiguousarray(ts, np.int64)
    L.orc_cluster_replay(h, n, fid.ctypes.data, acq.ctypes.data, prio.ctypes.data, ts.ctypes.data, out)
    a = np.frombuffer(out, dtype=np.int32).reshape(n, 3)
    return a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy()


@pytest.fixture(scope="module")
def eng_mod():
    from sentinel_amd import cluster
    return cluster


HOT_MODES = {"off": dict(hot_rules=False, small_batch=0), "on": dict(hot_rules=True, hot_min_requests=64, small_batch=0),
             "all": dict(hot_rules=True, hot_min_requests=1, small_batch=0),
             "small": dict(hot_rules=False, small_batch=4096)}


def make_engine(cluster, hot="off", **kw):
    """hot: the engine's path policy (decisions must not depend on it).  "off" (the default)
    sorts every request, "on" sends rules with >= 64 requests in the previous batch down the
    hot/cold split, "all" every rule seen in the previous batch (up to 4096), "small" orders
    batches of up to 4096 requests in one workgroup (k_small_sort) and sorts larger ones."""
    kw.setdefault("max_batch", 1 << 20)
    kw.update(HOT_MODES[hot])
    return cluster.Engine(**kw)


def engine_rules(cluster, eng, rules, namespace_conn=None):
    mgr = cluster.ClusterFlowRuleManager(eng)
    if namespace_conn:
        for ns, c in namespace_conn.items():
            mgr.set_connected_count(ns, c)
    for ns, rs in rules.items():
        fr = [cluster.FlowRule(resource=f"r{r['flow_id']}", count=r["count"], cluster_mode=True,
                               cluster_config=cluster.ClusterFlowConfig(
                                   flow_id=r["flow_id"], threshold_type=r.get("threshold_type", 0),
                                   sample_count=r.get("sample_count", 10),
                                   window_interval_ms=r.get("window_interval_ms", 1000))) for r in rs]
        mgr.load_rules(ns, fr)
    return mgr


def assert_same(gpu, orc, fid, ts, ctx=""):
    st, rem, wait = orc
    bad = np.nonzero((gpu["status"] != st) | (gpu["remaining"] != rem) | (gpu["wait_in_ms"] != wait))[0]
    if bad.size:
        i = bad[0]
        raise AssertionError(f"{ctx}: {bad.size} mismatches; first at {i}: flow={fid[i]} ts={ts[i]} "
                             f"gpu=({gpu['status'][i]},{gpu['remaining'][i]},{gpu['wait_in_ms'][i]}) "
                             f"oracle=({st[i]},{rem[i]},{wait[i]})")


def assert_metrics(cluster, eng, oh, flow_ids, now):
    svc = cluster.DefaultTokenService(eng)
    L = H.lib()
    for f in flow_ids:
        g = svc.metric_sums(int(f), now)
        o = [L.orc_cluster_metric_sum(oh, int(f), ev, now) for ev in range(7)]
        assert g == o, (f, g, o)


def random_rules(rng, n, ids=None, mixed_geometry=False):
    rs = []
    ids = ids if ids is not None else range(1, n + 1)
    for fid in ids:
        r = {"flow_id": int(fid), "count": float(rng.integers(1, 60)), "threshold_type": 1}
        if mixed_geometry:
            sc = int(rng.choice([1, 2, 5, 10, 20]))
            r["sample_count"] = sc
            r["window_interval_ms"] = int(sc * rng.choice([10, 50, 100, 200]))
            if rng.random() < 0.2:
                r["count"] = float(rng.integers(1, 60)) + 0.5
        rs.append(r)
    return rs


def test_cluster_flow_checker_kat_sequence(eng_mod):
    """CST/flow/ClusterFlowCheckerTest.java:37-75 sequence (disabled upstream) on the GPU."""
    c = eng_mod
    rule = [{"flow_id": 98765, "count": 5, "threshold_type": 1, "sample_count": 5, "window_interval_ms": 1000}]
    seq = [(0, 0, "OK"), (0, 0, "OK"), (200, 0, "OK"), (400, 1, "OK"), (400, 0, "OK"), (400, 1, "BLOCKED"),
           (600, 0, "BLOCKED"), (600, 0, "BLOCKED"), (800, 0, "BLOCKED"), (800, 1, "SHOULD_WAIT"),
           (800, 0, "BLOCKED"), (1000, 0, "OK")]
    for base in (T0, T0 + 123, T0 + 199):
        for one_by_one in (True, False):
            eng = make_engine(c)
            engine_rules(c, eng, {"default": rule})
            svc = c.DefaultTokenService(eng)
            ts = [base + d for d, _, _ in seq]
            pr = [p for _, p, _ in seq]
            if one_by_one:
                got = [svc.request_token(98765, 1, bool(p), t).status for t, p in zip(ts, pr)]
            else:
                got = list(svc.request_tokens([98765] * len(seq), [1] * len(seq), pr, ts)["status"])
            want = [H.TOKEN_STATUS[s] for _, _, s in seq]
            assert got == want, (base, one_by_one, got)
            eng.close()


def test_request_validation(eng_mod):
    c = eng_mod
    eng = make_engine(c)
    engine_rules(c, eng, {"default": [{"flow_id": 7, "count": 3, "threshold_type": 1}]})
    svc = c.DefaultTokenService(eng)
    r = svc.request_tokens([0, -5, 7, 7, 99, 7], [1, 1, 0, -3, 1, 1], [0] * 6, [T0] * 6)
    assert list(r["status"]) == [-4, -4, -4, -4, 3, 0]
    assert r["remaining"][5] == 2


@pytest.mark.parametrize("hot", ["off", "on", "all", "small"])
@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("mixed", [False, True])
@pytest.mark.parametrize("ids", ["dense", "sparse"])
def test_random_traces_bit_exact(eng_mod, seed, mixed, ids, hot):
    """Random rules (mixed window geometries, fractional counts), acquire mix (incl. counts
    beyond the packed 7-bit field), 10 % prioritized, bursts: every decision and counter equals
    the oracle.  ids="dense" exercises the direct flowId table, "sparse" the hash probe."""
    c = eng_mod
    rng = np.random.default_rng(seed)
    nr = 300
    idmul = 1 if ids == "dense" else 1_000_003
    rules = random_rules(rng, nr, ids=[i * idmul for i in range(1, nr + 1)], mixed_geometry=mixed)
    n = 60_000
    fid = rng.integers(1, nr + 40, size=n)          # some ids without rules
    fid[rng.random(n) < 0.002] = 0                  # BAD_REQUEST
    busy = rng.random(n) < 0.5
    fid[busy] = rng.integers(1, 6, size=busy.sum())  # hot rules -> long runs
    acq = np.where(rng.random(n) < 0.9, 1, rng.integers(1, 6, size=n)) if mixed else np.ones(n, np.int64)
    if mixed:
        acq[rng.random(n) < 0.002] = 300            # beyond the packed acquire field: replayed
    acq[rng.random(n) < 0.001] = 0                  # BAD_REQUEST
    fid = np.where(fid > 0, fid * idmul, fid)
    prio = (rng.random(n) < 0.1).astype(np.uint8)
    ts = T0 + np.cumsum(rng.integers(0, 3, size=n))
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot=hot, max_batch=1 << 16)
    engine_rules(c, eng, {"default": rules})
    svc = c.DefaultTokenService(eng)
    for lo in range(0, n, 20_000):  # several batches continue the same state (and move the hot set)
        sl = slice(lo, lo + 20_000)
        g = svc.request_tokens(fid[sl], acq[sl], prio[sl], ts[sl])
        o = oracle_replay(oh, fid[sl], acq[sl], prio[sl], ts[sl])
        assert_same(g, o, fid[sl], ts[sl], f"seed={seed} batch@{lo}")
    assert_metrics(c, eng, oh, [i * idmul for i in range(1, nr + 1)], int(ts[-1]))
    H.lib().orc_cluster_free(oh)
    eng.close()


def test_avg_local_threshold_and_reload(eng_mod):
    """AVG_LOCAL (count * connectedCount) and ClusterFlowRuleManager reload
    semantics: kept flowIds keep their metric, dropped ones lose it."""
    c = eng_mod
    rng = np.random.default_rng(7)
    rules = [{"flow_id": i, "count": float(rng.integers(1, 20)), "threshold_type": int(i % 2)} for i in range(1, 41)]
    conn = {"default": 3}
    oh = oracle_cluster({"default": rules}, namespace_conn=conn)
    eng = make_engine(c, max_batch=1 << 15)
    mgr = engine_rules(c, eng, {"default": rules}, namespace_conn=conn)
    svc = c.DefaultTokenService(eng)

    def batch(t0, n):
        fid = rng.integers(1, 45, size=n)
        acq = np.ones(n, np.int64)
        prio = (rng.random(n) < 0.2).astype(np.uint8)
        ts = t0 + np.sort(rng.integers(0, 1500, size=n))
        g = svc.request_tokens(fid, acq, prio, ts)
        o = oracle_replay(oh, fid, acq, prio, ts)
        assert_same(g, o, fid, ts)
        return int(ts[-1])

    t = batch(T0, 5000)
    # reload: drop 1..10, keep 11..40 (new counts), add 41..50
    rules2 = [{"flow_id": i, "count": float(rng.integers(1, 20)), "threshold_type": 1} for i in range(11, 51)]
    arr = H.cluster_rules_array(rules2)
    H.lib().orc_cluster_load_rules(oh, b"default", arr, len(rules2))
    mgr.load_rules("default", [c.FlowRule(count=r["count"], cluster_mode=True, cluster_config=c.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1)) for r in rules2])
    t = batch(t + 1, 5000)
    assert_metrics(c, eng, oh, range(11, 51), t)
    H.lib().orc_cluster_free(oh)
    eng.close()


@pytest.mark.parametrize("geometry", ["uniform", "mixed"])
@pytest.mark.parametrize("clock", ["sorted", "regress"])
def test_cold_partition_bit_exact(eng_mod, geometry, clock):
    """The hot path's cold partition (rule slots from 2^15 up: one scatter pass into slot bins, each bin
    ordered inside k_cold_fused's workgroup): 40k rules, Zipf-skewed traffic whose hot ids sit next to
    each other in the slot space (uneven bins), acquire counts and prioritized requests mixed, with
    mixed window geometries (per-rule parameter loads) or the uniform layout (the threshold from the
    record header); "regress" sends batches whose clock goes back inside the batch, so the key pass
    re-classifies every request as cold (the fallback) and single bins hold tens of thousands."""
    c = eng_mod
    rng = np.random.default_rng(11 if geometry == "uniform" else 12)
    nr = 40_000
    rules = random_rules(rng, nr, mixed_geometry=geometry == "mixed")
    for r in rules:
        r["count"] = float(rng.integers(1, 400))
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot="on", max_batch=1 << 18, max_rules=1 << 16)
    engine_rules(c, eng, {"default": rules})
    svc = c.DefaultTokenService(eng)
    n = 1 << 18
    t = T0
    for b in range(4):
        rank = np.minimum(rng.zipf(1.2, size=n), nr)
        fid = rank.astype(np.int64)                     # hot ids adjacent in flowId (and slot) order
        cold = rng.random(n) < 0.3
        fid[cold] = rng.integers(1, nr + 1, size=int(cold.sum()))
        acq = np.where(rng.random(n) < 0.95, 1, rng.integers(1, 4, size=n)).astype(np.int64)
        prio = (rng.random(n) < 0.05).astype(np.uint8)
        ts = t + np.sort(rng.integers(0, 400, size=n))
        if clock == "regress" and b % 2 == 1:
            k = rng.integers(1000, n - 1000)
            ts[k:k + 500] -= 30                         # back in time inside the batch
        t = int(ts.max()) + 1
        g = svc.request_tokens(fid, acq, prio, ts)
        o = oracle_replay(oh, fid, acq, prio, ts)
        assert_same(g, o, fid, ts, f"{geometry}/{clock} batch {b}")
    assert_metrics(c, eng, oh, list(range(1, 200)) + list(rng.integers(1, nr + 1, size=300)), t)
    H.lib().orc_cluster_free(oh)
    eng.close()


@pytest.mark.parametrize("hot", ["on", "all"])
def test_time_regression_and_gaps(eng_mod, hot):
    """Clock going backwards (detached windows) and long idle gaps."""
    c = eng_mod
    rules = [{"flow_id": 1, "count": 4, "threshold_type": 1, "sample_count": 5, "window_interval_ms": 500},
             {"flow_id": 2, "count": 2, "threshold_type": 1}]
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot=hot, max_batch=1 << 12)
    engine_rules(c, eng, {"default": rules})
    svc = c.DefaultTokenService(eng)
    ts = np.array([T0, T0 + 10, T0 + 250, T0 + 120, T0 + 130, T0 + 5000, T0 + 4000, T0 + 5001, T0 + 90000,
                   T0 + 90000, T0 + 90100] * 3, dtype=np.int64)
    fid = np.where(np.arange(len(ts)) % 3 == 2, 2, 1).astype(np.int64)
    prio = np.array([0, 1] * (len(ts) // 2) + [1] * (len(ts) % 2), dtype=np.uint8)
    acq = np.ones(len(ts), np.int64)
    for rep in range(3):  # the same pattern again, later: batches 2 and 3 run with both rules hot
        tsr = ts + rep * 200_000
        g = svc.request_tokens(fid, acq, prio, tsr)
        o = oracle_replay(oh, fid, acq, prio, tsr)
        assert_same(g, o, fid, tsr, f"rep {rep}")
    H.lib().orc_cluster_free(oh)
    eng.close()


@pytest.mark.parametrize("hot", ["on", "all"])
def test_zipf_c3_slice_bit_exact(eng_mod, hot):
    """C3 trace slice (100k rules, 2^21 requests, Zipf(1.1), 1 % prioritized)."""
    from sentinel_amd.workload import ClusterTrace
    c = eng_mod
    tr = ClusterTrace(n_rules=100_000, lam=10_000_000)
    fid_r, cnt = tr.rules()
    rules = [{"flow_id": int(f), "count": float(x), "threshold_type": 1} for f, x in zip(fid_r, cnt)]
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot=hot, max_batch=1 << 20, max_rules=1 << 17)
    c.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
    svc = c.DefaultTokenService(eng)
    for b in range(3):
        fid, acq, prio, ts = tr.events(b << 20, 1 << 20)
        g = svc.request_tokens(fid, acq, prio, ts)
        o = oracle_replay(oh, fid, acq, prio, ts)
        assert_same(g, o, fid, ts, f"batch {b}")
    seen = np.unique(fid)[:200]
    assert_metrics(c, eng, oh, seen, int(ts[-1]))
    H.lib().orc_cluster_free(oh)
    eng.close()


def test_host_batches_pipelined(eng_mod):
    """Host-buffer batches of more than one staging chunk (2^20 requests) take the page-locked pipeline
    (engine.cpp run_host_batch_pipelined: chunked H2D / D2H, device-side time offsets), a ragged last
    chunk included; one whose times span more than u32 offsets takes the chunked path.  Bit-exact
    against the oracle, metrics included."""
    from sentinel_amd.workload import ClusterTrace
    c = eng_mod
    tr = ClusterTrace(n_rules=50_000, lam=10_000_000)
    fid_r, cnt = tr.rules()
    rules = [{"flow_id": int(f), "count": float(x), "threshold_type": 1} for f, x in zip(fid_r, cnt)]
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot="on", max_batch=1 << 22, max_rules=1 << 16)
    c.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
    svc = c.DefaultTokenService(eng)
    lo = 0
    from sentinel_amd import _lib
    L = _lib.load()
    for k, n in enumerate([3 * (1 << 20) + 12345, 1 << 20, (1 << 20) + 7, (1 << 21) + 3]):
        fid, acq, prio, ts = tr.events(lo, n)
        lo += n
        if k == 2:  # a jump past the u32 span half way: the chunked path
            ts = ts.copy()
            ts[n // 2:] += 1 << 33
        if k == 3:  # registered buffers: DMA straight from / to them (run_host_batch_registered)
            fid, acq, prio, ts = (np.ascontiguousarray(x, dt) for x, dt in
                                  ((fid, np.int64), (acq, np.int32), (prio, np.uint8), (ts, np.int64)))
            out = np.zeros(n, dtype=c.TOKEN_DTYPE)
            arrs = (fid, acq, prio, ts, out)
            for x in arrs:
                assert L.sga_host_register(eng.handle, x.ctypes.data, x.nbytes) == 0
            rc = L.sga_request_tokens(eng.handle, fid.ctypes.data, acq.ctypes.data, prio.ctypes.data, ts.ctypes.data,
                                      n, out.ctypes.data)
            for x in arrs:
                assert L.sga_host_unregister(eng.handle, x.ctypes.data) == 0
            assert rc == 0
            g = out
        else:
            g = svc.request_tokens(fid, acq, prio, ts)
        o = oracle_replay(oh, fid, acq, prio, ts)
        assert_same(g, o, fid, ts, f"host batch {k} ({n} requests)")
    assert_metrics(c, eng, oh, np.unique(fid)[:100], int(ts[-1]))
    H.lib().orc_cluster_free(oh)
    eng.close()


def test_rls_descriptors(eng_mod):
    """Envoy RLS: SimpleClusterFlowChecker per descriptor, NO_RULE -> OK, no short-circuit."""
    from sentinel_amd.javautil import rls_key
    c = eng_mod
    rls = c.EnvoyRlsService
    keys = [rls_key("d", [("k", f"v{i}")]) for i in range(8)]
    fids = [rls.generate_flow_id(k) for k in keys]
    rules = [{"flow_id": f, "count": 3.0, "threshold_type": 1, "sample_count": 1, "window_interval_ms": 1000}
             for f in fids[:6]]
    eng = make_engine(c, max_batch=1 << 12)
    engine_rules(c, eng, {"default": rules})
    oh = oracle_cluster({"default": rules})
    svc = rls(eng)
    rng = np.random.default_rng(3)
    nreq = 400
    ndesc = rng.integers(1, 5, size=nreq)
    off = np.concatenate([[0], np.cumsum(ndesc)]).astype(np.uint32)
    dfid = np.array([fids[i] for i in rng.integers(0, 8, size=off[-1])], dtype=np.int64)
    hits = rng.integers(0, 3, size=nreq).astype(np.int32)
    hits[5] = -1
    ts = T0 + np.arange(nreq) * 7
    code, st, rem = svc.should_rate_limit(off, dfid, hits, ts, with_remaining=True)
    L = H.lib()
    for r in range(nreq):
        if hits[r] < 0:
            assert code[r] == -1
            assert all(st[d] == 3 and rem[d] == 0 for d in range(off[r], off[r + 1]))
            continue
        a = 1 if hits[r] == 0 else int(hits[r])
        blocked = False
        for d in range(off[r], off[r + 1]):
            res = L.orc_cluster_request_token_simple(oh, int(dfid[d]), a, int(ts[r]))
            assert (st[d], rem[d]) == (res.status, res.remaining), (r, d, st[d], rem[d], res.status, res.remaining)
            blocked |= res.status not in (0, 3)  # NO_RULE_EXISTS passes
        assert code[r] == (2 if blocked else 1)
    L.orc_cluster_free(oh)
    eng.close()


@pytest.mark.parametrize("seed", [41, 42])
def test_namespace_limiter(eng_mod, seed):
    """GlobalRequestLimiter pre-pass: two limited namespaces and one unlimited, requests
    without rules and bad requests interleaved, clock regressions, a limit change
    mid-stream (applyMaxQpsChange) -- statuses and metrics equal the oracle."""
    c = eng_mod
    rng = np.random.default_rng(seed)
    rules = {"ns-a": random_rules(rng, 0, ids=range(1, 51)), "ns-b": random_rules(rng, 0, ids=range(51, 101)),
             "ns-c": random_rules(rng, 0, ids=range(101, 151))}
    oh = oracle_cluster(rules)
    L = H.lib()
    eng = make_engine(c, max_batch=1 << 14)
    engine_rules(c, eng, rules)
    lim = c.GlobalRequestLimiter(eng)
    for ns, q in (("ns-a", 40.0), ("ns-b", 7.5)):
        L.orc_cluster_set_namespace_limit(oh, ns.encode(), q)
        lim.init_if_absent(ns, q)
    svc = c.DefaultTokenService(eng)
    n = 40_000
    fid = rng.integers(1, 160, size=n)
    fid[rng.random(n) < 0.003] = -1
    acq = np.where(rng.random(n) < 0.95, 1, 2)
    prio = (rng.random(n) < 0.05).astype(np.uint8)
    ts = T0 + np.cumsum(rng.integers(0, 2, size=n))
    back = rng.random(n) < 0.01
    ts[back] -= rng.integers(1, 400, size=back.sum())
    for k, lo in enumerate(range(0, n, 10_000)):
        if k == 2:
            L.orc_cluster_set_namespace_limit(oh, b"ns-a", 12.0)
            L.orc_cluster_set_namespace_limit(oh, b"ns-b", 12.0)
            lim.apply_max_qps_change(12.0)
        sl = slice(lo, lo + 10_000)
        g = svc.request_tokens(fid[sl], acq[sl], prio[sl], ts[sl])
        o = oracle_replay(oh, fid[sl], acq[sl], prio[sl], ts[sl])
        assert_same(g, o, fid[sl], ts[sl], f"limiter seed={seed} batch {k}")
        assert (o[0] == -2).any()
    assert_metrics(c, eng, oh, range(1, 151), int(ts.max()))
    L.orc_cluster_free(oh)
    eng.close()


@pytest.mark.parametrize("hot", ["on", "all"])
def test_hot_rules_skew_prio_mixed(eng_mod, hot):
    """Hot-rule path under heavy skew: a few rules carry most requests (runs spanning many tiles and
    several window buckets), 5 % prioritized with tight thresholds (SHOULD_WAIT inside hot runs),
    mixed acquire counts on some hot rules (their runs replayed), requests without rules, and a
    rule reload between batches (the hot set is forgotten and chosen again)."""
    c = eng_mod
    rng = np.random.default_rng(11)
    nr = 6000
    rules = [{"flow_id": i, "count": float(rng.integers(5, 400)), "threshold_type": 1} for i in range(1, nr + 1)]
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot=hot, max_batch=1 << 17)
    mgr = engine_rules(c, eng, {"default": rules})
    svc = c.DefaultTokenService(eng)
    t = T0
    for b in range(6):
        n = 100_000
        z = rng.zipf(1.3, size=n)
        fid = np.where(z <= nr + 50, z, rng.integers(1, nr + 1, size=n)).astype(np.int64)
        acq = np.ones(n, np.int64)
        mixed = (fid % 7 == 3) & (rng.random(n) < 0.3)
        acq[mixed] = rng.integers(2, 5, size=int(mixed.sum()))
        prio = (rng.random(n) < 0.05).astype(np.uint8)
        ts = t + np.sort(rng.integers(0, 700, size=n))
        t = int(ts[-1]) + int(rng.integers(0, 300))
        g = svc.request_tokens(fid, acq, prio, ts)
        o = oracle_replay(oh, fid, acq, prio, ts)
        assert_same(g, o, fid, ts, f"hot={hot} batch {b}")
        if b == 3:  # reload: counts change for the first 100 flowIds, metrics kept
            for r in rules[:100]:
                r["count"] = float(rng.integers(5, 400))
            arr = H.cluster_rules_array(rules)
            H.lib().orc_cluster_load_rules(oh, b"default", arr, len(rules))
            mgr.load_rule_arrays("default", np.array([r["flow_id"] for r in rules], np.int64),
                                 np.array([r["count"] for r in rules]))
    assert_metrics(c, eng, oh, range(1, 60), t)
    H.lib().orc_cluster_free(oh)
    eng.close()


@pytest.mark.parametrize("hot", ["off", "on"])
def test_c3_full_size_sampled_rules_bit_exact(eng_mod, hot):
    """BASELINE C3 at full size: 1M cluster rules, two batches of 2^24 Zipf(1.1) requests.  Rules
    are independent (GLOBAL thresholds, no namespace limiter), so the requests of a sample of
    rules -- the 16 hottest ranks and 2000 random flowIds -- replayed alone by the oracle must get
    the same TokenResults; every other request is checked for the size-independent properties
    (status domain, waitInMs, non-negative remaining, metric counters of sampled rules)."""
    from sentinel_amd.workload import ClusterTrace
    c = eng_mod
    tr = ClusterTrace()
    fid_r, cnt = tr.rules()
    rng = np.random.default_rng(99)
    sample = np.unique(np.concatenate([tr.perm[:16] + 1, rng.integers(1, tr.n + 1, size=2000)])).astype(np.int64)
    rules = [{"flow_id": int(f), "count": float(cnt[f - 1]), "threshold_type": 1} for f in sample]
    oh = oracle_cluster({"default": rules})
    eng = make_engine(c, hot=hot, max_batch=1 << 24, max_rules=1 << 20)
    c.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
    svc = c.DefaultTokenService(eng)
    for b in range(2):
        fid, acq, prio, ts = tr.events(b << 24, 1 << 24)
        g = svc.request_tokens(fid, acq, prio, ts)
        st = g["status"]
        assert np.isin(st, [0, 1, 2]).all()
        assert (g["wait_in_ms"][st == 2] == 100).all() and (g["wait_in_ms"][st != 2] == 0).all()
        assert (g["remaining"][st == 0] >= 0).all() and (g["remaining"][st != 0] == 0).all()
        m = np.isin(fid, sample)
        o = oracle_replay(oh, fid[m], acq[m], prio[m], ts[m])
        sub = {k: g[k][m] for k in ("status", "remaining", "wait_in_ms")}
        assert_same(sub, o, fid[m], ts[m], f"hot={hot} batch {b} ({int(m.sum())} sampled requests)")
    assert_metrics(c, eng, oh, sample[:64], int(ts[-1]))
    H.lib().orc_cluster_free(oh)
    eng.close()


def test_pipelined_device_batches_match_sync(eng_mod):
    """sga_request_tokens_device_async (stage A of batch b + 1 beside stage B of batch b, two
    scratch sets) decides exactly like one synchronous sga_request_tokens_device per batch:
    identical TokenResults for every batch and identical metric counters afterwards; the sampled
    rules' requests also equal the oracle's replay."""
    import torch
    from sentinel_amd import _lib
    from sentinel_amd.workload import ClusterTrace
    c = eng_mod
    L = _lib.load()
    dev = torch.device("cuda", 0)
    tr = ClusterTrace(n_rules=200_000, lam=20_000_000)
    fid_r, cnt = tr.rules()
    nb, m = 7, 1 << 19
    host = [tr.events(b * m, m) for b in range(nb)]
    res = {}
    for mode in ("sync", "async"):
        eng = make_engine(c, max_batch=m, max_rules=1 << 18)
        c.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
        fn = L.sga_request_tokens_device if mode == "sync" else L.sga_request_tokens_device_async
        keep, outs = [], []
        for b, (f, a, p, ts) in enumerate(host):
            base = int(ts[0])
            d = (torch.from_numpy(f).to(dev), torch.from_numpy(a).to(dev), torch.from_numpy(p).to(dev),
                 torch.from_numpy((ts - base).astype(np.int32)).to(dev))
            o = torch.zeros(m, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            rc = fn(eng.handle, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), base, d[3].data_ptr(), m,
                    o.data_ptr(), None)
            assert rc == 0, (mode, b, rc, L.sga_last_error(eng.handle))
            keep.append(d)
            outs.append(o)
        assert L.sga_sync(eng.handle) == 0
        torch.cuda.synchronize()
        res[mode] = [o.cpu().numpy() for o in outs]
        sample = np.unique(np.concatenate([tr.perm[:8] + 1, np.arange(1, 200_001, 997)])).astype(np.int64)
        res[mode + "_metrics"] = [c.DefaultTokenService(eng).metric_sums(int(x), int(host[-1][3][-1])) for x in sample]
        eng.close()
    for b in range(nb):
        assert np.array_equal(res["sync"][b], res["async"][b]), f"batch {b}"
    assert res["sync_metrics"] == res["async_metrics"]
    # and the sampled rules against the oracle
    rules = [{"flow_id": int(x), "count": float(cnt[x - 1]), "threshold_type": 1} for x in sample]
    oh = oracle_cluster({"default": rules})
    for b, (f, a, p, ts) in enumerate(host):
        sel = np.isin(f, sample)
        o = oracle_replay(oh, f[sel], a[sel], p[sel], ts[sel])
        r = res["async"][b].view(np.uint64)[sel]
        got = {"status": ((r >> np.uint64(48)) & np.uint64(0xFF)).astype(np.int8).astype(np.int32),
               "remaining": (r & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32),
               "wait_in_ms": ((r >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16).astype(np.int32)}
        assert_same(got, o, f[sel], ts[sel], f"async batch {b}")
    H.lib().orc_cluster_free(oh)


def _decode(r):
    r = r.view(np.uint64)
    return {"status": ((r >> np.uint64(48)) & np.uint64(0xFF)).astype(np.int8).astype(np.int32),
            "remaining": (r & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32),
            "wait_in_ms": ((r >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16).astype(np.int32)}


@pytest.mark.parametrize("script", ["plain", "interleaved"])
def test_pipelined_entry_matches_sync_and_oracle(eng_mod, script):
    """sga_request_tokens_device_pipelined (batch b + 1's key pass and sorts beside batch b's decisions, two
    scratch sets and dense tables) decides exactly like one sga_request_tokens_device per batch.  "interleaved"
    puts engine calls between the batches -- metric reads (they rotate windows), a batch whose clock goes back
    (the precheck keeps it off the hot path), a rule reload, a host-API batch -- each of which must join the
    pipeline.  Every batch's TokenResults, the metric counters afterwards, and the sampled rules against the
    oracle replaying the same calls."""
    import torch
    from sentinel_amd import _lib
    from sentinel_amd.workload import ClusterTrace
    c = eng_mod
    L = _lib.load()
    dev = torch.device("cuda", 0)
    tr = ClusterTrace(n_rules=200_000, lam=20_000_000)
    fid_r, cnt = tr.rules()
    nb, m = 9, 1 << 19
    host = [tr.events(b * m, m) for b in range(nb)]
    if script == "interleaved":  # batch 5 replays batch 4's times shifted back by 300 ms
        f5, a5, p5, t5 = host[5]
        host[5] = (f5, a5, p5, host[4][3] - 300)
    sample = np.unique(np.concatenate([tr.perm[:8] + 1, np.arange(1, 200_001, 997)])).astype(np.int64)
    res = {}
    for mode in ("sync", "pipe"):
        eng = make_engine(c, hot="on", max_batch=m, max_rules=1 << 18)
        mgr = c.ClusterFlowRuleManager(eng)
        mgr.load_rule_arrays("default", fid_r, cnt)
        svc = c.DefaultTokenService(eng)
        fn = L.sga_request_tokens_device if mode == "sync" else L.sga_request_tokens_device_pipelined
        inp = torch.cuda.Stream(dev)
        keep, outs, extra = [], [], []
        for b, (f, a, p, ts) in enumerate(host):
            base = int(ts.min())
            with torch.cuda.stream(inp):
                d = (torch.from_numpy(f).to(dev), torch.from_numpy(a).to(dev), torch.from_numpy(p).to(dev),
                     torch.from_numpy((ts - base).astype(np.int32)).to(dev))
                o = torch.zeros(m, dtype=torch.int64, device=dev)
            rc = fn(eng.handle, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), base, d[3].data_ptr(), m,
                    o.data_ptr(), C.c_void_p(inp.cuda_stream))
            assert rc == 0, (mode, b, rc, L.sga_last_error(eng.handle))
            keep.append(d)
            outs.append(o)
            if script == "interleaved":
                if b == 2:  # metric reads rotate the sampled rules' windows at a later time
                    extra.append([svc.metric_sums(int(x), int(ts.max()) + 150) for x in sample[:16]])
                if b == 6:  # a reload: every rule kept, half the counts changed
                    cnt2 = cnt.copy()
                    cnt2[::2] = np.maximum(cnt2[::2] // 2, 1)
                    mgr.load_rule_arrays("default", fid_r, cnt2)
                if b == 7:  # a host-API batch between two pipelined ones
                    g = svc.request_tokens(f[:5000], a[:5000], p[:5000], ts[:5000] + 1)
                    extra.append(g["status"].tolist())
        assert L.sga_stream_wait(eng.handle, C.c_void_p(inp.cuda_stream)) == 0
        torch.cuda.synchronize()
        res[mode] = [o.cpu().numpy() for o in outs]
        res[mode + "_extra"] = extra
        res[mode + "_metrics"] = [svc.metric_sums(int(x), int(host[-1][3].max())) for x in sample]
        eng.close()
    for b in range(nb):
        assert np.array_equal(res["sync"][b], res["pipe"][b]), f"batch {b}"
    assert res["sync_extra"] == res["pipe_extra"]
    assert res["sync_metrics"] == res["pipe_metrics"]
    if script == "plain":  # the sampled rules against the oracle
        rules = [{"flow_id": int(x), "count": float(cnt[x - 1]), "threshold_type": 1} for x in sample]
        oh = oracle_cluster({"default": rules})
        for b, (f, a, p, ts) in enumerate(host):
            sel = np.isin(f, sample)
            o = oracle_replay(oh, f[sel], a[sel], p[sel], ts[sel])
            assert_same({k: v[sel] for k, v in _decode(res["pipe"][b]).items()}, o, f[sel], ts[sel],
                        f"pipelined batch {b}")
        H.lib().orc_cluster_free(oh)


def test_coalescing_queue_threads_equal_ticket_order(eng_mod):
    """sga_token_submit / sga_poll from 8 threads at once (the Netty worker pattern of
    FlowRequestProcessor.java:43): every request is decided once, and the decisions and the rules'
    metrics equal the oracle replaying the requests one by one in ticket order."""
    import threading
    c = eng_mod
    rng = np.random.default_rng(77)
    rules = {"default": random_rules(rng, 0, ids=range(1, 41))}
    eng = make_engine(c, max_batch=1 << 12)
    engine_rules(c, eng, rules)
    svc = c.DefaultTokenService(eng)
    n_thr, per = 8, 1500
    got = [[] for _ in range(n_thr)]

    def worker(k):
        r = np.random.default_rng(1000 + k)
        for i in range(per):
            fid = int(r.integers(1, 45))  # some ids without a rule
            acq = int(r.integers(1, 3))
            pr = bool(r.random() < 0.1)
            now = T0 + i  # each thread's clock moves forward; threads interleave
            t = svc.submit(fid, acq, pr, now)
            res = None
            while res is None:
                res = svc.poll(t)
            got[k].append((t, fid, acq, pr, now, res))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(n_thr)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    allr = sorted(x for g in got for x in g)
    assert len(allr) == n_thr * per and len({x[0] for x in allr}) == len(allr)
    oh = oracle_cluster(rules)
    L = H.lib()
    for t, fid, acq, pr, now, res in allr:
        o = L.orc_cluster_request_token(oh, fid, acq, 1 if pr else 0, now)
        assert (res.status, res.remaining, res.wait_in_ms) == (o.status, o.remaining, o.wait_in_ms), (t, fid, now)
    assert_metrics(c, eng, oh, range(1, 41), T0 + per)
    L.orc_cluster_free(oh)
    one = svc.request_token(1, 1, False, T0 + 10_000)
    assert one.status in (0, 1)
    eng.close()


def test_coalescing_queue_bad_request_and_abandoned_tickets(eng_mod):
    """a request the batch would reject (ts < 0) is refused at submit for its caller only, the
    other queued requests are decided; tickets whose callers never poll are reclaimed when the ring wraps
    (a later poll of such a ticket answers EINVAL), so producers never spin forever."""
    from sentinel_amd._lib import EngineError
    c = eng_mod
    rules = {"default": [{"flow_id": 1, "count": 1e9, "threshold_type": 1}]}
    eng = make_engine(c, max_batch=1 << 12)
    engine_rules(c, eng, rules)
    svc = c.DefaultTokenService(eng)
    good = [svc.submit(1, 1, False, T0 + i) for i in range(5)]
    with pytest.raises(EngineError):
        svc.submit(1, 1, False, -5)
    res = [svc.poll(t) for t in good]
    while any(r is None for r in res):
        res = [r if r is not None else svc.poll(t) for r, t in zip(res, good)]
    assert all(r.status == 0 for r in res)
    # abandon a ticket, wrap the ring (65536 slots) with polled requests, then poll the abandoned one
    lost = svc.submit(1, 1, False, T0 + 100)
    cap = 1 << 16
    for k in range(cap + 10):
        t = svc.submit(1, 1, False, T0 + 200 + k // 1000)
        r = None
        while r is None:
            r = svc.poll(t)
    with pytest.raises(EngineError):
        svc.poll(lost)
    eng.close()
