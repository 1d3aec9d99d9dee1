"""CPU checks of the oracle's ClusterParamFlowChecker restatement (oracle/oracle_cparam.c) on
hand-derived sequences of the reference semantics (CS/flow/ClusterParamFlowChecker.java:42-87):
per-value QPS windows, hot-item thresholds, all-or-nothing collections, remaining = -1 for
several values, AVG_LOCAL thresholds scaled by the connected count, validation codes."""
import ctypes as C

import numpy as np
import pytest

from tests import oracle_harness as H

T0 = 1_700_000_000_000


def make(rules, ns="default", conn=None):
    L = H.lib()
    h = L.orc_cluster_new(1.0, 1.0)
    if conn is not None:
        L.orc_cluster_set_connected_count(h, ns.encode(), conn)
    keep = []
    arr = H.cluster_param_rules_array(rules, keep)
    assert L.orc_cluster_load_param_rules(h, ns.encode(), arr, len(rules)) == len(rules)
    return L, h, keep


def req(L, h, fid, acq, values, now):
    v = (C.c_int64 * max(1, len(values)))(*values)
    r = L.orc_cluster_request_param_token(h, fid, acq, v, len(values), now)
    return r.status, r.remaining


def test_per_value_window_and_hot_items():
    L, h, _ = make([{"flow_id": 5, "count": 3, "threshold_type": 1, "hot": {9: 1}}])
    got = [req(L, h, 5, 1, [1], T0 + i) for i in range(4)]
    assert got == [(0, 2), (0, 1), (0, 0), (1, 0)]
    assert [req(L, h, 5, 1, [9], T0 + 10 + i)[0] for i in range(2)] == [0, 1]
    assert req(L, h, 5, 1, [2], T0 + 20) == (0, 2)          # another value has its own window
    assert req(L, h, 5, 1, [1], T0 + 1000) == (0, 2)        # a second later the window rolled
    assert L.orc_cluster_param_sum(h, 5, 1, T0 + 1000) == 1
    L.orc_cluster_free(h)


def test_collections_all_or_nothing():
    L, h, _ = make([{"flow_id": 5, "count": 2, "threshold_type": 1}])
    assert req(L, h, 5, 1, [1, 2], T0) == (0, -1)            # remaining unsupported for several values
    assert req(L, h, 5, 1, [1], T0) == (0, 0)
    assert req(L, h, 5, 1, [2, 1], T0) == (1, 0)             # value 1 exhausted: nothing is added
    assert L.orc_cluster_param_sum(h, 5, 2, T0) == 1
    assert req(L, h, 5, 1, [2, 2], T0) == (0, -1)            # duplicates are added twice
    assert L.orc_cluster_param_sum(h, 5, 2, T0) == 3
    L.orc_cluster_free(h)


def test_avg_local_and_validation():
    L, h, _ = make([{"flow_id": 5, "count": 2, "threshold_type": 0}], conn=0)
    assert req(L, h, 5, 1, [1], T0) == (1, 0)                # 2 x 0 connected clients
    L.orc_cluster_set_connected_count(h, b"default", 2)
    assert req(L, h, 5, 1, [1], T0) == (0, 3)                # 2 x 2 - 0 - 1 (the block added nothing)
    assert req(L, h, 0, 1, [1], T0)[0] == -4
    assert req(L, h, 5, 0, [1], T0)[0] == -4
    assert req(L, h, 5, 1, [], T0)[0] == -4
    assert req(L, h, 6, 1, [1], T0)[0] == 3
    L.orc_cluster_free(h)


def test_replay_matches_single_calls():
    rules = [{"flow_id": f, "count": 4, "threshold_type": 1} for f in (1, 2)]
    L, h1, _ = make(rules)
    _, h2, _ = make(rules)
    rng = np.random.default_rng(3)
    n = 500
    fid = rng.integers(1, 3, size=n).astype(np.int64)
    acq = np.ones(n, np.int32)
    ts = (T0 + np.cumsum(rng.integers(0, 20, size=n))).astype(np.int64)
    off = np.arange(n + 1, dtype=np.uint32)
    vals = rng.integers(0, 5, size=n).astype(np.int64)
    out = (H.OrcTokenResult * n)()
    L.orc_cluster_param_replay(h1, n, fid.ctypes.data, acq.ctypes.data, off.ctypes.data, vals.ctypes.data,
                               ts.ctypes.data, out)
    ref = np.frombuffer(out, dtype=np.int32).reshape(-1, 3)
    for i in range(n):
        assert req(L, h2, int(fid[i]), 1, [int(vals[i])], int(ts[i])) == (ref[i, 0], ref[i, 1])
    L.orc_cluster_free(h1)
    L.orc_cluster_free(h2)


def test_top_values():
    """ClusterParamMetric.getTopValues(number): merged valid buckets, largest first, qps = sum /
    intervalInSecond, zero-count values never listed; equal sums -> smaller value key first."""
    L, h, _ = make([{"flow_id": 11, "count": 100, "threshold_type": 1, "sample_count": 2,
                     "window_interval_ms": 1000}])
    for v, k, t in ((1001, 5, 0), (7, 2, 0), (7, 1, 600), (2, 3, 600), (9, 1, 700)):
        for i in range(k):
            assert req(L, h, 11, 1, [v], T0 + t + i)[0] == 0
    vals, qps = (C.c_int64 * 8)(), (C.c_double * 8)()
    n = L.orc_cluster_param_top_values(h, 11, T0 + 800, 3, vals, qps)
    assert [(vals[i], qps[i]) for i in range(n)] == [(1001, 5.0), (2, 3.0), (7, 3.0)]
    n = L.orc_cluster_param_top_values(h, 11, T0 + 1200, 8, vals, qps)  # first bucket deprecated
    assert [(vals[i], qps[i]) for i in range(n)] == [(2, 3.0), (7, 1.0), (9, 1.0)]
    assert L.orc_cluster_param_top_values(h, 11, T0 + 5000, 8, vals, qps) == 0
    assert L.orc_cluster_param_top_values(h, 99, T0, 8, vals, qps) == 0  # no metric
    L.orc_cluster_free(h)


def test_bucket_map_lru_small_capacity():
    """Each bucket map is a strict LRU (ClusterParamMetric.java:37-88): capacity 3, one bucket, count 2.
    getSum's get and addValue's putIfAbsent are accesses; a new value into a full map evicts the least
    recently accessed one, whose count is gone (hand-derived sequence)."""
    L = H.lib()
    L.orc_cluster_set_param_capacity(3)
    try:
        L2, h, _ = make([{"flow_id": 5, "count": 2, "threshold_type": 1, "sample_count": 1,
                          "window_interval_ms": 1000}])
    finally:
        L.orc_cluster_set_param_capacity(0)
    seq = [1, 2, 3, 1, 4, 2, 1, 5, 4, 3, 1]
    got = [req(L, h, 5, 1, [v], T0 + i) for i, v in enumerate(seq)]
    # t3: value 1 read+added (order 2,3,1); t4: 4 evicts 2; t5: 2 is new again (evicts 3);
    # t6: value 1 at 2 -> blocked, but its get moves it to the MRU end; t7: 5 evicts 4; t8: 4 evicts 2;
    # t9: 3 evicts 1; t10: value 1 is new again
    assert got == [(0, 1), (0, 1), (0, 1), (0, 0), (0, 1), (0, 1), (1, 0), (0, 1), (0, 1), (0, 1), (0, 1)]
    assert [L.orc_cluster_param_sum(h, 5, v, T0 + 20) for v in (1, 2, 3, 4, 5)] == [1, 0, 1, 1, 0]
    L.orc_cluster_free(h)


@pytest.mark.parametrize("name", ["exhaust_then_evict", "exhaust_no_evict_at_capacity", "blocked_get_moves_to_mru",
                                  "two_buckets", "random_stream"])
def test_lru_golden_vectors(name):
    """The oracle's bucket maps (capacity 4000) against the independent strict-LRU model's vectors
    (tests/golden/make_cparam_lru_golden.py)."""
    doc = load_lru_golden(name)
    L, h, _ = make([golden_rule(doc)])
    ev = doc["events"]
    n = len(ev)
    fid = np.full(n, doc["flow_id"], np.int64)
    acq = np.full(n, doc["acquire"], np.int32)
    ts = np.array([t for _, t in ev], np.int64)
    off = np.arange(n + 1, dtype=np.uint32)
    vals = np.array([v for v, _ in ev], np.int64)
    out = (H.OrcTokenResult * n)()
    L.orc_cluster_param_replay(h, n, fid.ctypes.data, acq.ctypes.data, off.ctypes.data, vals.ctypes.data,
                               ts.ctypes.data, out)
    ref = np.frombuffer(out, dtype=np.int32).reshape(-1, 3)[:, :2]
    exp = np.array(doc["expect"], np.int32)
    bad = np.nonzero((ref != exp).any(axis=1))[0]
    assert bad.size == 0, (name, bad[:5], ref[bad[:5]], exp[bad[:5]])
    for v, t, s in doc["sums"]:
        assert L.orc_cluster_param_sum(h, doc["flow_id"], v, t) == s, (v, t, s)
    L.orc_cluster_free(h)


def load_lru_golden(name):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", f"cparamlru_{name}.json")) as fh:
        return json.load(fh)


def golden_rule(doc):
    r = doc["rule"]
    return {"flow_id": doc["flow_id"], "count": float(r["count"]), "threshold_type": 1,
            "sample_count": r["sample_count"], "window_interval_ms": r["window_interval_ms"],
            "hot": {int(k): v for k, v in r.get("hot", {}).items()}}
