"""CPU checks of the oracle's ClusterParamFlowChecker restatement (oracle/oracle_cparam.c) on
hand-derived sequences of the reference semantics (CS/flow/ClusterParamFlowChecker.java:42-87):
per-value QPS windows, hot-item thresholds, all-or-nothing collections, remaining = -1 for
several values, AVG_LOCAL thresholds scaled by the connected count, validation codes."""
import ctypes as C

import numpy as np

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
