"""GPU parity of the device-resident Envoy RLS entry (sga_rls_should_rate_limit_device) against the
oracle's SimpleClusterFlowChecker replay (SentinelEnvoyRlsServiceImpl.shouldRateLimit,
envoy/rls/SentinelEnvoyRlsServiceImpl.java:52-90): per descriptor status and remaining, per request
the response code, over several batches (the clock continues), with hitsAddend 0 (counts as 1) and
negative (onError: nothing checked, code -1) requests and descriptors without a rule."""
import numpy as np
import pytest

from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def test_rls_device_matches_oracle():
    import torch
    from sentinel_amd import cluster
    rng = np.random.default_rng(107)
    n_rules = 5000
    fids = np.arange(1, n_rules + 1, dtype=np.int64) * 7919 + 2147483647
    counts = rng.integers(5, 200, size=n_rules)
    eng = cluster.Engine(max_batch=1 << 16)
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fids, counts, threshold_type=1, sample_count=1)
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    arr = H.cluster_rules_array([{"flow_id": int(f), "count": float(c), "threshold_type": 1, "sample_count": 1}
                                 for f, c in zip(fids, counts)])
    L.orc_cluster_load_rules(oh, b"default", arr, n_rules)
    svc = cluster.EnvoyRlsService(eng)
    dev = torch.device("cuda", 0)
    p = 1.0 / np.arange(1, n_rules + 1) ** 1.1
    p /= p.sum()
    t = T0
    for batch in range(4):
        nreq = int(rng.integers(1000, 6000))
        ndesc = rng.integers(1, 5, size=nreq)
        off = np.concatenate([[0], np.cumsum(ndesc)]).astype(np.uint32)
        dfid = fids[rng.choice(n_rules, size=int(off[-1]), p=p)]
        dfid[rng.random(len(dfid)) < 0.02] = 42  # no rule
        hits = rng.integers(0, 4, size=nreq).astype(np.int32)
        hits[rng.random(nreq) < 0.01] = -1
        ts = t + np.sort(rng.integers(0, 1500, size=nreq)).astype(np.int64)
        t = int(ts.max()) + 1
        base = int(ts.min())
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        code, st, rem = svc.should_rate_limit_device(T(off.view(np.int32)), T(dfid), T(hits), base,
                                                     T((ts - base).astype(np.uint32).view(np.int32)))
        torch.cuda.synchronize()
        # oracle: every descriptor of a checked request is one SimpleClusterFlowChecker call
        chk = np.repeat(hits >= 0, ndesc)
        acq = np.repeat(np.where(hits <= 0, 1, hits), ndesc).astype(np.int32)
        dts = np.repeat(ts, ndesc).astype(np.int64)
        sel = np.nonzero(chk)[0]
        f_s, a_s, t_s = (np.ascontiguousarray(x[sel]) for x in (dfid, acq, dts))
        out = (H.OrcTokenResult * max(1, len(sel)))()
        L.orc_cluster_replay_simple(oh, len(sel), f_s.ctypes.data, a_s.ctypes.data, t_s.ctypes.data, out)
        exp = np.frombuffer(out, dtype=np.dtype([("status", np.int32), ("remaining", np.int32), ("wait", np.int32)]))
        es = np.full(len(dfid), 3, np.int64)  # skipped descriptors: NO_RULE_EXISTS, remaining 0
        er = np.zeros(len(dfid), np.int64)
        es[sel] = exp["status"][:len(sel)]
        er[sel] = exp["remaining"][:len(sel)]
        assert np.array_equal(st.cpu().numpy().astype(np.int64), es), batch
        assert np.array_equal(rem.cpu().numpy().astype(np.int64), er), batch
        blocked = np.add.reduceat((es != 0) & (es != 3), off[:-1].astype(np.int64)) > 0
        want = np.where(hits < 0, -1, np.where(blocked, 2, 1))
        assert np.array_equal(code.cpu().numpy(), want), batch
        assert blocked.any() and (~blocked).any()
    L.orc_cluster_free(oh)
    eng.close()
