"""BASELINE.json configurations C1, C2, C4 and C5 at their stated sizes on the GPU, bit-exact against
the oracle replay of the same stream (C3 is test_c3_full_size_* in
test_cluster_parity_gpu.py).

Streams are generated window by window (tests/local_trace.generate_windows): entries are decided by a
generator oracle, the ones that pass exit later with a response time (and an error flag), so exits
follow real entries as StatisticSlot.exit does.  The engine then replays the whole stream through the
C-ABI in max_batch chunks and a fresh oracle replays it in one pass; decisions and wait times of every
event, every resource's MetricNode rows (StatisticNode.metrics at the end), the node views of the
hottest resources and every breaker's state must be equal.

  C1  HelloWorld: one resource, QPS FlowRule count 20, DefaultController, 1M entries (~1 per ms).
  C2  100k FlowRules 40 % DefaultController / 30 % RateLimiter / 30 % WarmUp over 100k resources,
      Zipf(1.1) traffic, 2^22 entries with exits, 5 % of them acquiring 2..5.
  C4  10k ParamFlowRules (90 % QPS default / 10 % throttle), Zipf parameter values over 10M folded to at
      most 4000 distinct values per rule (inside the CacheMap capacity min(4000 * duration, 200000), so
      the reference's map never evicts: the pinned mode of SURVEY.md 8(d)).
  C5  (a) Envoy RLS: 100k descriptor rules, requests of 1..4 descriptors, SimpleClusterFlowChecker per
      descriptor; (b) DegradeSlot: 10k DegradeRules, 50 % slow-RT / 50 % exception-ratio breakers,
      log-normal response times, 5 % errors.
"""
import numpy as np
import pytest

from tests import local_trace as lt
from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _zipf(rng, n_items, size, s=1.1):
    p = 1.0 / np.arange(1, n_items + 1) ** s
    p /= p.sum()
    return rng.choice(n_items, size=size, p=p)


def _local(n_res, flow=(), param=(), degrade=(), max_batch=1 << 20):
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import LocalSentinel
    from tests.test_local_parity_gpu import _load
    eng = Engine(max_batch=max_batch)
    s = LocalSentinel(eng, [f"r{i}" for i in range(n_res)])
    _load(s, flow=list(flow) or None, param=list(param) or None, degrade=list(degrade) or None)
    return eng, s


def _check_local(n_res, st, flow=(), param=(), degrade=(), max_batch=1 << 20, hot_nodes=64):
    orc = lt.Oracle(n_res, list(flow), list(param), list(degrade))
    exp_d, exp_w = orc.replay(st)
    eng, s = _local(n_res, flow, param, degrade, max_batch)
    n = len(st["kind"])
    got_d = np.zeros(n, np.int8)
    got_w = np.zeros(n, np.int32)
    for lo in range(0, n, max_batch):  # the engine sees the stream in max_batch chunks
        sub = {k: np.ascontiguousarray(v[lo:lo + max_batch]) for k, v in st.items()}
        d, w = s.submit(sub["kind"], sub["resource"], sub["ts"], sub["acquire"], sub["flags"], sub["rt"],
                        sub["param"])
        got_d[lo:lo + len(d)] = d
        got_w[lo:lo + len(w)] = w
    bad = np.nonzero((got_d != exp_d) | (got_w != exp_w))[0]
    assert len(bad) == 0, (f"{len(bad)} of {n} events differ; first at {bad[0]}: kind={st['kind'][bad[0]]} "
                           f"res={st['resource'][bad[0]]} gpu=({got_d[bad[0]]},{got_w[bad[0]]}) "
                           f"oracle=({exp_d[bad[0]]},{exp_w[bad[0]]})")
    now = int(st["ts"].max()) + 1
    got = [(m.timestamp, s.resource_id(m.resource), m.pass_qps, m.block_qps, m.success_qps, m.exception_qps, m.rt,
            m.occupied_pass_qps) for m in s.metrics(now, cap=1 << 20)]
    exp = orc.metrics(now, cap=1 << 20)
    assert got == exp, (len(got), len(exp))
    hot = np.argsort(-np.bincount(st["resource"].astype(np.int64), minlength=n_res))[:hot_nodes]
    for rid in hot:
        v = s.node(int(rid), now)
        assert [getattr(v, g) for g in lt.NODE_GETTERS] == orc.node(int(rid), now), int(rid)
    if degrade:
        for r in degrade:
            rid = r["resource"]
            assert s.circuit_breaker_state(rid, 0) == orc.cb_state(rid, 0), rid
    orc.close()
    eng.close()
    return exp_d


def test_c1_hello_world_1m_entries():
    rng = np.random.default_rng(101)
    n = 1_000_000
    flow = [{"resource": 0, "count": 20.0}]
    ts = T0 + np.cumsum(rng.integers(0, 3, size=n))  # ~1 entry per ms
    gen = lt.Oracle(1, flow)
    st = lt.generate_windows(gen, np.zeros(n), ts, np.ones(n), np.zeros(n, np.uint8), np.zeros(n, np.uint64),
                             rng.integers(5, 60, size=n), rng.random(n) < 0.02, window_ms=5)
    gen.close()
    d = _check_local(1, st, flow=flow, max_batch=1 << 20)
    ent = st["kind"] == 0
    assert (d[ent] == 0).sum() > 10_000 and (d[ent] == 1).sum() > 100_000  # 20 QPS passes, the rest blocks


def test_c2_100k_mixed_controllers_zipf():
    rng = np.random.default_rng(102)
    n_res, n = 100_000, 1 << 22
    flow = []
    for r in range(n_res):
        u = r % 10
        if u < 4:
            flow.append({"resource": r, "count": float(rng.integers(5, 500))})
        elif u < 7:
            flow.append({"resource": r, "count": float(rng.integers(5, 500)), "control_behavior": 2,
                         "max_queueing_time_ms": int(rng.choice([20, 500]))})
        else:
            flow.append({"resource": r, "count": float(rng.integers(5, 500)), "control_behavior": 1,
                         "warm_up_period_sec": int(rng.integers(1, 11))})
    res = _zipf(rng, n_res, n)
    ts = T0 + (np.arange(n) // 1000)  # 1M entries per virtual second
    acq = np.where(rng.random(n) < 0.05, rng.integers(2, 6, size=n), 1)
    gen = lt.Oracle(n_res, flow)
    st = lt.generate_windows(gen, res, ts, acq, np.zeros(n, np.uint8), np.zeros(n, np.uint64),
                             rng.integers(1, 40, size=n), rng.random(n) < 0.01, window_ms=1)
    gen.close()
    d = _check_local(n_res, st, flow=flow, max_batch=1 << 21)
    ent = st["kind"] == 0
    assert (d[ent] == 0).any() and (d[ent] == 1).any() and (st["kind"] == 1).sum() > 100_000


@pytest.mark.parametrize("log_n", [22, 24])
def test_c2_bench_mix_bit_exact(log_n):
    """bench.py --config c2's own mix (bench_local._cfg_c2): count U{5..5000} -- RateLimiter rules above
    2000 QPS pace acquire-1 entries at zero cost in k_lwave --, lambda 10^7 entries per virtual second,
    WarmUp 10 s, maxQueueingTimeMs 500, 5 % acquiring 2..5, at 2^22 entries per batch and at the bench's own
    2^24 (the hottest resources' later windows, k_lwave's grid at the benched batch size).  As the bench does:
    one batch of entries, then the exits of the entries that passed (exit time = entry time + a geometric
    RT), on the engine and on the oracle; every decision and wait equal, then the metric rows and the
    hottest nodes."""
    import bench_local as bl
    rng = np.random.default_rng(102)
    cfg = bl._cfg_c2(rng, n=1 << log_n)
    b = cfg["batch"]
    n_res, flow = cfg["n_res"], cfg["flow"]
    ent = {"kind": np.zeros(b.n, np.uint8), "resource": b.res, "ts": b.ts, "acquire": b.acq, "flags": b.flags,
           "rt": np.zeros(b.n, np.int64), "param": b.param}
    orc = lt.Oracle(n_res, flow)
    exp_d, exp_w = orc.replay({k: np.ascontiguousarray(v) for k, v in ent.items()})
    eng, s = _local(n_res, flow, max_batch=b.n)
    d, w = s.submit(ent["kind"], ent["resource"], ent["ts"], ent["acquire"], ent["flags"], ent["rt"], ent["param"])
    bad = np.nonzero((d != exp_d) | (w != exp_w))[0]
    assert len(bad) == 0, (f"{len(bad)} of {b.n} entries differ; first at {bad[0]}: res={b.res[bad[0]]} "
                           f"gpu=({d[bad[0]]},{w[bad[0]]}) oracle=({exp_d[bad[0]]},{exp_w[bad[0]]})")
    rl0 = [r["resource"] for r in flow if r.get("control_behavior") == 2 and r["count"] > 2000]
    assert np.isin(b.res, rl0).sum() > 10_000  # the zero-cost pacing path saw real traffic
    passed = (exp_d == 0) | (exp_d == 4)
    k = np.nonzero(passed[b.exit_of])[0]  # exits in exit-time order, of the entries that passed
    e = b.exit_of[k]
    ex = {"kind": np.ones(len(k), np.uint8), "resource": b.res[e], "ts": b.exit_ts[k], "acquire": b.acq[e],
          "flags": b.exit_flags[k], "rt": b.exit_rt[k], "param": b.param[e]}
    ex = {k: np.ascontiguousarray(v) for k, v in ex.items()}
    exp_xd, _ = orc.replay(ex)
    xd, _ = s.submit(ex["kind"], ex["resource"], ex["ts"], ex["acquire"], ex["flags"], ex["rt"], ex["param"])
    assert (xd == exp_xd).all()
    now = int(max(b.ts.max(), ex["ts"].max())) + 1
    got = [(m.timestamp, s.resource_id(m.resource), m.pass_qps, m.block_qps, m.success_qps, m.exception_qps, m.rt,
            m.occupied_pass_qps) for m in s.metrics(now, cap=1 << 20)]
    assert got == orc.metrics(now, cap=1 << 20)
    hot = np.argsort(-np.bincount(b.res.astype(np.int64), minlength=n_res))[:64]
    for rid in hot:
        v = s.node(int(rid), now)
        assert [getattr(v, g) for g in lt.NODE_GETTERS] == orc.node(int(rid), now), int(rid)
    orc.close()
    eng.close()


def test_c4_10k_param_rules_pinned():
    rng = np.random.default_rng(104)
    n_res, n = 10_000, 1 << 22
    param = [{"resource": r, "count": float(rng.integers(1, 100)),
              **({"control_behavior": 2, "max_queueing_time_ms": int(rng.choice([0, 50, 200]))} if r % 10 == 9 else {})}
             for r in range(n_res)]
    res = _zipf(rng, n_res, n)
    vals = _zipf(rng, 10_000_000, n) % 4000  # at most 4000 distinct values per rule: no CacheMap eviction
    ts = T0 + (np.arange(n) // 1000)
    gen = lt.Oracle(n_res, [], param)
    st = lt.generate_windows(gen, res, ts, np.ones(n), np.full(n, 4, np.uint8), vals.astype(np.uint64),
                             rng.integers(1, 30, size=n), np.zeros(n, bool), window_ms=1)
    gen.close()
    d = _check_local(n_res, st, param=param, max_batch=1 << 21)
    ent = st["kind"] == 0
    assert (d[ent] == 0).any() and (d[ent] == 2).any()  # ParamFlowException blocks happen


def test_c5b_10k_degrade_rules_lognormal_rt():
    rng = np.random.default_rng(105)
    n_res, n = 10_000, 1 << 21
    degrade = [{"resource": r, "grade": 0 if r % 2 == 0 else 1, "count": 50.0 if r % 2 == 0 else 0.3,
                "time_window": int(rng.integers(1, 4)), "min_request_amount": 5, "slow_ratio_threshold": 0.5,
                "stat_interval_ms": 1000} for r in range(n_res)]
    res = _zipf(rng, n_res, n)
    ts = T0 + (np.arange(n) // 1000)
    rt = np.clip(np.round(rng.lognormal(mean=3.0, sigma=1.0, size=n)), 1, 5000).astype(np.int64)
    gen = lt.Oracle(n_res, [], [], degrade)
    st = lt.generate_windows(gen, res, ts, np.ones(n), np.zeros(n, np.uint8), np.zeros(n, np.uint64), rt,
                             rng.random(n) < 0.05, window_ms=1)
    gen.close()
    d = _check_local(n_res, st, degrade=degrade, max_batch=1 << 20)
    ent = st["kind"] == 0
    assert (d[ent] == 3).any() and (d[ent] == 0).any()  # breakers open and close


def test_c5b_bench_config_full_batch_two_steps():
    """bench.py --config c5b at its benched size: 2^22 entries, then the exits of the passed ones in time order,
    for two steps (the second 2^22 later in time).  Most flows are breaker-only and one-sided per batch, so the
    long ones go over the whole GPU in tiles (k_cbt_*) and the short ones to one-wave k_cb_flows<1>.  Every
    decision and wait, the metric rows, the hottest nodes and every breaker's state equal the oracle's replay."""
    import bench_local as bl
    bl.SHARD = (0, 1)
    rng = np.random.default_rng(107)
    cfg = bl._cfg_c5b(rng)
    b = cfg["batch"]
    n_res, degrade = cfg["n_res"], cfg["degrade"]
    orc = lt.Oracle(n_res, [], [], degrade)
    eng, s = _local(n_res, degrade=degrade, max_batch=b.n)
    span = b.t_hi - b.t_lo + 1
    blocked = 0
    for step in range(2):
        off = step * span
        ent = {"kind": np.zeros(b.n, np.uint8), "resource": b.res, "ts": b.ts + off, "acquire": b.acq,
               "flags": b.flags, "rt": np.zeros(b.n, np.int64), "param": b.param}
        ent = {k: np.ascontiguousarray(v) for k, v in ent.items()}
        exp_d, exp_w = orc.replay(ent)
        d, w = s.submit(ent["kind"], ent["resource"], ent["ts"], ent["acquire"], ent["flags"], ent["rt"], ent["param"])
        bad = np.nonzero((d != exp_d) | (w != exp_w))[0]
        assert len(bad) == 0, (f"step {step}: {len(bad)} of {b.n} entries differ; first at {bad[0]}: "
                               f"res={b.res[bad[0]]} gpu=({d[bad[0]]},{w[bad[0]]}) oracle=({exp_d[bad[0]]},{exp_w[bad[0]]})")
        blocked += int((exp_d == 3).sum())
        k = np.nonzero(exp_d[b.exit_of] == 0)[0]  # the passed entries' exits, in time order
        e = b.exit_of[k]
        ex = {"kind": np.ones(len(k), np.uint8), "resource": b.res[e], "ts": b.exit_ts[k] + off, "acquire": b.acq[e],
              "flags": b.exit_flags[k], "rt": b.exit_rt[k], "param": b.param[e]}
        ex = {kk: np.ascontiguousarray(v) for kk, v in ex.items()}
        exp_xd, _ = orc.replay(ex)
        xd, _ = s.submit(ex["kind"], ex["resource"], ex["ts"], ex["acquire"], ex["flags"], ex["rt"], ex["param"])
        assert (xd == exp_xd).all(), step
    assert blocked > 0  # breakers open
    now = int(b.t_hi + span) + 1
    got = [(m.timestamp, s.resource_id(m.resource), m.pass_qps, m.block_qps, m.success_qps, m.exception_qps, m.rt,
            m.occupied_pass_qps) for m in s.metrics(now, cap=1 << 20)]
    assert got == orc.metrics(now, cap=1 << 20)
    hot = np.argsort(-np.bincount(b.res.astype(np.int64), minlength=n_res))[:64]
    for rid in hot:
        v = s.node(int(rid), now)
        assert [getattr(v, g) for g in lt.NODE_GETTERS] == orc.node(int(rid), now), int(rid)
    for r in degrade:
        assert s.circuit_breaker_state(r["resource"], 0) == orc.cb_state(r["resource"], 0), r["resource"]
    orc.close()
    eng.close()


def test_c5a_rls_100k_descriptors():
    from sentinel_amd import cluster
    rng = np.random.default_rng(106)
    n_rules, nreq = 100_000, 1 << 20
    fids = np.arange(1, n_rules + 1, dtype=np.int64) * 7919 + 2147483647
    counts = rng.integers(10, 1000, size=n_rules)
    eng = cluster.Engine(max_batch=1 << 22)
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fids, counts, threshold_type=1, sample_count=1)
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    arr = H.cluster_rules_array([{"flow_id": int(f), "count": float(c), "threshold_type": 1, "sample_count": 1}
                                 for f, c in zip(fids, counts)])
    L.orc_cluster_load_rules(oh, b"default", arr, n_rules)
    ndesc = rng.integers(1, 5, size=nreq)
    off = np.concatenate([[0], np.cumsum(ndesc)]).astype(np.uint32)
    dfid = fids[_zipf(rng, n_rules, int(off[-1]))]
    dfid[rng.random(len(dfid)) < 0.01] = 42  # descriptors without a rule: NO_RULE_EXISTS answers OK
    hits = rng.integers(0, 4, size=nreq).astype(np.int32)  # hitsAddend 0 counts as 1
    ts = T0 + (np.arange(nreq) // 500)
    svc = cluster.EnvoyRlsService(eng)
    code, st, rem = svc.should_rate_limit(off, dfid, hits, ts, with_remaining=True)
    acq = np.repeat(np.where(hits == 0, 1, hits), ndesc).astype(np.int32)
    dts = np.repeat(ts, ndesc).astype(np.int64)
    out = (H.OrcTokenResult * len(dfid))()
    L.orc_cluster_replay_simple(oh, len(dfid), dfid.ctypes.data, acq.ctypes.data, dts.ctypes.data, out)
    exp = np.frombuffer(out, dtype=np.dtype([("status", np.int32), ("remaining", np.int32), ("wait", np.int32)]))
    es = exp["status"].astype(np.int64)
    er = exp["remaining"].astype(np.int64)
    assert np.array_equal(np.asarray(st, np.int64), es)
    assert np.array_equal(np.asarray(rem, np.int64), er)
    blocked = np.add.reduceat((es != 0) & (es != 3), off[:-1].astype(np.int64)) > 0
    assert np.array_equal(np.asarray(code), np.where(blocked, 2, 1))
    assert blocked.any() and (~blocked).any()
    L.orc_cluster_free(oh)
    eng.close()


def test_c4args_vectors_blocks_revokes_full_batch():
    """bench.py --config c4args at its benched size (2^22 entries): C4 pinned with 5 % whole argument vectors
    (SGA_EV_ARGS, the exits the same), 0.1 % blocks by a slot before the engine (kind 2) and 0.2 % of the passed
    entries revoked (kind 3 at the entry's time).  None of them sends the chunk to the one-lane replay: the vectors
    are restated as their one value, the blocks and revokes join the per-value segments (ParamFlowChecker.java
    :48-130, StatisticSlot.java:121-135).  Every decision and wait, the metric rows and the hottest nodes equal
    the oracle's replay."""
    import bench_local as bl
    bl.SHARD = (0, 1)
    rng = np.random.default_rng(104)
    cfg = bl._cfg_c4args(rng)
    b = cfg["batch"]
    n_res, param = cfg["n_res"], cfg["param"]
    ent = {"kind": b.kind, "resource": b.res, "ts": b.ts, "acquire": b.acq, "flags": b.flags,
           "rt": np.zeros(b.n, np.int64), "param": b.param, "param_values": b.pvals}
    ent = {k: np.ascontiguousarray(v) for k, v in ent.items()}
    orc = lt.Oracle(n_res, [], param)
    exp_d, exp_w = orc.replay(ent)
    eng, s = _local(n_res, param=param, max_batch=b.n)
    d, w = s.submit(ent["kind"], ent["resource"], ent["ts"], ent["acquire"], ent["flags"], ent["rt"], ent["param"],
                    ent["param_values"])
    bad = np.nonzero((d != exp_d) | (w != exp_w))[0]
    assert len(bad) == 0, (f"{len(bad)} of {b.n} entries differ; first at {bad[0]}: res={b.res[bad[0]]} "
                           f"kind={b.kind[bad[0]]} flags={b.flags[bad[0]]} gpu=({d[bad[0]]},{w[bad[0]]}) "
                           f"oracle=({exp_d[bad[0]]},{exp_w[bad[0]]})")
    passed = ((exp_d == 0) | (exp_d == 4)) & (b.kind != 2)
    k = np.nonzero(passed[b.exit_of])[0]  # exits (and revokes) in time order, of the entries that passed
    e = b.exit_of[k]
    ex = {"kind": b.exit_kind[k], "resource": b.res[e], "ts": b.exit_ts[k], "acquire": b.acq[e],
          "flags": b.exit_flags[k], "rt": b.exit_rt[k], "param": b.param[e], "param_values": b.pvals}
    ex = {kk: np.ascontiguousarray(v) for kk, v in ex.items()}
    assert (ex["kind"] == 3).sum() > 1000 and (b.kind == 2).sum() > 1000 and (b.flags & 32).any()
    exp_xd, _ = orc.replay(ex)
    xd, _ = s.submit(ex["kind"], ex["resource"], ex["ts"], ex["acquire"], ex["flags"], ex["rt"], ex["param"],
                     ex["param_values"])
    assert (xd == exp_xd).all()
    now = int(max(b.ts.max(), ex["ts"].max())) + 1
    got = [(m.timestamp, s.resource_id(m.resource), m.pass_qps, m.block_qps, m.success_qps, m.exception_qps, m.rt,
            m.occupied_pass_qps) for m in s.metrics(now, cap=1 << 20)]
    assert got == orc.metrics(now, cap=1 << 20)
    hot = np.argsort(-np.bincount(b.res.astype(np.int64), minlength=n_res))[:64]
    for rid in hot:
        v = s.node(int(rid), now)
        assert [getattr(v, g) for g in lt.NODE_GETTERS] == orc.node(int(rid), now), int(rid)
    ent_d = exp_d[b.kind == 0]
    assert (ent_d == 0).any() and (ent_d == 2).any()
    orc.close()
    eng.close()
