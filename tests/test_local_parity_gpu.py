"""GPU parity of the local path (StatisticSlot + ParamFlowSlot + FlowSlot + DegradeSlot)
against the oracle, through the C-ABI (sga_submit_events / sga_query_node).

Bar: decisions, wait times, node statistics and breaker states bit-identical to the
oracle replay of the same stream (all integer state; derived doubles are computed
from the same integers with the same operations, so they compare exactly too).
"""
import numpy as np
import pytest

from tests import local_trace as lt
from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _engine(max_batch=1 << 16):
    from sentinel_amd.cluster import Engine
    return Engine(max_batch=max_batch)


def _sentinel(n_res, max_batch=1 << 16):
    from sentinel_amd.local import LocalSentinel
    eng = _engine(max_batch)
    return eng, LocalSentinel(eng, [f"r{i}" for i in range(n_res)])


def _load(s, flow=None, param=None, degrade=None):
    from sentinel_amd.local import DegradeRuleManager, FlowRuleManager, ParamFlowRuleManager
    from sentinel_amd.rules import DegradeRule, FlowRule, ParamFlowItem, ParamFlowRule
    if flow is not None:
        from sentinel_amd.rules import ClusterFlowConfig
        FlowRuleManager(s).load_rules([FlowRule(resource=f"r{r['resource']}", count=r["count"], grade=r.get("grade", 1),
                                                control_behavior=r.get("control_behavior", 0),
                                                warm_up_period_sec=r.get("warm_up_period_sec", 10),
                                                max_queueing_time_ms=r.get("max_queueing_time_ms", 500),
                                                cluster_mode=bool(r.get("cluster_mode", False)),
                                                cluster_config=ClusterFlowConfig(
                                                    flow_id=r.get("cluster_flow_id"),
                                                    sample_count=r.get("cluster_sample_count", 10),
                                                    window_interval_ms=r.get("cluster_window_ms", 1000),
                                                    fallback_to_local_when_fail=r.get("cluster_fallback", True)))
                                       for r in flow])
    if param is not None:
        ParamFlowRuleManager(s).load_rules([
            ParamFlowRule(resource=f"r{r['resource']}", grade=r.get("grade", 1), count=r["count"],
                          param_idx=r.get("param_idx", 0), control_behavior=r.get("control_behavior", 0),
                          max_queueing_time_ms=r.get("max_queueing_time_ms", 0), burst_count=r.get("burst_count", 0),
                          duration_in_sec=r.get("duration_in_sec", 1),
                          param_flow_item_list=[ParamFlowItem(int(k), int(v)) for k, v in r.get("hot", {}).items()])
            for r in param])
    if degrade is not None:
        DegradeRuleManager(s).load_rules([
            DegradeRule(resource=f"r{r['resource']}", grade=r.get("grade", 0), count=r["count"],
                        time_window=r.get("time_window", 1), min_request_amount=r.get("min_request_amount", 5),
                        slow_ratio_threshold=r.get("slow_ratio_threshold", 1.0),
                        stat_interval_ms=r.get("stat_interval_ms", 1000))
            for r in degrade])


def _submit(s, st):
    return s.submit(st["kind"], st["resource"], st["ts"], st["acquire"], st["flags"], st["rt"], st["param"])


def _assert_same(st, got, exp, what=""):
    gd, gw = got
    ed, ew = exp
    bad = np.nonzero((gd != ed) | (gw != ew))[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} of {len(gd)} events differ; first at {i}: kind={st['kind'][i]} "
                             f"res={st['resource'][i]} ts={st['ts'][i]} acq={st['acquire'][i]} "
                             f"flags={st['flags'][i]} gpu=({gd[i]},{gw[i]}) oracle=({ed[i]},{ew[i]})")


def _assert_nodes(s, orc, n_res, now):
    for rid in range(n_res):
        v = s.node(rid, now)
        got = [getattr(v, g) for g in lt.NODE_GETTERS]
        exp = orc.node(rid, now)
        assert got == exp, (rid, list(zip(lt.NODE_GETTERS, got, exp)))


def _run(n_res, flow=(), param=(), degrade=(), max_batch=1 << 16, **gen_kw):
    gen = lt.Oracle(n_res, flow, param, degrade)
    st = lt.generate(gen, n_res, t0=T0, **gen_kw)
    gen.close()
    orc = lt.Oracle(n_res, flow, param, degrade)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, max_batch)
    _load(s, list(flow), list(param), list(degrade))
    got = _submit(s, st)
    _assert_same(st, got, exp, "decisions")
    t_end = int(st["ts"].max())
    _assert_nodes(s, orc, n_res, t_end)
    for rid in range(n_res):
        for k in range(4):
            assert s.circuit_breaker_state(rid, k) == orc.cb_state(rid, k), (rid, k)
    orc.close()
    eng.close()
    return st, exp


def test_hello_world_20_qps():
    # README quick start: FlowRule(count=20, QPS) and one entry per ms
    st, (d, _) = _run(1, flow=[{"resource": 0, "count": 20}], n_entries=3000, seed=1, gap_mean=1.0, rt_max=5)
    assert (d[st["kind"] == 0] == 0).sum() > 0


def _random_flow_rules(rng, n_res, thread_ok=True):
    rules = []
    for r in range(n_res):
        k = rng.integers(0, 7)
        nr = 2 if rng.random() < 0.15 else 1
        for _ in range(nr):
            if k == 0 and thread_ok:
                rules.append({"resource": r, "grade": 0, "count": int(rng.integers(1, 6))})
            elif k in (1, 2):
                rules.append({"resource": r, "count": float(rng.choice([5, 10, 20.5, 100]))})
            elif k == 3:
                rules.append({"resource": r, "count": float(rng.choice([10, 50])), "control_behavior": 1,
                              "warm_up_period_sec": int(rng.integers(1, 5))})
            elif k == 4:
                rules.append({"resource": r, "count": float(rng.choice([5, 20, 333])), "control_behavior": 2,
                              "max_queueing_time_ms": int(rng.choice([20, 500]))})
            elif k == 5:
                rules.append({"resource": r, "count": float(rng.choice([10, 40])), "control_behavior": 3,
                              "warm_up_period_sec": 2, "max_queueing_time_ms": 300})
            # k == 6: no rule
    return rules


@pytest.mark.parametrize("seed,max_batch", [(11, 1 << 16), (12, 4096), (13, 1000)])
def test_mixed_controllers(seed, max_batch):
    rng = np.random.default_rng(seed)
    n_res = 40
    flow = _random_flow_rules(rng, n_res)
    _run(n_res, flow=flow, max_batch=max_batch, n_entries=15000, seed=seed, gap_mean=0.4, prio_pct=0.15,
         acq_max=3, err_pct=0.1, rt_max=40, regress_pct=0.01)


@pytest.mark.parametrize("seed", [21, 22])
def test_param_flow(seed):
    rng = np.random.default_rng(seed)
    n_res = 12
    param = []
    for r in range(n_res):
        kind = r % 6
        if kind == 0:
            param.append({"resource": r, "count": 5, "burst_count": int(rng.integers(0, 4))})
        elif kind == 1:
            param.append({"resource": r, "count": 3, "duration_in_sec": 2, "hot": {1: 10, 2: 0}})
        elif kind == 2:
            param.append({"resource": r, "count": 4, "control_behavior": 2, "max_queueing_time_ms": 200})
        elif kind == 3:
            param.append({"resource": r, "grade": 0, "count": 2, "hot": {0: 4}})
        elif kind == 4:
            param.append({"resource": r, "count": 6, "param_idx": -1})
            param.append({"resource": r, "count": 1, "param_idx": 1})  # args.length <= idx: skipped
    flow = [{"resource": r, "count": 30} for r in range(0, n_res, 3)]
    _run(n_res, flow=flow, param=param, n_entries=12000, seed=seed, gap_mean=0.5, acq_max=2, rt_max=30,
         params=5, prio_pct=0.05)


@pytest.mark.parametrize("seed", [23, 24])
def test_param_heavy_resources(seed):
    """Parameter-only resources with thousands of events per batch (k_lheavy): the rule check of
    each event is decided by the lane owning its value, the statistics by one lane in order.
    Token buckets (burst, hot items, duration 2 s), throttling, a thread-grade rule beside them
    (stays on the sequential path), many values, and batches smaller than the stream."""
    n_res = 5
    param = [{"resource": 0, "count": 4, "burst_count": 2},
             {"resource": 1, "count": 3, "duration_in_sec": 2, "hot": {1: 10, 2: 0, 7: 1}},
             {"resource": 2, "count": 5, "control_behavior": 2, "max_queueing_time_ms": 300},
             {"resource": 3, "grade": 0, "count": 2},
             {"resource": 4, "count": 2, "param_idx": -1}]
    for mb in (1 << 16, 6000):
        _run(n_res, param=param, n_entries=30000, seed=seed, gap_mean=0.05, acq_max=2, rt_max=20, params=120,
             max_batch=mb)


@pytest.mark.parametrize("seed", [31, 32])
def test_circuit_breakers(seed):
    n_res = 9
    degrade = []
    for r in range(n_res):
        g = r % 3
        if g == 0:
            degrade.append({"resource": r, "grade": 0, "count": 20, "time_window": 1, "slow_ratio_threshold": 0.4,
                            "min_request_amount": 3, "stat_interval_ms": 1000})
        elif g == 1:
            degrade.append({"resource": r, "grade": 1, "count": 0.3, "time_window": 2, "min_request_amount": 4,
                            "stat_interval_ms": 500})
        else:
            degrade.append({"resource": r, "grade": 2, "count": 3, "time_window": 1, "stat_interval_ms": 2000})
            degrade.append({"resource": r, "grade": 0, "count": 100, "time_window": 3, "slow_ratio_threshold": 1.0})
    flow = [{"resource": 0, "count": 50}, {"resource": 4, "grade": 0, "count": 3}]
    _run(n_res, flow=flow, degrade=degrade, n_entries=10000, seed=seed, gap_mean=0.7, err_pct=0.35, rt_max=60)


@pytest.mark.parametrize("seed", [33, 34])
def test_breaker_heavy_resources(seed):
    """Breaker-only resources with thousands of events per batch (k_lheavy): breakers event by
    event in arrival order, node statistics applied per 500 ms bucket run; slow-RT, error-ratio
    and error-count breakers (two on one resource), batches smaller than the stream."""
    n_res = 4
    degrade = [{"resource": 0, "grade": 0, "count": 25, "time_window": 1, "slow_ratio_threshold": 0.3,
                "min_request_amount": 5, "stat_interval_ms": 1000},
               {"resource": 1, "grade": 1, "count": 0.25, "time_window": 1, "min_request_amount": 4,
                "stat_interval_ms": 500},
               {"resource": 2, "grade": 2, "count": 6, "time_window": 1, "stat_interval_ms": 700},
               {"resource": 2, "grade": 0, "count": 40, "time_window": 2, "slow_ratio_threshold": 0.8},
               {"resource": 3, "grade": 1, "count": 0.5, "time_window": 3, "min_request_amount": 10}]
    for mb in (1 << 16, 5000):
        _run(n_res, degrade=degrade, n_entries=30000, seed=seed, gap_mean=0.05, err_pct=0.3, rt_max=60,
             max_batch=mb)


@pytest.mark.parametrize("seed", [35, 36])
def test_breaker_heavy_open_close_cycles(seed):
    """One breaker per hot resource that trips, stays OPEN, probes HALF_OPEN and closes many times
    within a batch (the C5 pattern): k_lheavy alternates CLOSED bulk parts (entries pass up to the
    tripping exit), OPEN bulk parts (entries blocked up to the retry time, exits only count) and
    lane-0 replays while HALF_OPEN."""
    n_res = 3
    degrade = [{"resource": 0, "grade": 0, "count": 30, "time_window": 1, "slow_ratio_threshold": 0.5,
                "min_request_amount": 5, "stat_interval_ms": 1000},
               {"resource": 1, "grade": 1, "count": 0.3, "time_window": 1, "min_request_amount": 5,
                "stat_interval_ms": 400},
               {"resource": 2, "grade": 2, "count": 10, "time_window": 2, "stat_interval_ms": 1000}]
    for mb in (1 << 16, 3000):
        _run(n_res, degrade=degrade, n_entries=40000, seed=seed, gap_mean=0.02, err_pct=0.3, rt_max=60,
             max_batch=mb)


@pytest.mark.parametrize("seed,regress", [(31, 0.0), (32, 0.002)])
def test_pacing_heavy_resources(seed, regress):
    """RateLimiterController-only resources with thousands of entries per batch go to k_lwave (one wave
    per resource, a ballot finds each window's next passing entry); acquire 1..3 (cost differs per
    entry), queues of 0 / 20 / 500 ms, a zero-count rule (every entry blocks), exits interleaved, and
    clock regressions (those runs take the per-event chain).  Resource 5 is above 2000 QPS: its acquire-1
    entries cost Math.round(1000 / 2500.0) = 0 ms, the zero-cost pacing of C2's bench mix."""
    n_res = 6
    flow = [{"resource": 0, "count": 50.0, "control_behavior": 2, "max_queueing_time_ms": 500},
            {"resource": 1, "count": 7.5, "control_behavior": 2, "max_queueing_time_ms": 20},
            {"resource": 2, "count": 200.0, "control_behavior": 2, "max_queueing_time_ms": 0},
            {"resource": 3, "count": 0.0, "control_behavior": 2, "max_queueing_time_ms": 100},
            {"resource": 4, "count": 1000.0, "control_behavior": 2, "max_queueing_time_ms": 500},
            {"resource": 5, "count": 2500.0, "control_behavior": 2, "max_queueing_time_ms": 500}]
    _run(n_res, flow=flow, max_batch=1 << 15, n_entries=40000, seed=seed, gap_mean=0.05, acq_max=3, rt_max=20,
         err_pct=0.05, regress_pct=regress)


@pytest.mark.parametrize("seed", [41, 42])
def test_pacing_saturated_windows(seed):
    """Saturated RateLimiter resources with tens of thousands of entries per second-run: k_lwave<1> walks
    k_lwsum's window summaries, skipping windows whose costly entries all block and whose zero-cost entries
    pass behind the queue (their waits L - t from the skipped state, k_lresults RUN_WIN).  acquireCount 0
    entries (pass, no state), 1 and 2..6 (cost per entry), rules whose acquire-1 entries cost 0 ms (count
    2500, 4000), 1 ms, 20 ms and a 1 ms queue; arrival rates from 5 to 40 entries per ms; two batches."""
    rng = np.random.default_rng(seed)
    flow = [{"resource": 0, "count": 2500.0, "control_behavior": 2, "max_queueing_time_ms": 500},
            {"resource": 1, "count": 999.0, "control_behavior": 2, "max_queueing_time_ms": 500},
            {"resource": 2, "count": 50.0, "control_behavior": 2, "max_queueing_time_ms": 500},
            {"resource": 3, "count": 4000.0, "control_behavior": 2, "max_queueing_time_ms": 1},
            {"resource": 4, "count": 700.0, "control_behavior": 2, "max_queueing_time_ms": 37}]
    n_res = len(flow)
    n = 160_000
    res = rng.choice(n_res, size=n, p=[0.35, 0.25, 0.15, 0.15, 0.10]).astype(np.uint32)
    ts = T0 + np.sort(rng.integers(0, 4000, size=n)).astype(np.int64)
    u = rng.random(n)
    acq = np.where(u < 0.02, 0, np.where(u < 0.9, 1, rng.integers(2, 7, size=n))).astype(np.int32)
    st = {"kind": np.zeros(n, np.uint8), "resource": res, "ts": ts, "acquire": acq, "flags": np.zeros(n, np.uint8),
          "rt": np.zeros(n, np.int64), "param": np.zeros(n, np.uint64)}
    orc = lt.Oracle(n_res, flow, (), ())
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 17)
    _load(s, flow)
    got = _submit(s, st)
    _assert_same(st, got, exp, "decisions")
    _assert_nodes(s, orc, n_res, int(ts.max()))
    passed = exp[0] == 0
    assert passed.sum() > 1000 and (~passed).sum() > 1000
    orc.close()
    eng.close()


@pytest.mark.parametrize("seed,regress", [(33, 0.0), (34, 0.002)])
def test_mixed_acquire_heavy_resources(seed, regress):
    """DefaultController / WarmUpController resources with thousands of entries per batch and mixed
    acquire counts (no closed form): k_lwave decides each window by one prefix sum up to its first
    block, then a ballot per further pass; prioritized entries and clock regressions keep the
    per-event chain."""
    n_res = 6
    flow = [{"resource": 0, "count": 120.0},
            {"resource": 1, "count": 9.0},
            {"resource": 2, "count": 300.0, "control_behavior": 1, "warm_up_period_sec": 2},
            {"resource": 3, "count": 40.0, "control_behavior": 1, "warm_up_period_sec": 5},
            {"resource": 4, "count": 2000.0}]
    _run(n_res, flow=flow, max_batch=1 << 15, n_entries=40000, seed=seed, gap_mean=0.05, acq_max=4, rt_max=20,
         err_pct=0.05, regress_pct=regress, prio_pct=0.002 if regress else 0.0)


def test_rule_reload_between_batches():
    n_res = 10
    rng = np.random.default_rng(5)
    flow1 = _random_flow_rules(rng, n_res)
    flow2 = _random_flow_rules(rng, n_res)
    deg1 = [{"resource": r, "grade": 2, "count": 2, "time_window": 1} for r in range(n_res)]
    deg2 = deg1[:5] + [{"resource": r, "grade": 1, "count": 0.5, "time_window": 1} for r in range(5, n_res)]
    par1 = [{"resource": r, "count": 3} for r in range(n_res)]
    par2 = par1[::2] + [{"resource": r, "count": 4, "burst_count": 1} for r in range(1, n_res, 2)]
    gen = lt.Oracle(n_res, flow1, par1, deg1)
    s1 = lt.generate(gen, n_res, 4000, 1, T0, gap_mean=0.5, err_pct=0.3, rt_max=20, params=4)
    gen.load(flow2, par2, deg2)
    s2 = lt.generate(gen, n_res, 4000, 2, T0, gap_mean=0.5, err_pct=0.3, rt_max=20, params=4,
                     t_start=int(s1["ts"].max()) + 1)
    gen.close()
    orc = lt.Oracle(n_res, flow1, par1, deg1)
    eng, s = _sentinel(n_res)
    _load(s, flow1, par1, deg1)
    _assert_same(s1, _submit(s, s1), orc.replay(s1), "before reload")
    orc.load(flow2, par2, deg2)
    _load(s, flow2, par2, deg2)
    _assert_same(s2, _submit(s, s2), orc.replay(s2), "after reload")
    _assert_nodes(s, orc, n_res, int(s2["ts"].max()))
    orc.close()
    eng.close()


def _fast_path_stream(n_res, n, seed, rate_per_ms):
    """QPS Default / WarmUp rules only: exits never change a decision, so exits of
    the passed entries can be added after an entries-only oracle replay."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, n_res + 1) ** 1.1
    w /= w.sum()
    res = rng.choice(n_res, size=n, p=w).astype(np.uint32)
    ts = T0 + np.sort(rng.integers(0, int(n / rate_per_ms), size=n)).astype(np.int64)
    ent = {"kind": np.zeros(n, np.uint8), "resource": res, "ts": ts, "acquire": np.ones(n, np.int32),
           "flags": np.zeros(n, np.uint8), "rt": np.zeros(n, np.int64), "param": np.zeros(n, np.uint64)}
    return ent, rng


def test_fast_path_large_stream():
    n_res, n = 4096, 1 << 20
    rng0 = np.random.default_rng(3)
    flow = []
    for r in range(n_res):
        if r % 5 == 4:
            flow.append({"resource": r, "count": float(rng0.integers(5, 200)), "control_behavior": 1,
                         "warm_up_period_sec": int(rng0.integers(1, 4))})
        elif r % 7 != 6:
            flow.append({"resource": r, "count": float(rng0.integers(1, 500))})
    ent, rng = _fast_path_stream(n_res, n, 3, rate_per_ms=200)
    o1 = lt.Oracle(n_res, flow)
    d, _ = o1.replay(ent)
    o1.close()
    passed = np.nonzero(d == 0)[0]
    rt = rng.integers(0, 80, size=len(passed))
    ex = {"kind": np.ones(len(passed), np.uint8), "resource": ent["resource"][passed],
          "ts": ent["ts"][passed] + rt, "acquire": np.ones(len(passed), np.int32),
          "flags": (rng.random(len(passed)) < 0.1).astype(np.uint8) * 2, "rt": rt.astype(np.int64),
          "param": np.zeros(len(passed), np.uint64)}
    st = lt.concat(ent, ex)
    order = np.lexsort((st["kind"], st["ts"]))
    st = {k: v[order] for k, v in st.items()}
    orc = lt.Oracle(n_res, flow)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, max_batch=1 << 20)
    _load(s, flow)
    got = _submit(s, st)
    _assert_same(st, got, exp, "fast path")
    now = int(st["ts"].max())
    for rid in list(range(64)) + list(range(n_res - 64, n_res)):
        v = s.node(rid, now)
        assert [getattr(v, g) for g in lt.NODE_GETTERS] == orc.node(rid, now), rid
    orc.close()
    eng.close()


def test_edge_cases():
    from sentinel_amd import EngineError
    eng, s = _sentinel(3)
    _load(s, [{"resource": 0, "count": 1}])
    d, w = s.submit([], [], [], [])
    assert len(d) == 0
    # unknown resource id: no node, no rules -> pass
    d, w = s.submit([0, 0], [7, 0], [T0, T0], [1, 1])
    assert list(d) == [0, 0]
    d, w = s.submit([0], [0], [T0 + 1], [1])
    assert list(d) == [1]
    with pytest.raises(EngineError):
        s.submit([0], [0], [T0], [-1])
    with pytest.raises(EngineError):
        s.submit([0], [0], [-5], [1])
    # SphU-style API
    from sentinel_amd.local import FlowException
    e = None
    with pytest.raises(FlowException):
        e = s.entry("r0", T0 + 2)
    assert e is None
    ok = s.entry("r1", T0 + 2)
    ok.trace_error()
    ok.exit(T0 + 9)
    v = s.node("r1", T0 + 9)
    assert v.total_exception == 1 and v.total_success == 1 and v.avg_rt == 7.0 and v.cur_thread_num == 0
    eng.close()


@pytest.mark.parametrize("server", [1, 0])
def test_cluster_mode_flow_rules(server):
    """FlowSlot with cluster-mode rules (FlowRuleChecker.passClusterCheck / applyTokenResult /
    fallbackToLocalOrPass, FlowRuleChecker.java:168-230).  server=1: the embedded token server is the
    same engine's cluster path -- OK passes, SHOULD_WAIT passes after waitInMs, BLOCKED blocks,
    NO_RULE_EXISTS (a flowId without a cluster rule) falls back to the local rater or passes;
    server=0: no token service, every cluster rule falls back.  Decisions, wait times, node views and
    the cluster rules' metrics equal the oracle (whose FlowSlot asks its own token server)."""
    from sentinel_amd import cluster as CL
    from sentinel_amd.local import ClusterStateManager
    from tests.test_cluster_parity_gpu import assert_metrics, engine_rules, oracle_cluster
    rng = np.random.default_rng(91 + server)
    n_res = 12
    flow, crules = [], []
    for r in range(n_res):
        fid = 1000 + r
        if r % 3 == 0:
            flow.append({"resource": r, "count": float(rng.choice([5, 20]))})
        else:
            flow.append({"resource": r, "count": float(rng.choice([3, 10])), "cluster_mode": True,
                         "cluster_flow_id": fid, "cluster_fallback": r % 3 == 1,
                         "control_behavior": int(rng.choice([0, 2])), "max_queueing_time_ms": 300})
            if r % 4 != 2:  # the others have no cluster rule: NO_RULE_EXISTS -> fallback
                crules.append({"flow_id": fid, "count": float(rng.choice([4, 15, 40])), "threshold_type": 1})
        if r % 5 == 4:  # a second, local rule after the cluster one
            flow.append({"resource": r, "count": 25.0})
    rules = {"default": crules}
    L = lt.lib()
    gen = lt.Oracle(n_res, flow)
    ohg = oracle_cluster(rules)
    L.orc_flow_set_cluster(gen.h, ohg, server)
    st = lt.generate(gen, n_res, n_entries=12000, seed=17 + server, t0=T0, gap_mean=0.5, prio_pct=0.2,
                     acq_max=2, rt_max=30)
    gen.close()
    orc = lt.Oracle(n_res, flow)
    oh = oracle_cluster(rules)
    L.orc_flow_set_cluster(orc.h, oh, server)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 14)
    engine_rules(CL, eng, rules)
    _load(s, flow)
    if server:
        ClusterStateManager(s).set_to_server()
    got = _submit(s, st)
    _assert_same(st, got, exp, f"cluster-mode rules, server={server}")
    t_end = int(st["ts"].max())
    _assert_nodes(s, orc, n_res, t_end)
    assert_metrics(CL, eng, oh, [c["flow_id"] for c in crules], t_end)
    d = exp[0][st["kind"] == 0]
    assert (d == 0).any() and (d == 1).any()
    H.lib().orc_cluster_free(oh)
    H.lib().orc_cluster_free(ohg)
    orc.close()
    eng.close()


def test_collection_and_array_parameters():
    """ParamFlowChecker.passLocalCheck with a Collection / array argument (ParamFlowChecker.java:79-106):
    every element is checked in order and the entry passes only if all pass (the elements before a
    failing one keep their token updates); ParameterMetric counts a thread for every element and the
    exit releases them (ParameterMetric.java:125-230).  Lists of 0..4 values (SGA_EV_PARAM_LIST),
    single values and entries without arguments are mixed over default, throttle and thread-grade
    rules with hot items; decisions, waits and node views equal the oracle."""
    rng = np.random.default_rng(61)
    n_res, n = 16, 40000
    param = []
    for r in range(n_res):
        k = r % 4
        if k == 0:
            param.append({"resource": r, "count": float(rng.integers(2, 20)), "hot": {3: 50, 7: 1}})
        elif k == 1:
            param.append({"resource": r, "count": float(rng.integers(2, 10)), "control_behavior": 2,
                          "max_queueing_time_ms": int(rng.choice([0, 100]))})
        elif k == 2:
            param.append({"resource": r, "grade": 0, "count": float(rng.integers(1, 4)), "hot": {5: 2}})
        else:
            param.append({"resource": r, "count": float(rng.integers(5, 40)), "burst_count": 3,
                          "duration_in_sec": int(rng.choice([1, 2]))})
    res = rng.integers(0, n_res, size=n)
    ts = T0 + np.sort(rng.integers(0, 20_000, size=n))
    kind = rng.random(n)
    flags = np.zeros(n, np.uint8)
    pv = np.zeros(n, np.uint64)
    values = []
    for i in range(n):
        if kind[i] < 0.35:  # a Collection / array argument
            m = int(rng.integers(0, 5))
            pv[i] = (len(values) << 32) | m
            values.extend(int(x) for x in rng.integers(0, 12, size=m))
            flags[i] = 4 | 16
        elif kind[i] < 0.9:
            pv[i] = int(rng.integers(0, 12))
            flags[i] = 4
    values = np.array(values, dtype=np.uint64)
    gen = lt.Oracle(n_res, [], param)
    st = lt.generate_windows(gen, res, ts, rng.integers(1, 3, size=n), flags, pv, rng.integers(2, 80, size=n),
                             rng.random(n) < 0.05, window_ms=2, param_values=values)
    gen.close()
    orc = lt.Oracle(n_res, [], param)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 14)
    _load(s, param=param)
    got = s.submit(st["kind"], st["resource"], st["ts"], st["acquire"], st["flags"], st["rt"], st["param"],
                   param_values=st["param_values"])
    _assert_same(st, got, exp, "collection parameters")
    _assert_nodes(s, orc, n_res, int(st["ts"].max()))
    d = exp[0][st["kind"] == 0]
    lst = (st["flags"][st["kind"] == 0] & 16) != 0
    assert (d[lst] == 2).any() and (d[lst] == 0).any()
    orc.close()
    eng.close()


def test_event_queue_threads_equal_ticket_order():
    """sga_event_submit / sga_event_poll from 8 threads at once (SphU.entry / Entry.exit from application threads,
    CtSph.java:117-168): each thread enters, waits for its decision, then exits what passed, with argument
    vectors, blocks outside the engine and revokes among them.  Every event is decided once, and the decisions,
    waits and node views equal the oracle replaying all events one by one in ticket order."""
    import threading
    n_res = 12
    flow = [{"resource": r, "count": 8.0, **({"grade": 0, "count": 3} if r % 4 == 1 else {})} for r in range(0, n_res, 2)]
    param = [{"resource": r, "count": 4.0, "param_idx": 0} for r in range(1, n_res, 3)]
    degrade = [{"resource": 3, "grade": 2, "count": 3, "min_request_amount": 3, "time_window": 1}]
    eng, s = _sentinel(n_res, 1 << 12)
    _load(s, flow, param, degrade)
    n_thr, per = 8, 300
    got = [[] for _ in range(n_thr)]

    def worker(k):
        r = np.random.default_rng(500 + k)
        for i in range(per):
            res = int(r.integers(0, n_res))
            now = T0 + 3 * i + int(r.integers(0, 3))
            acq = int(r.integers(1, 3))
            words, fl, pv = None, 8 if r.random() < 0.3 else 0, 0
            u = r.random()
            if u < 0.2:  # a whole argument vector: (scalar v, scalar x) or (list [v, w])
                v = int(r.integers(0, 6))
                args = [v, int(r.integers(0, 100))] if r.random() < 0.7 else [[v, int(r.integers(0, 6))]]
                lw = []
                pv = lt.encode_args(args, lw)
                words, fl = np.array(lw, np.uint64), fl | 32
            elif u < 0.6:
                pv, fl = int(r.integers(0, 6)), fl | 4
            kind = 2 if r.random() < 0.03 else 0
            t = s.event_submit(kind, res, now, acq, fl, 0, pv, words)
            d = None
            while d is None:
                d = s.event_poll(t)
            got[k].append((t, kind, res, now, acq, fl, 0, pv, words, d))
            if kind == 0 and d[0] in (0, 4):  # passed: exit later (or revoked by a later slot)
                rev = r.random() < 0.1
                xt = now if rev else now + int(r.integers(1, 20))
                xfl = (fl & (4 | 8 | 32)) | (2 if (not rev and r.random() < 0.2) else 0)
                xrt = 0 if rev else xt - now
                t2 = s.event_submit(3 if rev else 1, res, xt, acq, xfl, xrt, pv, words)
                d2 = None
                while d2 is None:
                    d2 = s.event_poll(t2)
                got[k].append((t2, 3 if rev else 1, res, xt, acq, xfl, xrt, pv, words, d2))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(n_thr)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    allr = sorted((x for g in got for x in g), key=lambda x: x[0])
    assert len({x[0] for x in allr}) == len(allr)
    orc = lt.Oracle(n_res, flow, param, degrade)
    for (t, kind, res, now, acq, fl, rt, pv, words, d) in allr:
        ev = {"kind": np.array([kind], np.uint8), "resource": np.array([res], np.uint32),
              "ts": np.array([now], np.int64), "acquire": np.array([acq], np.int32),
              "flags": np.array([fl], np.uint8), "rt": np.array([rt], np.int64), "param": np.array([pv], np.uint64)}
        if words is not None:
            ev["param_values"] = words
        ed, ew = orc.replay(ev)
        assert (d[0], d[1]) == (int(ed[0]), int(ew[0])), (t, kind, res, now, fl, d, int(ed[0]), int(ew[0]))
    end = max(x[3] for x in allr) + 1
    _assert_nodes(s, orc, n_res, end)
    kinds = [x[1] for x in allr]
    assert kinds.count(3) > 20 and kinds.count(2) > 20
    orc.close()
    eng.close()


def test_event_post_exits_threads_equal_ticket_order():
    """sga_event_post: 8 threads enter through sga_event_submit / sga_event_poll and post their exits, revokes
    and blocks without waiting (what GpuStatisticSlot's exit path calls).  Every posted event is decided in
    ticket order before the thread's later events; the node views read afterwards (a query waits for the queued
    events) and every entry's decision equal the oracle replaying all events one by one in ticket order."""
    import threading
    n_res = 12
    flow = [{"resource": r, "count": 8.0, **({"grade": 0, "count": 3} if r % 4 == 1 else {})} for r in range(0, n_res, 2)]
    param = [{"resource": r, "count": 4.0, "param_idx": 0} for r in range(1, n_res, 3)]
    degrade = [{"resource": 3, "grade": 2, "count": 3, "min_request_amount": 3, "time_window": 1}]
    eng, s = _sentinel(n_res, 1 << 12)
    _load(s, flow, param, degrade)
    n_thr, per = 8, 300
    got = [[] for _ in range(n_thr)]

    def worker(k):
        r = np.random.default_rng(700 + k)
        for i in range(per):
            res = int(r.integers(0, n_res))
            now = T0 + 3 * i + int(r.integers(0, 3))
            acq = int(r.integers(1, 3))
            words, fl, pv = None, 8 if r.random() < 0.3 else 0, 0
            u = r.random()
            if u < 0.2:
                v = int(r.integers(0, 6))
                args = [v, int(r.integers(0, 100))] if r.random() < 0.7 else [[v, int(r.integers(0, 6))]]
                lw = []
                pv = lt.encode_args(args, lw)
                words, fl = np.array(lw, np.uint64), fl | 32
            elif u < 0.6:
                pv, fl = int(r.integers(0, 6)), fl | 4
            if r.random() < 0.03:  # blocked by a slot before the engine: posted
                t = s.event_post(2, res, now, acq, fl, 0, pv, words)
                got[k].append((t, 2, res, now, acq, fl, 0, pv, words, None))
                continue
            t = s.event_submit(0, res, now, acq, fl, 0, pv, words)
            d = None
            while d is None:
                d = s.event_poll(t)
            got[k].append((t, 0, res, now, acq, fl, 0, pv, words, d))
            if d[0] in (0, 4):  # passed: exit (or revoke), posted
                rev = r.random() < 0.1
                xt = now if rev else now + int(r.integers(1, 20))
                xfl = (fl & (4 | 8 | 32)) | (2 if (not rev and r.random() < 0.2) else 0)
                xrt = 0 if rev else xt - now
                t2 = s.event_post(3 if rev else 1, res, xt, acq, xfl, xrt, pv, words)
                got[k].append((t2, 3 if rev else 1, res, xt, acq, xfl, xrt, pv, words, None))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(n_thr)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    allr = sorted((x for g in got for x in g), key=lambda x: x[0])
    assert len({x[0] for x in allr}) == len(allr)
    orc = lt.Oracle(n_res, flow, param, degrade)
    for (t, kind, res, now, acq, fl, rt, pv, words, d) in allr:
        ev = {"kind": np.array([kind], np.uint8), "resource": np.array([res], np.uint32),
              "ts": np.array([now], np.int64), "acquire": np.array([acq], np.int32),
              "flags": np.array([fl], np.uint8), "rt": np.array([rt], np.int64), "param": np.array([pv], np.uint64)}
        if words is not None:
            ev["param_values"] = words
        ed, ew = orc.replay(ev)
        if d is not None:
            assert (d[0], d[1]) == (int(ed[0]), int(ew[0])), (t, kind, res, now, fl, d, int(ed[0]), int(ew[0]))
    end = max(x[3] for x in allr) + 1
    _assert_nodes(s, orc, n_res, end)  # the node queries wait for the posted events
    kinds = [x[1] for x in allr]
    assert kinds.count(1) > 500 and kinds.count(3) > 20 and kinds.count(2) > 20
    with pytest.raises(Exception):
        s.event_post(0, 0, T0, 1)  # an entry needs its decision
    orc.close()
    eng.close()
