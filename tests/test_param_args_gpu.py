"""GPU parity of ParamFlowSlot over whole argument vectors (SGA_EV_ARGS, a16) and of cluster-mode parameter
rules decided by the embedded token server, against the oracle (tests/test_param_args_oracle.py pins the
oracle's restatement of ParamFlowSlot.java:56-92 / ParamFlowChecker.java:48-130,305-343 by hand-derived
cases).  Decisions, waits and every node view must be identical."""
import numpy as np
import pytest

from tests import local_trace as lt
from tests import oracle_harness as H
from tests.test_local_parity_gpu import T0, _assert_nodes, _assert_same, _load, _sentinel, _submit

pytestmark = pytest.mark.gpu


def _submit_args(s, st):
    return s.submit(st["kind"], st["resource"], st["ts"], st["acquire"], st["flags"], st["rt"], st["param"],
                    st["param_values"])


def _rules(rng, n_res):
    rules = []
    for r in range(n_res):
        kind = r % 6
        if kind == 0:
            rules.append({"resource": r, "count": float(rng.integers(2, 6)), "param_idx": 1})
        elif kind == 1:
            rules.append({"resource": r, "count": float(rng.integers(2, 6)), "param_idx": -1, "burst_count": 1})
        elif kind == 2:  # two rules: index 0 then index 2
            rules.append({"resource": r, "count": 4.0, "param_idx": 0})
            rules.append({"resource": r, "count": 2.0, "param_idx": 2, "hot": {3: 6}})
        elif kind == 3:  # thread grade on the second argument
            rules.append({"resource": r, "grade": 0, "count": 2.0, "param_idx": 1, "hot": {1: 4}})
        elif kind == 4:  # throttle on the last argument
            rules.append({"resource": r, "count": 5.0, "param_idx": -1, "control_behavior": 2,
                          "max_queueing_time_ms": 150})
        else:
            rules.append({"resource": r, "count": 3.0, "param_idx": -2})
    return rules


@pytest.mark.parametrize("seed", [3, 4])
def test_argument_vectors_match_oracle(seed):
    rng = np.random.default_rng(seed)
    n_res = 12
    rules = _rules(rng, n_res)
    gen = lt.Oracle(n_res, [], rules)
    st = lt.generate_args(gen, n_res, 6000, seed=seed, t0=T0, gap_mean=0.4, acq_max=2, prio_pct=0.05)
    gen.close()
    orc = lt.Oracle(n_res, [], rules)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 14)
    _load(s, param=rules)
    got = _submit_args(s, st)
    _assert_same(st, got, exp, f"argument vectors seed {seed}")
    _assert_nodes(s, orc, n_res, int(st["ts"].max()))
    d = exp[0][st["kind"] == 0]
    assert (d == 2).sum() > 50 and (d == 0).sum() > 50
    orc.close()
    eng.close()


def test_sticky_index_on_parallel_paths():
    """applyRealParamIdx on the engine's parallel paths (one lane per resource, heavy resources): rule -1
    whose resource's first entry carries no argument becomes index 1, so later single-argument entries
    (the round-2 param form) pass; a resource whose first entry carries one argument gets index 0."""
    n_res = 3
    rules = [{"resource": 0, "count": 2.0, "param_idx": -1}, {"resource": 1, "count": 2.0, "param_idx": -1},
             {"resource": 2, "count": 2.0, "param_idx": -1}]
    n = 6000
    res = np.array([0, 1, 2] + [int(x) for x in np.random.default_rng(1).integers(0, 3, size=n - 3)], np.uint32)
    ts = T0 + np.arange(n, dtype=np.int64) // 8
    flags = np.full(n, 4, np.uint8)
    flags[0] = 0  # resource 0: first entry without the argument
    param = (np.arange(n, dtype=np.uint64) % 5)
    st = {"kind": np.zeros(n, np.uint8), "resource": res, "ts": ts, "acquire": np.ones(n, np.int32),
          "flags": flags, "rt": np.zeros(n, np.int64), "param": param}
    orc = lt.Oracle(n_res, [], rules)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 14)
    _load(s, param=rules)
    got = s.submit(st["kind"], st["resource"], st["ts"], st["acquire"], st["flags"], st["rt"], st["param"])
    _assert_same(st, got, exp, "sticky paramIdx")
    assert (exp[0][res == 0] == 0).all()       # resource 0's rule reads args[1]: never limited
    assert (exp[0][res == 1] == 2).any()       # resource 1's rule reads args[0]
    _assert_nodes(s, orc, n_res, int(ts.max()))
    orc.close()
    eng.close()


@pytest.mark.parametrize("server,cap", [(1, None), (0, None), (1, 6)])
def test_cluster_mode_param_rules(server, cap):
    """Cluster-mode QPS parameter rules (ParamFlowChecker.passClusterCheck, :305-333): with the embedded server
    the same engine's cluster parameter path (requestParamToken -> ClusterParamFlowChecker) decides in event
    order -- OK passes, BLOCKED blocks, NO_RULE_EXISTS (a flowId without a cluster rule) falls back to the
    local check or passes (fallbackToLocalOrPass, :335-343); without a server every rule falls back.
    Decisions, node views and the cluster parameter metrics equal the oracle.  cap: the embedded server's
    bucket maps hold 6 values (ClusterParamMetric maxCapacity), so they evict in LRU order."""
    from sentinel_amd import cluster as CL
    from sentinel_amd.local import ClusterStateManager
    from tests.test_cluster_param_gpu import to_param_rules
    rng = np.random.default_rng(71 + server)
    n_res = 10
    rules, crules = [], []
    for r in range(n_res):
        fid = 700 + r
        if r % 4 == 3:
            rules.append({"resource": r, "count": 3.0, "param_idx": 0})
            continue
        rules.append({"resource": r, "count": float(rng.integers(1, 4)), "param_idx": r % 2, "cluster_mode": True,
                      "cluster_flow_id": fid, "cluster_fallback": r % 3 == 0})
        if r % 5 != 2:
            crules.append({"flow_id": fid, "count": float(rng.integers(2, 8)), "threshold_type": 1,
                           "hot": {2: 1}})
    L = lt.lib()
    srv_g = L.orc_cluster_new(1.0, 1.0)
    srv = L.orc_cluster_new(1.0, 1.0)
    keep = []
    H.lib().orc_cluster_set_param_capacity(cap or 0)
    try:
        for h in (srv_g, srv):
            arr = H.cluster_param_rules_array(crules, keep)
            L.orc_cluster_load_param_rules(h, b"default", arr, len(crules))
    finally:
        H.lib().orc_cluster_set_param_capacity(0)
    gen = lt.Oracle(n_res, [], rules)
    L.orc_flow_set_cluster(gen.h, srv_g, server)
    domain = 4 if cap is None else 24
    st = lt.generate_args(gen, n_res, 5000, seed=13 + server, t0=T0, gap_mean=0.5, max_args=2, domain=domain)
    gen.close()
    orc = lt.Oracle(n_res, [], rules)
    L.orc_flow_set_cluster(orc.h, srv, server)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 14)
    if cap is not None:
        CL.ClusterParamFlowRuleManager(eng).set_param_capacity(cap)
    CL.ClusterParamFlowRuleManager(eng).load_rules("default", to_param_rules(CL, crules))  # embedded server's rules
    _load_cluster_params(s, rules)
    if server:
        ClusterStateManager(s).set_to_server()
    got = _submit_args(s, st)
    _assert_same(st, got, exp, f"cluster-mode parameter rules, server={server}")
    t_end = int(st["ts"].max())
    _assert_nodes(s, orc, n_res, t_end)
    pm = CL.ClusterParamFlowRuleManager(eng)
    for c in crules:
        for v in range(domain):
            assert pm.param_sum(c["flow_id"], v, t_end) == L.orc_cluster_param_sum(srv, c["flow_id"], v, t_end), (c, v)
    d = exp[0][st["kind"] == 0]
    assert (d == 0).any() and (d == 2).any()
    L.orc_cluster_free(srv)
    L.orc_cluster_free(srv_g)
    orc.close()
    eng.close()


def _load_cluster_params(s, rules):
    from sentinel_amd.local import ParamFlowRuleManager
    from sentinel_amd.rules import ParamFlowClusterConfig, ParamFlowItem, ParamFlowRule
    ParamFlowRuleManager(s).load_rules([
        ParamFlowRule(resource=f"r{r['resource']}", grade=r.get("grade", 1), count=r["count"],
                      param_idx=r.get("param_idx", 0), control_behavior=r.get("control_behavior", 0),
                      max_queueing_time_ms=r.get("max_queueing_time_ms", 0), burst_count=r.get("burst_count", 0),
                      duration_in_sec=r.get("duration_in_sec", 1),
                      param_flow_item_list=[ParamFlowItem(int(k), int(v)) for k, v in r.get("hot", {}).items()],
                      cluster_mode=bool(r.get("cluster_mode")),
                      cluster_config=ParamFlowClusterConfig(flow_id=r.get("cluster_flow_id"),
                                                            fallback_to_local_when_fail=bool(r.get("cluster_fallback"))))
        for r in rules])


def test_blocked_entries_outside_the_engine():
    """Event kind 2 (SGA_KIND_BLOCKED): an entry blocked by a slot outside the engine (AuthoritySlot ahead
    of the checks) is counted by StatisticSlot's BlockException branch only (StatisticSlot.java:121-135) --
    block QPS on the node and, inbound, on ENTRY_NODE; later decisions see those counts (block QPS feeds
    no controller, the node views must match)."""
    rng = np.random.default_rng(9)
    n_res = 4
    flow = [{"resource": r, "count": 5.0} for r in range(n_res)]
    n = 3000
    st = {"kind": (rng.random(n) < 0.2).astype(np.uint8) * 2, "resource": rng.integers(0, n_res, n).astype(np.uint32),
          "ts": T0 + np.arange(n, dtype=np.int64) // 3, "acquire": rng.integers(1, 3, n).astype(np.int32),
          "flags": np.where(rng.random(n) < 0.5, 8, 0).astype(np.uint8), "rt": np.zeros(n, np.int64),
          "param": np.zeros(n, np.uint64)}
    orc = lt.Oracle(n_res, flow)
    exp = orc.replay(st)
    eng, s = _sentinel(n_res, 1 << 14)
    _load(s, flow)
    got = s.submit(st["kind"], st["resource"], st["ts"], st["acquire"], st["flags"], st["rt"], st["param"])
    _assert_same(st, got, exp, "kind-2 blocks")
    _assert_nodes(s, orc, n_res, int(st["ts"].max()))
    assert s.node(0xFFFFFFFF, int(st["ts"].max())).total_block == orc.node(0xFFFFFFFF, int(st["ts"].max()))[9]
    orc.close()
    eng.close()


def test_thread_maps_many_indices_distinct_values():
    """One resource with parameter rules on five argument indices and a max_batch batch of entries whose
    arguments are all distinct: every entry claims a thread-count map slot per index (ParameterMetric
    .addThreadCount, ParameterMetric.java:184-230), 5 x 2^16 keys in one batch, so the thread table's
    growth budget must count the indices (FlowEngine::ensure_maps).  Then the exits.  Decisions, waits and
    node views equal the oracle, and the batch does not fail."""
    n_res, n, k_idx = 1, 1 << 16, 5
    rules = [{"resource": 0, "count": 3.0, "param_idx": k} for k in range(k_idx)]
    pv, words = [], []
    for i in range(n):
        words.append(lt.encode_args([i * k_idx + k + 1 for k in range(k_idx)], pv))
    ts = T0 + np.arange(n, dtype=np.int64) // 64
    st = {"kind": np.zeros(n, np.uint8), "resource": np.zeros(n, np.uint32), "ts": ts,
          "acquire": np.ones(n, np.int32), "flags": np.full(n, 32, np.uint8), "rt": np.zeros(n, np.int64),
          "param": np.array(words, np.uint64), "param_values": np.array(pv, np.uint64)}
    orc = lt.Oracle(n_res, [], rules)
    exp = orc.replay(st)
    ok = np.isin(exp[0], (0, 4))  # passed entries exit
    assert ok.all()
    ex = {k: v.copy() for k, v in st.items()}
    ex["kind"] = np.ones(n, np.uint8)
    ex["ts"] = ts + 5
    ex["rt"] = np.full(n, 5, np.int64)
    exp_x = orc.replay(ex)
    eng, s = _sentinel(n_res, n)
    _load(s, param=rules)
    got = _submit_args(s, st)
    _assert_same(st, got, exp, "distinct arguments on five indices (entries)")
    got_x = _submit_args(s, ex)
    _assert_same(ex, got_x, exp_x, "distinct arguments on five indices (exits)")
    _assert_nodes(s, orc, n_res, int(ex["ts"].max()))
    orc.close()
    eng.close()


@pytest.mark.parametrize("small", [True, False])
def test_revoked_entries_after_a_later_slot_block(small):
    """Event kind 3 (SGA_KIND_REVOKE): an entry the engine passed that a slot sorted after DegradeSlot then
    blocked.  The reference's StatisticSlot fires those slots before its pass accounting (StatisticSlot.java:
    71-84), so the entry counts only a block (:121-135): the revoke undoes the pass, the thread counts (node,
    ENTRY_NODE, parameter thread maps) and counts the block.  Rounds of entries, then revokes for some of the
    passed ones and exits for the rest; thread-grade flow and parameter rules see the released threads.
    Decisions, waits and node views equal the oracle's replay (oracle_ext.c kind 3)."""
    rng = np.random.default_rng(17)
    n_res = 4
    flow = [{"resource": 0, "grade": 0, "count": 3}, {"resource": 1, "count": 40.0}]
    param = [{"resource": 2, "grade": 0, "count": 2.0, "param_idx": 0}, {"resource": 3, "count": 5.0}]
    orc = lt.Oracle(n_res, flow, param)
    eng, s = _sentinel(n_res, 1 << 12)
    if not small:  # the rounds through the pipeline instead of the one-workgroup replay (k_lsmall)
        eng.set_small_batch(0)
    _load(s, flow, param)
    n_rev = n_pass = 0
    for k in range(30):
        n = 200
        t0 = T0 + k * 1000
        st = {"kind": np.zeros(n, np.uint8), "resource": rng.integers(0, n_res, n).astype(np.uint32),
              "ts": t0 + np.sort(rng.integers(0, 100, n)).astype(np.int64), "acquire": rng.integers(1, 3, n).astype(np.int32),
              "flags": (4 | np.where(rng.random(n) < 0.5, 8, 0)).astype(np.uint8), "rt": np.zeros(n, np.int64),
              "param": rng.integers(0, 3, n).astype(np.uint64)}
        exp = orc.replay(st)
        got = s.submit(st["kind"], st["resource"], st["ts"], st["acquire"], st["flags"], st["rt"], st["param"])
        _assert_same(st, got, exp, f"round {k} entries")
        passed = np.nonzero(exp[0] == 0)[0]
        rev = passed[rng.random(len(passed)) < 0.4]
        ext = np.setdiff1d(passed, rev)
        n_rev += len(rev)
        n_pass += len(passed)
        fx = {f: np.concatenate([st[f][rev], st[f][ext]]) for f in st}
        fx["kind"] = np.concatenate([np.full(len(rev), 3, np.uint8), np.ones(len(ext), np.uint8)])
        fx["rt"] = np.concatenate([np.zeros(len(rev), np.int64), rng.integers(1, 30, len(ext)).astype(np.int64)])
        fx["ts"] = np.concatenate([st["ts"][rev], t0 + 200 + fx["rt"][len(rev):]])
        order = np.argsort(fx["ts"], kind="stable")
        fx = {f: v[order] for f, v in fx.items()}
        exp_x = orc.replay(fx)
        got_x = s.submit(fx["kind"], fx["resource"], fx["ts"], fx["acquire"], fx["flags"], fx["rt"], fx["param"])
        _assert_same(fx, got_x, exp_x, f"round {k} revokes and exits")
        _assert_nodes(s, orc, n_res, t0 + 300)
    assert n_rev > 500 and n_pass > n_rev
    end = T0 + 30 * 1000
    assert s.node(0xFFFFFFFF, end).cur_thread_num == 0
    orc.close()
    eng.close()


@pytest.mark.parametrize("small", [True, False])
def test_revoked_probes_return_breakers_to_open(small):
    """Revokes of entries that were circuit-breaker probes (AbstractCircuitBreaker.java:117-139: the
    whenTerminate hook moves a breaker the blocked entry made HALF_OPEN back to OPEN, next retry kept).
    Exception-count and slow-RT breakers trip on erroring / slow exits; after each retry time the first entry
    probes, and revokes take some probes back. Decisions, waits and node views equal the oracle's replay."""
    rng = np.random.default_rng(23)
    n_res = 3
    degrade = [{"resource": 0, "grade": 2, "count": 2, "min_request_amount": 3, "time_window": 1},
               {"resource": 1, "grade": 0, "count": 20, "min_request_amount": 3, "time_window": 1,
                "slow_ratio_threshold": 0.5},
               {"resource": 2, "grade": 1, "count": 0.5, "min_request_amount": 3, "time_window": 1}]
    flow = [{"resource": 2, "count": 50.0}]
    orc = lt.Oracle(n_res, flow, [], degrade)
    eng, s = _sentinel(n_res, 1 << 12)
    if not small:
        eng.set_small_batch(0)
    _load(s, flow, None, degrade)
    reopened = 0
    for k in range(40):
        n = 60
        t0 = T0 + k * 700
        st = {"kind": np.zeros(n, np.uint8), "resource": rng.integers(0, n_res, n).astype(np.uint32),
              "ts": t0 + np.sort(rng.integers(0, 100, n)).astype(np.int64), "acquire": np.ones(n, np.int32),
              "flags": np.where(rng.random(n) < 0.5, 8, 0).astype(np.uint8), "rt": np.zeros(n, np.int64),
              "param": np.zeros(n, np.uint64)}
        exp = orc.replay(st)
        got = _submit(s, st)
        _assert_same(st, got, exp, f"round {k} entries")
        passed = np.nonzero(exp[0] == 0)[0]
        rev = passed[rng.random(len(passed)) < 0.5]
        ext = np.setdiff1d(passed, rev)
        fx = {f: np.concatenate([st[f][rev], st[f][ext]]) for f in st}
        fx["kind"] = np.concatenate([np.full(len(rev), 3, np.uint8), np.ones(len(ext), np.uint8)])
        err = rng.random(len(ext)) < 0.6
        fx["flags"] = fx["flags"] | np.concatenate([np.zeros(len(rev), np.uint8), np.where(err, 2, 0).astype(np.uint8)])
        fx["rt"] = np.concatenate([np.zeros(len(rev), np.int64), rng.integers(1, 60, len(ext)).astype(np.int64)])
        fx["ts"] = np.concatenate([st["ts"][rev], t0 + 150 + fx["rt"][len(rev):]])
        order = np.argsort(fx["ts"], kind="stable")
        fx = {f: v[order] for f, v in fx.items()}
        exp_x = orc.replay(fx)
        got_x = _submit(s, fx)
        _assert_same(fx, got_x, exp_x, f"round {k} revokes and exits")
        _assert_nodes(s, orc, n_res, t0 + 300)
        reopened += int((exp[0] == 3).sum() > 0 and len(rev) > 0)
    assert reopened > 5
    orc.close()
    eng.close()
