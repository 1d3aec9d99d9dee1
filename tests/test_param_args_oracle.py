"""ParamFlowSlot over whole argument vectors in the oracle (a16): ParamFlowSlot.applyRealParamIdx
(ParamFlowSlot.java:56-66, the rule's index rewritten at its first check), ParamFlowChecker.passCheck
(ParamFlowChecker.java:48-77: args.length <= paramIdx or a null value pass), per-index thread-count maps
(ParameterMetric.java:113-230) and their clearing on reload (ParamFlowRuleManager.java:122-150), and
cluster-mode parameter rules (ParamFlowChecker.passClusterCheck / fallbackToLocalOrPass, :305-343).
Expected decisions are derived by hand from those lines (no reference test covers them: parity is
defined by the restatement)."""
import ctypes as C

import numpy as np

from tests import local_trace as lt
from tests import oracle_harness as H

T0 = 1_700_000_000_000


class Flow:
    def __init__(self, n_res, param_rules, flow_rules=()):
        self.o = lt.Oracle(n_res, list(flow_rules), list(param_rules))
        self.L = self.o.L

    def ev(self, kind, rid, t, args, acq=1, rt=0):
        pv = []
        word = lt.encode_args(args, pv)
        arrs = [np.array([kind], np.uint8), np.array([rid], np.uint32), np.array([t], np.int64),
                np.array([acq], np.int32), np.array([32], np.uint8), np.array([rt], np.int64),
                np.array([word], np.uint64)]
        lv = np.ascontiguousarray(pv or [0], dtype=np.uint64)
        d = np.zeros(1, np.int8)
        w = np.zeros(1, np.int32)
        self.L.orc_flow_replay_args(self.o.h, 1, *[a.ctypes.data for a in arrs], lv.ctypes.data, d.ctypes.data,
                                    w.ctypes.data)
        return int(d[0])

    def entry(self, rid, t, *args, acq=1):
        return self.ev(0, rid, t, list(args), acq)

    def exit(self, rid, t, *args):
        return self.ev(1, rid, t, list(args))


def test_negative_index_fixed_by_first_check():
    """paramIdx -1: the first entry has no arguments -> -(-1) = 1 > length 0 -> the rule becomes paramIdx 1
    for good, so later one-argument entries are never limited (args.length 1 <= 1)."""
    f = Flow(2, [{"resource": 0, "count": 1, "param_idx": -1}, {"resource": 1, "count": 1, "param_idx": -1}])
    assert f.entry(0, T0) == 0
    assert f.L.orc_flow_param_idx(f.o.h, 0, 0) == 1
    assert [f.entry(0, T0 + 1, 7) for _ in range(4)] == [0, 0, 0, 0]
    # resource 1 first sees one argument: -1 -> 0, then count 1 per value per second
    assert f.entry(1, T0, 7) == 0
    assert f.L.orc_flow_param_idx(f.o.h, 1, 0) == 0
    assert f.entry(1, T0 + 1, 7) == 2
    assert f.entry(1, T0 + 1, 8) == 0
    assert f.entry(1, T0 + 2, 8, 99) == 2  # still index 0 with two arguments


def test_second_argument_and_nulls():
    """paramIdx 1 reads args[1]; a null args[1] passes (ParamFlowChecker.java:69-71); fewer arguments pass."""
    f = Flow(1, [{"resource": 0, "count": 2, "param_idx": 1}])
    assert [f.entry(0, T0, 5, 42) for _ in range(3)] == [0, 0, 2]
    assert f.entry(0, T0 + 1, 5, 43) == 0       # another value of args[1]
    assert f.entry(0, T0 + 1, 5, None) == 0     # null
    assert f.entry(0, T0 + 1, 5) == 0           # args.length 1 <= 1
    assert f.entry(0, T0 + 1, 6, [42, 43]) == 2  # a list: 42 is exhausted
    assert f.entry(0, T0 + 1001, 6, [42, 43]) == 0  # next second: both refilled, both pass


def test_thread_maps_per_index_and_reload_clears():
    """THREAD grade on paramIdx 1 counts args[1] (ParameterMetric.threadCountMap[1]); a reload that drops the
    rule clears that map (clearForRule -> threadCountMap.remove(paramIdx))."""
    rule = {"resource": 0, "grade": 0, "count": 1, "param_idx": 1}
    f = Flow(1, [rule])
    assert f.entry(0, T0, 1, 9) == 0
    assert f.entry(0, T0, 2, 9) == 2         # value 9 holds one thread
    assert f.entry(0, T0, 1, 10) == 0
    f.exit(0, T0 + 5, 1, 9)                   # releases value 9
    assert f.entry(0, T0 + 6, 3, 9) == 0
    # reload with a different rule: the old rule's thread map (index 1) goes; the new one starts empty
    keep = []
    rule2 = dict(rule, count=2)
    f.L.orc_flow_load_param_rules(f.o.h, H.param_rules_array([rule2], keep), 1)
    assert f.entry(0, T0 + 7, 1, 10) == 0 and f.entry(0, T0 + 7, 1, 10) == 0  # 10's old thread is gone
    assert f.entry(0, T0 + 7, 1, 10) == 2


def test_cluster_mode_param_rule_with_embedded_server():
    """Cluster-mode QPS parameter rules ask the embedded server (requestParamToken): OK passes, BLOCKED blocks;
    a flowId with no cluster rule answers NO_RULE_EXISTS -> fallbackToLocalOrPass: the local check when
    fallbackToLocalWhenFail, else pass.  Without a token service every rule falls back."""
    L = H.lib()
    rules = [{"resource": 0, "count": 1, "cluster_mode": True, "cluster_flow_id": 500},
             {"resource": 1, "count": 1, "cluster_mode": True, "cluster_flow_id": 501, "cluster_fallback": True},
             {"resource": 2, "count": 1, "cluster_mode": True, "cluster_flow_id": 502}]
    f = Flow(3, rules)
    srv = L.orc_cluster_new(1.0, 1.0)
    keep = []
    arr = H.cluster_param_rules_array([{"flow_id": 500, "count": 3, "threshold_type": 1}], keep)
    L.orc_cluster_load_param_rules(srv, b"default", arr, 1)
    L.orc_flow_set_cluster(f.o.h, srv, 1)
    assert [f.entry(0, T0, 7) for _ in range(4)] == [0, 0, 0, 2]  # the server's count 3 (not the local 1)
    assert [f.entry(1, T0, 7) for _ in range(2)] == [0, 2]        # NO_RULE_EXISTS -> local count 1
    assert [f.entry(2, T0, 7) for _ in range(3)] == [0, 0, 0]     # NO_RULE_EXISTS, no fallback -> pass
    L.orc_flow_set_cluster(f.o.h, srv, 0)
    assert f.entry(0, T0 + 1, 8) == 0 and f.entry(0, T0 + 1, 8) == 0  # no service, no fallback: pass
    assert f.entry(1, T0 + 1, 7) == 2                                  # no service: local (7 exhausted)
    L.orc_cluster_free(srv)


def test_generated_argument_streams_replay_identically():
    """The generator drives one oracle event by event; replaying the recorded stream on a fresh oracle gives
    the same decisions (the stream encoding round-trips)."""
    rules = [{"resource": r, "count": 2 + r % 3, "param_idx": [0, 1, -1, 2][r % 4]} for r in range(8)]
    rules += [{"resource": 3, "grade": 0, "count": 1, "param_idx": 1}]
    gen = lt.Oracle(8, [], rules)
    st = lt.generate_args(gen, 8, 3000, seed=5, t0=T0, gap_mean=0.3)
    dec_gen = gen.replay  # noqa: F841
    orc = lt.Oracle(8, [], rules)
    d, w = orc.replay(st)
    assert (d[st["kind"] == 0] == 2).any() and (d[st["kind"] == 0] == 0).any()
    gen.close()
    orc.close()


def test_revoke_undoes_the_pass_and_counts_the_block():
    """Kind 3 (SGA_KIND_REVOKE) in the oracle: after a passed entry and its revoke, the node holds what the
    reference's StatisticSlot records when a slot after the checks throws (StatisticSlot.java:71-84,121-135):
    no pass, no thread (node, ENTRY_NODE for an inbound entry, the parameter thread map), one block of the
    entry's count.  A thread-grade rule of 1 then passes the next entry again."""
    T = 1_700_000_000_000
    flow = [{"resource": 0, "grade": 0, "count": 1}]
    param = [{"resource": 0, "grade": 0, "count": 1.0, "param_idx": 0}]
    orc = lt.Oracle(1, flow, param)

    def ev(kind, t, acq=1):
        return {"kind": np.array([kind], np.uint8), "resource": np.zeros(1, np.uint32), "ts": np.array([t], np.int64),
                "acquire": np.array([acq], np.int32), "flags": np.array([4 | 8], np.uint8),
                "rt": np.zeros(1, np.int64), "param": np.array([7], np.uint64)}

    assert orc.replay(ev(0, T))[0][0] == 0
    assert orc.replay(ev(0, T + 1))[0][0] != 0  # the first entry holds the one thread
    orc.replay(ev(3, T))
    v = dict(zip(lt.NODE_GETTERS, orc.node(0, T + 2)))
    e = dict(zip(lt.NODE_GETTERS, orc.node(0xFFFFFFFF, T + 2)))
    assert v["cur_thread_num"] == 0 and e["cur_thread_num"] == 0
    assert v["pass_qps"] == 0 and e["pass_qps"] == 0
    assert v["block_qps"] == 2 and e["block_qps"] == 2  # the second entry's block + the revoked entry's
    assert orc.replay(ev(0, T + 3))[0][0] == 0  # thread and parameter thread counts released
    orc.close()


def test_revoked_probe_returns_its_breaker_to_open():
    """A revoked entry that was a breaker's HALF_OPEN probe: the reference's whenTerminate hook
    (AbstractCircuitBreaker.java:117-139, the issue-1638 workaround) sees the block error and moves the
    breaker back to OPEN without a new retry time, so the next entry past the retry time probes again
    (a breaker left HALF_OPEN would block every later entry)."""
    T = 1_700_000_000_000
    degrade = [{"resource": 0, "grade": 2, "count": 2, "min_request_amount": 3, "time_window": 1}]
    orc = lt.Oracle(1, [], [], degrade)

    def ev(kind, t, err=False):
        return {"kind": np.array([kind], np.uint8), "resource": np.zeros(1, np.uint32), "ts": np.array([t], np.int64),
                "acquire": np.ones(1, np.int32), "flags": np.array([2 if err else 0], np.uint8),
                "rt": np.array([1], np.int64), "param": np.zeros(1, np.uint64)}

    for _ in range(4):
        assert orc.replay(ev(0, T))[0][0] == 0
    for _ in range(4):
        orc.replay(ev(1, T + 1, err=True))  # three errors trip it at T + 1: OPEN, retry at T + 1001
    assert orc.replay(ev(0, T + 500))[0][0] == 3  # OPEN
    assert orc.replay(ev(0, T + 1500))[0][0] == 0  # the probe: HALF_OPEN
    assert orc.replay(ev(0, T + 1501))[0][0] == 3  # HALF_OPEN blocks
    orc.replay(ev(3, T + 1500))  # the probe is revoked: back to OPEN, retry time kept
    assert orc.replay(ev(0, T + 1600))[0][0] == 0  # a new probe
    orc.close()
