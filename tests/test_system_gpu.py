"""GPU parity: inbound traffic (EntryType.IN) and SystemSlot on the local path, HIP engine vs the
oracle on the same recorded streams.  Without system rules the decisions stay on the parallel
pipeline and Constants.ENTRY_NODE is updated by k_entry_stats (bucketed when time does not go
back inside a 1024-event tile, event by event otherwise); with system rules the batch is decided
by one lane in arrival order (k_lseq).  Decisions, waits, every node view (ENTRY_NODE included)
and the metrics rows must be identical."""
import numpy as np
import pytest

from tests import local_trace as lt

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
ENTRY = 0xFFFFFFFF


def _setup(n_res, flow, system=None, status=None):
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import FlowRuleManager, LocalSentinel, SystemRule, SystemRuleManager
    from sentinel_amd.rules import FlowRule
    eng = Engine(max_batch=1 << 14)
    s = LocalSentinel(eng, [f"r{i}" for i in range(n_res)])
    FlowRuleManager(s).load_rules([FlowRule(resource=f"r{r['resource']}", count=r["count"]) for r in flow])
    if system is not None:
        m = SystemRuleManager(s)
        m.load_rules([SystemRule(**r) for r in system])
        if status is not None:
            m.set_system_status(*status)
    return eng, s


def _oracles(n_res, flow, system=None, status=None):
    out = []
    for _ in range(2):
        o = lt.Oracle(n_res, flow)
        if system is not None:
            o.system(system, *(status if status is not None else (None, None)))
        out.append(o)
    return out


def _check(s, orc, n_res, stream, sizes, ctx):
    lo = 0
    k = 0
    while lo < len(stream["kind"]):
        hi = min(len(stream["kind"]), lo + sizes[k % len(sizes)])
        sub = lt.slice_stream(stream, lo, hi)
        dec, wait = s.submit(sub["kind"], sub["resource"], sub["ts"], sub["acquire"], sub["flags"], sub["rt"],
                             sub["param"])
        odec, owait = orc.replay(sub)
        bad = np.nonzero((dec != odec) | (wait != owait))[0]
        assert bad.size == 0, (ctx, lo, int(bad[0]), dec[bad[0]], odec[bad[0]])
        lo = hi
        k += 1
    now = int(stream["ts"].max()) + 1
    for r in list(range(n_res)) + [ENTRY]:
        got = s.node(r, now)
        exp = orc.node(r, now)
        assert [getattr(got, g) for g in lt.NODE_GETTERS] == exp, (ctx, r)
    got = [(m.timestamp, ENTRY if m.resource == "__total_inbound_traffic__" else s.resource_id(m.resource),
            m.pass_qps, m.block_qps, m.success_qps, m.exception_qps, m.rt, m.occupied_pass_qps)
           for m in s.metrics(now + 2000)]
    exp = orc.metrics(now + 2000)
    assert got == exp, ctx
    assert any(row[1] == ENTRY for row in exp), ctx


@pytest.mark.parametrize("regress", [0.0, 0.02], ids=["ordered", "regressions"])
def test_inbound_entry_node_parallel(regress):
    n_res = 12
    flow = [{"resource": r, "count": float(3 + 2 * r)} for r in range(0, n_res, 2)]
    gen, orc = _oracles(n_res, flow)
    st = lt.generate(gen, n_res, n_entries=9000, seed=21, t0=T0, gap_mean=0.4, err_pct=0.05, rt_max=40,
                     inbound_pct=0.6, regress_pct=regress, prio_pct=0.02)
    gen.close()
    eng, s = _setup(n_res, flow)
    assert (st["flags"] & 8).any() and (st["kind"] == 1).any()
    _check(s, orc, n_res, st, [4000, 1500, 3100, 700], f"regress={regress}")
    orc.close()
    eng.close()


@pytest.mark.parametrize("case", ["qps_thread_rt", "bbr_cpu"])
def test_system_rules_sequential(case):
    n_res = 8
    flow = [{"resource": r, "count": float(4 + r)} for r in range(0, n_res, 3)]
    if case == "qps_thread_rt":
        system, status = [{"qps": 40.0}, {"max_thread": 25}, {"avg_rt": 30}], None
    else:
        system, status = [{"highest_system_load": 1.5, "highest_cpu_usage": 0.9}], (2.0, 0.5)
    gen, orc = _oracles(n_res, flow, system, status)
    st = lt.generate(gen, n_res, n_entries=5000, seed=5, t0=T0, gap_mean=0.5, err_pct=0.05, rt_max=60,
                     inbound_pct=0.7, regress_pct=0.01)
    blocked = int((gen.last_decisions == 5).sum())
    gen.close()
    assert blocked > 0, "the trace must exercise SystemBlockException"
    eng, s = _setup(n_res, flow, system, status)
    _check(s, orc, n_res, st, [2500, 900], case)
    orc.close()
    eng.close()
