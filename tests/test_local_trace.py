"""CPU checks of the local-path test infrastructure: a generated stream replays on a
fresh oracle to exactly the decisions that generated it (the exits it carries are
the exits of passed entries), and the breakers/param maps it drives are exercised."""
import numpy as np

from tests import local_trace as lt

T0 = 1_700_000_000_000


def _roundtrip(n_res, flow=(), param=(), degrade=(), **kw):
    gen = lt.Oracle(n_res, flow, param, degrade)
    st = lt.generate(gen, n_res, t0=T0, **kw)
    gd = gen.last_decisions
    gen.close()
    orc = lt.Oracle(n_res, flow, param, degrade)
    d, w = orc.replay(st)
    orc.close()
    assert np.array_equal(d[st["kind"] == 0], gd)
    return st, d


def test_generated_stream_replays_to_its_own_decisions():
    flow = [{"resource": 0, "count": 5}, {"resource": 1, "grade": 0, "count": 2},
            {"resource": 2, "count": 10, "control_behavior": 2, "max_queueing_time_ms": 100}]
    param = [{"resource": 3, "count": 2, "burst_count": 1}]
    degrade = [{"resource": 4, "grade": 2, "count": 2, "time_window": 1}]
    st, d = _roundtrip(6, flow, param, degrade, n_entries=3000, seed=4, gap_mean=0.5, prio_pct=0.1, acq_max=2,
                       err_pct=0.3, rt_max=30, params=3, regress_pct=0.02)
    kinds = set(d[st["kind"] == 0].tolist())
    assert {0, 1, 2, 3} <= kinds, kinds
    # every exit belongs to a passed entry: exits per resource never exceed passes
    for r in range(6):
        ent = (st["kind"] == 0) & (st["resource"] == r)
        assert (st["kind"][st["resource"] == r] == 1).sum() == np.isin(d[ent], (0, 4)).sum()
