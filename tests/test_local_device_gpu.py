"""GPU parity of the device-resident local entry (sga_submit_events_device): the events already sit in
HBM, the chunk is launched without a host wait and the checks the host entry makes by scanning the
events (SystemSlot / Collection arguments -> arrival-order replay, inbound statistics, validation) are
made by k_lgate on the device.  Decisions, waits, node views and metrics must equal the oracle replay of
the same stream (and so the host entry, which the other local tests pin to the same oracle)."""
import numpy as np
import pytest

from tests import local_trace as lt

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
ENTRY = 0xFFFFFFFF


def _dev(s, sub, pvals=None, stream=None):
    """One chunk through LocalSentinel.submit_device; returns host numpy (decision, wait)."""
    import torch
    dev = torch.device("cuda", 0)
    ts = np.asarray(sub["ts"], np.int64)
    base = int(ts.min())
    off = (ts - base).astype(np.uint32).view(np.int32)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)  # noqa: E731
    kw = {}
    if pvals is not None:
        kw["param_values"] = t(np.asarray(pvals, np.uint64), np.int64)
    d, w = s.submit_device(t(np.asarray(sub["kind"], np.uint8), np.uint8),
                           t(np.asarray(sub["resource"], np.uint32), np.int32), base, t(off, np.int32),
                           t(np.asarray(sub["acquire"], np.int32), np.int32),
                           flags=t(np.asarray(sub["flags"], np.uint8), np.uint8),
                           rt=t(np.asarray(sub["rt"], np.int64), np.int64),
                           param=t(np.asarray(sub["param"], np.uint64), np.int64), stream=stream, **kw)
    if stream is not None:
        stream.synchronize()
    s.device_status()
    return d.cpu().numpy(), w.cpu().numpy()


def _sentinel(n_res, max_batch):
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import LocalSentinel
    eng = Engine(max_batch=max_batch)
    return eng, LocalSentinel(eng, [f"r{i}" for i in range(n_res)])


def _chunks(s, orc, st, sizes, ctx, pvals=None, stream=None):
    lo, k = 0, 0
    n = len(st["kind"])
    while lo < n:
        hi = min(n, lo + sizes[k % len(sizes)])
        sub = lt.slice_stream(st, lo, hi)
        if pvals is not None:
            sub["param_values"] = pvals
        d, w = _dev(s, sub, pvals, stream)
        od, ow = orc.replay(sub)
        bad = np.nonzero((d != od) | (w != ow))[0]
        assert bad.size == 0, (ctx, lo, int(bad[0]), int(d[bad[0]]), int(od[bad[0]]), int(w[bad[0]]), int(ow[bad[0]]))
        lo, k = hi, k + 1


def _nodes(s, orc, n_res, now, entry=False):
    for r in list(range(n_res)) + ([ENTRY] if entry else []):
        assert [getattr(s.node(r, now), g) for g in lt.NODE_GETTERS] == orc.node(r, now), r


@pytest.mark.parametrize("side_stream", [False, True], ids=["engine_stream", "caller_stream"])
def test_device_entry_flow_param_degrade(side_stream):
    import torch
    from tests.test_local_parity_gpu import _load, _random_flow_rules
    rng = np.random.default_rng(71)
    n_res = 30
    flow = _random_flow_rules(rng, n_res)
    param = [{"resource": r, "count": float(rng.integers(2, 9))} for r in range(0, n_res, 4)]
    degrade = [{"resource": r, "grade": r % 3, "count": [40.0, 0.3, 5.0][r % 3], "slow_ratio_threshold": 0.5,
                "time_window": 1, "min_request_amount": 3} for r in range(1, n_res, 5)]
    gen = lt.Oracle(n_res, flow, param, degrade)
    st = lt.generate(gen, n_res, n_entries=12000, seed=72, t0=T0, gap_mean=0.4, prio_pct=0.1, acq_max=3,
                     err_pct=0.1, rt_max=60, params=6, regress_pct=0.01)
    gen.close()
    orc = lt.Oracle(n_res, flow, param, degrade)
    eng, s = _sentinel(n_res, 1 << 13)
    _load(s, flow, param, degrade)
    stream = torch.cuda.Stream() if side_stream else None
    _chunks(s, orc, st, [4000, 1500, 3100, 700], "flow/param/degrade", stream=stream)
    now = int(st["ts"].max())
    _nodes(s, orc, n_res, now)
    for r in degrade:
        assert s.circuit_breaker_state(r["resource"], 0) == orc.cb_state(r["resource"], 0)
    orc.close()
    eng.close()


@pytest.mark.parametrize("case", ["inbound_parallel", "system_sequential"])
def test_device_entry_inbound_and_system(case):
    from tests.test_system_gpu import _oracles, _setup
    n_res = 10
    flow = [{"resource": r, "count": float(4 + r)} for r in range(0, n_res, 2)]
    system = [{"qps": 40.0}, {"max_thread": 25}] if case == "system_sequential" else None
    gen, orc = _oracles(n_res, flow, system)
    st = lt.generate(gen, n_res, n_entries=6000, seed=73, t0=T0, gap_mean=0.5, err_pct=0.05, rt_max=50,
                     inbound_pct=0.6, regress_pct=0.01, prio_pct=0.02)
    gen.close()
    eng, s = _setup(n_res, flow, system)
    _chunks(s, orc, st, [2500, 900, 1700], case)
    _nodes(s, orc, n_res, int(st["ts"].max()) + 1, entry=True)
    orc.close()
    eng.close()


def test_device_entry_collection_parameters():
    from tests.test_local_parity_gpu import _load
    rng = np.random.default_rng(74)
    n_res, n = 8, 12000
    param = [{"resource": r, "count": float(rng.integers(2, 12)), **({"grade": 0, "count": 2.0} if r % 4 == 2 else {})}
             for r in range(n_res)]
    res = rng.integers(0, n_res, size=n)
    ts = T0 + np.sort(rng.integers(0, 8000, size=n))
    flags = np.zeros(n, np.uint8)
    pv = np.zeros(n, np.uint64)
    values = []
    for i in range(n):
        u = rng.random()
        if u < 0.4:
            m = int(rng.integers(0, 4))
            pv[i] = (len(values) << 32) | m
            values.extend(int(x) for x in rng.integers(0, 9, size=m))
            flags[i] = 4 | 16
        elif u < 0.8:
            pv[i] = int(rng.integers(0, 9))
            flags[i] = 4
    values = np.array(values, dtype=np.uint64)
    gen = lt.Oracle(n_res, [], param)
    st = lt.generate_windows(gen, res, ts, rng.integers(1, 3, size=n), flags, pv, rng.integers(2, 60, size=n),
                             rng.random(n) < 0.05, window_ms=2, param_values=values)
    gen.close()
    vals = st.pop("param_values")
    orc = lt.Oracle(n_res, [], param)
    eng, s = _sentinel(n_res, 1 << 13)
    _load(s, param=param)
    _chunks(s, orc, st, [5000, 2000], "collections", pvals=vals)
    _nodes(s, orc, n_res, int(st["ts"].max()))
    orc.close()
    eng.close()


def test_device_entry_rejects_invalid_chunk():
    """acquire < 0 (the host entry's -EINVAL): the chunk answers -1, is not applied, and
    sga_events_device_status reports it once."""
    import torch
    from sentinel_amd import EngineError
    from tests.test_local_parity_gpu import _load
    n_res = 3
    eng, s = _sentinel(n_res, 1 << 10)
    _load(s, [{"resource": 0, "count": 2}])
    dev = torch.device("cuda", 0)
    k = torch.zeros(4, dtype=torch.uint8, device=dev)
    r = torch.zeros(4, dtype=torch.int32, device=dev)
    off = torch.zeros(4, dtype=torch.int32, device=dev)
    bad = torch.tensor([1, 1, -1, 1], dtype=torch.int32, device=dev)
    d, _ = s.submit_device(k, r, T0, off, bad)
    with pytest.raises(EngineError):
        s.device_status()
    assert d.cpu().tolist() == [-1, -1, -1, -1]
    s.device_status()  # reported once
    good = torch.ones(4, dtype=torch.int32, device=dev)
    d, _ = s.submit_device(k, r, T0, off, good)
    s.device_status()
    assert d.cpu().tolist() == [0, 0, 1, 1]  # count 2: the rejected chunk took no token
    assert s.node(0, T0).total_pass == 2
    eng.close()
