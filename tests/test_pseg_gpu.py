"""GPU parity of the per-segment paths of the local engine (flow.hip k_pseg_* and k_cb_flows) against the
oracle replay, batch by batch as the engine sees them.

* Parameter-only resources (one QPS ParamFlowRule): the events are grouped per (rule, value) segment.
  Long segments of entries with one acquire count and non-decreasing times are decided by stretches
  (k_pseg_long: token-bucket refills and throttle passes found by search); exit-only segments take the
  closed form of decreaseThreadCount; every other segment (mixed, irregular acquire counts, a clock that
  goes back) is walked event by event.  Cases: refills inside one batch, burst counts, hot items, throttle
  with and without queueing, irregular segments, exits that empty and refill the thread counts.
* Breaker-only resources (one DegradeRule) whose batch holds only entries or only exits: an OPEN breaker's
  probe (the first entry at or after the retry time), HALF_OPEN decided by the next exit, a CLOSED breaker
  tripped inside a long exit batch, a stat window that goes back in time.

Every decision and wait, the MetricNode rows, the node views and the breaker states must equal the oracle's
(tests/test_configs_fullsize_gpu._check_local's checks, with explicit batch boundaries)."""
import numpy as np
import pytest

from tests import local_trace as lt
from tests.test_configs_fullsize_gpu import T0, _local

pytestmark = pytest.mark.gpu

EV_ERROR, EV_HAS_PARAM = 2, 4


def _batch(kind, res, ts, acq=None, flags=None, rt=None, param=None):
    n = len(ts)
    return {"kind": np.full(n, kind, np.uint8) if np.isscalar(kind) else np.asarray(kind, np.uint8),
            "resource": np.asarray(np.broadcast_to(res, (n,)), np.uint32).copy(),
            "ts": np.asarray(ts, np.int64),
            "acquire": np.ones(n, np.int32) if acq is None else np.asarray(acq, np.int32),
            "flags": np.zeros(n, np.uint8) if flags is None else np.asarray(flags, np.uint8),
            "rt": np.zeros(n, np.int64) if rt is None else np.asarray(rt, np.int64),
            "param": np.zeros(n, np.uint64) if param is None else np.asarray(param, np.uint64)}


def _check_batches(n_res, batches, param=(), degrade=()):
    """Each batch one engine call; the oracle replays their concatenation."""
    st = {k: np.concatenate([b[k] for b in batches]) for k in batches[0]}
    orc = lt.Oracle(n_res, [], list(param), list(degrade))
    exp_d, exp_w = orc.replay(st)
    eng, s = _local(n_res, param=param, degrade=degrade, max_batch=max(len(b["kind"]) for b in batches))
    got_d, got_w, lo = [], [], 0
    for b in batches:
        d, w = s.submit(b["kind"], b["resource"], b["ts"], b["acquire"], b["flags"], b["rt"], b["param"])
        got_d.append(d)
        got_w.append(w)
    got_d, got_w = np.concatenate(got_d), np.concatenate(got_w)
    bad = np.nonzero((got_d != exp_d) | (got_w != exp_w))[0]
    assert len(bad) == 0, (f"{len(bad)} of {len(got_d)} differ; first at {bad[0]}: kind={st['kind'][bad[0]]} "
                           f"res={st['resource'][bad[0]]} gpu=({got_d[bad[0]]},{got_w[bad[0]]}) "
                           f"oracle=({exp_d[bad[0]]},{exp_w[bad[0]]})")
    now = int(st["ts"].max()) + 1
    got = [(m.timestamp, s.resource_id(m.resource), m.pass_qps, m.block_qps, m.success_qps, m.exception_qps, m.rt,
            m.occupied_pass_qps) for m in s.metrics(now, cap=1 << 16)]
    assert got == orc.metrics(now, cap=1 << 16)
    for rid in range(n_res):
        v = s.node(rid, now)
        assert [getattr(v, g) for g in lt.NODE_GETTERS] == orc.node(rid, now), rid
    for r in degrade:
        assert s.circuit_breaker_state(r["resource"], 0) == orc.cb_state(r["resource"], 0), r["resource"]
    orc.close()
    eng.close()
    return exp_d


def _param_stream(rng, n, n_res, n_vals, span_ms, acq=None):
    res = rng.integers(0, n_res, size=n)
    vals = np.minimum(rng.zipf(1.3, size=n) - 1, n_vals - 1)  # a few values with long segments
    ts = T0 + np.sort(rng.integers(0, span_ms, size=n))
    return res, vals.astype(np.uint64), ts, (np.ones(n, np.int32) if acq is None else acq)


@pytest.mark.parametrize("case", ["bucket", "burst", "throttle0", "throttle_queue", "hot_items", "duration2",
                                  "throttle_zero_cost"])
def test_long_entry_segments_then_exits(case):
    """Entries only (long regular segments spanning several refills), then the exits of half of them, then
    entries again: stretches, the exit closed form and the walk all meet the same maps."""
    rng = np.random.default_rng({"bucket": 1, "burst": 2, "throttle0": 3, "throttle_queue": 4, "hot_items": 5,
                                 "duration2": 6, "throttle_zero_cost": 7}[case])
    n_res, n = 3, 60_000
    rule = {"count": 40.0}
    if case == "burst":
        rule["burst_count"] = 25
    if case == "throttle0":
        rule.update(control_behavior=2, max_queueing_time_ms=0, count=30.0)
    if case == "throttle_queue":
        rule.update(control_behavior=2, max_queueing_time_ms=150, count=30.0)
    if case == "throttle_zero_cost":  # Math.round(1000 / 5000) = 0: every entry at or after the last pass passes
        rule.update(control_behavior=2, max_queueing_time_ms=0, count=5000.0)
    if case == "hot_items":
        rule["hot"] = {0: 500, 1: 0, 2: 3}
    if case == "duration2":
        rule["duration_in_sec"] = 2
    param = [dict(rule, resource=r) for r in range(n_res)]
    res, vals, ts, acq = _param_stream(rng, n, n_res, 50, 5_000)
    b1 = _batch(0, res, ts, acq=acq, flags=np.full(n, EV_HAS_PARAM), param=vals)
    sel = np.sort(rng.choice(n, n // 2, replace=False))
    b2 = _batch(1, res[sel], ts[sel] + 7_000, flags=np.full(len(sel), EV_HAS_PARAM), param=vals[sel],
                rt=rng.integers(1, 50, size=len(sel)))
    res3, vals3, ts3, acq3 = _param_stream(rng, n, n_res, 50, 3_000)
    b3 = _batch(0, res3, ts3 + 9_000, acq=acq3, flags=np.full(n, EV_HAS_PARAM), param=vals3)
    d = _check_batches(n_res, [b1, b2, b3], param=param)
    assert (d == 0).any() and (case == "throttle_zero_cost" or (d == 2).any())


@pytest.mark.parametrize("case", ["mixed_acquire", "clock_back", "mixed_kinds", "no_param_events"])
def test_irregular_segments_walk(case):
    rng = np.random.default_rng(20 + ["mixed_acquire", "clock_back", "mixed_kinds", "no_param_events"].index(case))
    n_res, n = 2, 40_000
    param = [{"resource": r, "count": 25.0, **({"control_behavior": 2, "max_queueing_time_ms": 40} if r else {})}
             for r in range(n_res)]
    acq = rng.integers(1, 4, size=n).astype(np.int32) if case == "mixed_acquire" else None
    res, vals, ts, acq = _param_stream(rng, n, n_res, 20, 4_000, acq)
    if case == "clock_back":
        ts = ts.copy()
        ts[n // 2:n // 2 + 500] -= 1_500  # a stretch of the batch from 1.5 s earlier
    kind = np.zeros(n, np.uint8)
    flags = np.full(n, EV_HAS_PARAM, np.uint8)
    if case == "mixed_kinds":
        kind = (rng.random(n) < 0.3).astype(np.uint8)
    if case == "no_param_events":
        flags[rng.random(n) < 0.2] = 0
    b = _batch(kind, res, ts, acq=acq, flags=flags, param=vals, rt=rng.integers(1, 30, size=n))
    b2 = _batch(1, res[:5000], ts[:5000] + 5_000, flags=flags[:5000], param=vals[:5000], rt=np.full(5000, 3))
    _check_batches(n_res, [b, b2], param=param)


def test_exit_closed_form_counts():
    """Exit-only segments against counts 0, 1, many and absent: decreaseThreadCount's put(0) of an absent
    value and remove at zero, then a THREAD-free QPS rule still blocks by tokens."""
    n_res = 1
    param = [{"resource": 0, "count": 3.0}]
    ent_v = np.repeat(np.arange(6, dtype=np.uint64), [0, 1, 2, 5, 9, 3])
    ts = T0 + np.arange(len(ent_v))
    b1 = _batch(0, 0, ts, flags=np.full(len(ent_v), EV_HAS_PARAM), param=ent_v)
    ex_v = np.repeat(np.arange(7, dtype=np.uint64), [3, 1, 4, 2, 9, 700, 5])  # more exits than passes
    b2 = _batch(1, 0, T0 + 100 + np.arange(len(ex_v)), flags=np.full(len(ex_v), EV_HAS_PARAM), param=ex_v,
                rt=np.full(len(ex_v), 2))
    b3 = _batch(0, 0, T0 + 2_000 + np.arange(len(ent_v)), flags=np.full(len(ent_v), EV_HAS_PARAM), param=ent_v)
    _check_batches(n_res, [b1, b2, b3], param=param)


@pytest.mark.parametrize("grade", [0, 1])
def test_breaker_flows_trip_probe_half_open(grade):
    """One breaker per resource, batches of only entries or only exits: CLOSED entries pass; a long exit
    batch trips it part-way; entries before the retry time block, the first after it probes; the probe's
    exit (bad on resource 0, good on resource 1) reopens or closes it; a last exit batch goes back in time."""
    rng = np.random.default_rng(40 + grade)
    n_res = 3
    if grade == 0:
        degrade = [{"resource": r, "grade": 0, "count": 50.0, "slow_ratio_threshold": 0.4, "min_request_amount": 20,
                    "stat_interval_ms": 1000, "time_window": 2} for r in range(n_res)]
    else:
        degrade = [{"resource": r, "grade": 1, "count": 0.25, "min_request_amount": 20, "stat_interval_ms": 1000,
                    "time_window": 2} for r in range(n_res)]
    n = 30_000
    res = rng.integers(0, n_res, size=n)
    t1 = T0 + np.sort(rng.integers(0, 3_000, size=n))
    b1 = _batch(0, res, t1)
    # exits: healthy for the first 2 s of each resource, then bad (slow or failing) on resources 0 and 1
    te = t1 + 4_000
    late = te >= T0 + 6_000
    badm = late & (res < 2)
    rt = np.where(badm & (grade == 0), 200, rng.integers(1, 30, size=n))
    fl = np.where(badm & (grade == 1) & (rng.random(n) < 0.6), EV_ERROR, 0).astype(np.uint8)
    b2 = _batch(1, res, te, flags=fl, rt=rt)
    # entries across the retry time (opened near T0 + 6 s, time window 2 s)
    t3 = T0 + 7_000 + np.sort(rng.integers(0, 3_000, size=n))
    res3 = rng.integers(0, n_res, size=n)
    b3 = _batch(0, res3, t3)
    # the probes' exits: resource 0 bad, resource 1 good, then more traffic
    k = 2_000
    res4 = np.concatenate([[0, 1], rng.integers(0, n_res, size=k)])
    t4 = T0 + 11_000 + np.arange(k + 2)
    rt4 = np.concatenate([[300 if grade == 0 else 5, 5], rng.integers(1, 30, size=k)])
    fl4 = np.concatenate([[EV_ERROR if grade == 1 else 0, 0], np.zeros(k)]).astype(np.uint8)
    b4 = _batch(1, res4, t4, flags=fl4, rt=rt4)
    # exits from an older stat window (a detached bucket) after newer ones
    t5 = np.concatenate([T0 + 12_500 + np.arange(500), T0 + 11_200 + np.arange(500)])
    b5 = _batch(1, rng.integers(0, n_res, size=1000), t5, rt=rng.integers(1, 30, size=1000))
    b6 = _batch(0, rng.integers(0, n_res, size=5000), T0 + 13_000 + np.arange(5000))
    _check_batches(n_res, [b1, b2, b3, b4, b5, b6], degrade=degrade)


@pytest.mark.parametrize("grade", [0, 1])
def test_breaker_long_exit_flows_tiles(grade):
    """Exit-only flows of >= 2 rounds (16384 exits) go over the whole GPU in tiles (k_cbt_*): a CLOSED breaker
    tripped inside a tile of its third window, a long healthy flow (only the counts move), an OPEN breaker's
    long flow (no trip, the counts carry on), a HALF_OPEN one (left to k_cb_flows), and windows that go back
    between tiles, inside a tile and against the breaker's own window (the whole flow back to the step-by-step
    walk).  Entries after each exit batch read the breakers' states and retry times."""
    rng = np.random.default_rng(70 + grade)
    n_res = 3
    if grade == 0:
        degrade = [{"resource": r, "grade": 0, "count": 50.0, "slow_ratio_threshold": 0.4, "min_request_amount": 20,
                    "stat_interval_ms": 1000, "time_window": 2} for r in range(n_res)]
    else:
        degrade = [{"resource": r, "grade": 1, "count": 0.25, "min_request_amount": 20, "stat_interval_ms": 1000,
                    "time_window": 2} for r in range(n_res)]

    def exits(res, ts, bad):
        ts = np.asarray(ts, np.int64)
        bad = np.asarray(bad, bool)
        n = len(ts)
        rt = np.where(bad & (grade == 0), 200, rng.integers(1, 30, size=n))
        fl = np.where(bad & (grade == 1), EV_ERROR, 0).astype(np.uint8)
        return _batch(1, res, ts, flags=fl, rt=rt)

    n = 60_000
    res = rng.choice(n_res, size=n, p=[0.6, 0.3, 0.1])
    t1 = T0 + np.sort(rng.integers(0, 3_000, size=n))
    b1 = _batch(0, res, t1)
    te = t1 + 4_000  # windows T0+4 s .. T0+7 s
    bad = (rng.random(n) < 0.1) | ((res == 0) & (te >= T0 + 6_000) & (rng.random(n) < 0.6))
    b2 = exits(res, te, bad)  # resource 0: ~36k exits, trips in its third window; 1: ~18k healthy; 2: ~6k
    b3 = _batch(0, rng.choice(n_res, size=20_000), T0 + 7_500 + np.sort(rng.integers(0, 3_000, size=20_000)))
    # the probes' exits (HALF_OPEN at the start: k_cb_flows), resource 0's bad so it opens again
    k = 20_000
    r4 = np.concatenate([[0, 1, 2], rng.choice(n_res, size=k, p=[0.9, 0.05, 0.05])])
    t4 = T0 + 10_600 + np.arange(k + 3) // 20
    b4 = exits(r4, t4, np.concatenate([[True, False, False], rng.random(k) < 0.05]))
    # OPEN at the start: a long flow of resource 0 only counts
    k = 30_000
    b5 = exits(np.zeros(k), T0 + 11_800 + np.arange(k) // 20, rng.random(k) < 0.5)
    # windows that go back: resource 1 between tiles, resource 0 inside a tile, resource 2 against its window
    a = T0 + 13_500 + np.arange(10_000) // 10
    r1 = exits(np.ones(20_000), np.concatenate([a, a - 1_000]), rng.random(20_000) < 0.05)
    t0b = T0 + 13_000 + np.arange(20_000) // 10
    t0b[3_000:3_100] -= 1_000
    r0 = exits(np.zeros(20_000), t0b, rng.random(20_000) < 0.05)
    b6 = {kk: np.concatenate([r1[kk], r0[kk]]) for kk in r1}
    b7 = exits(np.full(20_000, 2), T0 + 10_000 + np.arange(20_000) // 40, rng.random(20_000) < 0.05)
    b8 = _batch(0, rng.choice(n_res, size=5_000), T0 + 16_000 + np.arange(5_000))
    _check_batches(n_res, [b1, b2, b3, b4, b5, b6, b7, b8], degrade=degrade)


def test_missing_thread_count_entry_fails_the_batch():
    """The device check of k_pseg_key: a parameter event of a per-value segment flow whose thread-count entry
    is missing (fault-injected with SGA_PSEG_FORCE_MISS=1, never expected otherwise) fails the batch with
    SGA_EIO and the check's message, instead of leaving the event undecided.  Run in a child process (the
    knob is read once per process); the same batch without the knob succeeds."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys
sys.path.insert(0, {root!r})
import numpy as np
from tests.test_pseg_gpu import _batch, _param_stream, EV_HAS_PARAM
from tests.test_configs_fullsize_gpu import _local
rng = np.random.default_rng(3)
res, vals, ts, acq = _param_stream(rng, 20_000, 2, 20, 2_000)
b = _batch(0, res, ts, acq=acq, flags=np.full(len(ts), EV_HAS_PARAM), param=vals)
eng, s = _local(2, param=[{{"resource": r, "count": 30.0}} for r in range(2)], max_batch=1 << 15)
try:
    s.submit(b["kind"], b["resource"], b["ts"], b["acquire"], b["flags"], b["rt"], b["param"])
except Exception as e:
    print("ERROR", e)
else:
    print("OK")
eng.close()
"""
    out = {}
    for knob in ("0", "1"):
        # the fault-injection hook exists only in the test-only build (flow.hip SGA_TEST_HOOKS)
        env = dict(os.environ, SGA_PSEG_FORCE_MISS=knob, SGA_LIB_VARIANT="testhooks")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[knob] = r.stdout.strip().splitlines()[-1]
    assert out["0"] == "OK", out
    assert out["1"].startswith("ERROR") and "rc=-5" in out["1"] and "k_pseg_key device check" in out["1"], out
