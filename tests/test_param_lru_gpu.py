"""GPU parity for ParameterMetric's capacity-bounded CacheMaps (a19: ParameterMetric.java:37-39,95-121,
ConcurrentLinkedHashMapWrapper over CLHM 1.4.2, restated as strict LRU -- parity against CLHM itself is
unpinned, exact against the oracle's restatement, oracle/oracle_ext.c lru_*).

* The eviction vectors of tests/golden/lrukat_*.json (an independent pure-Python LRU model,
  tests/golden/make_lru_golden.py) replayed through the engine: one resource, one parameter rule,
  entries only, in small and large chunks (an owner crosses its capacity inside a batch and between
  batches, so both the count pass and the switch to LRU mode are exercised).
* A THREAD-grade rule whose thread-count map (capacity 4000) evicts: the count of an evicted value is
  lost, so the value passes again.
* C4 full mode: 10k ParamFlowRules with Zipf(1.1) values over 10^7 WITHOUT folding, entries and exits,
  bit-exact against the oracle (decisions, waits, metric rows, hot node views)."""
import glob
import json
import os

import numpy as np
import pytest

from tests import local_trace as lt
from tests.test_configs_fullsize_gpu import T0, _check_local, _local, _zipf

pytestmark = pytest.mark.gpu

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "lrukat_*.json")))


@pytest.mark.parametrize("chunk", [1 << 15, 1000])
@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[7:-5] for p in GOLD])
def test_lru_vectors_through_engine(path, chunk):
    doc = json.load(open(path))
    r = dict(doc["rule"])
    rule = {"resource": 0, "count": float(r.pop("count")), **r}
    ev = np.asarray(doc["events"], dtype=np.int64)
    n = len(ev)
    st = {"kind": np.zeros(n, np.uint8), "resource": np.zeros(n, np.uint32), "ts": ev[:, 1].copy(),
          "acquire": ev[:, 2].astype(np.int32), "flags": np.full(n, 4, np.uint8), "rt": np.zeros(n, np.int64),
          "param": ev[:, 0].astype(np.uint64)}
    eng, s = _local(1, param=[rule], max_batch=chunk)
    got_d = np.zeros(n, np.int8)
    got_w = np.zeros(n, np.int32)
    for lo in range(0, n, chunk):
        sub = {k: np.ascontiguousarray(v[lo:lo + chunk]) for k, v in st.items()}
        d, w = s.submit(sub["kind"], sub["resource"], sub["ts"], sub["acquire"], sub["flags"], sub["rt"],
                        sub["param"])
        got_d[lo:lo + len(d)] = d
        got_w[lo:lo + len(w)] = w
    eng.close()
    exp = np.asarray(doc["expect"], dtype=np.int64)
    want_d = np.where(exp[:, 0] == 1, 0, 2)  # pass / ParamFlowException
    bad = np.nonzero(got_d != want_d)[0]
    assert len(bad) == 0, f"{len(bad)} of {n} differ; first at {bad[0]}: event {ev[bad[0]]} got {got_d[bad[0]]}"
    ok = want_d == 0
    assert np.array_equal(got_w[ok], exp[ok, 1].astype(np.int32))


def test_thread_count_map_evicts_at_4000():
    """ParameterMetric.threadCountMap (capacity 4000): 5000 values enter (count 1 each, no exits); the
    oldest ones lose their count, so they pass again while the newest still block (THREAD grade, count 1)."""
    n_vals = 5000
    vals = np.concatenate([np.arange(1, n_vals + 1), [1, 2, n_vals, n_vals - 1, 500, 1500]]).astype(np.uint64)
    n = len(vals)
    st = {"kind": np.zeros(n, np.uint8), "resource": np.zeros(n, np.uint32),
          "ts": T0 + np.arange(n, dtype=np.int64), "acquire": np.ones(n, np.int32),
          "flags": np.full(n, 4, np.uint8), "rt": np.zeros(n, np.int64), "param": vals}
    param = [{"resource": 0, "grade": 0, "count": 1}]
    d = _check_local(1, st, param=param, max_batch=1 << 12, hot_nodes=1)
    tail = list(d[-6:])
    assert tail == [0, 0, 2, 2, 0, 2], tail  # values 1, 2, 500 were evicted; 1500, 4999, 5000 still counted


@pytest.mark.parametrize("n", [1 << 20, 1 << 22])
def test_c4_full_mode_10k_rules_unfolded_values(n):
    """BASELINE C4 as stated: 10k ParamFlowRules, Zipf(1.1) parameter values over 10^7 (no folding), so the
    hot rules' maps hold their 4000 (or 8000) most recently used values and evict on every new one."""
    rng = np.random.default_rng(204)
    n_res = 10_000
    param = [{"resource": r, "count": float(rng.integers(1, 100)),
              **({"control_behavior": 2, "max_queueing_time_ms": int(rng.choice([0, 50, 200]))} if r % 10 == 9 else {}),
              **({"duration_in_sec": 2} if r % 7 == 3 else {})}
             for r in range(n_res)]
    res = _zipf(rng, n_res, n)
    vals = _zipf(rng, 10_000_000, n)  # full mode: no % 4000
    ts = T0 + (np.arange(n) // 1000)
    gen = lt.Oracle(n_res, [], param)
    st = lt.generate_windows(gen, res, ts, np.ones(n), np.full(n, 4, np.uint8), vals.astype(np.uint64),
                             rng.integers(1, 30, size=n), np.zeros(n, bool), window_ms=1)
    gen.close()
    d = _check_local(n_res, st, param=param, max_batch=1 << 21)
    ent = st["kind"] == 0
    assert (d[ent] == 0).any() and (d[ent] == 2).any()
