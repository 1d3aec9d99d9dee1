"""The oracle's capacity-bounded LRU parameter maps (a19: ParameterMetric CacheMap,
ParameterMetric.java:37-39,95-120) against the eviction vectors of tests/golden/make_lru_golden.py
(an independent pure-Python strict-LRU model; parity vs CLHM 1.4.2 itself is unpinned)."""
import ctypes as C
import glob
import json
import os

import numpy as np
import pytest

from tests import oracle_harness as H

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "lrukat_*.json")))


def _lib():
    L = H.lib()
    L.orc_prule_map_size.restype = C.c_size_t
    L.orc_prule_map_size.argtypes = [C.c_void_p, C.c_int]
    L.orc_prule_map_keys.restype = C.c_size_t
    L.orc_prule_map_keys.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]
    L.orc_prule_map_evictions.restype = C.c_uint64
    L.orc_prule_map_evictions.argtypes = [C.c_void_p, C.c_int]
    L.orc_flow_param_map_size.restype = C.c_size_t
    L.orc_flow_param_map_size.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_int]
    return L


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[7:-5] for p in GOLD])
def test_lru_eviction_vectors(path):
    doc = json.load(open(path))
    L = _lib()
    keep = []
    rule = H.param_rule_struct(doc["rule"], keep)
    p = L.orc_prule_new(C.byref(rule))
    try:
        w = C.c_int64()
        got = []
        for v, t, a in doc["events"]:
            d = L.orc_prule_pass_single(p, v, a, t, 0, C.byref(w))
            got.append([d, w.value])
        bad = [i for i, (g, e) in enumerate(zip(got, doc["expect"])) if g != e]
        assert not bad, f"first mismatch at event {bad[0]}: {doc['events'][bad[0]]} got {got[bad[0]]} " \
                        f"expect {doc['expect'][bad[0]]}"
        assert L.orc_prule_map_size(p, 0) == doc["final_time_map_size"]
        assert L.orc_prule_map_size(p, 0) <= doc["capacity"]
        keys = np.zeros(16, dtype=np.uint64)
        n = L.orc_prule_map_keys(p, 0, keys.ctypes.data, None, 16)
        assert [int(k) for k in keys[:n]] == doc["final_time_map_lru_head"]
        if doc["rule"].get("control_behavior", 0) != 2:
            # the token map sees the time map's key sequence: same keys, same evictions
            assert L.orc_prule_map_size(p, 1) == L.orc_prule_map_size(p, 0)
            assert L.orc_prule_map_evictions(p, 1) == L.orc_prule_map_evictions(p, 0)
    finally:
        L.orc_prule_free(p)


def test_negative_control_unbounded_model_differs():
    """The eviction vectors are not satisfied by an unbounded map (the round-2 semantics)."""
    doc = json.load(open([g for g in GOLD if "exhaust_then_evict" in g][0]))
    tail = doc["expect"][-6:]
    assert [d for d, _ in tail] == [1, 1, 1, 1, 1, 0]  # an unbounded map would block all six


def test_thread_count_map_capacity_4000():
    """ParameterMetric.threadCountMap (capacity 4000, :115-120): a THREAD-grade rule's count for a
    value is lost once 4000 other values were added after it (LRU), so the value passes again."""
    L = _lib()
    keep = []
    f = L.orc_flow_new(1, 0)
    rules = H.param_rules_array([{"resource": 0, "grade": 0, "count": 1}], keep)
    assert L.orc_flow_load_param_rules(f, rules, 1) == 1
    T = 1_700_000_000_000
    w = C.c_int64()
    entry = lambda v, t: L.orc_flow_entry_p(f, 0, t, 1, 0, 1, v, C.byref(w))  # noqa: E731
    assert entry(1, T) == 0          # thread count of value 1 -> 1
    assert entry(1, T) != 0          # 1 + 1 > 1: blocked (getThreadCount reads value 1: MRU)
    for k in range(3999):
        assert entry(2 + k, T + 1) == 0
    assert L.orc_flow_param_map_size(f, 0, 0, 2) == 4000
    assert entry(1, T + 2) != 0      # still cached
    assert entry(5000, T + 2) == 0   # evicts the LRU value: 2 (value 1 was read after it)
    assert entry(2, T + 2) == 0      # value 2 lost its count -> passes
    assert L.orc_flow_param_map_size(f, 0, 0, 2) == 4000
    L.orc_flow_free(f)
