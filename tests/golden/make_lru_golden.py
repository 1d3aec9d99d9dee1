#!/usr/bin/env python3
"""Eviction known-answer vectors for the parameter maps' CacheMap.

The reference bounds each ParamFlowRule's time and token maps at min(4000 * durationInSec, 200000)
keys and each thread-count map at 4000 (ParameterMetric.java:37-39, 95-120), with LRU eviction by
concurrentlinkedhashmap-lru 1.4.2 -- a dependency the reference does not vendor, and no reference test
evicts.  These vectors are therefore NOT reference outputs: the expected decisions come from the small
pure-Python model below (collections.OrderedDict as the access-ordered map, strict LRU: a read or
write moves the key to the MRU end, an insert past capacity evicts the LRU end), written
independently of the C oracle, over ParamFlowChecker.passDefaultLocalCheck / passThrottleLocalCheck
(ParamFlowChecker.java:132-281).  They pin the oracle's LRU restatement (tests/test_oracle_lru.py);
parity with CLHM itself stays unpinned.

Run: python3 tests/golden/make_lru_golden.py  (writes tests/golden/lrukat_*.json)."""
import json
import os
import random
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))


class Lru:
    def __init__(self, cap):
        self.cap, self.d = cap, OrderedDict()

    def put_if_absent(self, k, v):  # None after an insert, else the present value (a read)
        if k in self.d:
            self.d.move_to_end(k)
            return self.d[k]
        self.d[k] = v
        while len(self.d) > self.cap:
            self.d.popitem(last=False)
        return None

    def get(self, k):
        if k in self.d:
            self.d.move_to_end(k)
            return self.d[k]
        return None

    def set(self, k, v):  # AtomicLong.set on a value object: no map access
        self.d[k] = v


def cap_of(duration):
    return min(4000 * duration, 200000)


def java_round(x):
    import math
    return math.floor(x + 0.5)


def default_check(time_m, token_m, rule, value, acq, now):
    token_count = int(rule["count"])
    if token_count == 0:
        return 0
    max_count = token_count + rule.get("burst_count", 0)
    if acq > max_count:
        return 0
    dur_ms = rule.get("duration_in_sec", 1) * 1000
    last = time_m.put_if_absent(value, now)
    if last is None:
        token_m.put_if_absent(value, max_count - acq)
        return 1
    pass_time = now - last
    if pass_time > dur_ms:
        old = token_m.put_if_absent(value, max_count - acq)
        if old is None:
            time_m.set(value, now)
            return 1
        to_add = (pass_time * token_count) // dur_ms
        new = max_count - acq if to_add + old > max_count else old + to_add - acq
        if new < 0:
            return 0
        token_m.set(value, new)
        time_m.set(value, now)
        return 1
    old = token_m.get(value)
    if old is None:
        raise AssertionError("time kept, token evicted: unreachable under strict LRU with equal capacities")
    if old - acq >= 0:
        token_m.set(value, old - acq)
        return 1
    return 0


def throttle_check(time_m, rule, value, acq, now):
    token_count = int(rule["count"])
    if token_count == 0:
        return 0, 0
    cost = java_round(1.0 * 1000 * acq * rule.get("duration_in_sec", 1) / token_count)
    last = time_m.put_if_absent(value, now)
    if last is None:
        return 1, 0
    expected = last + cost
    if expected <= now or expected - now < rule.get("max_queueing_time_ms", 0):
        time_m.get(value)
        wait = expected - now
        time_m.set(value, expected if wait > 0 else now)
        return 1, max(wait, 0)
    return 0, 0


def run(rule, events):
    cap = cap_of(rule.get("duration_in_sec", 1))
    time_m, token_m = Lru(cap), Lru(cap)
    out = []
    for v, t, a in events:
        if rule.get("control_behavior", 0) == 2:
            d, w = throttle_check(time_m, rule, v, a, t)
        else:
            d, w = default_check(time_m, token_m, rule, v, a, t), 0
        out.append([d, w])
    return out, sorted(time_m.d), list(time_m.d.keys())[:16]


def scenarios():
    T = 1_700_000_000_000
    out = []
    # 1. exhaust value 1, then 4000 distinct others: value 1 is the LRU key at the 4001st insert,
    #    evicted, and comes back as unseen (a fresh bucket) -> passes inside the same second
    ev = [(1, T, 1)] * 6 + [(2 + k, T + 1, 1) for k in range(4000)] + [(1, T + 2, 1)] * 6
    out.append(("exhaust_then_evict", {"count": 5}, ev))
    # 2. the same with 3999 others: value 1 is still cached and stays blocked
    ev = [(1, T, 1)] * 6 + [(2 + k, T + 1, 1) for k in range(3999)] + [(1, T + 2, 1)] * 2
    out.append(("exhaust_no_evict_at_capacity", {"count": 5}, ev))
    # 3. a read in the middle moves value 1 to the MRU end: value 2 is evicted instead
    ev = ([(1, T, 1)] * 6 + [(2 + k, T + 1, 1) for k in range(2000)] + [(1, T + 1, 1)] +
          [(2002 + k, T + 2, 1) for k in range(2000)] + [(1, T + 3, 1), (2, T + 3, 1)] * 2)
    out.append(("touch_moves_to_mru", {"count": 5}, ev))
    # 4. duration 2 -> capacity 8000
    ev = [(7, T, 3)] * 3 + [(100 + k, T + 5, 1) for k in range(8000)] + [(7, T + 6, 3)] * 2
    out.append(("duration2_capacity_8000", {"count": 6, "duration_in_sec": 2}, ev))
    # 5. throttle (time map only): an evicted value is re-admitted without waiting
    ev = [(9, T, 1), (9, T, 1)] + [(10 + k, T + 1, 1) for k in range(4000)] + [(9, T + 2, 1)]
    out.append(("throttle_evict", {"count": 10, "control_behavior": 2, "max_queueing_time_ms": 0}, ev))
    # 6. random Zipf-ish stream over 20k values, 60k events, ~3 virtual s (refills, blocks, evictions)
    rng = random.Random(0x4C5255)
    ev, t = [], T
    for i in range(30000):
        u = rng.random()
        v = int(20000 ** u) if u < 0.97 else rng.randrange(20000, 40000)
        t += rng.randrange(0, 2) if i % 7 else 0
        ev.append((v, t, 1 if rng.random() < 0.9 else rng.randrange(2, 4)))
    out.append(("random_stream_burst", {"count": 4, "burst_count": 2}, ev))
    return out


def main():
    for name, rule, events in scenarios():
        expect, keys_sorted, lru_head = run(rule, events)
        doc = {
            "source": "tests/golden/make_lru_golden.py (pure-Python strict-LRU model over ParamFlowChecker.java:"
                      "132-281 with ParameterMetric.java:37-39,95-120 capacities); parity vs CLHM 1.4.2 unpinned",
            "rule": rule, "capacity": cap_of(rule.get("duration_in_sec", 1)),
            "events": [list(e) for e in events], "expect": expect,
            "final_time_map_size": len(keys_sorted), "final_time_map_lru_head": lru_head,
        }
        with open(os.path.join(HERE, f"lrukat_{name}.json"), "w") as fh:
            json.dump(doc, fh, separators=(",", ":"))
        print(name, len(events), "events,", sum(d for d, _ in expect), "passed")


if __name__ == "__main__":
    main()
