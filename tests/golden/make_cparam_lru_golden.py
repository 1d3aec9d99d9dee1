#!/usr/bin/env python3
"""Eviction known-answer vectors for the cluster parameter metric's bucket maps.

ClusterParamMetric keeps, per LeapArray bucket, a ConcurrentLinkedHashMapWrapper of maxCapacity
DEFAULT_CLUSTER_MAX_CAPACITY = 4000 (ClusterParamMetric.java:37-49, ClusterParameterLeapArray.java:40-47):
getSum reads the value in every valid bucket (:52-62), addValue putIfAbsent's it into the current one
(:79-88), a bucket reset clears its map.  The LRU itself is concurrentlinkedhashmap-lru 1.4.2, which the
reference does not vendor, and no reference test evicts.  These vectors are therefore NOT reference
outputs: the expected results come from the small pure-Python model below (one OrderedDict per bucket as
the access-ordered map, strict LRU: a get or putIfAbsent of a present key moves it to the MRU end, an
insert past capacity evicts the LRU end), written independently of the C oracle, over
ClusterParamFlowChecker.acquireClusterToken (ClusterParamFlowChecker.java:42-87).  They pin the oracle's
restatement (tests/test_cluster_param_oracle.py) and the engine (tests/test_cluster_param_gpu.py);
parity with CLHM itself stays unpinned.

Run: python3 tests/golden/make_cparam_lru_golden.py  (writes tests/golden/cparamlru_*.json)."""
import json
import os
import random
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))
T0 = 1_700_000_000_000


class Metric:
    """ClusterParamMetric over ClusterParameterLeapArray(sampleCount, intervalInMs, capacity)."""

    def __init__(self, sample_count, interval, cap):
        self.S, self.interval, self.W, self.cap = sample_count, interval, interval // sample_count, cap
        self.start = [None] * sample_count
        self.maps = [OrderedDict() for _ in range(sample_count)]

    def current(self, t):  # LeapArray.currentWindow: the bucket index, None for a detached bucket
        idx, ws = (t // self.W) % self.S, t - t % self.W
        if self.start[idx] is None or ws > self.start[idx]:
            self.start[idx] = ws
            self.maps[idx] = OrderedDict()
            return idx
        return idx if ws == self.start[idx] else None

    def get_sum(self, v, t):
        self.current(t)
        s = 0
        for j in range(self.S):
            if self.start[j] is None or t - self.start[j] > self.interval:
                continue
            m = self.maps[j]
            if v in m:
                m.move_to_end(v)
                s += m[v]
        return s

    def add(self, v, c, t):
        idx = self.current(t)
        if idx is None:
            return
        m = self.maps[idx]
        if v in m:
            m.move_to_end(v)
            m[v] += c
            return
        m[v] = c
        while len(m) > self.cap:
            m.popitem(last=False)


def acquire(metric, rule, count, values, t):
    """(status, remaining): OK 0 / BLOCKED 1, ClusterParamFlowChecker.java:42-87 (GLOBAL threshold)."""
    remaining, passed = -1.0, True
    for v in values:
        thr = float(rule.get("hot", {}).get(v, rule["count"]))
        nxt = thr - metric.get_sum(v, t) / (metric.interval / 1000.0) - count
        remaining = nxt
        if nxt < 0:
            passed = False
            break
    if passed:
        for v in values:
            metric.add(v, count, t)
    if len(values) > 1:
        remaining = -1.0
    return (0, int(remaining)) if passed else (1, 0)


def scenarios():
    out = []
    cap = 4000
    # 1. value 1 exhausted, then 4000 distinct others in the same bucket: value 1 is the LRU key at the
    #    4000th insert, evicted, and passes again inside the same window
    ev = [(1, T0)] * 6 + [(2 + k, T0 + 1) for k in range(4000)] + [(1, T0 + 2)] * 6
    out.append(("exhaust_then_evict", {"count": 5, "sample_count": 10, "window_interval_ms": 1000}, ev, []))
    # 2. 3999 others: value 1 stays in the map and stays blocked
    ev = [(1, T0)] * 6 + [(2 + k, T0 + 1) for k in range(3999)] + [(1, T0 + 2)] * 2
    out.append(("exhaust_no_evict_at_capacity", {"count": 5, "sample_count": 10, "window_interval_ms": 1000}, ev, []))
    # 3. a blocked request's getSum still reads value 1 (moves it to the MRU end): value 2 goes instead
    ev = ([(1, T0)] * 6 + [(2 + k, T0 + 1) for k in range(2000)] + [(1, T0 + 1)] +
          [(2002 + k, T0 + 2) for k in range(2000)] + [(1, T0 + 3), (2, T0 + 3)] * 2)
    out.append(("blocked_get_moves_to_mru", {"count": 5, "sample_count": 10, "window_interval_ms": 1000}, ev, []))
    # 4. two buckets of 500 ms: the older bucket's reads (getSum over valid buckets) keep its keys
    #    fresh there; evictions happen per bucket
    ev = ([(k, T0 + k // 40) for k in range(4500)] +                       # bucket 0: 4500 keys -> 500 evicted
          [(k, T0 + 600) for k in range(0, 4500, 3)] +                     # bucket 1: reads bucket 0 too
          [(9000 + k, T0 + 700) for k in range(3000)] +
          [(k, T0 + 800) for k in range(0, 4500, 7)])
    out.append(("two_buckets", {"count": 3, "sample_count": 2, "window_interval_ms": 1000}, ev,
                [(k, T0 + 900) for k in range(0, 4500, 250)]))
    # 5. random stream: Zipf-ish over 3000 values plus a uniform tail over 10^6, 10000 requests a 250 ms
    #    bucket (about 6000 distinct values each), 1.5 virtual s, hot items
    rng = random.Random(0xC9A2)
    ev, t = [], T0
    for i in range(60000):
        u = rng.random()
        v = int(3000 ** (u / 0.45)) if u < 0.45 else rng.randrange(3000, 1_000_000)
        t += 1 if i % 40 == 0 else 0
        ev.append((v, t))
    out.append(("random_stream", {"count": 4, "sample_count": 4, "window_interval_ms": 1000, "hot": {1: 9, 2: 50}},
                ev, [(v, t + 10) for v in (1, 2, 3, 5, 8, 13, 21, 34)]))
    return out, cap


def main():
    scen, cap = scenarios()
    for name, rule, events, sums in scen:
        m = Metric(rule["sample_count"], rule["window_interval_ms"], cap)
        expect = [list(acquire(m, rule, 1, [v], t)) for v, t in events]
        sums_out = [[v, t, m.get_sum(v, t)] for v, t in sums]
        doc = {
            "source": "tests/golden/make_cparam_lru_golden.py (pure-Python strict-LRU model of ClusterParamMetric, "
                      "ClusterParamMetric.java:37-88, over ClusterParamFlowChecker.java:42-87); parity vs CLHM "
                      "1.4.2 unpinned",
            "rule": {k: ({str(a): b for a, b in v.items()} if k == "hot" else v) for k, v in rule.items()},
            "capacity": cap, "flow_id": 7, "acquire": 1,
            "events": [list(e) for e in events], "expect": expect, "sums": sums_out,
        }
        with open(os.path.join(HERE, f"cparamlru_{name}.json"), "w") as fh:
            json.dump(doc, fh, separators=(",", ":"))
        print(name, len(events), "requests,", sum(1 for s, _ in expect if s == 0), "passed")


if __name__ == "__main__":
    main()
