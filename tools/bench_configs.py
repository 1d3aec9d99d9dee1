"""Throughput of the other BASELINE.json configurations (C1, C2, C4, C5) on one MI355X, beside the
C oracle on a sample of the same stream (one host thread).  bench.py measures the headline (C3);
this tool records the rest for BASELINE.md.  Synthetic data, random rules; every number is the
host API (sga_submit_events / sga_rls_should_rate_limit) with host buffers, i.e. PCIe included.

Usage (GPU box): python3 tools/bench_configs.py [--quick] > gpurun_out/configs.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

T0 = 1_700_000_000_000


def zipf_ids(rng, n_items, size, s=1.1):
    p = 1.0 / np.arange(1, n_items + 1) ** s
    p /= p.sum()
    return rng.choice(n_items, size=size, p=p)


def stream(kind_n, resource, ts, acquire=None, flags=None, rt=None, param=None):
    n = len(resource)
    return {"kind": np.zeros(n, np.uint8) if kind_n is None else kind_n.astype(np.uint8),
            "resource": resource.astype(np.uint32), "ts": ts.astype(np.int64),
            "acquire": np.ones(n, np.int32) if acquire is None else acquire.astype(np.int32),
            "flags": np.zeros(n, np.uint8) if flags is None else flags.astype(np.uint8),
            "rt": np.zeros(n, np.int64) if rt is None else rt.astype(np.int64),
            "param": np.zeros(n, np.uint64) if param is None else param.astype(np.uint64)}


def time_gpu(s, st, chunk, reps=3):
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        for lo in range(0, len(st["kind"]), chunk):
            sl = slice(lo, lo + chunk)
            s.submit(st["kind"][sl], st["resource"][sl], st["ts"][sl], st["acquire"][sl], st["flags"][sl],
                     st["rt"][sl], st["param"][sl])
            print(f"  chunk @{lo}: {time.perf_counter() - t:.2f} s", file=sys.stderr, flush=True)
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    return best


def time_oracle(orc, st, sample):
    sub = {k: np.ascontiguousarray(v[:sample]) for k, v in st.items()}
    t = time.perf_counter()
    orc.replay(sub)
    return time.perf_counter() - t


def local_case(name, n_res, st, flow=(), param=(), degrade=(), chunk=1 << 22, sample=1 << 20, reps=2):
    """Fresh engine + oracle per repetition: the stream's time range restarts each time."""
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import LocalSentinel
    from tests import local_trace as lt
    from tests.test_local_parity_gpu import _load
    best = None
    for _ in range(reps):
        eng = Engine(max_batch=chunk)
        s = LocalSentinel(eng, [f"r{i}" for i in range(n_res)])
        _load(s, flow=list(flow) or None, param=list(param) or None, degrade=list(degrade) or None)
        dt = time_gpu(s, st, chunk, reps=1)
        best = dt if best is None else min(best, dt)
        eng.close()
    orc = lt.Oracle(n_res, list(flow), list(param), list(degrade))
    ct = time_oracle(orc, st, sample)
    orc.close()
    n = len(st["kind"])
    return {"config": name, "events": n, "gpu_s": best, "gpu_events_per_s": n / best,
            "cpu_sample": min(sample, n), "cpu_s": ct, "cpu_events_per_s": min(sample, n) / ct,
            "note": "sga_submit_events with host buffers (PCIe included); oracle = 1 host thread"}


def c1(rng, n):
    ts = T0 + np.cumsum(rng.integers(0, 3, size=n))  # ~1 event / ms
    st = stream(None, np.zeros(n, np.int64), ts)
    return local_case("C1 HelloWorld QPS 20 (DefaultController)", 1, st, flow=[{"resource": 0, "count": 20.0}],
                      chunk=1 << 20)


def c2(rng, n):
    n_res = 100_000
    res = zipf_ids(rng, n_res, n)
    ts = T0 + (np.arange(n) // 1000)  # 1M events per virtual second
    flow = []
    for r in range(n_res):
        b = r % 3
        flow.append({"resource": r, "count": float(rng.integers(5, 500)), "control_behavior": [0, 2, 1][b],
                     "max_queueing_time_ms": 500, "warm_up_period_sec": 10})
    st = stream(None, res, ts)
    return local_case("C2 100k FlowRules Default/RateLimiter/WarmUp, Zipf(1.1)", n_res, st, flow=flow)


def c4(rng, n):
    n_res = 10_000
    res = zipf_ids(rng, n_res, n)
    vals = zipf_ids(rng, 10_000_000, n) if n <= 4_000_000 else rng.integers(0, 10_000_000, size=n)
    ts = T0 + (np.arange(n) // 1000)
    param = [{"resource": r, "count": float(rng.integers(1, 100))} for r in range(n_res)]
    st = stream(None, res, ts, flags=np.full(n, 4), param=vals)
    return local_case("C4 10k ParamFlowRules x Zipf params over 10M values", n_res, st, param=param,
                      chunk=1 << 21)


def c5(rng, n):
    from sentinel_amd import cluster
    from tests import oracle_harness as H
    # Envoy RLS: 2 descriptors per request over 100k RLS rules (GLOBAL, sampleCount 1)
    n_rules = 100_000
    fids = np.arange(1, n_rules + 1, dtype=np.int64) * 7919 + 2147483647
    eng = cluster.Engine(max_batch=1 << 22)
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fids, rng.integers(10, 1000, size=n_rules),
                                                         threshold_type=1, sample_count=1)
    svc = cluster.EnvoyRlsService(eng)
    nreq = n // 2
    off = np.arange(0, 2 * nreq + 1, 2, dtype=np.uint32)
    dfid = fids[zipf_ids(rng, n_rules, 2 * nreq)]
    hits = np.ones(nreq, np.int32)
    ts = T0 + (np.arange(nreq) // 1000)
    best = None
    for rep in range(3):
        # each repetition continues the clock (a stream that restarts at T0 would go back in time
        # and send every rule through the per-request replay)
        ts_rep = ts + rep * (nreq // 1000 + 10_000)
        t = time.perf_counter()
        for lo in range(0, nreq, 1 << 20):
            hi = min(nreq, lo + (1 << 20))
            svc.should_rate_limit(off[lo:hi + 1] - off[lo], dfid[off[lo]:off[hi]], hits[lo:hi], ts_rep[lo:hi])
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    eng.close()
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    arr = H.cluster_rules_array([{"flow_id": int(f), "count": 100.0, "threshold_type": 1, "sample_count": 1}
                                 for f in fids])
    L.orc_cluster_load_rules(oh, b"default", arr, n_rules)
    k = min(200_000, 2 * nreq)
    t = time.perf_counter()
    for d in range(k):
        L.orc_cluster_request_token_simple(oh, int(dfid[d]), 1, int(ts[d // 2]))
    ct = time.perf_counter() - t
    L.orc_cluster_free(oh)
    rls = {"config": "C5a Envoy RLS, 2 descriptors/request, 100k rules", "descriptors": 2 * nreq, "gpu_s": best,
           "gpu_descriptors_per_s": 2 * nreq / best, "cpu_sample": k, "cpu_s": ct, "cpu_descriptors_per_s": k / ct,
           "note": "sga_rls_should_rate_limit, host buffers; oracle SimpleClusterFlowChecker via ctypes per call"}
    # DegradeSlot: 10k resources with RT / exception-ratio breakers, entries + exits with RT
    n_res = 10_000
    m = n // 2
    res = zipf_ids(rng, n_res, m)
    ts_e = T0 + (np.arange(m) // 1000)
    rt = rng.integers(1, 200, size=m)
    kind = np.zeros(2 * m, np.uint8)
    kind[1::2] = 1
    rr = np.repeat(res, 2)
    tt = np.repeat(ts_e, 2)
    tt[1::2] += rt
    order = np.argsort(tt, kind="stable")
    flags = np.zeros(2 * m, np.uint8)
    flags[1::2] = (rng.random(m) < 0.05) * 2
    rts = np.zeros(2 * m, np.int64)
    rts[1::2] = rt
    st = stream(kind[order], rr[order], tt[order], flags=flags[order], rt=rts[order])
    degrade = [{"resource": r, "grade": r % 2, "count": 100.0 if r % 2 == 0 else 0.5, "time_window": 2,
                "min_request_amount": 5, "slow_ratio_threshold": 0.5} for r in range(n_res)]
    deg = local_case("C5b DegradeSlot breakers, 10k resources, entries + exits", n_res, st, degrade=degrade)
    return [rls, deg]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    n = 1 << 20 if a.quick else 1 << 22
    rng = np.random.default_rng(1)
    for name, fn in (("c1", c1), ("c2", c2), ("c4", c4), ("c5", c5)):
        if a.only and name not in a.only.split(","):
            continue
        r = fn(rng, 1_000_000 if name == "c1" else n)
        for x in (r if isinstance(r, list) else [r]):
            print(json.dumps(x), flush=True)


if __name__ == "__main__":
    main()
