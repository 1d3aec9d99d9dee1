"""GPU debug harness for the hot path: prints the last batch's path (sga_cluster_batch_info) for a
few synthetic traces.  Usage: python3 tools/hot_debug.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sentinel_amd import cluster  # noqa: E402
from sentinel_amd.cluster import ClusterFlowRuleManager, DefaultTokenService  # noqa: E402


def run(n, rules, prio_frac, ts_step_per_req, batches=3, seed=1, hot_min=1):
    eng = cluster.Engine(max_batch=1 << 20, max_rules=1 << 16, hot_rules=True, hot_min_requests=hot_min)
    fid = np.arange(1, rules + 1, dtype=np.int64)
    ClusterFlowRuleManager(eng).load_rule_arrays("default", fid, np.full(rules, 50.0))
    svc = DefaultTokenService(eng)
    rng = np.random.default_rng(seed)
    t0 = 1_700_000_000_000
    for b in range(batches):
        f = rng.integers(1, rules + 1, size=n).astype(np.int64)
        a = np.ones(n, np.int32)
        p = (rng.random(n) < prio_frac).astype(np.uint8)
        ts = t0 + ((np.arange(n) + b * n) * ts_step_per_req).astype(np.int64)
        svc.request_tokens(f, a, p, ts)
        print(f"n={n} rules={rules} prio={prio_frac} step={ts_step_per_req} batch {b}: {eng.batch_info()}",
              flush=True)
    eng.close()


if __name__ == "__main__":
    run(100_000, 1000, 0.0, 0.001)
    run(100_000, 1000, 0.5, 0.001)
    run(100_000, 1000, 0.0, 0.0)
    run(300_000, 3000, 0.01, 0.01)
