import sys, numpy as np
sys.path.insert(0, '.')
import bench_local as bl
from sentinel_amd.cluster import Engine
from sentinel_amd.local import LocalSentinel
rng = np.random.default_rng(104)
cfg = bl._cfg_c4(rng)
b = cfg["batch"]
n = 1 << 20
eng = Engine(device=0, max_batch=n)
s = LocalSentinel(eng, [f"r{i}" for i in range(cfg["n_res"])])
bl._load_rules(s, cfg)
for step in range(3):
    off = step * 100000
    ts = b.ts[:n] + off
    d, w = s.submit(np.zeros(n, np.uint8), b.res[:n], ts, b.acq[:n], b.flags[:n], np.zeros(n, np.int64), b.param[:n])
    ok = (d == 0) | (d == 4)
    idx = np.nonzero(ok)[0]
    print("entries", step, ok.mean(), flush=True)
    s.submit(np.ones(len(idx), np.uint8), b.res[:n][idx], ts[idx] + 50, b.acq[:n][idx], b.flags[:n][idx], np.full(len(idx), 10, np.int64), b.param[:n][idx])
    print("exits", step, flush=True)
eng.close()
