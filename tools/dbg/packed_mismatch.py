"""Debug: the packed entry against the array entry on batch 0 of test_packed_entry_matches_arrays_and_oracle[on]."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from sentinel_amd import _lib, cluster
from sentinel_amd.workload import ClusterTrace
from tests.test_packed_device_gpu import _engine, _run, _decode

L = _lib.load()
dev = torch.device("cuda", 0)
tr = ClusterTrace(n_rules=3000, lam=3_000_000, prio_pct=5)
fid_r, cnt = tr.rules()
cnt = np.minimum(cnt, 500.0)
m = 200_000
rng = np.random.default_rng(7)
f, a, p, ts = tr.events(0, m)
f, a = f.copy(), a.copy()
k = rng.integers(0, m, size=m // 200)
f[k[: len(k) // 3]] = 0
f[k[len(k) // 3: 2 * len(k) // 3]] = 3000 + rng.integers(1, 1000, size=len(k[len(k) // 3: 2 * len(k) // 3]))
a[k[2 * len(k) // 3:]] = 0
j = rng.integers(0, m, size=m // 500)
a[j] = rng.choice([2, 3, 200, 65535], size=len(j))
r = rng.integers(0, m, size=m // 300)
a_arr = a.copy()
a_arr[r] = 0
mode = sys.argv[1] if len(sys.argv) > 1 else "on"
out = {}
for name, aa, rv, pk in (("arr", a_arr, None, False), ("pk", a, r, True), ("arr2", a_arr, None, False), ("pk_nores", a_arr, None, True)):
    eng = _engine(cluster, mode, max_batch=m)
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
    out[name] = _run(L, eng, dev, f, aa, p, ts, pk, rv)
    print(name, eng.batch_info())
    eng.close()
for x, y in (("arr", "arr2"), ("arr", "pk"), ("arr", "pk_nores")):
    bad = np.nonzero(out[x] != out[y])[0]
    print(x, "vs", y, "mismatches", len(bad))
    rs = set(r.tolist())
    for i in bad[:10]:
        print("  i", i, "f", f[i], "a", a[i], "a_arr", a_arr[i], "p", p[i], "resv", i in rs, "ts", ts[i] - ts.min(),
              x, _decode(out[x][i:i + 1]), y, _decode(out[y][i:i + 1]))
