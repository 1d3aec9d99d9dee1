"""Debug: C3 full-size, two batches through the packed entry; describe the requests that differ from the oracle."""
import numpy as np
import torch
from sentinel_amd import _lib, cluster
from sentinel_amd.workload import ClusterTrace, DeviceClusterGen, pack_requests
from tests import oracle_harness as H

L = _lib.load()
dev = torch.device("cuda", 0)
tr = ClusterTrace()
fid_r, cnt = tr.rules()
gen = DeviceClusterGen(dev)
m = 1 << 24
eng = cluster.Engine(device=0, max_batch=m + 1024, max_rules=1 << 20)
cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
host, outs = [], []
for b in range(2):
    f, a, p, t, base, n = gen.batch(b * m, m)
    rec = pack_requests(f, a, p, t)
    o = torch.zeros(n, dtype=torch.int64, device=dev)
    rc = L.sga_request_tokens_packed_device(eng.handle, rec.data_ptr(), base, n, o.data_ptr(), None)
    assert rc == 0
    assert L.sga_sync(eng.handle) == 0
    host.append((f.cpu().numpy(), a.cpu().numpy(), p.cpu().numpy(), t.cpu().numpy().astype(np.int64) + base))
    outs.append(o.cpu().numpy())
    print("batch", b, eng.batch_info(), flush=True)
orc = H.cluster_replay_sharded(fid_r, cnt, host, threads=16)
for b in range(2):
    r = outs[b].view(np.uint64)
    st = ((r >> np.uint64(48)) & np.uint64(0xFF)).astype(np.int8).astype(np.int32)
    rem = (r & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
    wt = ((r >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16).astype(np.int32)
    ost, orem, owt = orc[b]
    bad = np.nonzero((st != ost) | (rem != orem) | (wt != owt))[0]
    f, a, p, ts = host[b]
    print(f"batch {b}: {bad.size} mismatches; prio among bad {p[bad].mean() if bad.size else 0:.3f} (all {p.mean():.4f})")
    if bad.size:
        pairs = {}
        for i in bad:
            k = (int(st[i]), int(ost[i]))
            pairs[k] = pairs.get(k, 0) + 1
        print("  (gpu status, oracle status):", sorted(pairs.items(), key=lambda x: -x[1])[:8])
        fb = f[bad]
        u, c = np.unique(fb, return_counts=True)
        print("  distinct flows among bad", u.size, "top", list(zip(u[np.argsort(-c)][:8].tolist(), np.sort(c)[::-1][:8].tolist())))
        # for the top flow: its requests in order, gpu vs oracle
        top = u[np.argmax(c)]
        idx = np.nonzero(f == top)[0]
        bi = set(bad.tolist())
        first = [j for j in range(idx.size) if idx[j] in bi][:3]
        print("  top flow requests", idx.size, "first bad positions within flow", first)
        for j in first[:1]:
            for q in range(max(0, j - 4), min(idx.size, j + 6)):
                i = idx[q]
                print(f"    i={i} ts={ts[i]} acq={a[i]} prio={p[i]} gpu=({st[i]},{rem[i]},{wt[i]}) orc=({ost[i]},{orem[i]},{owt[i]})")
eng.close()
