"""Once-per-second metric aggregation across the GPUs of a node.

Each rank's engine writes its shard's snapshot into device memory
(sga_cluster_metric_nodes_device: ClusterMetricNodeGenerator.flowToMetricNode,
CS/flow/statistic/ClusterMetricNodeGenerator.java:75-91) and the ranks exchange them with one
all-gather -- RCCL over xGMI when the process group is "nccl" (ROCm), the only collective of the
engine and off the decision path.  Rank order is kept, so the merged list is the shards' lists
concatenated.
"""
import ctypes as C

import numpy as np

from . import _lib

CLUSTER_NODE_DTYPE = np.dtype([("flow_id", "<i8"), ("pass_qps", "<f8"), ("block_qps", "<f8"),
                               ("timestamp", "<i8")])


def all_gather_rows(local, group=None):
    """All-gathers a [k, w] int64 tensor whose k differs per rank; returns the [sum k, w]
    concatenation in rank order (on every rank).  One count exchange, one padded all-gather."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    k = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    ks = [int(x.item()) for x in ks]
    kmax = max(max(ks), 1)
    pad = torch.zeros((kmax, local.shape[1]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * kmax, local.shape[1]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, pad, group=group)
        parts = [out[r * kmax: r * kmax + ks[r]] for r in range(world)]
    else:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        parts = [bufs[r][: ks[r]] for r in range(world)]
    return torch.cat(parts, dim=0)


def cluster_metric_snapshot(engine, now: int, group=None) -> np.ndarray:
    """ClusterMetricNode of every active cluster flow rule of every rank's engine at `now`
    (structured array, CLUSTER_NODE_DTYPE).  Without a process group: this engine only."""
    import torch
    L = _lib.load()
    act = C.c_uint64()
    _lib.check(L.sga_cluster_stats(engine.handle, C.byref(act), None), engine.handle, "stats")
    cap = max(int(act.value), 1)
    dev = torch.device("cuda", torch.cuda.current_device())
    # a stream of our own: torch's default stream is the NULL handle, which the C-ABI reads as
    # "the engine's stream" -- the snapshot, the count read and the collective must share one
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        rows = torch.empty((cap, 4), dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(L.sga_cluster_metric_nodes_device(engine.handle, now, rows.data_ptr(), cap, cnt.data_ptr(),
                                                     side.cuda_stream), engine.handle, "clusterMetricNodes")
        n = int(cnt.item())
        local = rows[:n]
        if group is not None or _dist_ready():
            local = all_gather_rows(local, group)
        res = local.cpu().numpy()
    return res.view(CLUSTER_NODE_DTYPE).reshape(-1)


def _dist_ready():
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    except Exception:
        return False
