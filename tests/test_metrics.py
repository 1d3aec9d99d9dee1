"""Once-per-second metrics.

CPU: the all-gather used for the node-wide aggregation, with world_size-2 gloo groups (ragged row
counts per rank, rank order kept); MetricNode thin format.
GPU: StatisticNode.metrics() snapshots (lastFetchTime filtering, per-second buckets, rt = rtSum /
success) and ClusterMetricNodeGenerator.flowToMetricNode against the oracle; the snapshot through
a one-rank RCCL process group equals the direct one."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import local_trace as lt
from tests import oracle_harness as H

T0 = 1_700_000_000_000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gather_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from sentinel_amd.metrics import all_gather_rows
    k = 3 + 5 * rank
    local = torch.arange(k * 4, dtype=torch.int64).reshape(k, 4) + 1000 * rank
    out = all_gather_rows(local)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_rows_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    exp = np.concatenate([np.arange(k * 4).reshape(k, 4) + 1000 * r for r, k in ((0, 3), (1, 8))])
    assert np.array_equal(out, exp)


def test_metric_node_thin_string():
    from sentinel_amd.local import MetricNode
    m = MetricNode(1700000000000, "a|b", 5, 1, 4, 0, 12, 2)
    # MetricNode.toThinString (CORE/node/metric/MetricNode.java:160-176)
    assert m.to_thin_string() == "1700000000000|a_b|5|1|4|0|12|2|0|0"


@pytest.mark.gpu
def test_local_metrics_snapshots_match_oracle():
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import FlowRuleManager, LocalSentinel
    from sentinel_amd.rules import FlowRule
    n_res = 16
    flow = [{"resource": r, "count": float(5 + 3 * r)} for r in range(0, n_res, 2)]
    gen = lt.Oracle(n_res, flow)
    st = lt.generate(gen, n_res, n_entries=12000, seed=5, t0=T0, gap_mean=0.6, err_pct=0.05, rt_max=30)
    gen.close()
    orc = lt.Oracle(n_res, flow)
    eng = Engine(max_batch=1 << 16)
    s = LocalSentinel(eng, [f"r{i}" for i in range(n_res)])
    FlowRuleManager(s).load_rules([FlowRule(resource=f"r{r['resource']}", count=r["count"]) for r in flow])
    ts = st["ts"]
    polls = emitted = 0
    now = T0 + 137
    lo = 0
    while lo < len(ts):
        now += 1000 if polls % 3 else 2300  # irregular polling, as a late scheduler would
        hi = int(np.searchsorted(ts, now, side="left"))
        sub = {k: np.ascontiguousarray(v[lo:hi]) for k, v in st.items()}
        if hi > lo:
            s.submit(sub["kind"], sub["resource"], sub["ts"], sub["acquire"], sub["flags"], sub["rt"], sub["param"])
            orc.replay(sub)
        got = [(m.timestamp, s.resource_id(m.resource), m.pass_qps, m.block_qps, m.success_qps, m.exception_qps,
                m.rt, m.occupied_pass_qps) for m in s.metrics(now)]
        exp = orc.metrics(now)
        assert got == exp, (now - T0, got[:3], exp[:3])
        emitted += len(got)
        polls += 1
        lo = hi
    assert polls >= 4 and emitted > 2 * n_res
    orc.close()
    eng.close()


@pytest.mark.gpu
def test_cluster_metric_nodes_and_rccl_gather():
    import torch
    from sentinel_amd import cluster
    from sentinel_amd.metrics import cluster_metric_snapshot
    from sentinel_amd.workload import ClusterTrace
    tr = ClusterTrace(n_rules=3000, lam=2_000_000)
    fid_r, cnt = tr.rules()
    eng = cluster.Engine(max_batch=1 << 18)
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_r, cnt)
    f, a, p, ts = tr.events(0, 200_000)
    cluster.DefaultTokenService(eng).request_tokens(f, a, p, ts)
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    arr = H.cluster_rules_array([{"flow_id": int(x), "count": float(c), "threshold_type": 1}
                                 for x, c in zip(fid_r, cnt)])
    L.orc_cluster_load_rules(oh, b"default", arr, len(fid_r))
    out = (H.OrcTokenResult * len(f))()
    L.orc_cluster_replay(oh, len(f), np.ascontiguousarray(f).ctypes.data, np.ascontiguousarray(a).ctypes.data,
                         np.ascontiguousarray(p).ctypes.data, np.ascontiguousarray(ts).ctypes.data, out)
    now = int(ts[-1]) + 40
    torch.cuda.set_device(0)
    direct = cluster_metric_snapshot(eng, now)
    assert len(direct) == len(fid_r)
    by = {int(r["flow_id"]): r for r in direct}
    for fid in fid_r[:500]:
        r = by[int(fid)]
        # getAvg(BLOCK) then getAvg(PASS) at now, ClusterMetric.java:64-66 (interval 1 s)
        assert r["block_qps"] == L.orc_cluster_metric_sum(oh, int(fid), 1, now) / 1.0
        assert r["pass_qps"] == L.orc_cluster_metric_sum(oh, int(fid), 0, now) / 1.0
        assert r["timestamp"] == now
    # the same snapshot through a one-rank RCCL group (the once-per-second collective)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        gathered = cluster_metric_snapshot(eng, now + 1000, group=dist.group.WORLD)
    finally:
        dist.destroy_process_group()
    assert len(gathered) == len(fid_r)
    assert set(int(x) for x in gathered["flow_id"]) == set(int(x) for x in fid_r)
    L.orc_cluster_free(oh)
    eng.close()
