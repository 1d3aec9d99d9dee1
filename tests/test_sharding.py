"""Multi-GPU decomposition of the cluster path (DESIGN.md "Multi-GPU").

Rules shard by splitmix64(flowId) mod G; a rank owns its shard's rules and
decides exactly the requests routed to it.  Rules never interact (no namespace
limiter in the sharded configuration), so the per-request results of G shards
must equal those of one server holding every rule.  The CPU tests run that
property with world_size-2 gloo process groups (the bench's launch shape) over
the oracle; the GPU test runs it through the engine.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from sentinel_amd.workload import ClusterTrace, shard_of
from tests import oracle_harness as H

N_RULES = 20_000
N_EVENTS = 200_000
LAM = 2_000_000


def _rules_struct(fid, cnt):
    from sentinel_amd.cluster import CLUSTER_RULE_DTYPE
    rules = np.zeros(len(fid), dtype=CLUSTER_RULE_DTYPE)
    rules["flow_id"] = fid
    rules["count"] = cnt
    rules["threshold_type"] = 1
    rules["sample_count"] = 10
    rules["window_interval_ms"] = 1000
    rules["grade"] = 1
    import ctypes as C
    assert rules.itemsize == C.sizeof(H.OrcClusterRule)
    return rules


def _oracle_replay(fid_rules, cnt_rules, f, a, p, ts):
    import ctypes as C
    L = H.lib()
    rules = _rules_struct(fid_rules, cnt_rules)
    oh = L.orc_cluster_new(1.0, 1.0)
    L.orc_cluster_load_rules(oh, b"default", rules.ctypes.data_as(C.POINTER(H.OrcClusterRule)), len(rules))
    out = (H.OrcTokenResult * max(1, len(f)))()
    f, a, p, ts = [np.ascontiguousarray(x) for x in (f, a, p, ts)]
    L.orc_cluster_replay(oh, len(f), f.ctypes.data, a.ctypes.data, p.ctypes.data, ts.ctypes.data, out)
    L.orc_cluster_free(oh)
    return np.frombuffer(out, dtype=np.int32).reshape(-1, 3)[: len(f)].copy()


def test_shard_function_partitions_rules():
    fid = np.arange(1, 100_001, dtype=np.int64)
    for g in (1, 2, 4, 8):
        s = shard_of(fid, g)
        assert s.min() >= 0 and s.max() < g
        counts = np.bincount(s, minlength=g)
        assert counts.min() > 0.95 * len(fid) / g  # balanced


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    tr = ClusterTrace(n_rules=N_RULES, lam=LAM)
    fid_all, cnt_all = tr.rules()
    mine = shard_of(fid_all, world) == rank
    f, a, p, ts = tr.events(0, N_EVENTS)
    sel = np.nonzero(shard_of(f, world) == rank)[0]
    res = _oracle_replay(fid_all[mine], cnt_all[mine], f[sel], a[sel], p[sel], ts[sel])
    # the bench's reductions: max of per-rank times, sum of per-rank event counts
    t = torch.tensor([float(rank + 1), float(len(sel))], dtype=torch.float64)
    tmax = t[:1].clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tsum = t[1:].clone()
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    gathered = [None] * world
    dist.all_gather_object(gathered, (sel, res))
    if rank == 0:
        q.put((float(tmax[0]), float(tsum[0]), gathered))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_replay_equals_single_server(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, tsum, gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert tmax == float(world) and tsum == float(N_EVENTS)
    tr = ClusterTrace(n_rules=N_RULES, lam=LAM)
    fid_all, cnt_all = tr.rules()
    f, a, p, ts = tr.events(0, N_EVENTS)
    full = _oracle_replay(fid_all, cnt_all, f, a, p, ts)
    merged = np.zeros_like(full)
    seen = np.zeros(N_EVENTS, dtype=bool)
    for sel, res in gathered:
        merged[sel] = res
        seen[sel] = True
    assert seen.all()
    assert np.array_equal(merged, full)
    assert (full[:, 0] == 1).any() and (full[:, 0] == 0).any()  # both outcomes exercised


@pytest.mark.gpu
def test_engine_shards_equal_single_engine():
    from sentinel_amd import cluster
    g = 4
    tr = ClusterTrace(n_rules=N_RULES, lam=LAM)
    fid_all, cnt_all = tr.rules()
    f, a, p, ts = tr.events(0, N_EVENTS)
    full_eng = cluster.Engine(max_batch=1 << 18)
    cluster.ClusterFlowRuleManager(full_eng).load_rule_arrays("default", fid_all, cnt_all)
    full = cluster.DefaultTokenService(full_eng).request_tokens(f, a, p, ts)
    full_eng.close()
    for r in range(g):
        mine = shard_of(fid_all, g) == r
        sel = np.nonzero(shard_of(f, g) == r)[0]
        e = cluster.Engine(max_batch=1 << 18)
        cluster.ClusterFlowRuleManager(e).load_rule_arrays("default", fid_all[mine], cnt_all[mine])
        got = cluster.DefaultTokenService(e).request_tokens(f[sel], a[sel], p[sel], ts[sel])
        e.close()
        assert np.array_equal(got, full[sel]), r


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` run bare starts two ranks itself (torch.distributed.run child process,
    before any GPU call); both join one process group (SGA_BENCH_DRY stops them before the GPU)."""
    import json
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tempfile.mkdtemp()
    env = dict(os.environ, SGA_BENCH_DRY="1", SGA_BENCH_DRY_OUT=out)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.load(open(os.path.join(out, f))) for f in sorted(os.listdir(out))]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["gpus"] == 2 and d["rank_sum"] == 1 for d in lines)


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SGA_BENCH_DRY="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus=2" in r.stderr
