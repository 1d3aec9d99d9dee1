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


# ---- the local path (SphU.entry / Entry.exit through the slot chain): resources shard by
# splitmix64(resource id) mod G (bench_local.py).  Resources are independent without
# SystemRules and RELATE / CHAIN strategies (FlowRuleChecker.java:96-116 reads another resource's node: such
# resources must be co-located, which the engine leaves to the caller), so a shard's decisions equal one
# engine's on the same events.
L_RES, L_EVENTS = 2_000, 60_000


def _local_stream():
    """A C2-like mixed workload (Default / RateLimiter / WarmUp rules, Zipf resources, acquire 1-5), its entries
    then the exits of the entries that passed (masked by the deciding replay's own decisions)."""
    rng = np.random.default_rng(77)
    flow = []
    for r in range(L_RES):
        b = rng.random()
        c = float(rng.integers(5, 300))
        if b < 0.4:
            flow.append(dict(resource=r, count=c))
        elif b < 0.7:
            flow.append(dict(resource=r, count=c, control_behavior=2, max_queueing_time_ms=500))
        else:
            flow.append(dict(resource=r, count=c, control_behavior=1, warm_up_period_sec=10))
    p = 1.0 / np.arange(1, L_RES + 1) ** 1.1
    res = rng.choice(L_RES, size=L_EVENTS, p=p / p.sum())
    ts = 1_700_000_000_000 + np.arange(L_EVENTS) // 20
    acq = np.where(rng.random(L_EVENTS) < 0.05, rng.integers(2, 6, size=L_EVENTS), 1)
    rt = rng.geometric(0.2, size=L_EVENTS)
    return flow, res.astype(np.uint32), ts.astype(np.int64), acq.astype(np.int32), rt.astype(np.int64)


def _local_events(res, ts, acq, sel):
    n = len(sel)
    return {"kind": np.zeros(n, np.uint8), "resource": res[sel], "ts": ts[sel], "acquire": acq[sel],
            "flags": np.zeros(n, np.uint8), "rt": np.zeros(n, np.int64), "param": np.zeros(n, np.uint64)}


def _local_exits(res, ts, acq, rt, sel, dec):
    ok = sel[(dec == 0) | (dec == 4)]
    order = ok[np.argsort(ts[ok] + rt[ok], kind="stable")]
    n = len(order)
    return {"kind": np.ones(n, np.uint8), "resource": res[order], "ts": ts[order] + rt[order], "acquire": acq[order],
            "flags": np.zeros(n, np.uint8), "rt": rt[order], "param": np.zeros(n, np.uint64)}


def _local_replay(flow, res, ts, acq, rt, sel):
    from tests import local_trace as lt
    orc = lt.Oracle(L_RES, flow)
    dec, wait = orc.replay(_local_events(res, ts, acq, sel))
    ex = _local_exits(res, ts, acq, rt, sel, dec)
    orc.replay(ex)
    now = int(ts.max()) + 10_000
    nodes = {int(r): orc.node(int(r), now) for r in np.unique(res[sel])[:200]}
    orc.close()
    return dec, wait, nodes


def _local_rank_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    flow, res, ts, acq, rt = _local_stream()
    mine = shard_of(res.astype(np.int64), world) == rank
    sel = np.nonzero(mine)[0]
    own_rules = [r for r in flow if shard_of(np.array([r["resource"]]), world)[0] == rank]
    dec, wait, nodes = _local_replay(own_rules, res, ts, acq, rt, sel)
    gathered = [None] * world
    dist.all_gather_object(gathered, (sel, dec, wait, nodes))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_local_shards_equal_single_replay():
    """world 2 (gloo, the bench's launch shape): each rank replays the local oracle over its resource shard
    (its rules only, its events in arrival order, the exits of its passes); merged, every decision, wait and
    node view equals one oracle holding every rule."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    flow, res, ts, acq, rt = _local_stream()
    dec, wait, nodes = _local_replay(flow, res, ts, acq, rt, np.arange(L_EVENTS))
    md, mw = np.full(L_EVENTS, 99, np.int8), np.zeros(L_EVENTS, np.int32)
    for sel, d, w, nd in gathered:
        md[sel] = d
        mw[sel] = w
        for r, v in nd.items():
            if r in nodes:
                assert v == nodes[r], r
    assert np.array_equal(md, dec) and np.array_equal(mw, wait)
    assert (dec == 0).any() and (dec == 1).any()


def test_local_bench_gpus2_launches_and_routes():
    """`bench.py --config c5b --gpus 2` run bare starts two ranks (torch.distributed.run, before any GPU call);
    each builds its shard (SGA_BENCH_DRY stops it before the GPU): disjoint resource sets covering all 10k, every
    event on an own resource, both ranks' full per-GPU batches."""
    import json
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tempfile.mkdtemp()
    env = dict(os.environ, SGA_BENCH_DRY="1", SGA_BENCH_DRY_OUT=out)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--config", "c5b", "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.load(open(os.path.join(out, f))) for f in sorted(os.listdir(out))]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["events_on_own"] and d["world"] == 2 for d in lines)
    assert sum(d["own_resources"] for d in lines) == 10_000
    assert all(d["events_all_ranks"] == 2 * (1 << 22) for d in lines)


@pytest.mark.gpu
def test_local_engines_per_shard_equal_single_engine():
    """The local path through the engine: G = 2 engines on one device, each holding one resource shard's rules
    and deciding that shard's entries and exits, equal one engine holding every rule (decisions, waits)."""
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import FlowRuleManager, LocalSentinel
    from sentinel_amd.rules import FlowRule
    flow, res, ts, acq, rt = _local_stream()

    def run(rules, sel):
        eng = Engine(max_batch=1 << 17)
        s = LocalSentinel(eng, [f"r{i}" for i in range(L_RES)])
        FlowRuleManager(s).load_rules([FlowRule(resource=f"r{r['resource']}", **{k: v for k, v in r.items()
                                                                                 if k != "resource"}) for r in rules])
        e = _local_events(res, ts, acq, sel)
        d, w = s.submit(e["kind"], e["resource"], e["ts"], e["acquire"], e["flags"], e["rt"], e["param"])
        x = _local_exits(res, ts, acq, rt, sel, d)
        s.submit(x["kind"], x["resource"], x["ts"], x["acquire"], x["flags"], x["rt"], x["param"])
        now = int(ts.max()) + 10_000
        mine = set(np.unique(res[sel]).tolist())
        views = {int(r): s.node(int(r), now) for r in probe if int(r) in mine}
        eng.close()
        return d, w, views

    probe = np.unique(res)[:200]  # the resources whose node views are compared
    d1, w1, v1 = run(flow, np.arange(L_EVENTS))
    for rank in range(2):
        sel = np.nonzero(shard_of(res.astype(np.int64), 2) == rank)[0]
        own = [r for r in flow if shard_of(np.array([r["resource"]]), 2)[0] == rank]
        d, w, v = run(own, sel)
        assert np.array_equal(d, d1[sel]) and np.array_equal(w, w1[sel]), rank
        for r, view in v.items():
            assert view == v1[r], (rank, r)
