#!/usr/bin/env python3
"""Headline benchmark: admission decisions/s of the cluster token server at 1M
rules, Zipf(1.1) (BASELINE.json metric).

One process per GPU: `--gpus N` under torch.distributed.run (the driver's launch), or bare, in which
case this script starts the N ranks itself.  Rules shard by
splitmix64(flowId) mod N; every rank owns its shard's rules and decides the
requests routed to it (no data-path collective; "weak" scaling: each rank sees
a global batch of N * 2^24 requests at lambda = N * 1e8 requests per virtual
second, of which ~2^24 are its own).  A step = one DefaultTokenService batch
(sga_request_tokens_device) over one pre-generated, HBM-resident batch.

Prints ONE JSON line on rank 0 (the driver's contract) with `roofline` and
`cpu_baseline` objects.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PER_RANK_BATCH = 1 << 24
N_RULES = 1_000_000
LAMBDA_PER_GPU = 100_000_000
E_IN, E_OUT, S_FLOW = 12, 8, 704  # token request 12 B, token result 8 B, cluster flow 704 B
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: 8.0 TB/s spec
E2E_BATCHES = 6                   # host-buffer batches after the timed loop (PCIe included): 1 warmup + 2 timed
                                  # through pageable buffers, then the same through registered ones


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=PER_RANK_BATCH, help="requests per rank per step (avg)")
    ap.add_argument("--rules", type=int, default=N_RULES)
    ap.add_argument("--cpu-sample", type=int, default=1 << 25, help="oracle replay sample (requests)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) batches")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the first two timed batches")
    ap.add_argument("--config", default="c3", choices=["c1", "c2", "c3", "c4", "c4args", "c4full", "c5a", "c5b"],
                    help="BASELINE.json configuration (SURVEY.md 8(d)); c3 = the headline, the others through "
                         "bench_local.py (c2 / c4 / c4full / c5b shard by resource over --gpus N)")
    return ap.parse_args()


def launch_ranks(args):
    """`--gpus N` without a launcher: start N ranks with torch.distributed.run as a child process
    (before this process touches the GPU) and exit with its code.  Rank 0 prints the line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.config != "c3":
        import bench_local
        bench_local.run(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}")
    n_gpus = world
    one_device = os.environ.get("SGA_BENCH_ONE_DEVICE") == "1"
    import torch
    import torch.distributed as dist
    if os.environ.get("SGA_BENCH_DRY") == "1":
        # launch check only (tests/test_sharding.py, CPU): every rank joins the process group,
        # all-reduces its rank and reports, before anything touches a GPU
        if world > 1:
            dist.init_process_group("gloo")
        t = torch.tensor([rank], dtype=torch.int64)
        if world > 1:
            dist.all_reduce(t)
        line = json.dumps({"dry": True, "rank": rank, "world": world, "gpus": args.gpus, "rank_sum": int(t.item())})
        out_dir = os.environ.get("SGA_BENCH_DRY_OUT")
        if out_dir:  # one file per rank: the ranks' stdout lines may interleave
            with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as fh:
                fh.write(line)
        else:
            print(line, flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    coll = None       # process group of the metric all-gather
    coll_backend = None
    if world > 1:
        dist.init_process_group("gloo")  # barriers and the max-over-ranks timing (CPU tensors)
        # RCCL over xGMI for the once-per-virtual-second metric all-gather; RCCL needs one device per
        # rank, so the one-GPU rehearsal of the N-rank path gathers over gloo instead
        coll_backend = "gloo" if one_device else "nccl"
        coll = dist.new_group(backend=coll_backend)
    if one_device:
        local = 0  # rehearsal of the N-rank path on a one-GPU box (every rank on device 0)
    torch.cuda.set_device(local)

    from sentinel_amd import _lib, cluster
    from sentinel_amd.workload import ClusterTrace, DeviceClusterGen, pack_requests, shard_of

    lam = LAMBDA_PER_GPU * n_gpus
    glob_batch = args.batch * n_gpus
    dev = torch.device("cuda", local)

    # ---- rules of this shard (C3: flowId 1..1M, GLOBAL, count U{10..10000}, 10 x 100 ms)
    tr = ClusterTrace(n_rules=args.rules, lam=lam)
    fid_all, cnt_all = tr.rules()
    mine = shard_of(fid_all, n_gpus) == rank

    # ---- pre-generate warmup+steps batches in HBM (untimed), plus the end-to-end batches that follow
    # the timed ones in virtual time (host buffers through sga_request_tokens, after the timed loop).
    # The timed entry takes the packed 12-byte records (sga_token_request, SURVEY.md 8(d) E_in);
    # SGA_BENCH_UNPACKED=1 times the four-array entry instead (A/B).
    unpacked = os.environ.get("SGA_BENCH_UNPACKED", "0") == "1"
    n_e2e = 0 if args.no_e2e else E2E_BATCHES
    nb = args.warmup + args.steps
    nb_all = nb + n_e2e
    gen = DeviceClusterGen(dev, n_rules=args.rules, lam=lam, n_shards=n_gpus, shard=rank)
    batches, packed = [], []
    touched = []
    max_n = 0
    for b in range(nb_all):
        f, a, p, t, ts_base, n, nt = gen.batch(b * glob_batch, glob_batch, touched=True)
        touched.append(nt)
        batches.append((f, a, p, t, ts_base, n))
        packed.append(pack_requests(f, a, p, t) if b < nb and not unpacked else None)
        max_n = max(max_n, n)
    gen.tmp = None

    eng = cluster.Engine(device=local, max_batch=max_n + 1024, max_rules=max(1 << 16, int(mine.sum()) + 1))
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fid_all[mine], cnt_all[mine])
    L = _lib.load()
    estream = L.sga_engine_stream(eng.handle)
    # every batch its own result buffer (the first two timed batches are checked against the oracle afterwards)
    outs = [torch.empty(max(batches[b][5], 1), dtype=torch.int64, device=dev) for b in range(nb)]

    # HIP events on the engine stream: around the whole timed region and around every batch
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipEventSynchronize.argtypes = [C.c_void_p]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    hip.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]

    def new_event():
        ev = C.c_void_p()
        hip.hipEventCreate(C.byref(ev))
        return ev

    def elapsed_ms(e0, e1):
        ms = C.c_float()
        hip.hipEventElapsedTime(C.byref(ms), e0, e1)
        return ms.value

    ev0, ev1 = new_event(), new_event()
    bev = [(new_event(), new_event()) for _ in range(args.steps)]

    # once per virtual second: ClusterMetricNodeGenerator snapshot of this shard into HBM
    # (sga_cluster_metric_nodes_device) + the node-wide all-gather (RCCL over xGMI at N > 1)
    step_virtual_ms = glob_batch * 1000.0 / lam
    metric_every = max(1, int(round(1000.0 / step_virtual_ms)))
    if os.environ.get("SGA_BENCH_METRIC_EVERY"):  # diagnostics only (A/B of the snapshot's cost); never in a reported line
        metric_every = int(os.environ["SGA_BENCH_METRIC_EVERY"])
    act = C.c_uint64()
    _lib.check(L.sga_cluster_stats(eng.handle, C.byref(act), None), eng.handle, "stats")
    cap_rows = max(int(act.value), 1)
    if world > 1:
        caps = torch.tensor([cap_rows], dtype=torch.int64)
        dist.all_reduce(caps, op=dist.ReduceOp.MAX)
        cap_rows = int(caps.item())
    side = torch.cuda.Stream(dev)
    rows = torch.zeros((cap_rows, 4), dtype=torch.int64, device=dev)
    cnt_rows = torch.zeros(2, dtype=torch.int32, device=dev)
    gdev = dev if coll_backend != "gloo" else torch.device("cpu")
    gathered = torch.empty((world * cap_rows, 4), dtype=torch.int64, device=gdev) if world > 1 else None
    gcount = torch.empty(world * 2, dtype=torch.int32, device=gdev) if world > 1 else None
    mev = []

    ev_q = new_event()

    def metric_snapshot(now):
        e0, e1 = new_event(), new_event()
        # the snapshot's time starts once the engine stream's queued batches are done (the call
        # orders itself after them; e0 would otherwise time that wait as well)
        hip.hipEventRecord(ev_q, estream)
        hip.hipStreamWaitEvent(C.c_void_p(side.cuda_stream), ev_q, 0)
        hip.hipEventRecord(e0, C.c_void_p(side.cuda_stream))
        _lib.check(L.sga_cluster_metric_nodes_device(eng.handle, now, rows.data_ptr(), cap_rows, cnt_rows.data_ptr(),
                                                     C.c_void_p(side.cuda_stream)), eng.handle, "clusterMetricNodes")
        if world > 1:
            with torch.cuda.stream(side):
                if coll_backend == "gloo":
                    dist.all_gather(list(gathered.chunk(world)), rows.cpu(), group=coll)
                    dist.all_gather(list(gcount.chunk(world)), cnt_rows.cpu(), group=coll)
                else:
                    dist.all_gather_into_tensor(gathered, rows, group=coll)
                    dist.all_gather_into_tensor(gcount, cnt_rows, group=coll)
        hip.hipEventRecord(e1, C.c_void_p(side.cuda_stream))
        mev.append((e0, e1))

    # one sga_request_tokens_device per batch; SGA_BENCH_PIPE=1 uses the pipelined device entry instead (a batch's
    # key pass and sorts beside the previous batch's decisions: measured slower on MI355X, the two stages compete
    # for the same CUs -- DESIGN.md 3); the timed region ends after sga_stream_wait + a device synchronize
    pipe = os.environ.get("SGA_BENCH_PIPE", "0") == "1"
    in_torch = torch.cuda.Stream(dev)  # the inputs are complete (made before the loop); a stream of their own
    in_stream = C.c_void_p(in_torch.cuda_stream)
    entry = L.sga_request_tokens_device_pipelined if pipe else L.sga_request_tokens_device

    def step(b, k=None):
        f, a, p, t, ts_base, n = batches[b]
        o = outs[b]
        if k is not None:
            hip.hipEventRecord(bev[k][0], estream)
        if packed[b] is not None and not pipe:
            rc = L.sga_request_tokens_packed_device(eng.handle, packed[b].data_ptr(), ts_base, n, o.data_ptr(), None)
        else:
            rc = entry(eng.handle, f.data_ptr(), a.data_ptr(), p.data_ptr(), ts_base, t.data_ptr(), n, o.data_ptr(),
                       in_stream if pipe else None)
        if rc != 0:
            raise RuntimeError(f"sga_request_tokens_device rc={rc}: {L.sga_last_error(eng.handle)}")
        if k is not None:
            hip.hipEventRecord(bev[k][1], estream)
            if (k + 1) % metric_every == 0:
                metric_snapshot(int(ts_base + step_virtual_ms))

    for b in range(args.warmup):
        step(b)
    _lib.check(L.sga_stream_wait(eng.handle, in_stream), eng.handle, "stream_wait")
    if args.warmup > 0:
        # the snapshot path is warmed up like the batches (its first call pays one-time setup:
        # events, the kernel's first launch); the timed loop still runs it every metric_every steps
        metric_snapshot(int(batches[args.warmup - 1][4] + step_virtual_ms))
        mev.clear()
    torch.cuda.synchronize(dev)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    hip.hipEventRecord(ev0, estream)
    tq = []
    for k, b in enumerate(range(args.warmup, nb)):
        tq.append(time.perf_counter())
        step(b, k)
    tq.append(time.perf_counter())
    _lib.check(L.sga_stream_wait(eng.handle, in_stream), eng.handle, "stream_wait")
    hip.hipEventRecord(ev1, estream)
    if os.environ.get("SGA_BENCH_DEBUG"):  # diagnostics: host time to queue each step (ms)
        print("queue ms per step:", [round((tq[i + 1] - tq[i]) * 1e3, 3) for i in range(len(tq) - 1)], file=sys.stderr)
    torch.cuda.synchronize(dev)
    t_end = time.perf_counter()
    if world > 1:
        dist.barrier()
    hip.hipEventSynchronize(ev1)
    ms_ev = elapsed_ms(ev0, ev1)
    ms_batches = sum(elapsed_ms(e0, e1) for e0, e1 in bev)
    ms_metrics = [elapsed_ms(e0, e1) for e0, e1 in mev]
    coll_world, flows_gathered = None, None
    if mev:
        if world > 1:
            coll_world = dist.get_world_size(coll)
            flows_gathered = int(gcount.view(world, 2)[:, 0].to(torch.int64).sum().item())
        else:
            coll_world, flows_gathered = 1, int(cnt_rows[0].item())

    e2e = run_e2e(L, eng, batches[nb:], dev) if n_e2e else None

    wall = t_end - t_start
    my_events = sum(batches[b][5] for b in range(args.warmup, nb))
    my_touched = sum(touched[b] for b in range(args.warmup, nb))
    stats = torch.tensor([wall, ms_ev / 1e3, ms_batches / 1e3, float(my_events), float(my_touched)],
                         dtype=torch.float64)
    if world > 1:
        tmax = stats[:3].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = stats[3:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        stats = torch.cat([tmax, tsum])
    wall_max, gpu_max, batches_max, total_events, total_touched = [float(x) for x in stats]

    path = eng.batch_info()  # which path the last timed batch took (hot path or plain sort)

    # correctness spot-check of the last batch's statuses (cheap invariants)
    res = outs[nb - 1][: batches[nb - 1][5]].cpu().numpy().view(np.uint64)
    status = ((res >> np.uint64(48)) & np.uint64(0xFF)).astype(np.int8)
    frac_ok = float((status == 0).mean())

    # the headline checks itself: the first two timed batches against the oracle (every request, the
    # sharded replay of this rank's trace from batch 0), rank 0
    parity = None
    if rank == 0 and not args.no_parity and args.steps >= 1:
        parity = check_parity(batches, outs, args.warmup, min(2, args.steps), fid_all[mine], cnt_all[mine])

    cpu_baseline, router = None, None
    if rank == 0 and not args.no_cpu:
        # every N: rank 0 replays a bounded sample of its own shard stream of the same trace
        cpu_baseline, router = run_cpu_baseline(args, n_gpus)

    # HBM traffic per step from the committed rocprofv3 PMC passes of this pipeline
    # (tools/pmc_bench.sh -> tools/pmc_summary.py --json; per-kernel corrected counters)
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "traffic_c3.json")
    if os.path.exists(tpath) and args.batch == PER_RANK_BATCH and args.rules == N_RULES:
        with open(tpath) as fh:
            tj = json.load(fh)
        traffic, traffic_src = tj["traffic_bytes_per_step"], "profiles/traffic_c3.json (" + tj.get("run", "") + ")"

    if rank == 0:
        value = total_events / wall_max
        per_gpu_events = total_events / n_gpus
        per_gpu_touched = total_touched / n_gpus
        bytes_alg = per_gpu_events * (E_IN + E_OUT) + per_gpu_touched * 2 * S_FLOW  # per GPU, all timed steps
        # achieved / frac on the timed wall clock (max over ranks) -- the driver's own clock; the HIP-event
        # figure (sum of the batches' engine-stream event pairs) is reported beside it
        achieved = bytes_alg / wall_max / 1e9
        achieved_ev = bytes_alg / batches_max / 1e9
        line = {
            "metric": "admission decisions/sec at 1M rules Zipf(1.1), 1/2/4/8 GPU; % HBM peak",
            "value": value,
            "unit": "decisions/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic C3 trace (Zipf(1.1) flowIds, 1% prioritized, acquire 1), generated on GPU",
            "config": {"workload": "C3 cluster token server: DefaultTokenService.requestToken batches, "
                                   "1M cluster FlowRules (GLOBAL, count U{10..10000}, 10x100ms), sharded by flowId",
                       "rules": args.rules, "requests_per_step_per_gpu": args.batch,
                       "global_requests_per_step": args.batch * n_gpus, "lambda_per_virtual_s": lam,
                       "parallelism": f"shard{n_gpus}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "sga_request_tokens_device pipeline (hot path + cold sort path); achieved = "
                                   "bytes_alg / timed wall clock (ms_per_step)",
                         "achieved_hip_events": achieved_ev, "frac_hip_events": achieved_ev / HBM_PEAK_GBS,
                         "bytes_alg_per_step_per_gpu": bytes_alg / args.steps,
                         "touched_rules_per_step_per_gpu": per_gpu_touched / args.steps,
                         "gpu_ms_per_step": batches_max / args.steps * 1e3,
                         "engine_stream_ms_per_step": gpu_max / args.steps * 1e3},
            "cpu_baseline": cpu_baseline,
            "metric_allgather": {"every_steps": metric_every, "calls": len(ms_metrics),
                                 "ms_per_call": (sum(ms_metrics) / len(ms_metrics)) if ms_metrics else None,
                                 "backend": coll_backend or "none (one rank)", "group_size": coll_world,
                                 "flows_gathered_last_call": flows_gathered,
                                 "rows_per_rank": cap_rows,
                                 "what": "sga_cluster_metric_nodes_device (ClusterMetricNodeGenerator over the "
                                         "shard's flows) + all_gather_into_tensor, once per virtual second, "
                                         "inside the timed loop on a side stream"},
            "host_router": router,
            "end_to_end_host_buffers": e2e,
            "ok_fraction_last_batch": frac_ok,
            "parity_sample": parity,
            "entry": "sga_request_tokens_device (four arrays)" if (unpacked or pipe) else
                     "sga_request_tokens_packed_device (12-B sga_token_request records)",
            "last_batch_path": path,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def check_parity(batches, outs, first, count, rule_fid, rule_cnt):
    """Oracle (oracle/sentinel_oracle.c, ClusterFlowChecker restatement) replay of this rank's trace from
    batch 0 through the timed batches [first, first + count), sharded by flowId over 16 host threads; the
    timed batches' TokenResults (status, remaining, waitInMs) compared request by request."""
    import time as _t
    try:
        from tests import oracle_harness as H
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}
    t0 = _t.perf_counter()
    host = []
    for b in range(first + count):
        f, a, p, t, ts_base, n = batches[b]
        host.append((f.cpu().numpy(), a.cpu().numpy(), p.cpu().numpy(), t.cpu().numpy().astype(np.int64) + ts_base))
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    orc = H.cluster_replay_sharded(rule_fid, rule_cnt, host, threads=threads)
    mism, total = 0, 0
    for b in range(first, first + count):
        r = outs[b][: batches[b][5]].cpu().numpy().view(np.uint64)
        st = ((r >> np.uint64(48)) & np.uint64(0xFF)).astype(np.int8).astype(np.int32)
        rem = (r & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
        wait = ((r >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16).astype(np.int32)
        o = orc[b]
        mism += int(((st != o[0]) | (rem != o[1]) | (wait != o[2])).sum())
        total += len(st)
    return {"timed_batches": list(range(first, first + count)), "requests": total, "mismatches": mism,
            "seconds": _t.perf_counter() - t0,
            "what": "every TokenResult (status, remaining, waitInMs) of these timed batches vs the oracle replaying "
                    "this rank's trace from batch 0 (tests/oracle_harness.py cluster_replay_sharded, %d threads)"
                    % threads}


def run_e2e(L, eng, bats, dev):
    """SURVEY.md 8(d), last bullet: the same C3 batches through host buffers -- sga_request_tokens
    (H2D of flowId/acquire/prio/ts, the pipeline, D2H of the 8-B TokenResults), PCIe included.
    Batches follow the timed ones in virtual time, one synchronous call each.  The first three go
    through pageable buffers (engine-staged), the last three through buffers the caller registered
    with sga_host_register beforehand (a front end's long-lived pool: DMA straight from / to them);
    the first batch of each three is an untimed warmup.  Never `value`: reported beside it."""
    import torch
    from sentinel_amd import _lib
    hosts = []
    for f, a, p, t, ts_base, n in bats:
        ts = (t.to(torch.int64) + ts_base).cpu().numpy()
        hosts.append((f.cpu().numpy(), a.cpu().numpy(), p.cpu().numpy(), ts, n))
    torch.cuda.synchronize(dev)
    outs = [np.zeros(n * 2, dtype=np.int32) for *_, n in hosts]  # the caller's result buffers, allocated up front
    half = len(hosts) // 2
    regs = []
    for (f, a, p, ts, n), out in list(zip(hosts, outs))[half:]:
        for arr in (f, a, p, ts, out):
            _lib.check(L.sga_host_register(eng.handle, arr.ctypes.data, arr.nbytes), eng.handle, "host_register")
            regs.append(arr)

    def timed(pairs):
        total, secs = 0, 0.0
        for k, ((f, a, p, ts, n), out) in enumerate(pairs):
            t0 = time.perf_counter()
            rc = L.sga_request_tokens(eng.handle, f.ctypes.data, a.ctypes.data, p.ctypes.data, ts.ctypes.data, n,
                                      out.ctypes.data)
            dt = time.perf_counter() - t0
            _lib.check(rc, eng.handle, "requestTokens (host buffers)")
            if k > 0:  # the first is the warmup
                secs += dt
                total += n
        return total, secs

    tp, sp = timed(list(zip(hosts, outs))[:half])
    tr, sr = timed(list(zip(hosts, outs))[half:])
    for arr in regs:
        L.sga_host_unregister(eng.handle, arr.ctypes.data)
    return {"value": tr / sr, "unit": "decisions/s", "batches": half - 1, "requests": tr,
            "ms_per_batch": sr / (half - 1) * 1e3,
            "bytes_pcie_per_request": 8 + 4 + 1 + 8 + 8,
            "pageable": {"value": tp / sp, "ms_per_batch": sp / (half - 1) * 1e3, "batches": half - 1,
                         "bytes_pcie_per_request": 8 + 4 + 4 + 1 + 8,
                         "what": "the same call over pageable buffers: host threads stage 2^20-request chunks "
                                 "(times as int32 deltas) through page-locked slots while the DMA engine moves the "
                                 "previous chunk, the results come back the same way (run_host_batch_pipelined)"},
            "what": "sga_request_tokens over host buffers the caller registered once with sga_host_register "
                    "(int64 flowId, int32 acquire, uint8 prio, int64 ts in; 8-B TokenResult out): H2D straight "
                    "from them, the pipeline, D2H straight into the result buffer (run_host_batch_registered); one "
                    "synchronous call per 2^24-request batch, one GPU, after one warmup batch; the batches follow "
                    "the timed ones in virtual time"}


def _time_router(f, n_shards, threads):
    from sentinel_amd import _lib
    L = _lib.load()
    f = np.ascontiguousarray(f, dtype=np.int64)
    order = np.empty(len(f), dtype=np.uint32)
    off = np.empty(n_shards + 1, dtype=np.uint64)
    t0 = time.perf_counter()
    rc = L.sga_route_shards(f.ctypes.data, len(f), n_shards, threads, order.ctypes.data, off.ctypes.data)
    dt = time.perf_counter() - t0
    if rc != 0:
        return {"error": f"sga_route_shards rc={rc}"}
    return {"requests": int(len(f)), "shards": n_shards, "threads": threads, "seconds": dt,
            "requests_per_s": len(f) / dt,
            "what": "sga_route_shards: stable counting sort of a global batch by splitmix64(flowId) mod G "
                    "(host-side event routing, SURVEY.md 8(e)), timed on a sample of the C3 trace"}


def _time_wire_decode(f, n_shards):
    """One host thread decoding FLOW frames (the token server's Netty frames) into engine batches: plain
    (sga_wire_decode) and routed inside the decode into n_shards per-GPU batches (sga_wire_decode_sharded) --
    the host-fed node's way around a separate routing pass."""
    from sentinel_amd import token_server as ts
    f = np.asarray(f[: 1 << 20], dtype=np.int64)
    fr = np.zeros(len(f), dtype=[("len", ">u2"), ("xid", ">i4"), ("type", "u1"), ("fid", ">i8"), ("cnt", ">i4"),
                                 ("prio", "u1")])
    fr["len"], fr["xid"], fr["type"], fr["fid"], fr["cnt"] = 18, np.arange(len(f)), 1, f, 1
    buf = fr.tobytes()
    out = {"frames": int(len(f)), "shards": n_shards, "threads": 1}
    def one_pass(name, bs):
        at, t = 0, 0.0
        while at < len(buf):
            for b in bs:
                b.reset()
            chunk = buf[at:at + 18 * 65536 + 2]
            t0 = time.perf_counter()
            if name == "plain":
                _, used = bs[0].decode(chunk)
            else:
                _, used = ts.decode_sharded(chunk, bs)
            t += time.perf_counter() - t0
            if used == 0:
                break
            at += used
        return t

    for name in ("plain", "sharded"):
        bs = [ts.WireBatch(1 << 16, 1, 1) for _ in range(n_shards if name == "sharded" else 1)]
        one_pass(name, bs)  # touches the batches' pages
        out[f"{name}_frames_per_s"] = len(f) / min(one_pass(name, bs) for _ in range(3))
    out["what"] = ("one thread decoding 2^20 FLOW frames of the C3 trace's flowIds into engine batches: plain "
                   "(sga_wire_decode) and routed to 8 per-GPU batches inside the decode (sga_wire_decode_sharded); "
                   "best of three passes after one untimed, per-call Python overhead included")
    return out


def run_cpu_baseline(args, n_gpus):
    """CPU restatement of the same path on this host (the reference's JMH harness needs a JDK,
    which the image lacks).  Bounded sample: the first `cpu_sample` requests of rank 0's shard
    stream of the same C3 trace at 1M rules.
      1 thread : the single-threaded C oracle (oracle/sentinel_oracle.c, ClusterFlowChecker
                 restatement) replays the sample in order;
      T threads: the sample's rules split by splitmix64(flowId) mod T, one oracle instance per
                 thread replaying its sub-stream (rules are independent, as on the GPUs);
                 ctypes releases the GIL, so the threads run in parallel.  `value` is this one."""
    import threading
    try:
        from tests import oracle_harness as H
        from sentinel_amd.workload import ClusterTrace, shard_of
    except Exception as e:  # pragma: no cover
        return {"value": None, "error": str(e)}
    L = H.lib()
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    tr = ClusterTrace(n_rules=args.rules, lam=LAMBDA_PER_GPU * n_gpus)
    fid_all, cnt_all = tr.rules()
    mine = shard_of(fid_all, n_gpus) == 0
    fid_m, cnt_m = fid_all[mine], cnt_all[mine]

    def new_oracle(sel):
        from sentinel_amd.cluster import CLUSTER_RULE_DTYPE
        rules = np.zeros(int(sel.sum()), dtype=CLUSTER_RULE_DTYPE)
        rules["flow_id"] = fid_m[sel]
        rules["count"] = cnt_m[sel]
        rules["threshold_type"] = 1
        rules["sample_count"] = 10
        rules["window_interval_ms"] = 1000
        rules["grade"] = 1
        assert rules.itemsize == C.sizeof(H.OrcClusterRule), "oracle rule layout mismatch"
        oh = L.orc_cluster_new(1.0, 1.0)
        L.orc_cluster_load_rules(oh, b"default", rules.ctypes.data_as(C.POINTER(H.OrcClusterRule)), len(rules))
        return oh

    # the bounded sample (generation untimed)
    chunks, total, g, chunk = [], 0, 0, 1 << 22
    while total < args.cpu_sample:
        f, a, p, ts = tr.events(g, chunk)
        g += chunk
        sel = shard_of(f, n_gpus) == 0
        f, a, p, ts = [np.ascontiguousarray(x[sel]) for x in (f, a, p, ts)]
        chunks.append((f, a, p, ts))
        total += len(f)

    def replay(oh, parts):
        for f, a, p, ts in parts:
            out = (H.OrcTokenResult * max(1, len(f)))()
            L.orc_cluster_replay(oh, len(f), f.ctypes.data, a.ctypes.data, p.ctypes.data, ts.ctypes.data, out)

    oh = new_oracle(np.ones(len(fid_m), dtype=bool))
    t0 = time.perf_counter()
    replay(oh, chunks)
    dt1 = time.perf_counter() - t0
    L.orc_cluster_free(oh)

    sub = shard_of(fid_m, threads)
    ohs = [new_oracle(sub == k) for k in range(threads)]
    parts = [[] for _ in range(threads)]
    for f, a, p, ts in chunks:
        fs = shard_of(f, threads)
        for k in range(threads):
            m = fs == k
            parts[k].append(tuple(np.ascontiguousarray(x[m]) for x in (f, a, p, ts)))
    ths = [threading.Thread(target=replay, args=(ohs[k], parts[k])) for k in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dtn = time.perf_counter() - t0
    for o in ohs:
        L.orc_cluster_free(o)
    # contended: the reference's own concurrency design (oracle/oracle_contended.c: LongAdder cells, CAS window
    # rotation under LeapArray's updateLock) -- T threads share every rule and window, request i on thread i mod T
    fa, aa, pa, ta = [np.ascontiguousarray(np.concatenate([c[k] for c in chunks])) for k in range(4)]
    fn = L.orc_contended_cluster
    fn.restype = C.c_double
    fn.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_void_p,
                   C.c_void_p, C.c_void_p, C.c_void_p]
    rf, rc = np.ascontiguousarray(fid_m, np.int64), np.ascontiguousarray(cnt_m, np.float64)
    aa, pa, ta = aa.astype(np.int32), pa.astype(np.uint8), ta.astype(np.int64)
    dtc = fn(threads, len(rf), rf.ctypes.data, rc.ctypes.data, 10, 1000, len(fa), fa.ctypes.data, aa.ctypes.data,
             pa.ctypes.data, ta.ctypes.data, None)
    router = _time_router(np.concatenate([c[0] for c in chunks]), 8, threads)
    router["wire_decode"] = _time_wire_decode(np.concatenate([c[0] for c in chunks]), 8)
    v_shard, v_cont = total / dtn, total / dtc
    return {"value": max(v_shard, v_cont), "unit": "decisions/s", "cores": threads, "kind": "port",
            "variant": "contended" if v_cont >= v_shard else "shard-parallel",
            "value_shard_parallel": v_shard, "value_contended": v_cont, "value_1thread": total / dt1,
            "sample": f"{total} requests of the rank-0 shard stream of the same C3 trace (1M rules): "
                      f"value_contended = {threads} threads sharing every rule and window (oracle/oracle_contended.c: "
                      f"the reference's LongAdder cells and CAS / updateLock window rotation, request i on thread "
                      f"i mod {threads}); value_shard_parallel = {threads} threads over disjoint rule subsets "
                      f"(splitmix64(flowId) mod {threads}), one single-threaded C oracle each "
                      f"(oracle/sentinel_oracle.c); value_1thread = one oracle thread in arrival order; value = the "
                      f"larger of the two {threads}-thread figures (variant names it); reference JMH harness "
                      f"unavailable (no JDK on host)",
            "seconds": dtn, "seconds_contended": dtc, "seconds_1thread": dt1}, router


if __name__ == "__main__":
    main()
