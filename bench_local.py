"""`python bench.py --config c1|c2|c4|c4full|c5a|c5b [--gpus N]`: the other BASELINE.json configurations
 through the device-resident entries, one JSON line each (bench.py's contract).

Multi-GPU (c2, c4, c4full, c5b): resources shard by splitmix64(resource id) mod G, one process
per GPU (bench.py's launcher), each rank holding its shard's rules and deciding its shard's events -- resources
are independent on the local path without SystemRules or RELATE / CHAIN strategies, so there is no exchange.
Weak scaling: each rank's batch has the full per-GPU size, drawn from the configuration's distribution
restricted to its own resources (the share of a G-times larger global batch routed to it).

A step is one pass of the local slot chain over one pre-generated, HBM-resident batch: the batch's
entries (sga_submit_events_device), then the exits of the entries that passed (their resource id is
masked to "unknown", a no-op, on the device when the entry was blocked -- a blocked SphU.entry
returns no Entry to exit).  C5a is the Envoy RLS service (sga_rls_should_rate_limit_device).  Every
step shifts the batch's clock past the previous one, so each step is new virtual time.

value = entries (C5a: descriptors) decided per second of wall time over the K timed steps.
roofline.achieved = the algorithmic bytes of SURVEY.md 8(d) (N*(E_in+E_out) + per batch, per touched
key, 2*S_k) / the GPU time of the steps (torch events on the one stream every call runs on).
cpu_baseline = the C oracle (oracle/, test infrastructure) replaying a bounded sample of the same
batch on one host thread."""
import json
import os
import time

import numpy as np

T0 = 1_700_000_000_000
HBM_PEAK_GBS = 8000.0
KIND_ENTRY, KIND_EXIT = 0, 1
EV_ERROR, EV_HAS_PARAM, EV_ARGS = 2, 4, 32
# E_in / E_out and per-key state bytes S_k
E_ENTRY, E_PARAM_ENTRY, E_EXIT, E_DEC = 12, 20, 12, 1
E_RLS_IN, E_RLS_OUT, S_RLS = 12, 8, 72
S_NODE, S_WARMUP_EXTRA, S_RL, S_WU, S_WURL = 192, 64, 8, 16, 24
S_PARAM, S_PARAM_THROTTLE, S_BREAKER = 24, 16, 32


SHARD = (0, 1)  # (rank, G) of this process (run_local sets it before building the configuration)


def own_resources(n_res):
    """The resource ids this rank owns: splitmix64(id) mod G == rank (all of them on one GPU)."""
    from sentinel_amd.workload import shard_of
    rank, g = SHARD
    if g == 1:
        return np.ones(n_res, bool)
    return shard_of(np.arange(n_res, dtype=np.int64), g) == rank


def _zipf(rng, n_items, size, s=1.1, mask=None):
    """Zipf(s) over n_items; with `mask`, the distribution restricted to those items (a shard's events)."""
    p = 1.0 / np.arange(1, n_items + 1) ** s
    if mask is not None:
        p = np.where(mask, p, 0.0)
    p /= p.sum()
    return rng.choice(n_items, size=size, p=p)


class Batch:
    """One batch: entries, then exits (exit i belongs to entry exit_of[i]); host arrays.  kind: 0 entries, or 2 (a
    block by a slot outside the engine: no exit follows); revoke: a passed entry that a slot after the engine's
    checks blocked -- its exit is a kind 3 revoke at the entry's time; pvals: the argument vectors' words
    (SGA_EV_ARGS entries; their exits carry the same vector)."""

    def __init__(self, res, ts, acq=None, flags=None, param=None, exit_rt=None, exit_err=None, kind=None,
                 revoke=None, pvals=None):
        n = len(res)
        self.n = n
        self.res = res.astype(np.uint32)
        self.ts = ts.astype(np.int64)
        self.acq = (np.ones(n) if acq is None else acq).astype(np.int32)
        self.flags = (np.zeros(n) if flags is None else flags).astype(np.uint8)
        self.param = (np.zeros(n) if param is None else param).astype(np.uint64)
        self.kind = None if kind is None else kind.astype(np.uint8)
        self.pvals = None if pvals is None else np.ascontiguousarray(pvals, np.uint64)
        self.exit_of = None
        self.exit_kind = None
        if exit_rt is not None:
            exit_rt = exit_rt.astype(np.int64)
            if revoke is not None:
                exit_rt = np.where(revoke, 0, exit_rt)  # the revoke carries the entry's time
            ets = self.ts + exit_rt
            order = np.argsort(ets, kind="stable")
            self.exit_of = order.astype(np.int64)
            self.exit_ts = ets[order]
            self.exit_rt = exit_rt[order]
            self.exit_flags = (self.flags[order] & (EV_HAS_PARAM | EV_ARGS)) | \
                (np.zeros(n, np.uint8) if exit_err is None else (exit_err[order] * EV_ERROR).astype(np.uint8))
            if revoke is not None:
                self.exit_kind = np.where(revoke[order], 3, 1).astype(np.uint8)
                self.exit_flags = np.where(revoke[order], self.exit_flags & (EV_HAS_PARAM | EV_ARGS),
                                           self.exit_flags).astype(np.uint8)
        self.t_lo = int(min(self.ts.min(), self.exit_ts.min() if self.exit_of is not None else self.ts.min()))
        self.t_hi = int(max(self.ts.max(), self.exit_ts.max() if self.exit_of is not None else self.ts.max()))


def _cfg_c1(rng, erng=None):
    erng = erng or rng
    n = 1_000_000
    ts = T0 + np.arange(n) // 20  # lambda = 20 events / ms, 50 virtual s
    b = Batch(np.zeros(n), ts, exit_rt=erng.integers(0, 6, size=n))
    return dict(name="C1 HelloWorld: 1 FlowRule QPS 20 DefaultController, 1M entries + exits",
                n_res=1, flow=[dict(resource=0, count=20.0)], batch=b, sample=n, contended=True)


def _cfg_c2(rng, erng=None, n=1 << 24):
    erng = erng or rng  # rng: the rules (the same on every rank), erng: this rank's events
    n_res = 100_000
    flow = []
    beh = rng.random(n_res)
    cnt = rng.integers(5, 5001, size=n_res)
    own = own_resources(n_res)
    for r in range(n_res):
        if not own[r]:
            continue
        if beh[r] < 0.4:
            flow.append(dict(resource=r, count=float(cnt[r])))
        elif beh[r] < 0.7:
            flow.append(dict(resource=r, count=float(cnt[r]), control_behavior=2, max_queueing_time_ms=500))
        else:
            flow.append(dict(resource=r, count=float(cnt[r]), control_behavior=1, warm_up_period_sec=10))
    res = _zipf(erng, n_res, n, mask=None if SHARD[1] == 1 else own)
    ts = T0 + np.arange(n) // 10_000  # lambda = 1e7 / virtual s (per GPU)
    acq = np.where(erng.random(n) < 0.05, erng.integers(2, 6, size=n), 1)
    b = Batch(res, ts, acq=acq, exit_rt=erng.geometric(1.0 / 5.0, size=n))
    return dict(name="C2 100k FlowRules 40% Default / 30% RateLimiter(500 ms) / 30% WarmUp(10 s), Zipf(1.1), "
                     "2^24 entries + exits per batch",
                n_res=n_res, flow=flow, batch=b, sample=1 << 21)


def _cfg_c4(rng, erng=None):
    return _cfg_c4_common(rng, erng or rng, fold=True)


def _cfg_c4_common(rng, erng, fold):
    n_res, n = 10_000, 1 << 22
    param = []
    own = own_resources(n_res)
    for r in range(n_res):
        p = dict(resource=r, count=float(rng.integers(5, 101)))
        if rng.random() < 0.1:
            p.update(control_behavior=2, max_queueing_time_ms=0)
        if own[r]:
            param.append(p)
    res = _zipf(erng, n_res, n, mask=None if SHARD[1] == 1 else own)
    vals = _zipf(erng, 10_000_000, n)
    if fold:
        vals = vals % 4000  # pinned mode: <= 4000 keys per rule (no CacheMap eviction)
    ts = T0 + np.arange(n) // 10_000
    b = Batch(res, ts, flags=np.full(n, EV_HAS_PARAM), param=vals, exit_rt=erng.integers(1, 30, size=n))
    return dict(name="C4 10k ParamFlowRules (90% default / 10% throttle), Zipf(1.1) values over 10^7 folded to "
                     "<= 4000 per rule (pinned mode), 2^22 entries + exits per batch",
                n_res=n_res, param=param, batch=b, sample=1 << 20)


def _cfg_c4args(rng, erng=None):
    """C4 pinned with what a JVM feeding the engine through GpuStatisticSlot sends besides plain entries: 5 % of
    the entries pass their whole argument vector (SphU.entry(res, v, extra): SGA_EV_ARGS, the exits the same),
    0.1 % are blocks by a slot before the engine (kind 2), 0.2 % of the passed entries are revoked by a slot after
    it (kind 3 at the entry's time instead of an exit)."""
    erng = erng or rng
    cfg = _cfg_c4_common(rng, erng, fold=True)
    b = cfg["batch"]
    n = b.n
    args = erng.random(n) < 0.05
    blocked = (erng.random(n) < 0.001) & ~args
    revoke = (erng.random(n) < 0.002) & ~blocked
    extra = erng.integers(0, 1000, size=n).astype(np.uint64)
    ia = np.nonzero(args)[0]
    pvals = np.zeros(4 * len(ia), np.uint64)  # per vector: (scalar, v), (scalar, extra)
    pvals[1::4] = b.param[ia]
    pvals[3::4] = extra[ia]
    flags, param = b.flags.copy(), b.param.copy()
    flags[ia] = EV_ARGS
    param[ia] = (np.arange(len(ia), dtype=np.uint64) * np.uint64(4)) << np.uint64(32) | np.uint64(2)
    kind = np.where(blocked, 2, 0).astype(np.uint8)
    rt = np.zeros(n, np.int64)
    rt[b.exit_of] = b.exit_rt  # each entry's RT back in entry order
    cfg["batch"] = Batch(b.res, b.ts, flags=flags, param=param, exit_rt=rt, kind=kind, revoke=revoke, pvals=pvals)
    cfg["name"] = ("C4 args: C4 pinned, 5% of the entries with a whole argument vector (SGA_EV_ARGS, exits the "
                   "same), 0.1% blocks by a slot before the engine (kind 2), 0.2% of the passed entries revoked "
                   "(kind 3), 2^22 entries + exits per batch")
    return cfg


def _cfg_c4full(rng, erng=None):
    cfg = _cfg_c4_common(rng, erng or rng, fold=False)
    cfg["name"] = ("C4 full mode: 10k ParamFlowRules (90% default / 10% throttle), Zipf(1.1) values over 10^7 "
                   "unfolded (the CacheMaps hold their min(4000 * duration, 200000) most recently used values and "
                   "evict: strict LRU), 2^22 entries + exits per batch")
    return cfg


def _cfg_c5b(rng, erng=None):
    erng = erng or rng
    n_res, n = 10_000, 1 << 22
    degrade = []
    own = own_resources(n_res)
    for r in range(n_res):
        if not own[r]:
            continue
        if r % 2 == 0:
            degrade.append(dict(resource=r, grade=0, count=50.0, slow_ratio_threshold=0.5, min_request_amount=5,
                                stat_interval_ms=1000, time_window=5))
        else:
            degrade.append(dict(resource=r, grade=1, count=0.2, min_request_amount=5, stat_interval_ms=1000,
                                time_window=5))
    res = _zipf(erng, n_res, n, mask=None if SHARD[1] == 1 else own)
    ts = T0 + np.arange(n) // 10_000
    rt = np.clip(np.round(erng.lognormal(mean=np.log(20.0), sigma=1.0, size=n)), 1, 10_000)
    b = Batch(res, ts, exit_rt=rt, exit_err=erng.random(n) < 0.03)
    return dict(name="C5b DegradeSlot: 10k DegradeRules (50% slow-RT 50 ms / 50% exception ratio 0.2), lognormal "
                     "RT (median 20 ms), 3% errors, 2^22 entries + exits per batch",
                n_res=n_res, degrade=degrade, batch=b, sample=1 << 20)


def _load_rules(s, cfg):
    from sentinel_amd.local import DegradeRuleManager, FlowRuleManager, ParamFlowRuleManager
    from sentinel_amd.rules import DegradeRule, FlowRule, ParamFlowRule
    if cfg.get("flow"):
        FlowRuleManager(s).load_rules([FlowRule(resource=f"r{r['resource']}", **{k: v for k, v in r.items()
                                                                                  if k != "resource"})
                                       for r in cfg["flow"]])
    if cfg.get("param"):
        ParamFlowRuleManager(s).load_rules([ParamFlowRule(resource=f"r{r['resource']}",
                                                          **{k: v for k, v in r.items() if k != "resource"})
                                            for r in cfg["param"]])
    if cfg.get("degrade"):
        DegradeRuleManager(s).load_rules([DegradeRule(resource=f"r{r['resource']}",
                                                      **{k: v for k, v in r.items() if k != "resource"})
                                          for r in cfg["degrade"]])


def _state_bytes(cfg, b):
    """Sum over the batch's touched keys of 2 * S_k."""
    touched = np.unique(b.res)
    per_res = np.full(cfg["n_res"], S_NODE, np.int64)
    for r in cfg.get("flow", []):
        cb = r.get("control_behavior", 0)
        per_res[r["resource"]] += {0: 0, 1: S_WARMUP_EXTRA + S_WU, 2: S_RL, 3: S_WARMUP_EXTRA + S_WURL}[cb]
    for r in cfg.get("degrade", []):
        per_res[r["resource"]] += S_BREAKER
    total = int(per_res[touched].sum())
    if cfg.get("param"):
        thr = np.zeros(cfg["n_res"], bool)
        for r in cfg["param"]:
            thr[r["resource"]] = r.get("control_behavior", 0) == 2
        val = b.param.astype(np.uint64)
        if b.pvals is not None:  # an argument vector's value: its argument 0
            av = (b.flags & EV_ARGS) != 0
            val = val.copy()
            val[av] = b.pvals[(val[av] >> np.uint64(32)).astype(np.int64) + 1]
        keys = np.unique(b.res.astype(np.uint64) << np.uint64(32) | val)
        kr = (keys >> np.uint64(32)).astype(np.int64)
        total += int(np.where(thr[kr], S_PARAM_THROTTLE, S_PARAM).sum())
    return 2 * total


def _threads():
    import os
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))


class _Shard:
    """One oracle instance and its share of the sample: the entries (of the first m) whose resource is in
    sel_res, then the exits of those that passed, masked by its own decisions.  Rules and streams are
    built before any timing; entries() and exits() are the timed replays."""

    def __init__(self, cfg, b, m, sel_res):
        from tests import local_trace as lt
        self.b, self.m = b, m
        self.orc = lt.Oracle(cfg["n_res"], cfg.get("flow", []), cfg.get("param", []), cfg.get("degrade", []))
        idx = np.nonzero(sel_res[b.res[:m]])[0] if sel_res is not None else np.arange(m)
        self.idx = idx
        self.ent = {k: np.ascontiguousarray(v) for k, v in
                    {"kind": np.zeros(len(idx), np.uint8) if b.kind is None else b.kind[idx],
                     "resource": b.res[idx], "ts": b.ts[idx],
                     "acquire": b.acq[idx], "flags": b.flags[idx], "rt": np.zeros(len(idx), np.int64),
                     "param": b.param[idx]}.items()}
        if b.pvals is not None:
            self.ent["param_values"] = b.pvals
        self.ex = None
        self.n_ev = len(idx)

    def entries(self):
        self.dec, self.wait = self.orc.replay(self.ent)

    def build_exits(self):
        b = self.b
        if b.exit_of is None:
            return
        passed = np.zeros(b.n, bool)
        passed[self.idx] = (self.dec == 0) | (self.dec == 4)
        if b.kind is not None:
            passed &= b.kind != 2
        pos = np.empty(b.n, np.int64)
        pos[b.exit_of] = np.arange(b.n)
        sel = b.exit_of[b.exit_of < self.m]
        order = np.sort(pos[sel[passed[sel]]])
        self.ex = {k: np.ascontiguousarray(v) for k, v in
                   {"kind": np.ones(len(order), np.uint8) if b.exit_kind is None else b.exit_kind[order],
                    "resource": b.res[b.exit_of[order]],
                    "ts": b.exit_ts[order], "acquire": b.acq[b.exit_of[order]], "flags": b.exit_flags[order],
                    "rt": b.exit_rt[order], "param": b.param[b.exit_of[order]]}.items()}
        if b.pvals is not None:
            self.ex["param_values"] = b.pvals
        self.n_ev += len(order)

    def exits(self):
        if self.ex is not None:
            self.orc.replay(self.ex)

    def close(self):
        self.orc.close()


def _timed(shards, fn):
    import threading
    ths = [threading.Thread(target=lambda s=s: getattr(s, fn)()) for s in shards]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return time.perf_counter() - t0


def _cpu_contended_hello(cfg, b, m, T, passed):
    """C1 with T threads sharing the one resource (oracle/oracle_contended.c: StatisticNode over LongAdder cells,
    LeapArray's CAS / updateLock rotation, DefaultController.canPass): the sample's entries and the exits of the
    single-threaded replay's passes, event i on thread i mod T."""
    import ctypes as C
    from tests import oracle_harness as H
    L = H.lib()
    fn = L.orc_contended_hello
    fn.restype = C.c_double
    fn.argtypes = [C.c_int, C.c_double, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    kind = np.zeros(m, np.uint8)
    ts, rt = np.ascontiguousarray(b.ts[:m], np.int64), np.zeros(m, np.int64)
    if b.exit_of is not None:  # exits of the sample's passed entries (one-thread replay), merged in time order
        sel = b.exit_of[b.exit_of < m]
        sel = sel[passed[sel]]
        pos = np.argsort(np.concatenate([b.ts[:m], b.ts[sel] + b.exit_rt[np.argsort(b.exit_of)][sel]]), kind="stable")
        kind = np.concatenate([kind, np.ones(len(sel), np.uint8)])[pos]
        rt = np.concatenate([rt, b.exit_rt[np.argsort(b.exit_of)][sel]])[pos]
        ts = np.concatenate([ts, b.ts[sel] + b.exit_rt[np.argsort(b.exit_of)][sel]])[pos]
    kind, ts, rt = (np.ascontiguousarray(x) for x in (kind, ts.astype(np.int64), rt.astype(np.int64)))
    dt = fn(T, float(cfg["flow"][0]["count"]), len(kind), kind.ctypes.data, ts.ctypes.data, rt.ctypes.data, None)
    return {"value_contended": m / dt, "events_contended": int(len(kind)),
            "contended": f"{T} threads on the one resource (oracle/oracle_contended.c: LongAdder cells, CAS / "
                         f"updateLock window rotation), the sample's {m} entries and their exits, event i on thread "
                         f"i mod {T}; value_contended counts entries"}


def _cpu_local(cfg, b):
    """The C oracle on the host: one thread replaying the first `sample` entries (then their exits, masked by
    its own decisions as the GPU masks by its decisions), and T threads over disjoint resource subsets
    (resource mod T; resources are independent without SystemRules, as on the GPUs) -- the shard-parallel
    analogue of the reference's multi-threaded path.  Only the replays are timed (rule loads and stream
    building are not).  `value` is the larger of the two figures."""
    m = min(cfg["sample"], b.n)
    one = _Shard(cfg, b, m, None)
    dt1 = _timed([one], "entries")
    one_dec, one_wait = one.dec.copy(), one.wait.copy()
    one.build_exits()
    dt1 += _timed([one], "exits")
    n1 = one.n_ev
    one.close()
    T = _threads()
    res_of = np.arange(cfg["n_res"]) % T
    shards = [_Shard(cfg, b, m, res_of == k) for k in range(T)]
    dtn = _timed(shards, "entries")
    for sh in shards:
        sh.build_exits()
    dtn += _timed(shards, "exits")
    busy = sum(1 for sh in shards if len(sh.idx))
    for sh in shards:
        sh.close()
    extra = {}
    if cfg.get("contended"):  # C1: the reference's own concurrency design on one shared resource
        extra = _cpu_contended_hello(cfg, b, m, T, (one_dec == 0) | (one_dec == 4))
    return one_dec, one_wait, {"value": max(m / dtn, m / dt1, extra.get("value_contended", 0.0)),
            "unit": "decisions/s", "cores": T, "kind": "port",
            "value_1thread": m / dt1, "value_threads": m / dtn, "events_per_s_1thread": n1 / dt1,
            "threads_with_work": busy, **extra,
            "sample": f"the first {m} entries of the batch and the exits of those that passed ({n1} events), "
                      f"replayed by the C oracle (oracle/ slot-chain restatement): {T} threads over disjoint "
                      f"resource subsets (resource mod {T}; {busy} with events), value_1thread = one thread in "
                      f"arrival order; value = the larger of the two"}


def run_local(args, cfg_name):
    global SHARD
    import torch
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import LocalSentinel
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}")
    if world > 1 and cfg_name == "c1":
        raise SystemExit("bench.py: C1 is one resource (nothing to shard); run it with --gpus 1")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # barriers and the max-over-ranks timing (CPU tensors)
        if os.environ.get("SGA_BENCH_ONE_DEVICE") == "1":
            local = 0  # rehearsal of the N-rank path on a one-GPU box
    SHARD = (rank, world)
    seed = {"c1": 101, "c2": 102, "c4": 104, "c4args": 104, "c4full": 104, "c5b": 105}[cfg_name]
    # the rules (count, controller, grade of each resource) come from the base seed on every rank, so a shard's
    # rules are the single-GPU workload's restricted to the shard; only the event stream is drawn per rank (one
    # rank: one generator for both, the same draws as before)
    rng = np.random.default_rng(seed)
    erng = rng if world == 1 else np.random.default_rng([seed, rank, world])
    cfg = {"c1": _cfg_c1, "c2": _cfg_c2, "c4": _cfg_c4, "c4args": _cfg_c4args, "c4full": _cfg_c4full,
           "c5b": _cfg_c5b}[cfg_name](rng, erng)
    b = cfg["batch"]
    if os.environ.get("SGA_BENCH_DRY") == "1":  # launch and routing check only (tests, CPU)
        own = own_resources(cfg["n_res"])
        line = {"dry": True, "rank": rank, "world": world, "config": cfg_name, "events": int(b.n),
                "own_resources": int(own.sum()), "events_on_own": bool(own[b.res].all()),
                "rules": len(cfg.get("flow", []) or cfg.get("param", []) or cfg.get("degrade", []))}
        if dist is not None:
            t = torch.tensor([float(b.n)], dtype=torch.float64)
            dist.all_reduce(t)
            line["events_all_ranks"] = float(t.item())
        out_dir = os.environ.get("SGA_BENCH_DRY_OUT")
        if out_dir:
            with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as fh:
                fh.write(json.dumps(line))
        else:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return None
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    eng = Engine(device=local, max_batch=b.n)
    s = LocalSentinel(eng, [f"r{i}" for i in range(cfg["n_res"])])
    _load_rules(s, cfg)
    stream = torch.cuda.Stream(dev)  # every call and the exit masking run on this one stream
    torch.cuda.set_stream(stream)

    def up(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)

    span = b.t_hi - b.t_lo + 1000
    e_kind = up(b.kind, np.uint8) if b.kind is not None else torch.zeros(b.n, dtype=torch.uint8, device=dev)
    pvals = up(b.pvals, np.int64) if b.pvals is not None else None
    e_res, e_acq = up(b.res, np.int32), up(b.acq, np.int32)
    e_flags, e_param = up(b.flags, np.uint8), up(b.param, np.int64)
    e_off = up((b.ts - b.t_lo).astype(np.uint32), np.int32)
    dec = torch.empty(b.n, dtype=torch.int8, device=dev)
    wait = torch.empty(b.n, dtype=torch.int32, device=dev)
    has_exit = b.exit_of is not None
    if has_exit:
        x_kind = up(b.exit_kind, np.uint8) if b.exit_kind is not None else torch.ones(b.n, dtype=torch.uint8, device=dev)
        x_of = up(b.exit_of, np.int64)
        x_blocked = (e_kind[x_of] == 2) if b.kind is not None else None  # a block outside the engine: no exit
        x_res_all = e_res[x_of]
        x_acq = e_acq[x_of].contiguous()
        x_param = e_param[x_of].contiguous()
        x_flags = up(b.exit_flags, np.uint8)
        x_rt = up(b.exit_rt, np.int64)
        x_off = up((b.exit_ts - b.t_lo).astype(np.uint32), np.int32)
        x_dec = torch.empty(b.n, dtype=torch.int8, device=dev)
        unknown = torch.tensor(cfg["n_res"], dtype=torch.int32, device=dev)

    def step(k):
        base = b.t_lo + k * span
        s.submit_device(e_kind, e_res, base, e_off, e_acq, flags=e_flags, param=e_param, param_values=pvals,
                        decision=dec, wait=wait, stream=stream)
        if has_exit:
            d = dec[x_of]
            ok = (d == 0) | (d == 4)
            if x_blocked is not None:
                ok &= ~x_blocked
            x_res = torch.where(ok, x_res_all, unknown)
            s.submit_device(x_kind, x_res, base, x_off, x_acq, flags=x_flags, rt=x_rt, param=x_param,
                            param_values=pvals, decision=x_dec, wait=None, stream=stream)

    # the first step runs on a fresh engine, as the oracle's one-thread replay of the sample does: its
    # decisions and waits of the sample's entries are kept for the parity check below
    first = {}

    def keep_first():
        torch.cuda.synchronize(dev)
        m = min(cfg["sample"], b.n)
        first["dec"], first["wait"] = dec[:m].cpu().numpy(), wait[:m].cpu().numpy()

    for k in range(args.warmup):
        step(k)
        if k == 0:
            keep_first()
    torch.cuda.synchronize(dev)
    s.device_status()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    s.device_status()  # raises if a chunk was rejected or a parameter map filled
    if not first:  # no warmup step: the first timed step was the fresh one (its arrays were overwritten since)
        first = None
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    d = dec.cpu().numpy()
    n_ent_rank = b.n * args.steps
    n_ent = n_ent_rank
    if dist is not None:  # max of the ranks' times, sum of their entries
        tmax = torch.tensor([wall, gpu_s], dtype=torch.float64)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = torch.tensor([float(n_ent_rank)], dtype=torch.float64)
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        wall, gpu_s = float(tmax[0]), float(tmax[1])
        n_ent = int(tsum[0])
    n_exit = int(((d == 0) | (d == 4)).sum()) * args.steps if has_exit else 0
    e_in = E_PARAM_ENTRY if cfg.get("param") else E_ENTRY
    # per GPU (rank 0's shard): the roofline is a per-GPU figure
    bytes_alg = n_ent_rank * (e_in + E_DEC) + n_exit * E_EXIT + _state_bytes(cfg, b) * args.steps
    achieved = bytes_alg / gpu_s / 1e9
    cpu, parity = None, None
    if not args.no_cpu and rank == 0:
        o_dec, o_wait, cpu = _cpu_local(cfg, b)
        if first:
            bad_d = int((first["dec"] != o_dec).sum())
            bad_w = int((first["wait"] != o_wait).sum())
            parity = {"entries": int(len(o_dec)), "decision_mismatches": bad_d, "wait_mismatches": bad_w,
                      "what": "the first (fresh-engine) step's decisions and waits of the sample's entries against "
                              "the C oracle's one-thread replay of the same entries (cpu_baseline's replay)"}
            if bad_d or bad_w:
                raise AssertionError(f"bench sample differs from the oracle: {parity}")
    eng.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return None
    # HBM traffic per step from the committed rocprofv3 PMC passes of this line (tools/pmc_configs.sh)
    traffic, traffic_src = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", f"traffic_{cfg_name}.json")
    if os.path.exists(tpath):
        with open(tpath) as fh:
            tj = json.load(fh)
        traffic, traffic_src = tj["traffic_bytes_per_step"], f"profiles/traffic_{cfg_name}.json ({tj.get('run', '')})"
    return {
        "metric": f"admission decisions/sec, config {cfg_name.upper()} (SURVEY.md 8(d)); % HBM peak",
        "value": n_ent / wall, "unit": "decisions/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int64", "data": "synthetic (numpy, seeded), staged in HBM before the timed region",
        "config": {"workload": cfg["name"], "entries_per_step_per_gpu": b.n,
                   "exits_per_step": n_exit // max(1, args.steps), "resources": cfg["n_res"],
                   "parallelism": f"shard{world}",
                   "sharding": "resources by splitmix64(resource id) mod G, no exchange (weak scaling)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "sga_submit_events_device pipeline (entries, then masked exits), torch events on "
                               "the stream every call runs on",
                     "bytes_alg_per_step": bytes_alg / args.steps, "gpu_ms_per_step": gpu_s / args.steps * 1e3,
                     "lower_bound_bytes_per_step": (n_ent * (e_in + E_DEC) + n_exit * E_EXIT) / args.steps},
        "cpu_baseline": cpu,
        "parity_sample": parity,
        "pass_fraction": float(((d == 0) | (d == 4)).mean()),
    }


def run_rls(args):
    """C5a: Envoy RLS, 100k descriptor rules (count U{10..1000}), 1-4 descriptors per request,
    hitsAddend 1, Zipf(1.1) descriptors; 2^20 requests per step."""
    import torch
    from sentinel_amd import cluster
    from tests import oracle_harness as H
    rng = np.random.default_rng(0x53454E55)
    n_rules, nreq = 100_000, 1 << 20
    fids = np.arange(1, n_rules + 1, dtype=np.int64) * 7919 + 2147483647
    counts = rng.integers(10, 1001, size=n_rules)
    ndesc = rng.integers(1, 5, size=nreq)
    off = np.concatenate([[0], np.cumsum(ndesc)]).astype(np.uint32)
    nd = int(off[-1])
    dfid = fids[_zipf(rng, n_rules, nd)]
    hits = np.ones(nreq, np.int32)
    ts = (np.arange(nreq) // 4_000).astype(np.int64)  # 1e7 descriptors / virtual s
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = cluster.Engine(device=0, max_batch=nd)
    cluster.ClusterFlowRuleManager(eng).load_rule_arrays("default", fids, counts, threshold_type=1, sample_count=1)
    svc = cluster.EnvoyRlsService(eng)
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_off, d_fid, d_hits, d_ts = up(off.view(np.int32)), up(dfid), up(hits), up(ts.astype(np.uint32).view(np.int32))
    span = int(ts.max()) + 1000
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    out = {}

    def step(k):
        out["r"] = svc.should_rate_limit_device(d_off, d_fid, d_hits, T0 + k * span, d_ts, stream=stream)

    first = {}  # the fresh engine's first step, per descriptor: status and remaining (the parity check below)
    for k in range(max(1, args.warmup)):
        step(k)
        if k == 0:
            torch.cuda.synchronize(dev)
            first["st"] = out["r"][1].cpu().numpy().astype(np.int32)
            first["rem"] = out["r"][2].cpu().numpy()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    w0 = max(1, args.warmup)
    for k in range(w0, w0 + args.steps):
        step(k)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    code = out["r"][0].cpu().numpy()
    touched = len(np.unique(dfid))
    bytes_alg = (nd * (E_RLS_IN + E_RLS_OUT) + 2 * touched * S_RLS) * args.steps
    achieved = bytes_alg / gpu_s / 1e9
    eng.close()
    cpu, parity = None, None
    if not args.no_cpu:
        L = H.lib()
        oh = L.orc_cluster_new(1.0, 1.0)
        arr = H.cluster_rules_array([{"flow_id": int(f), "count": float(c), "threshold_type": 1, "sample_count": 1}
                                     for f, c in zip(fids, counts)])
        L.orc_cluster_load_rules(oh, b"default", arr, n_rules)
        m = min(nd, 1 << 21)
        dts = (T0 + np.repeat(ts, ndesc))[:m].astype(np.int64)
        f_s = np.ascontiguousarray(dfid[:m])
        a_s = np.ones(m, np.int32)
        res = (H.OrcTokenResult * m)()
        t0 = time.perf_counter()
        L.orc_cluster_replay_simple(oh, m, f_s.ctypes.data, a_s.ctypes.data, dts.ctypes.data, res)
        dt = time.perf_counter() - t0
        L.orc_cluster_free(oh)
        ores = np.frombuffer(res, dtype=np.int32).reshape(m, 3)
        parity = {"descriptors": int(m), "status_mismatches": int((first["st"][:m] != ores[:, 0]).sum()),
                  "remaining_mismatches": int((first["rem"][:m] != ores[:, 1]).sum()),
                  "what": "the first (fresh-engine) step's status and remaining of the sample's descriptors against "
                          "the C oracle's one-thread SimpleClusterFlowChecker replay (cpu_baseline's replay)"}
        if parity["status_mismatches"] or parity["remaining_mismatches"]:
            raise AssertionError(f"bench sample differs from the oracle: {parity}")
        # T threads over disjoint flowId subsets (one oracle each, rules independent)
        import threading
        T = _threads()
        part = (f_s % T).astype(np.int64)
        shards = []
        for k in range(T):
            sel = part == k
            ohk = L.orc_cluster_new(1.0, 1.0)
            L.orc_cluster_load_rules(ohk, b"default", arr, n_rules)
            shards.append((ohk, np.ascontiguousarray(f_s[sel]), np.ascontiguousarray(a_s[sel]),
                           np.ascontiguousarray(dts[sel]), (H.OrcTokenResult * max(1, int(sel.sum())))()))

        def work(k):
            ohk, f, a, t, r = shards[k]
            L.orc_cluster_replay_simple(ohk, len(f), f.ctypes.data, a.ctypes.data, t.ctypes.data, r)

        ths = [threading.Thread(target=work, args=(k,)) for k in range(T)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dtn = time.perf_counter() - t0
        for sh in shards:
            L.orc_cluster_free(sh[0])
        cpu = {"value": m / dtn, "unit": "descriptors/s", "cores": T, "kind": "port", "value_1thread": m / dt,
               "sample": f"the first {m} descriptors of the batch, replayed by the C oracle's "
                         f"SimpleClusterFlowChecker restatement (oracle/sentinel_oracle.c): {T} threads over "
                         f"disjoint flowId subsets (flowId mod {T}); value_1thread = one thread in order"}
    return {
        "metric": "admission decisions/sec, config C5A (Envoy RLS descriptors, SURVEY.md 8(d)); % HBM peak",
        "value": nd * args.steps / wall, "unit": "descriptors/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic (numpy, seeded), staged in HBM",
        "config": {"workload": "C5a Envoy RLS: 100k descriptor rules (count U{10..1000}, sampleCount 1), 1-4 "
                               "descriptors per request, Zipf(1.1), 2^20 requests per step",
                   "requests_per_step": nreq, "descriptors_per_step": nd, "parallelism": "shard1"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "sga_rls_should_rate_limit_device pipeline, torch events on its stream",
                     "bytes_alg_per_step": bytes_alg / args.steps, "gpu_ms_per_step": gpu_s / args.steps * 1e3},
        "cpu_baseline": cpu,
        "parity_sample": parity,
        "over_limit_fraction": float((code == 2).mean()),
    }


def run(args):
    name = args.config.lower()
    if name == "c5a" and args.gpus != 1:
        raise SystemExit("bench.py: --config c5a runs on one GPU")
    line = run_rls(args) if name == "c5a" else run_local(args, name)
    if line is not None:
        print(json.dumps(line), flush=True)
