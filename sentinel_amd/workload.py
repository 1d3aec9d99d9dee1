"""Synthetic workloads of SURVEY.md §8(d) (C1-C5), shared by tests and bench.py.

Not part of the decision path.  Counter-based randomness so any slice of a
trace can be generated independently (and identically by the GPU generator in
csrc/workload.hip, up to libm last-ulp differences in the Zipf sampler):
  u64(stream, i) = splitmix64(seed + stream * 0xD1B54A32D192ED03 + i * 0x9E3779B97F4A7C15)
Zipf(s) uses Hormann-Derflinger rejection-inversion (as published; the same
algorithm as Apache Commons RNG's RejectionInversionZipfSampler); rank -> id
goes through a seeded permutation so hot ids spread across shards.
"""
import numpy as np

MASTER_SEED = 0x53454E54494E454C
T0 = 1_700_000_000_000

S_ZIPF, S_PRIO, S_COUNT, S_PERM, S_ACQ, S_MIX, S_EXIT = range(1, 8)

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rng_u64(stream, idx, seed=MASTER_SEED):
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + np.uint64(stream) * np.uint64(0xD1B54A32D192ED03) + idx * np.uint64(0x9E3779B97F4A7C15)
    return splitmix64(x)


def rng_unit(stream, idx, seed=MASTER_SEED):
    return (rng_u64(stream, idx, seed) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


class Zipf:
    def __init__(self, n, s=1.1):
        self.n = int(n)
        self.s = float(s)
        self.hx1 = self.H(1.5) - 1.0
        self.hn = self.H(self.n + 0.5)
        self.sval = 2.0 - self.Hinv(self.H(2.5) - self.h(2.0))

    def h(self, x):
        return np.exp(-self.s * np.log(x))

    @staticmethod
    def _helper1(x):
        x = np.asarray(x, dtype=np.float64)
        small = np.abs(x) <= 1e-8
        with np.errstate(divide="ignore", invalid="ignore"):
            big = np.log1p(x) / x
        return np.where(small, 1.0 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x)), big)

    @staticmethod
    def _helper2(x):
        x = np.asarray(x, dtype=np.float64)
        small = np.abs(x) <= 1e-8
        with np.errstate(divide="ignore", invalid="ignore"):
            big = np.expm1(x) / x
        return np.where(small, 1.0 + x * 0.5 * (1.0 + x * (1.0 / 3.0) * (1.0 + 0.25 * x)), big)

    def H(self, x):
        lx = np.log(x)
        return self._helper2((1.0 - self.s) * lx) * lx

    def Hinv(self, x):
        t = np.maximum(x * (1.0 - self.s), -1.0)
        return np.exp(self._helper1(t) * x)

    def sample(self, stream, idx, seed=MASTER_SEED):
        """1-based ranks for event indices idx (vectorised, deterministic per index)."""
        idx = np.asarray(idx, dtype=np.uint64)
        out = np.zeros(idx.shape, dtype=np.int64)
        pending = np.arange(idx.size)
        for attempt in range(64):
            if pending.size == 0:
                break
            with np.errstate(over="ignore"):
                sub = idx[pending] * np.uint64(64) + np.uint64(attempt)
            u01 = rng_unit(stream, sub, seed)
            u = self.hn + u01 * (self.hx1 - self.hn)
            x = self.Hinv(u)
            k = np.floor(x + 0.5).astype(np.int64)
            k = np.clip(k, 1, self.n)
            ok = (k - x <= self.sval) | (u >= self.H(k + 0.5) - self.h(k.astype(np.float64)))
            out[pending[ok]] = k[ok]
            pending = pending[~ok]
        if pending.size:
            out[pending] = 1
        return out


def permutation(n, stream=S_PERM, seed=MASTER_SEED):
    """Seeded permutation of 0..n-1 (sort of random keys)."""
    keys = rng_u64(stream, np.arange(n, dtype=np.uint64), seed)
    return np.argsort(keys, kind="stable").astype(np.int64)


# ------------------------------------------------------------------ C3
class ClusterTrace:
    """C3: n_rules cluster FlowRules (flowId 1..n, GLOBAL, count U{10..10000},
    sampleCount 10, 1000 ms); requestToken(flowId ~ Zipf(1.1), 1, prio 1 %)
    at lambda events per virtual second starting at T0."""

    def __init__(self, n_rules=1_000_000, lam=100_000_000, prio_pct=1, seed=MASTER_SEED, s=1.1,
                 acquire_mix=False, count_lo=10, count_hi=10000):
        self.n = n_rules
        self.lam = lam
        self.prio_pct = prio_pct
        self.seed = seed
        self.zipf = Zipf(n_rules, s)
        self.perm = permutation(n_rules, seed=seed)
        self.acquire_mix = acquire_mix
        self.count_lo, self.count_hi = count_lo, count_hi

    def rules(self):
        fid = np.arange(1, self.n + 1, dtype=np.int64)
        span = self.count_hi - self.count_lo + 1
        count = (self.count_lo + (rng_u64(S_COUNT, fid.astype(np.uint64), self.seed) % np.uint64(span))).astype(
            np.float64)
        return fid, count

    def events(self, start, m):
        idx = np.arange(start, start + m, dtype=np.uint64)
        rank = self.zipf.sample(S_ZIPF, idx, self.seed)
        fid = self.perm[rank - 1] + 1
        if self.prio_pct:
            prio = ((rng_u64(S_PRIO, idx, self.seed) % np.uint64(100)) < np.uint64(self.prio_pct)).astype(np.uint8)
        else:
            prio = np.zeros(m, dtype=np.uint8)
        if self.acquire_mix:  # 95 % acquire 1, 5 % U{2..5}
            r = rng_u64(S_ACQ, idx, self.seed)
            acq = np.where((r % np.uint64(100)) < np.uint64(95), 1, 2 + ((r >> np.uint64(8)) % np.uint64(4))).astype(
                np.int32)
        else:
            acq = np.ones(m, dtype=np.int32)
        ts = (T0 + (idx.astype(np.int64) * 1000) // self.lam).astype(np.int64)
        return fid.astype(np.int64), acq, prio, ts


def shard_of(flow_id, n_shards):
    """Rules shard by flowId hash across GPUs: splitmix64(flowId) mod G."""
    return (splitmix64(np.asarray(flow_id, dtype=np.int64).astype(np.uint64)) % np.uint64(n_shards)).astype(np.int64)


# ------------------------------------------------------------------ C3 on the device
class DeviceClusterGen:
    """The C3 trace generated in HBM by libsga_workload.so (sgaw_gen_cluster: the same Zipf(1.1)
    flowIds, 1 % prioritized, acquire 1 at lambda requests per virtual second), one rank's share
    (splitmix64(flowId) mod n_shards == shard) of each global batch.  Benchmark / test input only."""

    def __init__(self, dev, n_rules=1_000_000, lam=100_000_000, n_shards=1, shard=0, seed=MASTER_SEED,
                 prio_pct=1, s=1.1):
        import ctypes as C
        import os

        import torch

        class SgawParams(C.Structure):
            _fields_ = [("seed", C.c_uint64), ("t0", C.c_int64), ("lambda_", C.c_int64), ("n_rules", C.c_int64),
                        ("zipf_s", C.c_double), ("prio_pct", C.c_int32), ("n_shards", C.c_int32),
                        ("shard", C.c_int32), ("reserved", C.c_int32)]

        self.C, self.torch, self.dev = C, torch, dev
        self.lam, self.n_rules = lam, n_rules
        self.wl = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsga_workload.so"))
        self.wl.sgaw_gen_cluster.restype = C.c_int
        self.wl.sgaw_gen_cluster.argtypes = [C.POINTER(SgawParams), C.c_uint64, C.c_uint32, C.c_void_p, C.c_int64,
                                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p]
        self.wl.sgaw_flow_histogram.restype = C.c_int
        self.wl.sgaw_flow_histogram.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int64, C.c_void_p]
        self.params = SgawParams(seed, T0, lam, n_rules, s, prio_pct, n_shards, shard, 0)
        self.perm = torch.from_numpy(permutation(n_rules, seed=seed)).to(dev)
        self.cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.hist = None
        self.tmp = None

    def ts_base(self, start):
        return T0 + (start * 1000) // self.lam

    def batch(self, start, m, touched=False):
        """Global requests [start, start + m): this shard's (flowId int64, acquire int32, prio u8, time offset
        int32 from ts_base(start)) on the device, ts_base, n (and the number of distinct flowIds if touched)."""
        torch, C = self.torch, self.C
        if self.tmp is None or self.tmp.numel() < 4 * m + 4096:
            self.tmp = torch.empty(4 * m + 4096, dtype=torch.int32, device=self.dev)
        f = torch.empty(m, dtype=torch.int64, device=self.dev)
        a = torch.empty(m, dtype=torch.int32, device=self.dev)
        p = torch.empty(m, dtype=torch.uint8, device=self.dev)
        t = torch.empty(m, dtype=torch.int32, device=self.dev)
        stream = torch.cuda.current_stream(self.dev)
        base = self.ts_base(start)
        rc = self.wl.sgaw_gen_cluster(C.byref(self.params), start, m, self.perm.data_ptr(), base, f.data_ptr(),
                                      a.data_ptr(), p.data_ptr(), t.data_ptr(), self.cnt.data_ptr(),
                                      self.tmp.data_ptr(), C.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"sgaw_gen_cluster rc={rc}")
        torch.cuda.synchronize(self.dev)
        n = int(self.cnt.item())
        out = (f[:n].clone(), a[:n].clone(), p[:n].clone(), t[:n].clone(), base, n)
        if touched:
            if self.hist is None:
                self.hist = torch.zeros(self.n_rules + 1, dtype=torch.int32, device=self.dev)
            self.wl.sgaw_flow_histogram(f.data_ptr(), n, self.hist.data_ptr(), self.n_rules,
                                        C.c_void_p(stream.cuda_stream))
            torch.cuda.synchronize(self.dev)
            out = out + (int((self.hist > 0).sum().item()),)
        return out


def pack_requests(f, a, p, t):
    """sga_token_request records (include/sentinel_amd.h) from device arrays: int32 [n, 3] =
    (flowId u32, time offset u32, acquire u16 | prioritized << 16).  Requires 0 <= flowId < 2^32 and
    0 <= acquire < 2^16 (the packed entry's domain)."""
    import torch
    n = f.numel()
    if n:  # outside the domain a value would wrap into a different valid request
        if int(f.min()) < 0 or int(f.max()) >= 1 << 32:
            raise ValueError("pack_requests: flowId outside [0, 2^32)")
        if int(a.min()) < 0 or int(a.max()) >= 1 << 16:
            raise ValueError("pack_requests: acquireCount outside [0, 2^16)")
        if int(p.min()) < 0 or int(p.max()) > 1:
            raise ValueError("pack_requests: prioritized must be 0 or 1")
    out = torch.empty((n, 3), dtype=torch.int32, device=f.device)
    out[:, 0] = f.to(torch.int64).to(torch.int32)
    out[:, 1] = t.to(torch.int32)
    out[:, 2] = a.to(torch.int32) | (p.to(torch.int32) << 16)
    torch.cuda.synchronize(f.device)  # the engine reads them on its own stream
    return out
