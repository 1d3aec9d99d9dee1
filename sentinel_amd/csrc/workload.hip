// Synthetic C3 workload generator on the GPU (bench support; see include/sga_workload.h).
#include "../../include/sga_workload.h"
#include "common.hpp"
#include "radix_sort.hpp"

namespace {

using namespace sga;

constexpr int kT = 256;

__device__ __forceinline__ uint64_t rng_u64(uint64_t seed, uint64_t stream, uint64_t i) {
    return splitmix64(seed + stream * 0xD1B54A32D192ED03ULL + i * 0x9E3779B97F4A7C15ULL);
}
__device__ __forceinline__ double rng_unit(uint64_t seed, uint64_t stream, uint64_t i) {
    return (double)(rng_u64(seed, stream, i) >> 11) * (1.0 / 9007199254740992.0);
}

struct ZipfDev {
    double s, hx1, hn, sval;
    int64_t n;
    __device__ __host__ double h(double x) const { return exp(-s * log(x)); }
    __device__ __host__ static double helper1(double x) {
        return fabs(x) > 1e-8 ? log1p(x) / x : 1.0 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x));
    }
    __device__ __host__ static double helper2(double x) {
        return fabs(x) > 1e-8 ? expm1(x) / x : 1.0 + x * 0.5 * (1.0 + x * (1.0 / 3.0) * (1.0 + 0.25 * x));
    }
    __device__ __host__ double H(double x) const {
        const double lx = log(x);
        return helper2((1.0 - s) * lx) * lx;
    }
    __device__ __host__ double Hinv(double x) const {
        double t = x * (1.0 - s);
        if (t < -1.0) t = -1.0;
        return exp(helper1(t) * x);
    }
};

enum { S_ZIPF = 1, S_PRIO = 2 };

__device__ __forceinline__ int64_t zipf_rank(const ZipfDev &z, uint64_t seed, uint64_t i) {
    for (int attempt = 0; attempt < 64; ++attempt) {
        const double u01 = rng_unit(seed, S_ZIPF, i * 64ULL + (uint64_t)attempt);
        const double u = z.hn + u01 * (z.hx1 - z.hn);
        const double x = z.Hinv(u);
        int64_t k = (int64_t)floor(x + 0.5);
        if (k < 1) k = 1;
        else if (k > z.n) k = z.n;
        if ((double)k - x <= z.sval || u >= z.H((double)k + 0.5) - z.h((double)k)) return k;
    }
    return 1;
}

struct Ev {
    int64_t fid;
    bool mine;
};

__device__ __forceinline__ Ev gen_one(const sgaw_cluster_params &p, const ZipfDev &z, const int64_t *perm,
                                      uint64_t i) {
    const int64_t rank = zipf_rank(z, p.seed, i);
    Ev e;
    e.fid = perm[rank - 1] + 1;
    e.mine = p.n_shards <= 1 || (int32_t)(splitmix64((uint64_t)e.fid) % (uint64_t)p.n_shards) == p.shard;
    return e;
}

__global__ void k_flags(sgaw_cluster_params p, ZipfDev z, const int64_t *perm, uint64_t start, uint32_t m,
                        uint32_t *flags) {
    const uint32_t j = blockIdx.x * kT + threadIdx.x;
    if (j >= m) return;
    flags[j] = gen_one(p, z, perm, start + j).mine ? 1u : 0u;
}

__global__ void k_emit(sgaw_cluster_params p, ZipfDev z, const int64_t *perm, uint64_t start, uint32_t m,
                       const uint32_t *flags, const uint32_t *pos, int64_t ts_base, int64_t *fid, int32_t *acq,
                       uint8_t *prio, uint32_t *ts_off, uint32_t *count) {
    const uint32_t j = blockIdx.x * kT + threadIdx.x;
    if (j >= m) return;
    if (j == m - 1) *count = pos[j] + flags[j];
    if (!flags[j]) return;
    const uint64_t i = start + j;
    const Ev e = gen_one(p, z, perm, i);
    const uint32_t o = pos[j];
    fid[o] = e.fid;
    acq[o] = 1;
    prio[o] = (rng_u64(p.seed, S_PRIO, i) % 100ULL) < (uint64_t)p.prio_pct ? 1 : 0;
    const int64_t ts = p.t0 + (int64_t)(i * 1000ULL / (uint64_t)p.lambda);
    ts_off[o] = (uint32_t)(ts - ts_base);
}

__global__ void k_hist(const int64_t *fid, uint32_t m, uint32_t *hist, int64_t n) {
    const uint32_t j = blockIdx.x * kT + threadIdx.x;
    if (j >= m) return;
    const int64_t f = fid[j];
    if (f >= 0 && f <= n) atomicAdd(&hist[f], 1u);
}

}  // namespace

extern "C" int sgaw_gen_cluster(const sgaw_cluster_params *p, uint64_t start, uint32_t m, const int64_t *d_perm,
                                int64_t ts_base, int64_t *d_fid, int32_t *d_acq, uint8_t *d_prio, uint32_t *d_ts_off,
                                uint32_t *d_count, uint32_t *d_tmp, void *hip_stream) {
    if (!p || m == 0 || p->n_rules <= 0 || p->lambda <= 0) return -22;
    hipStream_t s = (hipStream_t)hip_stream;
    ZipfDev z;
    z.s = p->zipf_s;
    z.n = p->n_rules;
    z.hx1 = z.H(1.5) - 1.0;
    z.hn = z.H((double)p->n_rules + 0.5);
    z.sval = 2.0 - z.Hinv(z.H(2.5) - z.h(2.0));
    uint32_t *flags = d_tmp;
    uint32_t *pos = d_tmp + m;
    uint32_t *partial = d_tmp + 2 * (size_t)m;
    const uint32_t nb = (m + kT - 1) / kT;
    hipLaunchKernelGGL(k_flags, dim3(nb), dim3(kT), 0, s, *p, z, d_perm, start, m, flags);
    sga::exclusive_scan_u32(flags, pos, m, partial, s);
    hipLaunchKernelGGL(k_emit, dim3(nb), dim3(kT), 0, s, *p, z, d_perm, start, m, flags, pos, ts_base, d_fid, d_acq,
                       d_prio, d_ts_off, d_count);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int sgaw_flow_histogram(const int64_t *d_fid, uint32_t m, uint32_t *d_hist, int64_t n, void *hip_stream) {
    hipStream_t s = (hipStream_t)hip_stream;
    if (hipMemsetAsync(d_hist, 0, (size_t)(n + 1) * 4, s) != hipSuccess) return -5;
    if (m == 0) return 0;
    hipLaunchKernelGGL(k_hist, dim3((m + kT - 1) / kT), dim3(kT), 0, s, d_fid, m, d_hist, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
