// Calibration of the cold-rule record access (k_cold_fused's flows phase) on this box.
// 1M records of 768 B (the S = 10 layout: a 256-byte header of two 128-byte lines + the counter
// array), a list of `touched` distinct slots in ascending order (as a partition bin hands them to
// its lanes).  Per touched rule: read the header, sum the ten (start, PASS) pairs, write one pair
// and one 48-byte counter group (what run_fast stores).
//   lane   : one lane per rule, 16 int4 loads per lane (the current form)
//   trans  : per wave 64 rules; each load instruction fetches 4 headers whole (16 lanes per header,
//            8 full lines), LDS hands each lane its rule's 16 pieces (padded rows)
//   coop   : 16 lanes per rule, one int4 each, DPP row reduction; the wave's 64 rules in 16 steps
//            with all the loads issued first
//   lane2  : one lane per rule, 2 int4 loads (load count scaling)
// Usage: ./recbench [touched] [wg_threads]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kRecI4 = 48;  // 768 B
constexpr int kHdrI4 = 16;  // 256 B

__device__ __forceinline__ long long lo64(int4 v) { return (long long)(((unsigned long long)(unsigned)v.y << 32) | (unsigned)v.x); }
__device__ __forceinline__ long long hi64(int4 v) { return (long long)(((unsigned long long)(unsigned)v.w << 32) | (unsigned)v.z); }

__global__ void k_lane(int4 *rec, const uint32_t *__restrict__ sl, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int4 *r = rec + (size_t)sl[i] * kRecI4;
    int4 h[kHdrI4];
#pragma unroll
    for (int k = 0; k < kHdrI4; ++k) h[k] = r[k];
    long long s = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) s += hi64(h[k]);
    const int cj = (int)(lo64(h[10]) & 7);
    r[cj] = make_int4((int)s, 0, h[cj].z + 1, h[cj].w);
    int4 *g = r + kHdrI4 + 3 * cj;
    g[0] = h[11];
    g[1] = h[12];
    g[2] = h[13];
}

__global__ void k_lane2(int4 *rec, const uint32_t *__restrict__ sl, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int4 *r = rec + (size_t)sl[i] * kRecI4;
    const int4 a = r[0], b = r[10];
    const long long s = hi64(a) + lo64(b);
    const int cj = (int)(lo64(b) & 7);
    r[cj] = make_int4((int)s, 0, a.z + 1, a.w);
    int4 *g = r + kHdrI4 + 3 * cj;
    g[0] = b;
    g[1] = a;
    g[2] = b;
}

// per wave: 64 rules; rows of 17 int4 (one pad) so a lane's 16 reads spread over the banks
__global__ void k_trans(int4 *rec, const uint32_t *__restrict__ sl, uint32_t n) {
    extern __shared__ int4 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int4 *w = lds + (size_t)wave * 64 * 17;
    const uint32_t base = (blockIdx.x * (blockDim.x >> 6) + wave) * 64;
    if (base >= n) return;
    const int piece = lane & 15, sub = lane >> 4;
    int4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t ri = min(base + (uint32_t)(k * 4 + sub), n - 1);
        v[k] = rec[(size_t)sl[ri] * kRecI4 + piece];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) w[(k * 4 + sub) * 17 + piece] = v[k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    const uint32_t i = base + lane;
    int4 h[kHdrI4];
#pragma unroll
    for (int k = 0; k < kHdrI4; ++k) h[k] = w[lane * 17 + k];
    if (i >= n) return;
    int4 *r = rec + (size_t)sl[i] * kRecI4;
    long long s = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) s += hi64(h[k]);
    const int cj = (int)(lo64(h[10]) & 7);
    r[cj] = make_int4((int)s, 0, h[cj].z + 1, h[cj].w);
    int4 *g = r + kHdrI4 + 3 * cj;
    g[0] = h[11];
    g[1] = h[12];
    g[2] = h[13];
}

// 16 lanes per rule: lane piece k holds int4 k of the header; row reduction over pieces 0..9
__global__ void k_coop(int4 *rec, const uint32_t *__restrict__ sl, uint32_t n) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t base = (blockIdx.x * (blockDim.x >> 6) + wave) * 64;
    if (base >= n) return;
    const int piece = lane & 15, sub = lane >> 4;
    int4 v[16];
    uint32_t s_of[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t ri = min(base + (uint32_t)(k * 4 + sub), n - 1);
        s_of[k] = sl[ri];
        v[k] = rec[(size_t)s_of[k] * kRecI4 + piece];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t ri = base + (uint32_t)(k * 4 + sub);
        long long x = piece < 10 ? hi64(v[k]) : 0;
        // row sum over 16 lanes (xor shuffles inside the row)
        for (int o = 1; o < 16; o <<= 1) {
            const int lo = __shfl_xor((int)(unsigned)x, o, 16);
            const int hi = __shfl_xor((int)(unsigned)((unsigned long long)x >> 32), o, 16);
            x += (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
        }
        const int cj = __shfl(v[k].x, (lane & ~15) + 10, 64) & 7;
        if (ri < n) {
            int4 *r = rec + (size_t)s_of[k] * kRecI4;
            if (piece == cj) r[cj] = make_int4((int)x, 0, v[k].z + 1, v[k].w);
            if (piece >= 11 && piece <= 13) r[kHdrI4 + 3 * cj + (piece - 11)] = v[k];
        }
    }
}

// 4 lanes per rule: lane q of the quad loads pieces q, q + 4, q + 8, q + 12 (each instruction: 64 contiguous bytes
// per quad, 16 rules per wave); the pass sum is a quad reduction, each lane stores a piece of the group
__global__ void k_quad(int4 *rec, const uint32_t *__restrict__ sl, uint32_t n) {
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x);
    const uint32_t i = g >> 2;
    const int q = threadIdx.x & 3;
    if (i >= n) return;
    int4 *r = rec + (size_t)sl[i] * kRecI4;
    int4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = r[4 * k + q];
    long long s = hi64(v[0]) + hi64(v[1]) + (q < 2 ? hi64(v[2]) : 0);  // pairs q, q + 4, q + 8 (< 10)
    for (int o = 1; o < 4; o <<= 1) {
        const int lo = __shfl_xor((int)(unsigned)s, o, 4);
        const int hi = __shfl_xor((int)(unsigned)((unsigned long long)s >> 32), o, 4);
        s += (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
    }
    const int cj = __shfl(v[2].x, (threadIdx.x & ~3) + 2, 64) & 7;  // piece 10 (lane 2, register 2)
    if (q == (cj & 3)) r[cj] = make_int4((int)s, 0, v[cj >> 2].z + 1, v[cj >> 2].w);
    int4 *gp = r + kHdrI4 + 3 * cj;
    if (q < 3) gp[q] = v[3];
}

// lane-interleaved records: int4 k of slot s at ((s / 64) * kRecI4 + k) * 64 + s % 64 (a wave over 64 near slots
// loads each piece as a few contiguous kilobytes); one lane per touched rule as in k_lane
__device__ __forceinline__ size_t ilv(uint32_t s, int k) { return ((size_t)(s >> 6) * kRecI4 + k) * 64 + (s & 63); }
__global__ void k_ilv(int4 *rec, const uint32_t *__restrict__ sl, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s0 = sl[i];
    int4 h[kHdrI4];
#pragma unroll
    for (int k = 0; k < kHdrI4; ++k) h[k] = rec[ilv(s0, k)];
    long long s = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) s += hi64(h[k]);
    const int cj = (int)(lo64(h[10]) & 7);
    rec[ilv(s0, cj)] = make_int4((int)s, 0, h[cj].z + 1, h[cj].w);
    rec[ilv(s0, kHdrI4 + 3 * cj)] = h[11];
    rec[ilv(s0, kHdrI4 + 3 * cj + 1)] = h[12];
    rec[ilv(s0, kHdrI4 + 3 * cj + 2)] = h[13];
}

template <class F> float timeit(F f, int reps = 20) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}

int main(int argc, char **argv) {
    const uint32_t nslots = 1u << 20;
    const uint32_t touched = argc > 1 ? (uint32_t)atoi(argv[1]) : 700000u;
    const int wg = argc > 2 ? atoi(argv[2]) : 256;
    int4 *rec; uint32_t *sl, *slr;
    CK(hipMalloc(&rec, (size_t)nslots * kRecI4 * 16));
    CK(hipMemset(rec, 0, (size_t)nslots * kRecI4 * 16));
    std::vector<uint32_t> all(nslots);
    for (uint32_t k = 0; k < nslots; ++k) all[k] = k;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint32_t k = nslots - 1; k > 0; --k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; std::swap(all[k], all[x % (k + 1)]); }
    std::vector<uint32_t> pick(all.begin(), all.begin() + touched), rnd = pick;
    std::sort(pick.begin(), pick.end());
    CK(hipMalloc(&sl, touched * 4)); CK(hipMalloc(&slr, touched * 4));
    CK(hipMemcpy(sl, pick.data(), touched * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(slr, rnd.data(), touched * 4, hipMemcpyHostToDevice));
    const uint32_t nb = (touched + wg - 1) / wg;
    const size_t lds = (size_t)(wg / 64) * 64 * 17 * 16;
    const double mb = touched * (256.0 + 64.0) / 1e6;  // header read + pair/group written (algorithmic)
    for (int order = 0; order < 2; ++order) {
        const uint32_t *s = order ? slr : sl;
        const char *on = order ? "random" : "sorted";
        float t;
        t = timeit([&] { hipLaunchKernelGGL(k_lane, dim3(nb), dim3(wg), 0, 0, rec, s, touched); });
        printf("{\"mode\":\"lane\",\"order\":\"%s\",\"touched\":%u,\"wg\":%d,\"us\":%.2f,\"GBs\":%.1f}\n", on, touched, wg, t * 1e3, mb / t);
        t = timeit([&] { hipLaunchKernelGGL(k_ilv, dim3(nb), dim3(wg), 0, 0, rec, s, touched); });
        printf("{\"mode\":\"ilv\",\"order\":\"%s\",\"touched\":%u,\"wg\":%d,\"us\":%.2f,\"GBs\":%.1f}\n", on, touched, wg, t * 1e3, mb / t);
        t = timeit([&] { hipLaunchKernelGGL(k_lane2, dim3(nb), dim3(wg), 0, 0, rec, s, touched); });
        printf("{\"mode\":\"lane2\",\"order\":\"%s\",\"touched\":%u,\"wg\":%d,\"us\":%.2f,\"GBs\":%.1f}\n", on, touched, wg, t * 1e3, mb / t);
        t = timeit([&] { hipLaunchKernelGGL(k_trans, dim3(nb), dim3(wg), lds, 0, rec, s, touched); });
        printf("{\"mode\":\"trans\",\"order\":\"%s\",\"touched\":%u,\"wg\":%d,\"us\":%.2f,\"GBs\":%.1f}\n", on, touched, wg, t * 1e3, mb / t);
        t = timeit([&] { hipLaunchKernelGGL(k_quad, dim3((4 * touched + wg - 1) / wg), dim3(wg), 0, 0, rec, s, touched); });
        printf("{\"mode\":\"quad\",\"order\":\"%s\",\"touched\":%u,\"wg\":%d,\"us\":%.2f,\"GBs\":%.1f}\n", on, touched, wg, t * 1e3, mb / t);
        t = timeit([&] { hipLaunchKernelGGL(k_coop, dim3(nb), dim3(wg), 0, 0, rec, s, touched); });
        printf("{\"mode\":\"coop\",\"order\":\"%s\",\"touched\":%u,\"wg\":%d,\"us\":%.2f,\"GBs\":%.1f}\n", on, touched, wg, t * 1e3, mb / t);
    }
    return 0;
}
