// Calibration of the access patterns the token path uses, on this box (HIP events, 20 reps).
//   copy16   : 16 B/lane streaming read + write (the chip's streaming ceiling)
//   read_soa : the request arrays of the token path (8 + 4 + 4 + 1 B per request) -> 4 B written
//   gather8  : one 8 B gather per request from an 8 MB table at a Zipf(1.1)-like index stream
//   scatter8 : 8 B stores to random positions of a 134 MB array
// Usage: ./membench [n_requests]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>
#include <cmath>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_copy16(const int4 *__restrict__ a, int4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void k_read_soa(const int64_t *__restrict__ f, const int32_t *__restrict__ a, const uint32_t *__restrict__ t,
                           const uint8_t *__restrict__ p, uint32_t *__restrict__ o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = (uint32_t)f[i] ^ (uint32_t)a[i] ^ t[i] ^ p[i];
}
__global__ void k_gather8(const uint32_t *__restrict__ idx, const uint64_t *__restrict__ tab, uint32_t *__restrict__ o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = (uint32_t)tab[idx[i]];
}
__global__ void k_scatter8(const uint32_t *__restrict__ idx, uint64_t *__restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[idx[i]] = i;
}

template <class F> float timeit(F f) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 20; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / 20;
}

int main(int argc, char **argv) {
    size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (1u << 24);
    const size_t nt = 1u << 20;  // table entries (8 MB)
    int64_t *f; int32_t *a; uint32_t *t, *o, *idx, *pidx; uint8_t *p; uint64_t *tab, *out; int4 *c0, *c1;
    CK(hipMalloc(&f, n * 8)); CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&t, n * 4)); CK(hipMalloc(&p, n));
    CK(hipMalloc(&o, n * 4)); CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&pidx, n * 4)); CK(hipMalloc(&tab, nt * 8));
    CK(hipMalloc(&out, n * 8)); CK(hipMalloc(&c0, n * 16)); CK(hipMalloc(&c1, n * 16));
    std::vector<uint32_t> h(n), hp(n);
    // Zipf(1.1)-like index stream over nt entries (inverse CDF on a precomputed table), and a permutation
    std::vector<double> cdf(nt); double s = 0; for (size_t k = 0; k < nt; ++k) { s += std::pow(k + 1.0, -1.1); cdf[k] = s; }
    uint64_t x = 88172645463325252ull;
    std::vector<uint32_t> perm(nt); for (size_t k = 0; k < nt; ++k) perm[k] = k;
    for (size_t k = nt - 1; k > 0; --k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; std::swap(perm[k], perm[x % (k + 1)]); }
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const double u = (x >> 11) * (1.0 / 9007199254740992.0) * s;
        h[i] = perm[std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()];
        x ^= x << 13; x ^= x >> 7; x ^= x << 17; hp[i] = (uint32_t)(x % n);
    }
    CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(pidx, hp.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(f, 1, n * 8)); CK(hipMemset(a, 1, n * 4)); CK(hipMemset(t, 1, n * 4)); CK(hipMemset(p, 1, n)); CK(hipMemset(tab, 1, nt * 8));
    const int G = 4096, B = 256;
    float m;
    m = timeit([&] { hipLaunchKernelGGL(k_copy16, dim3(G), dim3(B), 0, 0, c0, c1, n); });
    printf("copy16    %8.1f us  %6.2f TB/s (read+write %zu MB)\n", m * 1e3, 2.0 * n * 16 / (m * 1e-3) / 1e12, 2 * n * 16 >> 20);
    m = timeit([&] { hipLaunchKernelGGL(k_read_soa, dim3(G), dim3(B), 0, 0, f, a, t, p, o, n); });
    printf("read_soa  %8.1f us  %6.2f TB/s (17 B in + 4 B out per request)\n", m * 1e3, 21.0 * n / (m * 1e-3) / 1e12);
    m = timeit([&] { hipLaunchKernelGGL(k_gather8, dim3(G), dim3(B), 0, 0, idx, tab, o, n); });
    printf("gather8   %8.1f us  %6.2f G gathers/s (zipf index over 8 MB, + 8 B streamed per request)\n", m * 1e3, n / (m * 1e-3) / 1e9);
    m = timeit([&] { hipLaunchKernelGGL(k_scatter8, dim3(G), dim3(B), 0, 0, pidx, out, n); });
    printf("scatter8  %8.1f us  %6.2f G stores/s (random 8 B over %zu MB)\n", m * 1e3, n / (m * 1e-3) / 1e9, n * 8 >> 20);
    return 0;
}
