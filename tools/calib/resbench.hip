// Calibration: how the cold TokenResults reach the result array (k_cold_fused today: one random 8-B store per
// cold request).  n = 2^24 requests, m cold ones (a random subset, visited in random order as a bin order does).
//   scatter    : out[idx[j]] = v                      (m random 8-B stores; today's form)
//   sorted+gat : res[j] = v (coalesced), then one input-order pass over all n: a 4-B code read, for a cold request
//                one random 8-B read res[pos[i]], every out[i] written (the hot results pass writes them anyway)
//   inorder    : the same input-order pass without the cold gathers (the hot results pass alone)
// Usage: ./resbench [m]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_scatter(const uint32_t *__restrict__ idx, uint64_t *__restrict__ out, uint32_t m) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) out[idx[j]] = 0x100000000ull | j;
}
__global__ void k_sorted(uint64_t *__restrict__ res, uint32_t m) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) res[j] = 0x100000000ull | j;
}
template <bool kGather>
__global__ void k_inorder(const uint32_t *__restrict__ code, const uint64_t *__restrict__ res, uint64_t *__restrict__ out,
                          uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = __builtin_nontemporal_load(&code[i]);
    uint64_t v = c;  // a hot request's result (stands in for the rank arithmetic)
    if (kGather && (c >> 31)) v = res[c & 0x7FFFFFFFu];
    if (!kGather && (c >> 31)) return;  // today: the cold results were already scattered
    __builtin_nontemporal_store(v, &out[i]);
}

template <class F> float timeit(F f) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 20; ++r) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / 20;
}

int main(int argc, char **argv) {
    const uint32_t n = 1u << 24;
    const uint32_t m = argc > 1 ? (uint32_t)atoi(argv[1]) : 3900000u;
    std::vector<uint32_t> all(n);
    for (uint32_t k = 0; k < n; ++k) all[k] = k;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint32_t k = n - 1; k > 0; --k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; std::swap(all[k], all[x % (k + 1)]); }
    std::vector<uint32_t> idx(all.begin(), all.begin() + m);  // cold requests, in "bin order" (random)
    std::vector<uint32_t> code(n);
    for (uint32_t k = 0; k < n; ++k) code[k] = k & 0xFFFFu;
    for (uint32_t j = 0; j < m; ++j) code[idx[j]] = 0x80000000u | j;  // cold: its sorted position
    uint32_t *d_idx, *d_code; uint64_t *d_out, *d_res;
    CK(hipMalloc(&d_idx, m * 4)); CK(hipMalloc(&d_code, n * 4)); CK(hipMalloc(&d_out, (size_t)n * 8)); CK(hipMalloc(&d_res, (size_t)m * 8));
    CK(hipMemcpy(d_idx, idx.data(), m * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_code, code.data(), n * 4, hipMemcpyHostToDevice));
    const int B = 256;
    float t_sc = timeit([&] { hipLaunchKernelGGL(k_scatter, dim3((m + B - 1) / B), dim3(B), 0, 0, d_idx, d_out, m); });
    float t_so = timeit([&] { hipLaunchKernelGGL(k_sorted, dim3((m + B - 1) / B), dim3(B), 0, 0, d_res, m); });
    float t_g = timeit([&] { hipLaunchKernelGGL(k_inorder<true>, dim3((n + B - 1) / B), dim3(B), 0, 0, d_code, d_res, d_out, n); });
    float t_h = timeit([&] { hipLaunchKernelGGL(k_inorder<false>, dim3((n + B - 1) / B), dim3(B), 0, 0, d_code, d_res, d_out, n); });
    printf("{\"m\":%u,\"scatter_us\":%.2f,\"sorted_us\":%.2f,\"inorder_gather_us\":%.2f,\"inorder_hot_only_us\":%.2f,"
           "\"today_us\":%.2f,\"sorted_gather_us\":%.2f}\n", m, t_sc * 1e3, t_so * 1e3, t_g * 1e3, t_h * 1e3,
           (t_sc + t_h) * 1e3, (t_so + t_g) * 1e3);
    return 0;
}
