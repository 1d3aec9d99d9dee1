// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE against known byte counts for the access
// patterns the engine uses (MI355X_MICROARCH.md: "other access widths are uncalibrated").  Tables
// are 2 GiB (past the 256 MiB Infinity Cache).  Run under rocprofv3 --pmc FETCH_SIZE (then
// WRITE_SIZE) and divide by the bytes printed per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
// coalesced 16 B per lane
__global__ void k_cal_stream16(const int4 *__restrict__ a, int *__restrict__ sink, size_t n) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i].x ^ a[i].w;
    if (acc == 0x12345678) sink[0] = acc;
}
// coalesced 4 B per lane
__global__ void k_cal_stream4(const int *__restrict__ a, int *__restrict__ sink, size_t n) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
    if (acc == 0x12345678) sink[0] = acc;
}
// one random 8 B read per lane (distinct 128 B lines)
__global__ void k_cal_rand8(const uint64_t *__restrict__ t, size_t lines, int *__restrict__ sink, size_t n) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= t[(mix64(i) % lines) * 16];
    if (acc == 0x12345678) sink[0] = (int)acc;
}
// one random 16 B read per lane
__global__ void k_cal_rand16(const int4 *__restrict__ t, size_t lines, int *__restrict__ sink, size_t n) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int4 v = t[(mix64(i) % lines) * 8];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x12345678) sink[0] = acc;
}
// a random 128 B line read whole by one lane (8 x 16 B)
__global__ void k_cal_rand128(const int4 *__restrict__ t, size_t lines, int *__restrict__ sink, size_t n) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int4 *p = t + (mix64(i) % lines) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= p[k].x ^ p[k].w;
    }
    if (acc == 0x12345678) sink[0] = acc;
}
// one random 8 B store per lane (distinct lines)
__global__ void k_cal_wrand8(uint64_t *__restrict__ t, size_t lines, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        t[(mix64(i) % lines) * 16] = i;
}
// coalesced 8 B stores
__global__ void k_cal_wstream8(uint64_t *__restrict__ t, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) t[i] = i;
}

int main() {
    const size_t bytes = (size_t)2 << 30, lines = bytes / 128;
    char *t;
    int *sink;
    CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(t, 1, bytes));
    const size_t n = (size_t)1 << 24;  // random accesses per kernel
    const dim3 g(4096), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_cal_stream16, g, b, 0, 0, (const int4 *)t, sink, bytes / 16);
        hipLaunchKernelGGL(k_cal_stream4, g, b, 0, 0, (const int *)t, sink, bytes / 4);
        hipLaunchKernelGGL(k_cal_rand8, g, b, 0, 0, (const uint64_t *)t, lines, sink, n);
        hipLaunchKernelGGL(k_cal_rand16, g, b, 0, 0, (const int4 *)t, lines, sink, n);
        hipLaunchKernelGGL(k_cal_rand128, g, b, 0, 0, (const int4 *)t, lines, sink, n);
        hipLaunchKernelGGL(k_cal_wrand8, g, b, 0, 0, (uint64_t *)t, lines, n);
        hipLaunchKernelGGL(k_cal_wstream8, g, b, 0, 0, (uint64_t *)t, bytes / 8);
    }
    CK(hipDeviceSynchronize());
    printf("{\"stream16_bytes\": %zu, \"stream4_bytes\": %zu, \"rand8_accesses\": %zu, \"rand16_accesses\": %zu, "
           "\"rand128_lines\": %zu, \"wrand8_accesses\": %zu, \"wstream8_bytes\": %zu}\n",
           bytes, bytes, n, n, n, n, bytes);
    return 0;
}
