// Does an LDS atomic add with return, issued by one wave instruction, hand out the old values of
// lanes that hit the same address in lane order?  Compares atomicAdd's return with the in-order
// rank (ballot match) over many random rounds.  Prints mismatches per key range.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k(uint32_t K, uint32_t rounds, uint32_t seed, unsigned long long *bad, int mode) {
    __shared__ uint32_t c[4][4096];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int h = lane; h < 4096; h += 64) c[w][h] = 0;
    __builtin_amdgcn_wave_barrier();
    unsigned long long nb = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
        uint32_t x = mix(seed ^ (blockIdx.x * 1315423911u) ^ (r * 2654435761u) ^ (threadIdx.x * 97u));
        uint32_t hid = x % K;
        if (mode == 1) hid = (x & 1) ? 7 : hid;                       // skewed
        const bool act = mode == 2 ? ((x >> 8) & 1) : true;             // half the lanes active
        uint32_t v = 0xFFFFFFFFu;
        // reference: in-order rank via reading the counter before and matching ids
        uint32_t before = c[w][hid];
        __builtin_amdgcn_wave_barrier();
        uint64_t peers = __ballot(act);
        for (int b = 0; b < 12; ++b) {
            const bool bit = (hid >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint64_t lt = (1ull << lane) - 1ull;
        const uint32_t expect = before + (uint32_t)__popcll(peers & lt);
        __builtin_amdgcn_wave_barrier();
        if (act) v = atomicAdd(&c[w][hid], 1u);
        __builtin_amdgcn_wave_barrier();
        if (act && v != expect) ++nb;
    }
    atomicAdd(bad, nb);
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 8);
    const uint32_t Ks[] = {1, 2, 4, 16, 64, 512, 4096};
    for (int mode = 0; mode < 3; ++mode)
        for (uint32_t K : Ks) {
            hipMemset(d, 0, 8);
            hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, K, 64u, 12345u + K, d, mode);
            unsigned long long h = 0;
            hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
            printf("mode %d K %4u: %llu mismatches of %llu lane-ops\n", mode, K, h, 4096ull * 256 * 64);
        }
    return 0;
}
