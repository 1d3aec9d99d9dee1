// Stable LSD radix sort of (u32 key, 12-byte payload) pairs on gfx950 -- kernel K0
// of DESIGN.md.  Used to segment a batch by rule slot while keeping arrival
// order inside each rule (the reference decides each rule's requests in
// arrival order; stability is what makes the segmented replay exact).
//
// Per pass (digit of D bits, RADIX = 2^D <= 2048):
//   hist    : one 256-thread workgroup per 4096-key tile, LDS digit counts,
//             written digit-major  hist[d * ntiles + tile]
//   scan    : exclusive scan of the digit-major histogram (global offsets)
//   scatter : each wave ranks its 1024 keys in 16 rounds of 64 with a
//             ballot-based match (D ballots per round), keeping wave-private
//             running digit counts in LDS; one barrier, a cross-wave prefix,
//             then a scatter of key + payload.  Only two workgroup barriers
//             per tile.
#include "radix_sort.hpp"

namespace sga {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kRounds = 16;  // items per lane
constexpr int kTile = kThreads * kRounds;  // 4096

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ULL << lane) - 1ULL; }

template <int D>
__global__ __launch_bounds__(kThreads) void k_rs_hist(const uint32_t *__restrict__ keys, uint32_t n, int shift,
                                                      uint32_t ntiles, uint32_t *__restrict__ hist) {
    constexpr int RADIX = 1 << D;
    __shared__ uint32_t h[RADIX];
    for (int d = threadIdx.x; d < RADIX; d += kThreads) h[d] = 0;
    __syncthreads();
    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * kTile;
#pragma unroll 4
    for (int r = 0; r < kRounds; ++r) {
        uint32_t e = base + r * kThreads + threadIdx.x;
        if (e < n) atomicAdd(&h[(keys[e] >> shift) & (RADIX - 1)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < RADIX; d += kThreads) hist[(size_t)d * ntiles + tile] = h[d];
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_rs_scatter(const uint32_t *__restrict__ keys_in,
                                                         const Payload *__restrict__ pay_in, uint32_t n, int shift,
                                                         uint32_t ntiles, const uint32_t *__restrict__ offsets,
                                                         uint32_t *__restrict__ keys_out,
                                                         Payload *__restrict__ pay_out) {
    constexpr int RADIX = 1 << D;
    __shared__ uint32_t goff[RADIX];
    __shared__ uint32_t wcnt[kWaves][RADIX];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x;
    for (int d = threadIdx.x; d < RADIX; d += kThreads) {
        goff[d] = offsets[(size_t)d * ntiles + tile];
#pragma unroll
        for (int w = 0; w < kWaves; ++w) wcnt[w][d] = 0;
    }
    __syncthreads();

    const uint32_t wbase = tile * kTile + wave * (kRounds * 64);
    uint32_t key[kRounds];
    uint32_t rank[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        const bool valid = e < n;
        key[r] = valid ? keys_in[e] : 0u;
        const uint32_t d = (key[r] >> shift) & (RADIX - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < D; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        uint32_t before = 0;
        if (valid) before = wcnt[wave][d];
        // the lowest peer publishes the new running count after every peer read it
        __builtin_amdgcn_wave_barrier();
        const uint32_t my = (uint32_t)__popcll(peers & lanemask_lt(lane));
        if (valid && my == 0) wcnt[wave][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        rank[r] = before + my;
    }
    __syncthreads();
    // per digit: exclusive prefix over waves (wave order == arrival order in the tile)
    for (int d = threadIdx.x; d < RADIX; d += kThreads) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t c = wcnt[w][d];
            wcnt[w][d] = s;
            s += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        if (e < n) {
            const uint32_t d = (key[r] >> shift) & (RADIX - 1);
            const uint32_t pos = goff[d] + wcnt[wave][d] + rank[r];
            keys_out[pos] = key[r];
            pay_out[pos] = pay_in[e];
        }
    }
}

// ---- device-wide exclusive scan of u32 (3 phases) --------------------------
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *total) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (wave == 0) {
        uint32_t w = lane < kScanThreads / 64 ? wsum[lane] : 0;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            uint32_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < kScanThreads / 64) wsum[lane] = w;
    }
    __syncthreads();
    const uint32_t wave_prefix = wave ? wsum[wave - 1] : 0;
    if (total) *total = wsum[kScanThreads / 64 - 1];
    const uint32_t r = wave_prefix + x - v;
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint32_t *__restrict__ in, uint32_t n,
                                                              uint32_t *__restrict__ partial) {
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i)
        if (base + i < n) s += in[base + i];
    uint32_t total;
    block_exclusive_scan(s, &total);
    if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_partials(uint32_t *__restrict__ partial, uint32_t nparts) {
    // single workgroup; loops if nparts > kScanTile
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nparts; base += kScanTile) {
        const uint32_t i0 = base + threadIdx.x * kScanItems;
        uint32_t v[kScanItems];
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) {
            v[i] = (i0 + i < nparts) ? partial[i0 + i] : 0;
            s += v[i];
        }
        uint32_t total;
        uint32_t pre = block_exclusive_scan(s, &total) + carry;
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) {
            if (i0 + i < nparts) partial[i0 + i] = pre;
            pre += v[i];
        }
        carry += total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const uint32_t *__restrict__ in, uint32_t n,
                                                             const uint32_t *__restrict__ partial,
                                                             uint32_t *__restrict__ out) {
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        v[i] = (base + i < n) ? in[base + i] : 0;
        s += v[i];
    }
    uint32_t pre = block_exclusive_scan(s, nullptr) + partial[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        if (base + i < n) out[base + i] = pre;
        pre += v[i];
    }
}

}  // namespace

size_t scan_partials_needed(size_t n) { return (n + kScanTile - 1) / kScanTile; }

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, uint32_t *partial, hipStream_t s) {
    if (n == 0) return;
    const uint32_t nb = (uint32_t)scan_partials_needed(n);
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(kScanThreads), 0, s, in, (uint32_t)n, partial);
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(kScanThreads), 0, s, partial, nb);
    hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(kScanThreads), 0, s, in, (uint32_t)n, partial, out);
}

size_t radix_tiles(size_t n) { return (n + kTile - 1) / kTile; }

size_t radix_hist_entries(size_t n, int bits) {
    const int npass = bits <= 0 ? 0 : (bits + kMaxDigitBits - 1) / kMaxDigitBits;
    const int d = npass ? (bits + npass - 1) / npass : 1;
    return ((size_t)1 << d) * radix_tiles(n);
}

template <int D>
static void pass(const uint32_t *kin, const Payload *pin, uint32_t *kout, Payload *pout, uint32_t n, int shift,
                 RadixScratch &sc, hipStream_t s) {
    const uint32_t nt = (uint32_t)radix_tiles(n);
    hipLaunchKernelGGL((k_rs_hist<D>), dim3(nt), dim3(kThreads), 0, s, kin, n, shift, nt, sc.hist);
    exclusive_scan_u32(sc.hist, sc.hist_scan, ((size_t)1 << D) * nt, sc.partial, s);
    hipLaunchKernelGGL((k_rs_scatter<D>), dim3(nt), dim3(kThreads), 0, s, kin, pin, n, shift, nt, sc.hist_scan, kout,
                       pout);
}

int radix_sort_pairs(uint32_t *keys, Payload *pay, uint32_t *keys_alt, Payload *pay_alt, size_t n, int bits,
                     RadixScratch &sc, hipStream_t s) {
    if (n == 0 || bits <= 0) return 0;
    const int npass = (bits + kMaxDigitBits - 1) / kMaxDigitBits;
    const int d = (bits + npass - 1) / npass;
    uint32_t *ks = keys, *kd = keys_alt;
    Payload *ps = pay, *pd = pay_alt;
    for (int p = 0; p < npass; ++p) {
        const int shift = p * d;
        switch (d) {
        case 1: pass<1>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 2: pass<2>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 3: pass<3>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 4: pass<4>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 5: pass<5>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 6: pass<6>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 7: pass<7>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 8: pass<8>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 9: pass<9>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        case 10: pass<10>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        default: pass<11>(ks, ps, kd, pd, (uint32_t)n, shift, sc, s); break;
        }
        uint32_t *tk = ks; ks = kd; kd = tk;
        Payload *tp = ps; ps = pd; pd = tp;
    }
    return npass;  // result is in (keys, pay) if npass even, else in the alt buffers
}

}  // namespace sga
