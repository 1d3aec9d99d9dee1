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

#include <cstdlib>

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

// ---- single-sweep passes (decoupled look-back) ------------------------------
// Per pass one kernel: a workgroup takes the next tile id from a counter, ranks its
// 4096 keys (same ballot match as above), publishes its per-digit counts, looks
// back over the previous tiles' published counts for its global digit offsets,
// then stages the tile in LDS in sorted order so that keys and payloads leave as
// contiguous per-digit segments (coalesced stores instead of one store per key).
// Digit totals of every pass come from one up-front histogram read of the keys.
constexpr uint32_t kFlagAgg = 1u << 30, kFlagPrefix = 2u << 30, kCountMask = (1u << 30) - 1;
constexpr int kMaxPasses = 3;

template <int D>
__global__ __launch_bounds__(kThreads) void k_rs_upfront(const uint32_t *__restrict__ keys, uint32_t n, int npass,
                                                         uint32_t *__restrict__ ghist) {
    constexpr int RADIX = 1 << D;
    __shared__ uint32_t h[kMaxPasses][RADIX];
    for (int d = threadIdx.x; d < kMaxPasses * RADIX; d += kThreads) (&h[0][0])[d] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kTile;
#pragma unroll 4
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = base + r * kThreads + threadIdx.x;
        if (e < n) {
            const uint32_t k = keys[e];
            for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(k >> (p * D)) & (RADIX - 1)], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * RADIX; i += kThreads) {
        const uint32_t v = (&h[0][0])[i];
        if (v) atomicAdd(&ghist[i], v);
    }
}

// exclusive scan of each pass's RADIX digit totals (one workgroup)
template <int D>
__global__ __launch_bounds__(kThreads) void k_rs_digit_base(uint32_t *__restrict__ ghist, int npass) {
    constexpr int RADIX = 1 << D;
    constexpr int DPT = RADIX >= kThreads ? RADIX / kThreads : 1;
    __shared__ uint32_t ws[kWaves];
    for (int p = 0; p < npass; ++p) {
        uint32_t *g = ghist + p * RADIX;
        uint32_t v[DPT];
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            const int d = threadIdx.x * DPT + k;
            v[k] = d < RADIX ? g[d] : 0;
            sum += v[k];
        }
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        uint32_t pre = x - sum;
        for (int w = 0; w < wave; ++w) pre += ws[w];
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            const int d = threadIdx.x * DPT + k;
            if (d < RADIX) g[d] = pre;
            pre += v[k];
        }
        __syncthreads();
    }
}

template <int D>
struct OnesweepSmem {
    static constexpr int RADIX = 1 << D;
    uint32_t wcnt[kWaves][RADIX];  // per-wave digit counts, then exclusive prefixes over waves
    uint32_t dstart[RADIX];        // tile-local exclusive digit start
    uint32_t gbase[RADIX];         // global position of the tile's first key of digit d
    uint32_t skey[kTile];
    Payload spay[kTile / 2];
    uint32_t tile;
};

// LB = true: decoupled look-back over `status`; LB = false: the tile's global digit offsets
// come precomputed in `digit_base` (digit-major scan of the per-tile histograms).
template <int D, bool LB>
__global__ __launch_bounds__(kThreads) void k_rs_onesweep(const uint32_t *__restrict__ keys_in,
                                                          const Payload *__restrict__ pay_in, uint32_t n, int shift,
                                                          const uint32_t *__restrict__ digit_base,
                                                          uint32_t *__restrict__ status, uint32_t *tile_ctr,
                                                          uint32_t *__restrict__ keys_out,
                                                          Payload *__restrict__ pay_out) {
    constexpr int RADIX = 1 << D;
    constexpr int DPT = RADIX >= kThreads ? RADIX / kThreads : 1;
    __shared__ OnesweepSmem<D> sm;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) sm.tile = LB ? atomicAdd(tile_ctr, 1u) : blockIdx.x;
    for (int d = threadIdx.x; d < RADIX; d += kThreads) {
#pragma unroll
        for (int w = 0; w < kWaves; ++w) sm.wcnt[w][d] = 0;
    }
    __syncthreads();
    const uint32_t tile = sm.tile;
    const uint32_t tbase = tile * kTile;
    const uint32_t tn = min((uint32_t)kTile, n - tbase);

    // ---- rank: wave-private running digit counts (arrival order kept)
    const uint32_t wbase = tbase + wave * (kRounds * 64);
    uint32_t key[kRounds];
    uint32_t pos[kRounds];
    Payload pv[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        const bool valid = e < n;
        key[r] = valid ? keys_in[e] : 0u;
        pv[r] = valid ? pay_in[e] : Payload{0, 0, 0, 0};
        const uint32_t d = (key[r] >> shift) & (RADIX - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < D; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        uint32_t before = 0;
        if (valid) before = sm.wcnt[wave][d];
        __builtin_amdgcn_wave_barrier();
        const uint32_t my = (uint32_t)__popcll(peers & lanemask_lt(lane));
        if (valid && my == 0) sm.wcnt[wave][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        pos[r] = before + my;
    }
    __syncthreads();

    // ---- per digit (blocked: thread t owns digits t*DPT ..): wave prefixes, tile totals,
    //      publish the aggregate, tile-local digit starts (block scan)
    uint32_t tot[DPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = threadIdx.x * DPT + k;
        uint32_t sacc = 0;
        if (d < RADIX) {
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = sm.wcnt[w][d];
                sm.wcnt[w][d] = sacc;
                sacc += c;
            }
            if (LB)
                __hip_atomic_store(&status[(size_t)tile * RADIX + d], (tile == 0 ? kFlagPrefix : kFlagAgg) | sacc,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        tot[k] = sacc;
        tsum += sacc;
    }
    {
        __shared__ uint32_t ws[kWaves];
        uint32_t x = tsum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        uint32_t pre = x - tsum;
        for (int w = 0; w < wave; ++w) pre += ws[w];
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            const int d = threadIdx.x * DPT + k;
            if (d < RADIX) sm.dstart[d] = pre;
            pre += tot[k];
        }
    }
    // ---- decoupled look-back: exclusive count of digit d over all previous tiles
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = threadIdx.x * DPT + k;
        if (d >= RADIX) continue;
        if (!LB) {
            sm.gbase[d] = digit_base[(size_t)d * gridDim.x + tile];
            continue;
        }
        uint32_t excl = 0;
        if (tile > 0) {
            int64_t t = (int64_t)tile - 1;
            while (true) {
                uint32_t v;
                do {
                    v = __hip_atomic_load(&status[(size_t)t * RADIX + d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((v >> 30) == 0) __builtin_amdgcn_s_sleep(1);
                } while ((v >> 30) == 0);
                excl += v & kCountMask;
                if ((v & kFlagPrefix) || t == 0) break;
                --t;
            }
            __hip_atomic_store(&status[(size_t)tile * RADIX + d], kFlagPrefix | (excl + tot[k]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        sm.gbase[d] = digit_base[d] + excl;
    }
    __syncthreads();

    // ---- stage keys in tile-sorted order, then write them out as digit segments
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        if (e < n) {
            const uint32_t d = (key[r] >> shift) & (RADIX - 1);
            pos[r] += sm.dstart[d] + sm.wcnt[wave][d];
            sm.skey[pos[r]] = key[r];
        }
    }
    __syncthreads();
    uint32_t gpos[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t i = r * kThreads + threadIdx.x;
        gpos[r] = 0;
        if (i < tn) {
            const uint32_t k = sm.skey[i];
            const uint32_t d = (k >> shift) & (RADIX - 1);
            gpos[r] = sm.gbase[d] + (i - sm.dstart[d]);
            keys_out[gpos[r]] = k;
        }
    }
    // ---- payloads in two halves of the tile (LDS budget)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const uint32_t lo = half * (kTile / 2);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kRounds; ++r) {
            const uint32_t e = wbase + r * 64 + lane;
            if (e < n && pos[r] >= lo && pos[r] < lo + kTile / 2) sm.spay[pos[r] - lo] = pv[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = half * (kRounds / 2); r < (half + 1) * (kRounds / 2); ++r) {
            const uint32_t i = r * kThreads + threadIdx.x;
            if (i < tn) pay_out[gpos[r]] = sm.spay[i - lo];
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


// Per-digit prefix over tiles (one workgroup per digit row of the digit-major histogram) and the
// row total; the sweep adds the digit offsets (scan of the totals).  One launch instead of the
// three of a flat scan over digits x tiles.
constexpr int kRowItems = 8;
__global__ __launch_bounds__(kThreads) void k_row_scan(const uint32_t *__restrict__ hist, uint32_t nt,
                                                       uint32_t *__restrict__ hist_scan, uint32_t *__restrict__ tot,
                                                       const uint32_t *__restrict__ dn) {
    // dn: live element count on the device -- tiles past it have no histogram column
    __shared__ uint32_t ws[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t *row = hist + (size_t)blockIdx.x * nt;
    uint32_t *orow = hist_scan + (size_t)blockIdx.x * nt;
    if (dn) nt = min(nt, (*dn + kTile - 1) / kTile);
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nt; base += kThreads * kRowItems) {
        const uint32_t i0 = base + threadIdx.x * kRowItems;
        uint32_t v[kRowItems], s = 0;
#pragma unroll
        for (int k = 0; k < kRowItems; ++k) {
            v[k] = i0 + k < nt ? row[i0 + k] : 0u;
            s += v[k];
        }
        uint32_t x = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        uint32_t pre = carry + x - s, total = 0;
        for (int w = 0; w < kWaves; ++w) {
            if (w < wave) pre += ws[w];
            total += ws[w];
        }
#pragma unroll
        for (int k = 0; k < kRowItems; ++k) {
            if (i0 + k < nt) orow[i0 + k] = pre;
            pre += v[k];
        }
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// ---- u64 elements with an embedded key (kernel K0 of the cluster path) -----
// The element carries everything the later stages need (rule slot, window-bucket delta,
// prioritized flag, acquire count, request index), so a pass moves 8 bytes per request.
// Per pass: tile histogram (fused into the producer for pass 0), digit-major scan, then a
// ranking + LDS-staged scatter kernel as above.
template <int D>
__global__ __launch_bounds__(kThreads) void k_rs64_hist(const uint64_t *__restrict__ el, uint32_t n, int shift,
                                                        uint32_t ntiles, uint32_t *__restrict__ hist,
                                                        const uint32_t *__restrict__ dn,
                                                        const uint32_t *__restrict__ tile_n) {
    // dn: element count on the device (a producer that compacts); tiles past it count nothing.
    // tile_n: segmented producer (as in k_rs64_sweep): wave w of tile t counts tile_n[4 t + w]
    // elements from its segment's start.
    // After the first pass equal keys sit next to each other, so one digit often fills a whole
    // wave: lanes with equal digits are matched by ballots (as in the sweep) and only the first
    // of them adds the group's size -- at most one LDS atomic per distinct digit per wave.
    constexpr int RADIX = 1 << D;
    __shared__ uint32_t h[RADIX];
    for (int d = threadIdx.x; d < RADIX; d += kThreads) h[d] = 0;
    __syncthreads();
    const uint32_t tile = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t wbase = tile * kTile + (threadIdx.x >> 6) * (kRounds * 64);
    if (dn) n = min(n, *dn);
    if (!tile_n && tile * kTile >= n) return;  // past the live elements (k_row_scan skips the tile)
    uint32_t wn;  // elements of this wave's segment
    if (tile_n) wn = tile_n[tile * kWaves + (threadIdx.x >> 6)];
    else wn = n > wbase ? min((uint32_t)(kRounds * 64), n - wbase) : 0u;
    wn = __builtin_amdgcn_readfirstlane(wn);
    uint64_t key[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        key[r] = (uint32_t)(r * 64 + lane) < wn ? el[e] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        if ((uint32_t)(r * 64) >= wn) continue;  // wave-uniform: past the segment's elements
        const bool valid = (uint32_t)(r * 64 + lane) < wn;
        const uint32_t d = (uint32_t)(key[r] >> shift) & (RADIX - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < D; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        if (valid && (peers & lanemask_lt(lane)) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    for (int d = threadIdx.x; d < RADIX; d += kThreads) hist[(size_t)d * ntiles + tile] = h[d];
}

// Global digit totals of every pass in one read of the elements (look-back mode).
template <int D>
__global__ __launch_bounds__(kThreads) void k_rs64_upfront(const uint64_t *__restrict__ el, uint32_t n, int shift,
                                                           int npass, uint32_t *__restrict__ ghist) {
    constexpr int RADIX = 1 << D;
    __shared__ uint32_t h[kMaxPasses * RADIX];
    for (int d = threadIdx.x; d < kMaxPasses * RADIX; d += kThreads) h[d] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kTile;
#pragma unroll 4
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = base + r * kThreads + threadIdx.x;
        if (e < n) {
            const uint64_t k = el[e];
            for (int p = 0; p < npass; ++p) atomicAdd(&h[p * RADIX + ((uint32_t)(k >> (shift + p * D)) & (RADIX - 1))], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * RADIX; i += kThreads)
        if (h[i]) atomicAdd(&ghist[i], h[i]);
}

template <int D>
struct Sweep64Smem {
    static constexpr int RADIX = 1 << D;
    uint32_t wcnt[kWaves][RADIX];  // per-wave running digit counts, then exclusive prefixes over waves
    uint32_t dstart[RADIX];        // tile-local exclusive digit start
    uint32_t gbase[RADIX];         // global output position of the tile's first element of digit d
    uint64_t sel[kTile];           // tile in sorted order
};

template <int D>
__global__ __launch_bounds__(kThreads) void k_rs64_sweep(const uint64_t *__restrict__ in, uint32_t n, int shift,
                                                         const uint32_t *__restrict__ digit_base,
                                                         uint64_t *__restrict__ out,
                                                         const uint32_t *__restrict__ tile_n,
                                                         const uint32_t *__restrict__ dn,
                                                         const uint32_t *__restrict__ digit_tot) {
    // tile_n: segmented producer -- wave w of tile t holds tile_n[t * kWaves + w] elements at
    // in[t * kTile + w * kRounds * 64 ..] (arrival order: segment w before w + 1);
    // dn: element count on the device.  Either may be null (contiguous input of n elements).
    // digit_tot: per-digit totals when digit_base holds per-digit (row) prefixes over tiles; the
    // digit offsets are then scanned here.  Null: digit_base is the full digit-major scan.
    constexpr int RADIX = 1 << D;
    constexpr int DPT = RADIX >= kThreads ? RADIX / kThreads : 1;
    __shared__ Sweep64Smem<D> sm;
    __shared__ uint32_t ws[kWaves];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (!tile_n && dn && blockIdx.x * (uint32_t)kTile >= min(n, *dn)) return;  // no live element
    uint32_t dexc[DPT];
    if (digit_tot) {
        __shared__ uint32_t ws2[kWaves];
        uint32_t v[DPT], s = 0;
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            const int d = threadIdx.x * DPT + k;
            v[k] = d < RADIX ? digit_tot[d] : 0u;
            s += v[k];
        }
        uint32_t x = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws2[wave] = x;
        __syncthreads();
        uint32_t pre = x - s;
        for (int w = 0; w < wave; ++w) pre += ws2[w];
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            dexc[k] = pre;
            pre += v[k];
        }
    } else {
#pragma unroll
        for (int k = 0; k < DPT; ++k) dexc[k] = 0;
    }
    for (int d = threadIdx.x; d < RADIX; d += kThreads) {
#pragma unroll
        for (int w = 0; w < kWaves; ++w) sm.wcnt[w][d] = 0;
    }
    __syncthreads();
    const uint32_t tile = blockIdx.x;
    const uint32_t tbase = tile * kTile;
    if (dn) n = min(n, *dn);
    const uint32_t wloc = wave * (kRounds * 64);
    uint32_t tn, wn;
    if (tile_n) {
        tn = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) tn += tile_n[tile * kWaves + w];
        wn = tile_n[tile * kWaves + wave];
    } else {
        tn = n > tbase ? min((uint32_t)kTile, n - tbase) : 0u;
        wn = tn > wloc ? tn - wloc : 0u;
    }
    const uint32_t wbase = tbase + wloc;
    // rounds past the wave's last element are skipped whole (wave-uniform): a segmented producer's
    // segments are often a quarter full
    wn = __builtin_amdgcn_readfirstlane(wn);
    uint64_t key[kRounds];
    uint32_t pos[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        key[r] = (uint32_t)(r * 64 + lane) < wn ? in[e] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        pos[r] = 0;
        if ((uint32_t)(r * 64) >= wn) continue;
        const bool valid = (uint32_t)(r * 64 + lane) < wn;
        const uint32_t d = (uint32_t)(key[r] >> shift) & (RADIX - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < D; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        uint32_t before = 0;
        if (valid) before = sm.wcnt[wave][d];
        __builtin_amdgcn_wave_barrier();
        const uint32_t my = (uint32_t)__popcll(peers & lanemask_lt(lane));
        if (valid && my == 0) sm.wcnt[wave][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        pos[r] = before + my;
    }
    __syncthreads();
    uint32_t tot[DPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = threadIdx.x * DPT + k;
        uint32_t sacc = 0;
        if (d < RADIX) {
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = sm.wcnt[w][d];
                sm.wcnt[w][d] = sacc;
                sacc += c;
            }
            sm.gbase[d] = digit_base[(size_t)d * gridDim.x + tile] + dexc[k];
        }
        tot[k] = sacc;
        tsum += sacc;
    }
    {
        uint32_t x = tsum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        uint32_t pre = x - tsum;
        for (int w = 0; w < wave; ++w) pre += ws[w];
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            const int d = threadIdx.x * DPT + k;
            if (d < RADIX) sm.dstart[d] = pre;
            pre += tot[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        if ((uint32_t)(r * 64 + lane) < wn) {
            const uint32_t d = (uint32_t)(key[r] >> shift) & (RADIX - 1);
            sm.sel[pos[r] + sm.dstart[d] + sm.wcnt[wave][d]] = key[r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t i = r * kThreads + threadIdx.x;
        if (i < tn) {
            const uint64_t k = sm.sel[i];
            const uint32_t d = (uint32_t)(k >> shift) & (RADIX - 1);
            out[sm.gbase[d] + (i - sm.dstart[d])] = k;
        }
    }
}


// Single pass per digit (decoupled look-back): the tile id comes from a counter (tiles start in
// order, so every look-back target has started), the tile publishes its per-digit counts as an
// aggregate, walks back over predecessors until an inclusive prefix, then publishes its own
// inclusive prefix.  Status words: flag (bits 31:30) | count, published by agent-scope atomic adds
// and polled with agent-scope loads (cross-XCD visible).  The wait is bounded: a look-back that
// gives up sets err[0] (never expected; the host API reports it) instead of hanging the GPU.
constexpr uint32_t kLbAgg = 1u << 30, kLbPrefix = 2u << 30, kLbCount = (1u << 30) - 1;

template <int D>
__global__ __launch_bounds__(kThreads) void k_rs64_sweep_lb(const uint64_t *__restrict__ in, uint32_t n, int shift,
                                                            const uint32_t *__restrict__ digit_base,
                                                            uint32_t *__restrict__ status, uint32_t *tile_ctr,
                                                            uint32_t *err, uint64_t *__restrict__ out) {
    constexpr int RADIX = 1 << D;
    constexpr int DPT = RADIX >= kThreads ? RADIX / kThreads : 1;
    __shared__ Sweep64Smem<D> sm;
    __shared__ uint32_t ws[kWaves];
    __shared__ uint32_t stile;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) stile = atomicAdd(tile_ctr, 1u);
    for (int d = threadIdx.x; d < RADIX; d += kThreads) {
#pragma unroll
        for (int w = 0; w < kWaves; ++w) sm.wcnt[w][d] = 0;
    }
    __syncthreads();
    const uint32_t tile = stile;
    const uint32_t tbase = tile * kTile;
    const uint32_t tn = min((uint32_t)kTile, n - tbase);
    const uint32_t wbase = tbase + wave * (kRounds * 64);
    uint64_t key[kRounds];
    uint32_t pos[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        key[r] = e < n ? in[e] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        const bool valid = e < n;
        const uint32_t d = (uint32_t)(key[r] >> shift) & (RADIX - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < D; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        uint32_t before = 0;
        if (valid) before = sm.wcnt[wave][d];
        __builtin_amdgcn_wave_barrier();
        const uint32_t my = (uint32_t)__popcll(peers & lanemask_lt(lane));
        if (valid && my == 0) sm.wcnt[wave][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        pos[r] = before + my;
    }
    __syncthreads();
    uint32_t tot[DPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = threadIdx.x * DPT + k;
        uint32_t sacc = 0;
        if (d < RADIX) {
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = sm.wcnt[w][d];
                sm.wcnt[w][d] = sacc;
                sacc += c;
            }
            // publish the aggregate (tile 0: its inclusive prefix right away)
            atomicAdd(&status[(size_t)tile * RADIX + d], (tile == 0 ? kLbPrefix : kLbAgg) | sacc);
        }
        tot[k] = sacc;
        tsum += sacc;
    }
    {
        uint32_t x = tsum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        uint32_t pre = x - tsum;
        for (int w = 0; w < wave; ++w) pre += ws[w];
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
            const int d = threadIdx.x * DPT + k;
            if (d < RADIX) sm.dstart[d] = pre;
            pre += tot[k];
        }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = threadIdx.x * DPT + k;
        if (d >= RADIX) continue;
        uint32_t excl = 0;
        if (tile > 0) {
            int64_t t = (int64_t)tile - 1;
            uint32_t spins = 0;
            while (true) {
                uint32_t v = __hip_atomic_load(&status[(size_t)t * RADIX + d], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                while ((v >> 30) == 0) {
                    if (++spins > (1u << 24)) {
                        atomicOr(err, 1u);
                        v = kLbPrefix;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    v = __hip_atomic_load(&status[(size_t)t * RADIX + d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                excl += v & kLbCount;
                if ((v & kLbPrefix) || t == 0) break;
                --t;
            }
            // aggregate -> inclusive prefix: add the difference of the two status words
            atomicAdd(&status[(size_t)tile * RADIX + d], (kLbPrefix | (excl + tot[k])) - (kLbAgg | tot[k]));
        }
        sm.gbase[d] = digit_base[d] + excl;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t e = wbase + r * 64 + lane;
        if (e < n) {
            const uint32_t d = (uint32_t)(key[r] >> shift) & (RADIX - 1);
            sm.sel[pos[r] + sm.dstart[d] + sm.wcnt[wave][d]] = key[r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t i = r * kThreads + threadIdx.x;
        if (i < tn) {
            const uint64_t k = sm.sel[i];
            const uint32_t d = (uint32_t)(k >> shift) & (RADIX - 1);
            out[sm.gbase[d] + (i - sm.dstart[d])] = k;
        }
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

// status array (tiles x RADIX) + up-front digit histograms and tile counters
size_t radix_hist_entries(size_t n, int bits) {
    const int npass = bits <= 0 ? 0 : (bits + kMaxDigitBits - 1) / kMaxDigitBits;
    const int d = npass ? (bits + npass - 1) / npass : 1;
    return ((size_t)1 << d) * radix_tiles(n) + (size_t)kMaxPasses * 2048 + 64;
}

static int max_digit_bits() {
    static const int v = [] {
        // A/B knob: widest digit per pass (default 8).  At least 8: 24-bit slot keys must sort in
        // kMaxPasses (3) passes.
        const char *e = getenv("SGA_RADIX_BITS");
        int b = e ? atoi(e) : 8;
        return b < 8 ? 8 : (b > kMaxDigitBits ? kMaxDigitBits : b);
    }();
    return v;
}

static int radix_mode() {
    static const int v = [] {
        const char *e = getenv("SGA_RADIX_MODE");  // A/B knob: 0 look-back, 1 staged scatter, 2 direct scatter
        return e ? atoi(e) : 1;
    }();
    return v;
}

template <int D>
static void sort_passes(uint32_t *&ks, Payload *&ps, uint32_t *&kd, Payload *&pd, uint32_t n, int npass,
                        RadixScratch &sc, hipStream_t s) {
    constexpr int RADIX = 1 << D;
    const uint32_t nt = (uint32_t)radix_tiles(n);
    const int mode = radix_mode();
    if (mode != 0) {
        for (int p = 0; p < npass; ++p) {
            hipLaunchKernelGGL((k_rs_hist<D>), dim3(nt), dim3(kThreads), 0, s, ks, n, p * D, nt, sc.hist);
            exclusive_scan_u32(sc.hist, sc.hist_scan, (size_t)RADIX * nt, sc.partial, s);
            if (mode == 1)
                hipLaunchKernelGGL((k_rs_onesweep<D, false>), dim3(nt), dim3(kThreads), 0, s, ks, ps, n, p * D,
                                   sc.hist_scan, nullptr, nullptr, kd, pd);
            else
                hipLaunchKernelGGL((k_rs_scatter<D>), dim3(nt), dim3(kThreads), 0, s, ks, ps, n, p * D, nt,
                                   sc.hist_scan, kd, pd);
            uint32_t *tk = ks; ks = kd; kd = tk;
            Payload *tp = ps; ps = pd; pd = tp;
        }
        return;
    }
    uint32_t *status = sc.hist;
    uint32_t *ghist = sc.hist_scan;                     // npass x RADIX digit totals -> bases
    uint32_t *ctr = sc.hist_scan + kMaxPasses * 2048;   // one tile counter per pass
    SGA_HIP_CHECK(hipMemsetAsync(ghist, 0, (kMaxPasses * 2048 + 64) * sizeof(uint32_t), s));
    hipLaunchKernelGGL((k_rs_upfront<D>), dim3(nt), dim3(kThreads), 0, s, ks, n, npass, ghist);
    hipLaunchKernelGGL((k_rs_digit_base<D>), dim3(1), dim3(kThreads), 0, s, ghist, npass);
    for (int p = 0; p < npass; ++p) {
        SGA_HIP_CHECK(hipMemsetAsync(status, 0, (size_t)nt * RADIX * sizeof(uint32_t), s));
        hipLaunchKernelGGL((k_rs_onesweep<D, true>), dim3(nt), dim3(kThreads), 0, s, ks, ps, n, p * D, ghist + p * RADIX,
                           status, ctr + p, kd, pd);
        uint32_t *tk = ks; ks = kd; kd = tk;
        Payload *tp = ps; ps = pd; pd = tp;
    }
}

int radix_sort_pairs(uint32_t *keys, Payload *pay, uint32_t *keys_alt, Payload *pay_alt, size_t n, int bits,
                     RadixScratch &sc, hipStream_t s) {
    if (n == 0 || bits <= 0) return 0;
    const int mb = max_digit_bits();
    const int npass = (bits + mb - 1) / mb;
    const int d = (bits + npass - 1) / npass;
    if (npass > kMaxPasses) return -1;
    uint32_t *ks = keys, *kd = keys_alt;
    Payload *ps = pay, *pd = pay_alt;
    const uint32_t nn = (uint32_t)n;
    switch (d) {
    case 1: sort_passes<1>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 2: sort_passes<2>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 3: sort_passes<3>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 4: sort_passes<4>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 5: sort_passes<5>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 6: sort_passes<6>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 7: sort_passes<7>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 8: sort_passes<8>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 9: sort_passes<9>(ks, ps, kd, pd, nn, npass, sc, s); break;
    case 10: sort_passes<10>(ks, ps, kd, pd, nn, npass, sc, s); break;
    default: sort_passes<11>(ks, ps, kd, pd, nn, npass, sc, s); break;
    }
    return npass;  // result is in (keys, pay) if npass even, else in the alt buffers
}


int radix64_digit_bits(int bits) {
    if (bits <= 0) return 1;
    const int mb = max_digit_bits();  // 8 by default; SGA_RADIX_BITS up to 11 (two passes for 21-bit keys)
    const int npass = (bits + mb - 1) / mb;
    return (bits + npass - 1) / npass;
}

size_t radix64_tiles(size_t n) { return (n + kTile - 1) / kTile; }

int radix64_lookback() {
    static const int v = [] {
        const char *e = getenv("SGA_RADIX_MODE");  // A/B knob: 0 single-pass look-back, 1 hist + scan + sweep
        return e ? (atoi(e) == 0) : 0;
    }();
    return v;
}

template <int D>
static int sort64_passes(uint64_t *a, uint64_t *alt, uint32_t n, int key_shift, int npass, RadixScratch &sc,
                         hipStream_t s, bool hist0_ready, const uint64_t *first_src = nullptr,
                         const uint32_t *tile_n0 = nullptr, const uint32_t *dn = nullptr) {
    constexpr int RADIX = 1 << D;
    const uint32_t nt = (uint32_t)radix64_tiles(n);
    if (first_src) {
        // pass 0 reads the producer's tile-compacted buffer, later passes alternate a <-> alt
        for (int p = 0; p < npass; ++p) {
            const int shift = key_shift + p * D;
            const uint64_t *src = p == 0 ? first_src : ((p & 1) ? a : alt);
            uint64_t *dst = (p & 1) ? alt : a;
            if (p > 0 || !hist0_ready)
                hipLaunchKernelGGL((k_rs64_hist<D>), dim3(nt), dim3(kThreads), 0, s, src, n, shift, nt, sc.hist,
                                   p == 0 ? nullptr : dn, p == 0 ? tile_n0 : nullptr);
            hipLaunchKernelGGL(k_row_scan, dim3(RADIX), dim3(kThreads), 0, s, sc.hist, nt, sc.hist_scan, sc.ghist,
                               p == 0 ? nullptr : dn);
            hipLaunchKernelGGL((k_rs64_sweep<D>), dim3(nt), dim3(kThreads), 0, s, src, n, shift, sc.hist_scan, dst,
                               p == 0 ? tile_n0 : nullptr, p == 0 ? nullptr : dn, sc.ghist);
        }
        return npass;
    }
    uint64_t *src = a, *dst = alt;
    if (radix64_lookback() && sc.ghist) {
        // global digit totals of every pass: counted by the producer into sc.ghist when hist0_ready
        if (!hist0_ready) {
            SGA_HIP_CHECK(hipMemsetAsync(sc.ghist, 0, kRadixGhistWords * sizeof(uint32_t), s));
            hipLaunchKernelGGL((k_rs64_upfront<D>), dim3(nt), dim3(kThreads), 0, s, src, n, key_shift, npass,
                               sc.ghist);
        }
        hipLaunchKernelGGL((k_rs_digit_base<D>), dim3(1), dim3(kThreads), 0, s, sc.ghist, npass);
        for (int p = 0; p < npass; ++p) {
            SGA_HIP_CHECK(hipMemsetAsync(sc.hist, 0, (size_t)nt * RADIX * sizeof(uint32_t), s));
            hipLaunchKernelGGL((k_rs64_sweep_lb<D>), dim3(nt), dim3(kThreads), 0, s, src, n, key_shift + p * D,
                               sc.ghist + p * RADIX, sc.hist, sc.ghist + kMaxPasses * 2048 + p, sc.err, dst);
            uint64_t *t = src;
            src = dst;
            dst = t;
        }
        return npass;
    }
    for (int p = 0; p < npass; ++p) {
        const int shift = key_shift + p * D;
        if (p > 0 || !hist0_ready)
            hipLaunchKernelGGL((k_rs64_hist<D>), dim3(nt), dim3(kThreads), 0, s, src, n, shift, nt, sc.hist,
                               nullptr, nullptr);
        hipLaunchKernelGGL(k_row_scan, dim3(RADIX), dim3(kThreads), 0, s, sc.hist, nt, sc.hist_scan, sc.ghist,
                           nullptr);
        hipLaunchKernelGGL((k_rs64_sweep<D>), dim3(nt), dim3(kThreads), 0, s, src, n, shift, sc.hist_scan, dst,
                           nullptr, nullptr, sc.ghist);
        uint64_t *t = src;
        src = dst;
        dst = t;
    }
    return npass;
}

int radix_sort_u64(uint64_t *a, uint64_t *alt, size_t n, int key_shift, int bits, RadixScratch &sc, hipStream_t s,
                   bool hist0_ready) {
    if (n == 0 || bits <= 0) return 0;
    const int d = radix64_digit_bits(bits);
    const int npass = (bits + d - 1) / d;
    if (npass > kMaxPasses) return -1;
    const uint32_t nn = (uint32_t)n;
    switch (d) {
    case 1: return sort64_passes<1>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 2: return sort64_passes<2>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 3: return sort64_passes<3>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 4: return sort64_passes<4>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 5: return sort64_passes<5>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 6: return sort64_passes<6>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 7: return sort64_passes<7>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 8: return sort64_passes<8>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 9: return sort64_passes<9>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    case 10: return sort64_passes<10>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    default: return sort64_passes<11>(a, alt, nn, key_shift, npass, sc, s, hist0_ready);
    }
}

}  // namespace sga

namespace sga {

int radix_sort_u64_tiled(const uint64_t *src, const uint32_t *tile_n0, const uint32_t *dn, uint64_t *a,
                         uint64_t *alt, size_t n, int key_shift, int bits, RadixScratch &sc, hipStream_t s,
                         bool hist0_ready) {
    if (n == 0 || bits <= 0) return 0;
    const int d = radix64_digit_bits(bits);
    const int npass = (bits + d - 1) / d;
    if (npass > kMaxPasses) return -1;
    const uint32_t nn = (uint32_t)n;
    switch (d) {
    case 1: return sort64_passes<1>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 2: return sort64_passes<2>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 3: return sort64_passes<3>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 4: return sort64_passes<4>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 5: return sort64_passes<5>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 6: return sort64_passes<6>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 7: return sort64_passes<7>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 8: return sort64_passes<8>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 9: return sort64_passes<9>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    case 10: return sort64_passes<10>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    default: return sort64_passes<11>(a, alt, nn, key_shift, npass, sc, s, hist0_ready, src, tile_n0, dn);
    }
}

}  // namespace sga
