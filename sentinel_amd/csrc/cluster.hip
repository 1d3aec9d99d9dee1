// Cluster token server decision path on gfx950 (kernels K0, K6 of DESIGN.md).
//
// Semantics restated from the reference (aliases as in SURVEY.md):
//   DefaultTokenService.requestToken        CS/flow/DefaultTokenService.java:39-50
//   ClusterFlowChecker.acquireClusterToken  CS/flow/ClusterFlowChecker.java:55-112
//   ClusterMetric (getSum/getAvg/tryOccupyNext/canOccupy)  CS/flow/statistic/metric/ClusterMetric.java:39-98
//   ClusterMetricLeapArray (reset + occupy transfer, valid head)  CS/flow/statistic/metric/ClusterMetricLeapArray.java:43-92
//   LeapArray.currentWindow / values / isWindowDeprecated  CORE/slots/statistic/base/LeapArray.java:121-222,294-373
//   SimpleClusterFlowChecker (Envoy RLS)   RLS/flow/SimpleClusterFlowChecker.java:33-65
//
// Batch algorithm (requests decided as if issued one by one in array order):
//   1 classify  : validate, flowId -> slot (open addressing), sort key = slot
//   2 sort      : stable LSD radix sort by slot (arrival order kept per rule)
//   3 runs      : segment the sorted batch into runs = maximal (slot, window
//                 bucket) groups; 3-phase segmented scan gives per-event run id
//                 and prioritized-prefix counts, per-run extents/min/max acquire
//   4 flows     : one lane per rule walks that rule's runs in time order.  For
//                 a run of equal acquire counts the pass prefix and the number
//                 of occupied (SHOULD_WAIT) requests are found by binary search
//                 over the exact Java double predicates (both are monotone in
//                 the position); other runs are replayed request by request.
//   5 results   : every event derives its TokenResult from its run record.
#include "cluster.hpp"
#include "cluster_exact.hpp"
#include "cparam_exact.hpp"

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <type_traits>

namespace sga {

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTileElems = kThreads * kItems;  // 4096

enum : uint8_t { RUN_FAST = 0, RUN_DONE = 1 };

__device__ __forceinline__ uint64_t lanemask_lt64(int lane) { return (1ULL << lane) - 1ULL; }

__device__ __forceinline__ HashEntry slot_lookup(const ClusterState &st, int64_t fid) {
    uint32_t h = (uint32_t)hash_flow_id(fid) & st.hmask;
    for (uint32_t probe = 0; probe <= st.hmask; ++probe) {
        const HashEntry e = st.htab[h];
        if (e.key == fid || e.key == 0) return e;
        h = (h + 1) & st.hmask;
    }
    return HashEntry{0, 0, 0};
}

// ---------------------------------------------------------------- packed sort element
// One u64 per request carries everything after classify needs, so the sort and the scans move
// 8 bytes per request:
//   [63:40] rule slot (invalid requests: nslots, sorted last)
//   [39:34] window-bucket delta  t / W - ts_base / W   (63 = escape: does not fit)
//   [33]    prioritized
//   [32:26] acquire count 1..127 (0 = escape: not representable, or the bucket escaped)
//   [25:0]  request index (max_batch <= 2^26)
// An escaped request forces its run onto the exact per-request replay, which re-reads the
// original arrays; run boundaries are (slot, bucket delta) changes, exact whenever no escape.
constexpr int kIdxBits = 26;
constexpr int kAcqShift = 26, kPrioShift = 33, kBdShift = 34, kSlotShift = 40;
constexpr uint32_t kAcqMax = 127, kBdEsc = 63;

__device__ __forceinline__ uint64_t el_pack(uint32_t slot, uint32_t bd, uint32_t prio, uint32_t acq7, uint32_t idx) {
    return ((uint64_t)slot << kSlotShift) | ((uint64_t)bd << kBdShift) | ((uint64_t)prio << kPrioShift) |
           ((uint64_t)acq7 << kAcqShift) | (uint64_t)idx;
}
__device__ __forceinline__ uint32_t el_slot(uint64_t e) { return (uint32_t)(e >> kSlotShift); }
__device__ __forceinline__ uint32_t el_runkey(uint64_t e) { return (uint32_t)(e >> kBdShift); }  // slot | bucket
__device__ __forceinline__ uint32_t el_prio(uint64_t e) { return (uint32_t)(e >> kPrioShift) & 1u; }
__device__ __forceinline__ int32_t el_acq(uint64_t e) { return (int32_t)((e >> kAcqShift) & kAcqMax); }
__device__ __forceinline__ uint32_t el_idx(uint64_t e) { return (uint32_t)e & ((1u << kIdxBits) - 1); }

// floor(a / b) for 0 <= a, 0 < b through one double division and an exact correction
// (a < 2^53); the int64 division sequence costs many more registers and cycles.
__device__ __forceinline__ int64_t div_pos(int64_t a, int64_t b) {
    if (a >= ((int64_t)1 << 53)) return a / b;
    int64_t q = (int64_t)((double)a / (double)b);
    const int64_t r = a - q * b;
    if (r < 0) --q;
    else if (r >= b) ++q;
    return q;
}

// ---------------------------------------------------------------- classify
// One workgroup per sort tile (4096 requests, kItems per thread strided by the block size so every
// load is coalesced).  Validation (DefaultTokenService.notValidRequest, :87-89) and
// ClusterFlowRuleManager.getFlowRuleById (open addressing) write BAD_REQUEST / NO_RULE_EXISTS
// results directly.  The tile's histogram of the first radix digit is produced here (hist_d > 0).
template <int kClsChunk>  // table lookups in flight per thread
__global__ __launch_bounds__(kThreads) void k_classify(ClusterState st, const int64_t *__restrict__ flow_id,
                                                       const int32_t *__restrict__ acquire,
                                                       const uint8_t *__restrict__ prio,
                                                       const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                       uint32_t n, int simple, uint32_t invalid_key,
                                                       uint64_t *__restrict__ el, uint64_t *__restrict__ out,
                                                       int hist_d, uint32_t ntiles, uint32_t *__restrict__ hist,
                                                       int lb_npass, uint32_t *__restrict__ ghist) {
    // hist_d > 0: this tile's histogram of the first digit (hist + scan sorts);
    // lb_npass > 0: the global totals of every digit (look-back sorts)
    __shared__ uint32_t h[1024];
    const uint32_t nh = lb_npass > 0 ? (uint32_t)lb_npass << hist_d : (hist_d > 0 ? 1u << hist_d : 0u);
    if (nh) {
        for (uint32_t d = threadIdx.x; d < nh; d += kThreads) h[d] = 0;
        __syncthreads();
    }
    const uint32_t tbase = blockIdx.x * kTileElems;
    // software pipeline: chunk c + 1's request fields load while chunk c's lookups resolve
    int64_t fid[kClsChunk], nfid[kClsChunk];
    int32_t acq[kClsChunk], nacq[kClsChunk];
    uint32_t tso[kClsChunk], pr[kClsChunk], ntso[kClsChunk], npr[kClsChunk];
    auto load_chunk = [&](int c, int64_t (&f)[kClsChunk], int32_t (&a)[kClsChunk], uint32_t (&t)[kClsChunk],
                          uint32_t (&p)[kClsChunk]) {
#pragma unroll
        for (int u = 0; u < kClsChunk; ++u) {
            const uint32_t i = tbase + (c + u) * kThreads + threadIdx.x;
            f[u] = i < n ? flow_id[i] : 0;
            a[u] = i < n ? acquire[i] : 0;
            t[u] = i < n ? ts_off[i] : 0;
            p[u] = (i < n && !simple && prio) ? prio[i] : 0;
        }
    };
    constexpr bool pipelined = true;
    if (pipelined) load_chunk(0, fid, acq, tso, pr);
    for (int c = 0; c < kItems; c += kClsChunk) {
        uint32_t hh[kClsChunk];
        HashEntry e[kClsChunk];
        if (!pipelined) load_chunk(c, fid, acq, tso, pr);
        if (st.dense_n) {  // dense flowIds: one 4-byte load, no probe sequence
            uint32_t d[kClsChunk];
#pragma unroll
            for (int u = 0; u < kClsChunk; ++u)
                d[u] = (fid[u] >= 1 && fid[u] <= (int64_t)st.dense_n) ? (uint32_t)st.dense[fid[u] - 1] : ~0u;
#pragma unroll
            for (int u = 0; u < kClsChunk; ++u) {
                hh[u] = 0;
                e[u] = d[u] == ~0u ? HashEntry{-1, 0, 0} : HashEntry{fid[u], d[u] & 0xFFFFFFu, st.wtab[d[u] >> 24]};
            }
        } else {
#pragma unroll
            for (int u = 0; u < kClsChunk; ++u) {
                hh[u] = (uint32_t)hash_flow_id(fid[u]) & st.hmask;
                e[u] = fid[u] > 0 ? st.htab[hh[u]] : HashEntry{0, 0, 0};
            }
        }
        if (pipelined && c + kClsChunk < kItems) load_chunk(c + kClsChunk, nfid, nacq, ntso, npr);
#pragma unroll
        for (int u = 0; u < kClsChunk; ++u) {
            const uint32_t i = tbase + (c + u) * kThreads + threadIdx.x;
            const bool valid = i < n;
            uint32_t key = invalid_key;
            if (valid) {
            const int64_t f = fid[u];
            const int32_t a = acq[u];
            int8_t status = TRS_OK;
            HashEntry he = e[u];
            if (!simple && (f <= 0 || a <= 0)) {
                status = TRS_BAD_REQUEST;
            } else {
                if (!st.dense_n && f > 0 && he.key != f && he.key != 0) {  // continue the linear probe
                    uint32_t q = hh[u];
                    for (uint32_t probe = 1; probe <= st.hmask; ++probe) {
                        q = (q + 1) & st.hmask;
                        he = st.htab[q];
                        if (he.key == f || he.key == 0) break;
                    }
                }
                if (he.key != f || f <= 0) status = TRS_NO_RULE_EXISTS;
            }
            if (status != TRS_OK) {
                out[i] = pack_result(status, 0, 0);
                el[i] = (uint64_t)invalid_key << kSlotShift;
            } else {
                key = he.slot;
                const uint32_t p = pr[u] ? 1u : 0u;
                const int64_t W = (int64_t)he.W;
                const int64_t bd = div_pos(ts_base + (int64_t)tso[u], W) - div_pos(ts_base, W);
                uint32_t a7 = (a >= 1 && a <= (int32_t)kAcqMax) ? (uint32_t)a : 0u;
                uint32_t bd6 = (uint32_t)bd;
                if (bd >= (int64_t)kBdEsc) {
                    bd6 = kBdEsc;
                    a7 = 0;
                }
                el[i] = el_pack(key, bd6, p, a7, i);
            }
            }
            if (lb_npass > 0) {
                if (valid)
                    for (int p = 0; p < lb_npass; ++p)
                        atomicAdd(&h[((uint32_t)p << hist_d) + ((key >> (p * hist_d)) & ((1u << hist_d) - 1))], 1u);
            } else if (hist_d > 0 && valid) {
                atomicAdd(&h[key & ((1u << hist_d) - 1)], 1u);
            }
        }
        if (pipelined) {
#pragma unroll
            for (int u = 0; u < kClsChunk; ++u) {
                fid[u] = nfid[u];
                acq[u] = nacq[u];
                tso[u] = ntso[u];
                pr[u] = npr[u];
            }
        }
    }
    if (nh) {
        __syncthreads();
        if (lb_npass > 0) {
            for (uint32_t i = threadIdx.x; i < nh; i += kThreads)
                if (h[i]) atomicAdd(&ghist[i], h[i]);
        } else {
            for (uint32_t d = threadIdx.x; d < nh; d += kThreads) hist[(size_t)d * ntiles + blockIdx.x] = h[d];
        }
    }
}

// ---------------------------------------------------------------- runs (segmented scan)
// A run = maximal group of sorted requests with the same (rule, window bucket).
// Scan value: run / flow heads and prioritized requests (plain counts); since the last run
// head: prioritized count and min / max acquire (segmented).
struct Agg {
    uint32_t nh, nf, np;  // run heads, flow heads, prioritized (all since the batch start)
    uint32_t flag;        // run head seen
    uint32_t cnt;         // prioritized since the last run head
    int32_t mn, mx;       // min / max acquire since the last run head
};

__device__ __forceinline__ Agg agg_identity() { return Agg{0, 0, 0, 0, 0, INT32_MAX, INT32_MIN}; }

__device__ __forceinline__ Agg agg_combine(const Agg &a, const Agg &b) {
    Agg r;
    r.nh = a.nh + b.nh;
    r.nf = a.nf + b.nf;
    r.np = a.np + b.np;
    r.flag = a.flag | b.flag;
    r.cnt = b.flag ? b.cnt : a.cnt + b.cnt;
    r.mn = b.flag ? b.mn : min(a.mn, b.mn);
    r.mx = b.flag ? b.mx : max(a.mx, b.mx);
    return r;
}

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
__device__ __forceinline__ uint32_t shfl_up_u32(uint32_t v, int o) { return (uint32_t)__shfl_up((int)v, o, 64); }

__device__ __forceinline__ Agg agg_shfl_up(const Agg &v, int o) {
    return Agg{shfl_up_u32(v.nh, o), shfl_up_u32(v.nf, o), shfl_up_u32(v.np, o), shfl_up_u32(v.flag, o),
               shfl_up_u32(v.cnt, o), __shfl_up(v.mn, o, 64), __shfl_up(v.mx, o, 64)};
}

__device__ __forceinline__ Agg agg_shfl(const Agg &v, int src) {
    return Agg{shfl_u32(v.nh, src), shfl_u32(v.nf, src), shfl_u32(v.np, src), shfl_u32(v.flag, src),
               shfl_u32(v.cnt, src), __shfl(v.mn, src, 64), __shfl(v.mx, src, 64)};
}

// inclusive scan over the 64 lanes of a wave (lane order = element order)
__device__ __forceinline__ Agg wave_incl_scan(Agg x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Agg y = agg_shfl_up(x, o);
        if (lane >= o) x = agg_combine(y, x);
    }
    return x;
}

// ordered reduction of the 64 lanes (result valid in every lane)
__device__ __forceinline__ Agg wave_reduce(Agg v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Agg y = agg_shfl(v, (lane + o) & 63);
        if (lane + o < 64 && (lane & (2 * o - 1)) == 0) v = agg_combine(v, y);
    }
    return agg_shfl(v, 0);
}

// Results-side scan value (a projection of Agg): run heads, prioritized since the run head,
// elements since the run head.
__device__ __forceinline__ RAgg ragg_combine(const RAgg &a, const RAgg &b) {
    return RAgg{a.nh + b.nh, a.flag | b.flag, b.flag ? b.cnt : a.cnt + b.cnt};
}

// Blocked arrangement: a 512-thread workgroup per 4096-request tile, each thread folds 8
// consecutive elements serially; only per-thread aggregates cross lanes (one wave scan per 512
// requests instead of one per 64).
constexpr int kRunThreads = 512;
constexpr int kPerThread = 8;
constexpr int kRunWaves = kRunThreads / 64;         // 8
constexpr int kWaveElems = 64 * kPerThread;         // 512 consecutive requests per wave
static_assert(kWaveElems * kRunWaves == kTileElems, "tile geometry");

__device__ __forceinline__ uint64_t el_load(const uint64_t *el, uint32_t e, uint32_t nlim, uint32_t invalid_key) {
    return e < nlim ? el[e] : ((uint64_t)invalid_key << kSlotShift);
}

__device__ __forceinline__ void el_load_blk(const uint64_t *el, uint32_t e0, uint32_t nlim, uint32_t invalid_key,
                                            uint64_t (&x)[kPerThread]) {
    if (e0 + kPerThread <= nlim) {
        const ulonglong2 *v = reinterpret_cast<const ulonglong2 *>(el + e0);
#pragma unroll
        for (int k = 0; k < kPerThread / 2; ++k) {
            const ulonglong2 t = v[k];
            x[2 * k] = t.x;
            x[2 * k + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kPerThread; ++k) x[k] = el_load(el, e0 + k, nlim, invalid_key);
    }
}

// Agg contribution of element x with predecessor px (has_prev = x is not element 0)
__device__ __forceinline__ Agg run_value(uint64_t x, uint64_t px, bool has_prev, bool valid) {
    if (!valid) return agg_identity();
    const bool fh = !has_prev || el_slot(x) != el_slot(px);
    const bool h = !has_prev || el_runkey(x) != el_runkey(px);
    const int32_t a = el_acq(x);
    const uint32_t p = el_prio(x);
    return Agg{h ? 1u : 0u, fh ? 1u : 0u, p, h ? 1u : 0u, p, a, a};
}

// Per tile: aggregate over its valid elements + count of valid elements.
__global__ __launch_bounds__(kRunThreads) void k_runs_up(const uint64_t *__restrict__ el, uint32_t n,
                                                      uint32_t invalid_key, Agg *__restrict__ tile_agg,
                                                      uint32_t *__restrict__ tile_valid,
                                                      const uint32_t *__restrict__ dn) {
    __shared__ Agg wagg[kRunWaves];
    __shared__ uint32_t wval[kRunWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (dn) n = min(n, *dn);  // hot path: the sorted cold elements come first, then prioritized hot ones
    if (dn && blockIdx.x * (uint32_t)kTileElems >= n) return;  // past the live tiles (k_runs_tiles stops there)
    const uint32_t e0 = blockIdx.x * kTileElems + threadIdx.x * kPerThread;
    uint64_t x[kPerThread];
    el_load_blk(el, e0, n, invalid_key, x);
    uint64_t px = el_load(el, e0 - 1, e0 > 0 ? min(e0, n) : 0, invalid_key);
    Agg acc = agg_identity();
    uint32_t nval = 0;
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
        const bool valid = el_slot(x[k]) != invalid_key;
        acc = agg_combine(acc, run_value(x[k], px, e0 + k > 0, valid));
        nval += valid ? 1u : 0u;
        px = x[k];
    }
    acc = wave_reduce(acc, lane);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nval += (uint32_t)__shfl_down((int)nval, o, 64);
    if (lane == 0) {
        wagg[wave] = acc;
        wval[wave] = nval;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        Agg t = agg_identity();
        uint32_t c = 0;
        for (int w = 0; w < kRunWaves; ++w) {
            t = agg_combine(t, wagg[w]);
            c += wval[w];
        }
        tile_agg[blockIdx.x] = t;
        tile_valid[blockIdx.x] = c;
    }
}

constexpr int kTileScanThreads = 1024;

// exclusive scan of one Agg per thread over a 1024-thread workgroup
__device__ Agg block_excl_scan_1024(const Agg &v, Agg *total) {
    constexpr int NW = kTileScanThreads / 64;
    __shared__ Agg wtot[NW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const Agg x = wave_incl_scan(v, lane);
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    Agg wpre = agg_identity();
    for (int w = 0; w < wave; ++w) wpre = agg_combine(wpre, wtot[w]);
    Agg lane_excl = agg_shfl_up(x, 1);
    if (lane == 0) lane_excl = agg_identity();
    Agg t = agg_identity();
    for (int w = 0; w < NW; ++w) t = agg_combine(t, wtot[w]);
    *total = t;
    __syncthreads();
    return agg_combine(wpre, lane_excl);
}

// Single workgroup: tile carries, nvalid / nruns / nflows.  Blocked: each thread folds a run of
// consecutive tiles serially, one block scan over the per-thread aggregates.
__global__ __launch_bounds__(kTileScanThreads) void k_runs_tiles(const Agg *__restrict__ tile_agg,
                                                                 const uint32_t *__restrict__ tile_valid,
                                                                 uint32_t ntiles, Agg *__restrict__ tile_carry,
                                                                 uint32_t *__restrict__ counters,
                                                                 const uint32_t *__restrict__ dn) {
    __shared__ uint32_t ws[kTileScanThreads / 64];
    if (dn) ntiles = min(ntiles, (*dn + kTileElems - 1) / kTileElems);  // live tiles only
    const uint32_t per = (ntiles + kTileScanThreads - 1) / kTileScanThreads;
    const uint32_t t0 = threadIdx.x * per, t1 = min(ntiles, t0 + per);
    Agg acc = agg_identity();
    uint32_t c = 0;
    for (uint32_t t = t0; t < t1; ++t) {
        acc = agg_combine(acc, tile_agg[t]);
        c += tile_valid[t];
    }
    Agg total;
    Agg run = block_excl_scan_1024(acc, &total);
    for (uint32_t t = t0; t < t1; ++t) {
        tile_carry[t] = run;
        run = agg_combine(run, tile_agg[t]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_down((int)c, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t nvalid = 0;
        for (int w = 0; w < kTileScanThreads / 64; ++w) nvalid += ws[w];
        counters[0] = nvalid;
        counters[1] = total.nh;
        counters[2] = total.nf;
    }
}

// Per tile: run and flow records, the list of prioritized positions, and each wave's carry
// (for k_results, which re-derives run ids and prioritized ranks instead of reading them).
__global__ __launch_bounds__(kRunThreads) void k_runs_down(const uint64_t *__restrict__ el, uint32_t invalid_key,
                                                        const Agg *__restrict__ tile_carry, BatchScratch sc) {
    __shared__ Agg wagg[kRunWaves];
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t e0 = base + threadIdx.x * kPerThread;
    uint64_t x[kPerThread];
    el_load_blk(el, e0, nvalid, invalid_key, x);
    const uint64_t first_prev = el_load(el, e0 - 1, e0 > 0 ? min(e0, nvalid) : 0, invalid_key);
    const uint64_t after = el_load(el, e0 + kPerThread, nvalid, invalid_key);
    Agg acc = agg_identity();
    {
        uint64_t px = first_prev;
#pragma unroll
        for (int k = 0; k < kPerThread; ++k) {
            acc = agg_combine(acc, run_value(x[k], px, e0 + k > 0, e0 + k < nvalid));
            px = x[k];
        }
    }
    const Agg incl = wave_incl_scan(acc, lane);
    Agg excl = agg_shfl_up(incl, 1);
    if (lane == 0) excl = agg_identity();
    if (lane == 63) wagg[wave] = incl;
    __syncthreads();
    Agg carry = tile_carry[blockIdx.x];
    for (int w = 0; w < wave; ++w) carry = agg_combine(carry, wagg[w]);
    // results-side carry at the wave's first request
    if (lane == 0) sc.wave_carry[blockIdx.x * kRunWaves + wave] = RAgg{carry.nh, carry.flag, carry.cnt};
    Agg run = agg_combine(carry, excl);
    uint64_t px = first_prev;
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
        const uint32_t e = e0 + k;
        if (e >= nvalid) break;
        const uint64_t cur = x[k];
        run = agg_combine(run, run_value(cur, px, e > 0, true));
        const uint32_t rid = run.nh - 1;
        const uint32_t p = el_prio(cur);
        const bool fh = e == 0 || el_slot(cur) != el_slot(px);
        const bool h = e == 0 || el_runkey(cur) != el_runkey(px);
        if (h) {
            const uint32_t bd = (uint32_t)((cur >> kBdShift) & kBdEsc);
            sc.run_start[rid] = e;
            sc.run_slot[rid] = el_slot(cur);
            sc.run_idx0[rid] = el_idx(cur);
            sc.run_bd[rid] = (uint8_t)bd;
            sc.run_p0[rid] = run.np - p;
        }
        if (fh) sc.flow_first_run[run.nf - 1] = rid;
        if (p) sc.plist[run.np - 1] = e;
        const uint64_t nx = k + 1 < kPerThread ? x[k + 1 < kPerThread ? k + 1 : k] : after;
        if (e + 1 >= nvalid || el_runkey(nx) != el_runkey(cur)) {
            sc.run_cp[rid] = run.cnt;
            sc.run_acq[rid] = (run.mn == run.mx) ? run.mn : 0;  // 0: mixed or escaped -> replay
        }
        px = cur;
    }
}

// ---------------------------------------------------------------- flows: resolve runs per rule
// x / intervalInSec, exact: the default 1 s window has intervalInSec = 1.0 and x / 1.0 == x, so a wave whose lanes
// all divide by 1.0 skips the double division (a uniform branch on a ballot; ~10 VALU per division otherwise)
__device__ __forceinline__ double div_isec(double x, double isec) {
    if (__all(isec == 1.0)) return x;
    return x / isec;
}

__device__ __forceinline__ bool pass_cond(double thr, double isec, int64_t sum, int32_t a) {
    // nextRemaining = globalThreshold - latestQps - acquireCount >= 0   ClusterFlowChecker.java:67-71
    return thr - div_isec((double)sum, isec) - (double)a >= 0;
}

// First k in [0, n] with !pass_cond(s0 + k*a): a closed-form guess corrected against the
// exact predicate (monotone in k), so the result equals the sequential one.
__device__ __forceinline__ uint32_t pass_prefix(double thr, double isec, int64_t s0, int32_t a, uint32_t n) {
    if (n == 0) return 0;
    if (a <= 0) return pass_cond(thr, isec, s0, a) ? n : 0u;
    // the guess only seeds the exact search below: an approximate reciprocal of a does
    const double g = floor(((thr - (double)a) * isec - (double)s0) * __builtin_amdgcn_rcp((double)a)) + 1.0;
    uint32_t k = 0;
    if (g >= (double)n) k = n;
    else if (g > 0) k = (uint32_t)g;
#pragma nounroll
    while (k > 0 && !pass_cond(thr, isec, s0 + (int64_t)(k - 1) * a, a)) --k;
#pragma nounroll
    while (k < n && pass_cond(thr, isec, s0 + (int64_t)k * a, a)) ++k;
    return k;
}

__device__ __forceinline__ int64_t i64_lo(const int4 &v) {
    return (int64_t)(((uint64_t)(uint32_t)v.y << 32) | (uint32_t)v.x);
}
__device__ __forceinline__ int64_t i64_hi(const int4 &v) {
    return (int64_t)(((uint64_t)(uint32_t)v.w << 32) | (uint32_t)v.z);
}

// Closed form for one run of equal acquire counts (no escape) without clock regression: the
// window is rotated once in registers (LeapArray.currentWindow incl. the occupy transfer of
// ClusterMetricLeapArray.resetWindowTo), the valid buckets summed, the pass prefix and the
// occupied (SHOULD_WAIT) count found over the exact Java predicates, and the current bucket's
// seven counters stored once.  Returns false (nothing touched) when the run is not eligible.

struct RunIn {
    uint32_t j0, n, cp_tot, p0;
    int32_t a;
    uint32_t bd;  // bucket delta of the run (its bucket = ts_base / W + bd)
};

// A rule's record between its runs (cold flows): the record header as the lane's last run left it
// -- the (start, PASS) pairs, the occupy state, the cached counter group with its tag and the
// threshold -- so the rule's later runs issue no record loads (one memory round trip per rule
// instead of one per run).  have = false: load from the record.
#ifndef SGA_CARRY_PAIRS
#define SGA_CARRY_PAIRS 0
#endif
// 1: later runs of a rule take the pairs from registers (64 more VGPRs live across runs: two waves per
// SIMD); 0: they reload the header (an L2 hit: the lane just wrote it), and the kernel fits three
constexpr bool kCarryPairs = SGA_CARRY_PAIRS;
template <int kMaxPairs>
struct RecCarry {
    int4 sp[kMaxPairs > 0 ? kMaxPairs : 1];
    int4 o0, o1;
    int4 cg[3];  // cached group: (WAITING, BLOCK), (PASS_REQUEST, BLOCK_REQUEST), (OCCUPIED_PASS, OCCUPIED_BLOCK)
    int4 meta;   // (tag, threshold)
    bool have;
};

__device__ __forceinline__ double f64_hi(const int4 &v) { return __longlong_as_double(i64_hi(v)); }

// prio_before(k): prioritized requests among the run's first k (asked only when some prioritized
// request is past the passing prefix).  kMaxPairs = 0: sampleCount above the register form, the
// pairs are loaded one by one every run.  hdr_thr: the threshold is the record's copy (Rec::thr),
// not thr_in (which the caller then did not load).
#ifndef SGA_SKIP_GROUP
#define SGA_SKIP_GROUP 0
#endif
constexpr bool kSkipGroup = SGA_SKIP_GROUP;  // profiling builds only (the array group then goes stale)
#ifndef SGA_HDR_CACHE_ALL
#define SGA_HDR_CACHE_ALL 0
#endif
constexpr bool kHdrCacheAll = SGA_HDR_CACHE_ALL;  // 1: every cold run rewrites the header's counter cache
template <class PrioBefore, int kMaxPairs>
__device__ __forceinline__ bool run_fast(const ClusterState &st, const SlotParam &P, const Rec &R, double thr_in,
                                         bool hdr_thr, int64_t qbase, const RunIn &ri, PrioBefore prio_before,
                                         RunOut &ro, RecCarry<kMaxPairs> &rc) {
    // Cluster rules have intervalInMs = sampleCount x windowLengthInMs (checkClusterField), so every
    // validity test below (isWindowDeprecated, getValidHead) gives the same answer for any time in
    // the run's bucket: the bucket start stands in for the first request's time.
    const int32_t a = ri.a;
    const int64_t q = qbase + ri.bd;  // bucket number
    const int64_t ws = q * P.W;
    const int64_t t0 = ws;
    const int64_t qs = div_pos(q, P.S);
    const int cj = (int)(q - qs * P.S);
    const int jh = cj + 1 == P.S ? 0 : cj + 1;  // LeapArray.getValidHead index ((t0 + W) / W) % S
    // First run of a rule: the header's loads are issued before any is used (one memory latency, not
    // one per dependent step), at clamped indices (a load under a branch is waited for before the
    // branch closes, which would serialise them): the (start, PASS) pair of every bucket, the occupy
    // state, the cached counter group and (tag, threshold) -- for S = 10 exactly the header's two
    // 128-byte lines.  Later runs take them from registers.
    const int4 *v = reinterpret_cast<const int4 *>(R.r);
    const int4 *hv = reinterpret_cast<const int4 *>(R.cache());
    if (!rc.have) {
        const int4 *ov = reinterpret_cast<const int4 *>(&R.occ());
        rc.o0 = ov[0];
        rc.o1 = ov[1];
        rc.cg[0] = hv[0];
        rc.cg[1] = hv[1];
        rc.cg[2] = hv[2];
        rc.meta = hv[3];
        if constexpr (kMaxPairs > 0) {
#pragma unroll
            for (int jj = 0; jj < kMaxPairs; ++jj) rc.sp[jj] = v[min(jj, P.S - 1)];
        }
    }
    const double thr = hdr_thr ? f64_hi(rc.meta) : thr_in;
    SlotOcc occ_ld;
    occ_ld.occ_pass = i64_lo(rc.o0);
    occ_ld.occ_preq = i64_hi(rc.o0);
    occ_ld.has_occ = rc.o1.x;
    occ_ld.pad = rc.o1.y;
    int4 cur;  // the current bucket's pair
    int64_t bp = 0, hstart = kAbsent, hpass = 0;
    {
        auto take = [&](int jj, const int4 &sp) {
            const int64_t w = i64_lo(sp), pv = i64_hi(sp);
            if (jj == jh) {
                hstart = w;
                hpass = pv;
            }
            if (jj != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval)) bp += pv;
        };
        if constexpr (kMaxPairs > 0) {
            cur = rc.sp[0];
#pragma unroll
            for (int jj = 1; jj < kMaxPairs; ++jj)
                if (jj == cj) cur = rc.sp[jj];
#pragma unroll
            for (int jj = 0; jj < kMaxPairs; ++jj)
                if (jj < P.S) take(jj, rc.sp[jj]);
        } else {
            cur = v[cj];
            for (int jj = 0; jj < P.S; ++jj) take(jj, v[jj]);
        }
    }
    const int64_t old = i64_lo(cur);
    if (a <= 0 || (old != kAbsent && ws < old)) return false;
    if (ri.cp_tot > 0 && (P.S <= 1 || 1000 / P.S <= 0)) return false;
    const bool rot = old == kAbsent || ws > old;
    int4 c01 = rc.cg[0], c23 = rc.cg[1], c45 = rc.cg[2];
    const bool tag_was_cur = i64_lo(rc.meta) == old;
    if (!rot && !tag_was_cur) {  // the current bucket's counters are not the cached group: the array
        const int4 *cv = reinterpret_cast<const int4 *>(R.group(cj));
        c01 = cv[0];
        c23 = cv[1];
        c45 = cv[2];
    }
    int64_t c[CEV_N];
    SlotOcc o{0, 0, 0, 0};
    bool occ_loaded = false, occ_dirty = false;
    if (rot) {
#pragma unroll
        for (int k = 0; k < CEV_N; ++k) c[k] = 0;
        if (old != kAbsent) {  // resetWindowTo + transferOccupyToBucket
            o = occ_ld;
            occ_loaded = true;
            if (o.has_occ) {
                c[CEV_OCCUPIED_PASS] += o.occ_pass;
                c[CEV_PASS] += o.occ_pass;
                c[CEV_PASS_REQUEST] += o.occ_preq;
                o.occ_pass = 0;
                o.occ_preq = 0;
                o.has_occ = 0;
                occ_dirty = true;
            }
        }
    } else {
        c[CEV_PASS] = i64_hi(cur);
        c[CEV_WAITING] = i64_lo(c01);
        c[CEV_BLOCK] = i64_hi(c01);
        c[CEV_PASS_REQUEST] = i64_lo(c23);
        c[CEV_BLOCK_REQUEST] = i64_hi(c23);
        c[CEV_OCCUPIED_PASS] = i64_lo(c45);
        c[CEV_OCCUPIED_BLOCK] = i64_hi(c45);
    }
    int64_t head;  // getValidHead after the rotation (the head is the current bucket when S == 1)
    if (jh == cj) head = c[CEV_PASS];
    else head = (hstart != kAbsent && !(t0 - hstart > (int64_t)P.interval)) ? hpass : 0;
    const int64_t s0 = bp + c[CEV_PASS];
    const uint32_t n = ri.n;
    const uint32_t f = pass_prefix(thr, P.isec, s0, a, n);
    // prioritized requests among the first f: the run's prioritized positions are
    // plist[p0 .. p0 + cp_tot) (ascending)
    uint32_t cpf = ri.cp_tot;
    if (f < n && ri.cp_tot > 0) cpf = prio_before(f);
    const uint32_t np_after = ri.cp_tot - cpf;
    uint32_t cw = 0;
    if (np_after > 0) {
        // WAITING over the same valid buckets (only runs with prioritized blocked requests read it;
        // validity is re-tested per bucket, so any sampleCount works)
        int64_t w0 = c[CEV_WAITING];
        if constexpr (kMaxPairs > 0) {
            // the S WAITING counters loaded together at clamped indices (one memory latency; a load per
            // bucket behind its validity test waited S latencies, and about every wave has a lane here),
            // validity from the pairs in registers
            int64_t wv[kMaxPairs];
#pragma unroll
            for (int jj = 0; jj < kMaxPairs; ++jj) wv[jj] = R.group(min(jj, P.S - 1))[0];
#pragma unroll
            for (int jj = 0; jj < kMaxPairs; ++jj) {
                const int64_t w = i64_lo(rc.sp[jj]);
                if (jj < P.S && jj != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval)) w0 += wv[jj];
            }
        } else {
#pragma nounroll
            for (int jj = 0; jj < P.S; ++jj) {
                const int64_t w = R.start(jj);
                if (jj != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval)) w0 += R.cnt(CEV_WAITING, jj);
            }
        }
        if (!occ_loaded) o = occ_ld;
        const double latest = div_isec((double)(s0 + (int64_t)f * a), P.isec);
        const double lim = st.max_occupy_ratio * thr;
        const int64_t occ0 = o.occ_pass;
        uint32_t l2 = 0, h2 = np_after;
#pragma nounroll
        while (l2 < h2) {
            const uint32_t cc = l2 + ((h2 - l2) >> 1);
            const int64_t add = (int64_t)cc * a;
            const bool ok = (div_isec((double)(w0 + add), P.isec) <= lim) &&
                            (latest + (double)((int64_t)a + occ0 + add) - (double)head <= thr);
            if (ok) l2 = cc + 1;
            else h2 = cc;
        }
        cw = l2;
        if (cw > 0) {
            o.occ_pass += (int64_t)cw * a;
            o.occ_preq += cw;
            o.has_occ = 1;
            occ_dirty = true;
        }
    }
    const uint32_t nblk = n - f - cw;
    c[CEV_PASS] += (int64_t)f * a;
    c[CEV_PASS_REQUEST] += f;
    c[CEV_OCCUPIED_PASS] += (int64_t)cpf * a;
    c[CEV_WAITING] += (int64_t)cw * a;
    c[CEV_BLOCK] += (int64_t)nblk * a;
    c[CEV_BLOCK_REQUEST] += nblk;
    c[CEV_OCCUPIED_BLOCK] += (int64_t)(np_after - cw) * a;
    // 16-byte stores: the (start, PASS) pair, the six other counters (one 48-byte group), the occupy state
    {
        const int64_t stv = rot ? ws : old;
        auto i4 = [](int64_t lo, int64_t hi) {
            return make_int4((int)(uint32_t)lo, (int)(uint32_t)((uint64_t)lo >> 32), (int)(uint32_t)hi,
                             (int)(uint32_t)((uint64_t)hi >> 32));
        };
        reinterpret_cast<int4 *>(R.r)[cj] = i4(stv, c[CEV_PASS]);
        rc.cg[0] = i4(c[CEV_WAITING], c[CEV_BLOCK]);
        rc.cg[1] = i4(c[CEV_PASS_REQUEST], c[CEV_BLOCK_REQUEST]);
        rc.cg[2] = i4(c[CEV_OCCUPIED_PASS], c[CEV_OCCUPIED_BLOCK]);
        rc.meta.x = (int)(uint32_t)stv;  // the cache now holds bucket cj (the threshold word is stored back as loaded)
        rc.meta.y = (int)(uint32_t)((uint64_t)stv >> 32);
        int4 *cg = reinterpret_cast<int4 *>(R.group(cj));  // the array (authoritative) and the header's cache
        int4 *ch = reinterpret_cast<int4 *>(R.cache());
        if (!kSkipGroup) {
            cg[0] = rc.cg[0];
            cg[1] = rc.cg[1];
            cg[2] = rc.cg[2];
        }
        // the header's cache: written when it must stay coherent (it already held this bucket) or when it is
        // the policy (kHdrCacheAll); otherwise left alone -- its tag then names another bucket, and the run
        // saves the partial write of the header's second line
        if (kHdrCacheAll || (!rot && tag_was_cur)) {
            ch[0] = rc.cg[0];
            ch[1] = rc.cg[1];
            ch[2] = rc.cg[2];
            ch[3] = rc.meta;
        }
        if (occ_dirty) {
            rc.o0 = i4(o.occ_pass, o.occ_preq);
            rc.o1 = make_int4(o.has_occ, o.pad, rc.o1.z, rc.o1.w);  // the spare word stored back unchanged
            int4 *ov = reinterpret_cast<int4 *>(&R.occ());
            ov[0] = rc.o0;
            ov[1] = rc.o1;
        }
        if constexpr (kMaxPairs > 0) {
            const int4 np = i4(stv, c[CEV_PASS]);
#pragma unroll
            for (int jj = 0; jj < kMaxPairs; ++jj)
                if (jj == cj) rc.sp[jj] = np;
        }
        rc.have = kCarryPairs && kMaxPairs > 0;
    }
    ro.s0 = s0;
    ro.thr = thr;
    ro.isec = P.isec;
    ro.f = f;
    ro.cpf = cpf;
    ro.cw = cw;
    ro.wait = (uint16_t)(1000 / P.S);
    ro.mode = RUN_FAST;
    return true;
}

__global__ __launch_bounds__(kRunThreads) void k_results(BatchScratch sc, const uint64_t *__restrict__ el,
                                                         uint32_t invalid_key, uint64_t *__restrict__ out) {
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (base + wave * kWaveElems >= nvalid) return;
    const uint32_t e0 = base + threadIdx.x * kPerThread;
    uint64_t x[kPerThread];
    el_load_blk(el, e0, nvalid, invalid_key, x);
    const uint64_t first_prev = el_load(el, e0 - 1, e0 > 0 ? min(e0, nvalid) : 0, invalid_key);
    RAgg acc{0, 0, 0};
    {
        uint64_t px = first_prev;
#pragma unroll
        for (int k = 0; k < kPerThread; ++k) {
            const uint32_t e = e0 + k;
            const bool valid = e < nvalid;
            const bool h = valid && (e == 0 || el_runkey(x[k]) != el_runkey(px));
            acc = ragg_combine(acc, RAgg{h ? 1u : 0u, h ? 1u : 0u, valid ? el_prio(x[k]) : 0u});
            px = x[k];
        }
    }
    RAgg v = acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const RAgg y{shfl_up_u32(v.nh, o), shfl_up_u32(v.flag, o), shfl_up_u32(v.cnt, o)};
        if (lane >= o) v = ragg_combine(y, v);
    }
    RAgg excl{shfl_up_u32(v.nh, 1), shfl_up_u32(v.flag, 1), shfl_up_u32(v.cnt, 1)};
    if (lane == 0) excl = RAgg{0, 0, 0};
    RAgg run = ragg_combine(sc.wave_carry[blockIdx.x * kRunWaves + wave], excl);
    // phase 1 (registers only): run id and prioritized-before count of each element
    uint32_t rid[kPerThread], pcb[kPerThread];
    {
        uint64_t px = first_prev;
#pragma unroll
        for (int k = 0; k < kPerThread; ++k) {
            const uint32_t e = e0 + k;
            const bool h = e < nvalid && (e == 0 || el_runkey(x[k]) != el_runkey(px));
            const uint32_t p = e < nvalid ? el_prio(x[k]) : 0u;
            run = ragg_combine(run, RAgg{h ? 1u : 0u, h ? 1u : 0u, p});
            px = x[k];
            rid[k] = run.nh - 1;
            pcb[k] = run.cnt - p;
        }
    }
    // phase 2: the run records of kResIlp elements are loaded together (one load per run change,
    // issued before any is used), then the results are computed and stored
    constexpr int kResIlp = 8;
#pragma unroll
    for (int k0 = 0; k0 < kPerThread; k0 += kResIlp) {
        RunOut ro[kResIlp];
        uint32_t rs[kResIlp];
#pragma unroll
        for (int u = 0; u < kResIlp; ++u) {
            const int k = k0 + u;
            if (e0 + k < nvalid && (u == 0 || rid[k] != rid[k - 1])) {
                ro[u] = sc.run_out[rid[k]];
                rs[u] = sc.run_start[rid[k]];
            } else if (u > 0) {
                ro[u] = ro[u - 1];
                rs[u] = rs[u - 1];
            }
        }
#pragma unroll
        for (int u = 0; u < kResIlp; ++u) {
            const int k = k0 + u;
            const uint32_t e = e0 + k;
            if (e >= nvalid || ro[u].mode != RUN_FAST) continue;
            const uint32_t local = e - rs[u];
            const int32_t a = el_acq(x[k]);
            uint64_t res;
            if (local < ro[u].f) {
                const int64_t sum = ro[u].s0 + (int64_t)local * a;
                res = pack_result(TRS_OK, j_d2i(ro[u].thr - (double)sum / ro[u].isec - (double)a), 0);
            } else if (el_prio(x[k]) && pcb[k] - ro[u].cpf < ro[u].cw) {
                res = pack_result(TRS_SHOULD_WAIT, 0, (int32_t)ro[u].wait);
            } else {
                res = pack_result(TRS_BLOCKED, 0, 0);
            }
            out[el_idx(x[k])] = res;
        }
    }
}

// ---------------------------------------------------------------- fused runs / flows / results
// One workgroup per 2048-element chunk of the sorted elements does what k_runs_* / k_flows /
// k_flows_slow / k_results did in five launches: it owns the rules whose first element lies in its
// chunk (the chunk's leading elements of a rule begun earlier belong to the previous chunk), so a
// rule that runs past the chunk end is followed to its end (region [h0, E)).
//   1 runs    : a blocked segmented scan over the region finds run heads (slot, bucket) and rule
//               heads; each run's length, prioritized count, first prioritized index and common
//               acquire count are written at its head position (run records indexed by position),
//               prioritized positions are compacted into plist[h0 ..), rule heads into LDS.
//   2 flows   : one lane per owned rule walks its runs in time order -- the closed form
//               (run_fast) or the exact per-request replay (request_exact) -- and the rule's
//               request count feeds the next batch's hot-set candidates.
//   3 results : the same scan again; every request reads its run's record and writes its
//               TokenResult (runs replayed in step 2 wrote theirs already).
// Run records live in LDS (runs starting within a chunk's length of h0; the later runs of a rule
// that continues past the chunk use global run arrays), run decisions in global scratch written
// and read by the same workgroup.  Elements with a slot >= nkey (invalid requests, prioritized hot
// requests) end the data.
// kFzChunk: elements per workgroup in chunk mode (and the run records kept in LDS); the runs / results scans
// walk blocks of kFzBlk elements, kFzPer per thread
constexpr int kFzThreads = 256, kFzPer = 4, kFzBlk = kFzThreads * kFzPer, kFzChunk = 2048;
constexpr int kFzShortRun = 4;  // SGA_FZ_DEBUG bit 256 (A/B): the round-4 form -- runs of at most this many
                                // requests answered by their flows lane, every other one by the results scan
constexpr int kFzDirect = 32;   // closed-form runs of at most this many requests: TokenResults from the flows lane
constexpr int kFzLong = 512;    // longer runs listed for the results phase (one wave per run); a full list
                                // sends further runs to their flows lane as well
constexpr uint32_t kFzHuge = 2048;  // listed runs answered by the whole workgroup (no SHOULD_WAIT among them)

// Profiling only (SGA_FZ_DEBUG bit 16): per-phase cycles of k_cold_fused summed over workgroups.
__device__ unsigned long long g_fz_phase[8];
__device__ __forceinline__ void fz_mark(int dbg, int ph, unsigned long long &t) {
    if (!(dbg & 16)) return;
    __syncthreads();
    const unsigned long long now = wall_clock64();
    if (threadIdx.x == 0 && ph > 0) atomicAdd(&g_fz_phase[ph - 1], now - t);
    if (threadIdx.x == 0 && ph == 3) atomicAdd(&g_fz_phase[7], 1ull);
    t = now;
}

struct FAgg {
    uint32_t hpos;  // (run head position + 1) of the last run head so far (0: none)
    uint32_t np;    // prioritized requests so far (region-relative)
    uint32_t hp;    // np before the last run head
    uint32_t flag;  // run head seen
    int32_t mn, mx; // acquire min / max since the last run head
};
__device__ __forceinline__ FAgg fagg_id() { return FAgg{0, 0, 0, 0, INT32_MAX, INT32_MIN}; }
__device__ __forceinline__ FAgg fagg_combine(const FAgg &a, const FAgg &b) {
    FAgg r;
    r.hpos = max(a.hpos, b.hpos);
    r.np = a.np + b.np;
    r.hp = b.flag ? a.np + b.hp : a.hp;
    r.flag = a.flag | b.flag;
    r.mn = b.flag ? b.mn : min(a.mn, b.mn);
    r.mx = b.flag ? b.mx : max(a.mx, b.mx);
    return r;
}
__device__ __forceinline__ FAgg fagg_shfl_up(const FAgg &v, int o) {
    return FAgg{shfl_up_u32(v.hpos, o), shfl_up_u32(v.np, o), shfl_up_u32(v.hp, o), shfl_up_u32(v.flag, o),
                __shfl_up(v.mn, o, 64), __shfl_up(v.mx, o, 64)};
}

// FAgg lane moves on DPP (identity where the source is outside the row / wave)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ FAgg fagg_dpp(const FAgg &v) {
    const FAgg id = fagg_id();
    auto mv = [](uint32_t old, uint32_t x) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, kCtrl, kRowMask, 0xf, false);
    };
    return FAgg{mv(id.hpos, v.hpos), mv(id.np, v.np), mv(id.hp, v.hp), mv(id.flag, v.flag),
                (int32_t)mv((uint32_t)id.mn, (uint32_t)v.mn), (int32_t)mv((uint32_t)id.mx, (uint32_t)v.mx)};
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void fagg_scan_step(FAgg &x) {
    x = fagg_combine(fagg_dpp<kCtrl, kRowMask>(x), x);
}

// Exclusive workgroup scan of one FAgg per thread (thread order = element order).  Returns the
// exclusive prefix; *total gets the workgroup total.  The wave scan is DPP (row shifts, then row
// broadcasts), not LDS shuffles.
__device__ __forceinline__ FAgg fagg_block_excl(const FAgg &v, FAgg *total, FAgg *wtot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    FAgg x = v;
    fagg_scan_step<0x111, 0xf>(x);
    fagg_scan_step<0x112, 0xf>(x);
    fagg_scan_step<0x114, 0xf>(x);
    fagg_scan_step<0x118, 0xf>(x);
    fagg_scan_step<0x142, 0xa>(x);
    fagg_scan_step<0x143, 0xc>(x);
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    FAgg pre = fagg_id(), t = fagg_id();
#pragma unroll
    for (int w = 0; w < kFzThreads / 64; ++w) {
        if (w < wave) pre = fagg_combine(pre, wtot[w]);
        t = fagg_combine(t, wtot[w]);
    }
    const FAgg ex = fagg_dpp<0x138, 0xf>(x);  // wave_shr:1, lane 0 gets the identity
    *total = t;
    __syncthreads();
    return fagg_combine(pre, ex);
}

// Bin mode's ordering (the cold partition): the workgroup's bin [B0, B1) of the partition output, in
// arrival order, sorted stably by the slot bits below the bin (lb <= kPartMaxLow) into es[B0, B1).
// Each wave takes a contiguous quarter; pass 1 counts its digits (ballot match: lanes with equal
// digits, the lowest adds the group), the counts become absolute bases (digit starts + earlier
// waves), pass 2 ranks every element (base + earlier lanes of its digit) and stores it.
__device__ __forceinline__ uint64_t match_lanes(uint32_t d, int bits, bool valid) {
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
    }
    return peers;
}
constexpr int kBinLds = 2560;  // k_cold_fused bin mode: bins of at most this many elements are ordered in LDS
constexpr int kBoRounds = 12;  // bin_order: rounds of 64 elements a wave holds in registers (bins of ~3k in one go)
// The ordered bin goes to es[pos - ebase] (es: the workgroup's LDS image of a bin that fits, ebase = B0, or
// the global element buffer, ebase = 0).
__device__ void bin_order(const uint64_t *__restrict__ in, uint64_t *es, uint32_t ebase, uint32_t B0, uint32_t B1,
                          int lb, uint32_t *pc, uint32_t *wsum) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kW = kFzThreads / 64;
    const uint32_t nd = 1u << lb, dm = nd - 1u;
    const uint64_t lt = lanemask_lt64(lane);
    for (uint32_t k = threadIdx.x; k < kW * nd; k += kFzThreads) pc[k] = 0;
    const uint32_t nb = B1 - B0;
    const uint32_t q = (((nb + kW - 1) / kW) + 63u) & ~63u;
    const uint32_t w0 = min(B1, B0 + (uint32_t)wave * q), w1 = min(B1, w0 + q);
    uint32_t *mine = pc + (uint32_t)wave * nd;
    // the wave's elements, kBoRounds rounds at a time, all loads in flight together (unconditional, at
    // clamped positions); a wave of a bin that fits keeps them for pass 2
    uint64_t x[kBoRounds];
    auto load = [&](uint32_t c0) {
#pragma unroll
        for (int r = 0; r < kBoRounds; ++r) {
            const uint32_t p = c0 + (uint32_t)r * 64 + lane;
            x[r] = in[p < w1 ? p : (w0 < w1 ? w0 : B0)];
        }
    };
    const bool one = w1 - w0 <= (uint32_t)(kBoRounds * 64);
    __syncthreads();
    for (uint32_t c0 = w0; c0 < w1; c0 += kBoRounds * 64) {
        load(c0);
#pragma unroll
        for (int r = 0; r < kBoRounds; ++r) {
            if (c0 + (uint32_t)r * 64 >= w1) break;  // wave-uniform
            const bool valid = c0 + (uint32_t)r * 64 + lane < w1;
            const uint32_t d = el_slot(x[r]) & dm;
            const uint64_t peers = match_lanes(d, lb, valid);
            if (valid && (peers & lt) == 0) mine[d] += (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    // digit totals -> digit starts (block scan over digits, kFzThreads x up to 4 digits), then each
    // wave's base per digit = B0 + digit start + the counts of the earlier waves
    constexpr int kDpt = (1 << kPartMaxLow) / kFzThreads;
    uint32_t tot[kDpt], ts = 0;
#pragma unroll
    for (int k = 0; k < kDpt; ++k) {
        const uint32_t d = threadIdx.x * kDpt + k;
        uint32_t t = 0;
        if (d < nd)
            for (int w = 0; w < kW; ++w) t += pc[w * nd + d];
        tot[k] = t;
        ts += t;
    }
    uint32_t y = ts;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t z = __shfl_up(y, o, 64);
        if (lane >= o) y += z;
    }
    if (lane == 63) wsum[wave] = y;
    __syncthreads();
    uint32_t pre = B0 + y - ts;
    for (int w = 0; w < wave; ++w) pre += wsum[w];
#pragma unroll
    for (int k = 0; k < kDpt; ++k) {
        const uint32_t d = threadIdx.x * kDpt + k;
        if (d < nd) {
            uint32_t run = pre;
            for (int w = 0; w < kW; ++w) {
                const uint32_t c = pc[w * nd + d];
                pc[w * nd + d] = run;
                run += c;
            }
        }
        pre += tot[k];
    }
    __syncthreads();
    for (uint32_t c0 = w0; c0 < w1; c0 += kBoRounds * 64) {
        if (!one) load(c0);
#pragma unroll
        for (int r = 0; r < kBoRounds; ++r) {
            if (c0 + (uint32_t)r * 64 >= w1) break;
            const bool valid = c0 + (uint32_t)r * 64 + lane < w1;
            const uint32_t d = el_slot(x[r]) & dm;
            const uint64_t peers = match_lanes(d, lb, valid);
            if (valid) es[mine[d] + (uint32_t)__popcll(peers & lt) - ebase] = x[r];
            __builtin_amdgcn_wave_barrier();
            if (valid && (peers & lt) == 0) mine[d] += (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();  // the bin in order before the runs read it
}

enum : int { kFzAll = 0, kFzBin = 1 };
// kFzAll: one workgroup per kFzChunk sorted elements (owning the rules whose first element lies in
// it); kFzBin: one workgroup per partition bin (el = the partition output; the bin is ordered into
// es first, and every rule of the bin is the workgroup's).
template <int kMode>
__global__ __launch_bounds__(kFzThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_cold_fused_t(ClusterState st, BatchScratch sc,
                                                             const uint64_t *__restrict__ el_in, uint32_t nhost,
                                                             const uint32_t *__restrict__ dn, uint32_t nkey,
                                                             const ReqIn in, int64_t ts_base,
                                                             int simple, uint32_t hot_min, uint64_t *__restrict__ out,
                                                             int dbg, uint64_t *__restrict__ es, int lb) {
    // Chunk mode keeps u32 run records for kFzChunk head positions; bin mode, sized for three workgroups
    // per CU (<= 53 KB of LDS each), keeps u16 records for the kBinLds positions of a bin that fits in
    // LDS (lengths, counts and the plist offset relative to h0 are then below 2^16) and none for a larger
    // bin (every run in the global run arrays).
    constexpr bool kBin = kMode == kFzBin;
    constexpr int kRl = kBin ? kBinLds : kFzChunk;           // run-record capacity (head positions)
    constexpr int kRules = kBin ? (1 << kPartMaxLow) : kFzChunk;  // rules per workgroup at most
    using RlT = typename std::conditional<kBin, uint16_t, uint32_t>::type;
    __shared__ uint32_t fheads[kRules + 1], fslot[kRules + 1];  // owned rules: first position, slot
    // run records of the runs that start in [h0, h0 + rl_cap): length, prioritized count, first
    // prioritized index (relative to h0 in bin mode), acquire count | bucket delta << 8
    __shared__ RlT rl_buf[4 * kRl];
    RlT *rl_n = rl_buf, *rl_cp = rl_buf + kRl, *rl_p0 = rl_buf + 2 * kRl, *rl_ab = rl_buf + 3 * kRl;
    __shared__ uint32_t s_long[kFzLong];  // closed-form runs the flows lanes left to the results phase (heads)
    __shared__ uint32_t s_nlong, s_huge;
    const bool scan_results = (dbg & 256) != 0;  // A/B: the round-4 results scan over every element
    __shared__ FAgg wtot[kFzThreads / 64];
    __shared__ uint32_t s_h0, s_E, s_wcnt[kFzThreads / 64];
    __shared__ uint32_t s_ncand, s_cbase, s_next, s_cand[2 * kFzThreads];
    // bin mode: the ordered bin, when it fits, stays in LDS (every later element read is an LDS read
    // through a flat pointer); a larger bin is ordered into the global buffer es
    __shared__ uint64_t sel[kBin ? kBinLds : 1];
    static_assert(!kBin || sizeof(rl_buf) >= (size_t)((kFzThreads / 64) << kPartMaxLow) * 4,
                  "bin_order's digit counts fit the run records");
    uint32_t rl_cap = kRl;  // head positions [h0, h0 + rl_cap) keep their run record in LDS
    uint32_t p0_rel = 0;    // bin mode: rl_p0 holds plist index - h0
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t *el = el_in;
    bool in_lds = false;    // bin mode: the ordered bin is the LDS image sel (element p at sel[p - lds_base])
    uint32_t lds_base = 0;
    // element p: an LDS read (ds_read) when the bin is in LDS -- a flat pointer into LDS would make every
    // element read wait for all outstanding global stores as well
    uint32_t h0, E;
    if constexpr (kMode == kFzBin) {
        const uint32_t B0 = sc.pstart[blockIdx.x], B1 = sc.pstart[blockIdx.x + 1];
        if (B0 >= B1) return;
        unsigned long long ot = 0;
        fz_mark(dbg, 0, ot);
        in_lds = B1 - B0 <= (uint32_t)kBinLds && !(dbg & 64);
        // (two calls, so each inlined copy knows its store's address space: ds_write into the LDS image)
        if (in_lds) bin_order(el_in, sel, B0, B0, B1, lb, reinterpret_cast<uint32_t *>(rl_buf), s_wcnt);
        else bin_order(el_in, es, 0u, B0, B1, lb, reinterpret_cast<uint32_t *>(rl_buf), s_wcnt);
        rl_cap = in_lds ? (uint32_t)kBinLds : 0u;
        p0_rel = B0;
        fz_mark(dbg, 4, ot);
        // element p of the bin: sel[p - B0] (LDS image) or es[p]
        el = es;
        lds_base = B0;
        h0 = B0;
        E = B1;
    } else {
    const uint32_t n = dn ? min(nhost, *dn) : nhost;
    const uint32_t c0 = blockIdx.x * kFzChunk;
    if (c0 >= n) return;
    const uint32_t c1 = min(n, c0 + kFzChunk);
    auto slot_at = [&](uint32_t p) -> uint32_t { return p < n ? el_slot(el[p]) : nkey; };
    // ---- ownership: the first rule head in the chunk (h0) and the end of the last owned rule (E)
    if (threadIdx.x == 0) {
        s_h0 = c1;
        s_E = c1;
    }
    __syncthreads();
    {
        uint32_t first_head = c1, first_inv = c1;
        for (uint32_t p = c0 + threadIdx.x; p < c1; p += kFzThreads) {
            const uint32_t s = el_slot(el[p]);
            if (s >= nkey) first_inv = min(first_inv, p);  // sorted: invalid / foreign keys form a suffix
            else if (p == 0 || el_slot(el[p - 1]) != s) first_head = min(first_head, p);
        }
        if (first_head < c1) atomicMin(&s_h0, first_head);
        if (first_inv < c1) atomicMin(&s_E, first_inv);
    }
    __syncthreads();
    h0 = s_h0;
    if (h0 >= s_E) return;  // uniform: the chunk holds no rule head
    if (s_E == c1 && c1 < n) {  // the last owned rule may continue past the chunk
        const uint32_t ls = el_slot(el[c1 - 1]);
        if (el_slot(el[c1]) == ls) {  // uniform
            __syncthreads();
            if (threadIdx.x == 0) s_E = 0xFFFFFFFFu;
            __syncthreads();
            // one chunk ahead with the whole workgroup, then (long rules only) gallop + bisect
            for (uint32_t p = c1 + threadIdx.x; p < min(n, c1 + kFzChunk); p += kFzThreads)
                if (el_slot(el[p]) != ls) {
                    atomicMin(&s_E, p);
                    break;
                }
            __syncthreads();
            if (threadIdx.x == 0 && s_E == 0xFFFFFFFFu) {
                uint32_t lo = min(n, c1 + kFzChunk), step = kFzChunk;  // slot(el[lo - 1]) == ls
                uint32_t hi = lo;
                while (true) {  // gallop: first probe with slot != ls (or n)
                    hi = (uint32_t)min((uint64_t)n, (uint64_t)lo + step);
                    if (hi >= n || slot_at(hi) != ls) break;
                    lo = hi + 1;
                    step *= 2;
                }
                while (lo < hi) {  // first position in [lo, hi] with slot != ls
                    const uint32_t m = lo + (hi - lo) / 2;
                    if (slot_at(m) != ls) hi = m;
                    else lo = m + 1;
                }
                s_E = lo;
            }
        }
    }
    __syncthreads();
    E = s_E;
    }
    // element p of the sorted cold elements: a ds_read of the bin's LDS image, or a global load.  The two
    // pointers keep their address spaces, so the choice stays a branch: one flat load for both would wait for
    // every outstanding global store as well.
    using LdsU64 = __attribute__((address_space(3))) uint64_t;
    using GlbU64 = __attribute__((address_space(1))) const uint64_t;
    const LdsU64 *lds_el = (const LdsU64 *)(sel) - lds_base;
    const GlbU64 *glb_el = (const GlbU64 *)el;
    auto EL = [&](uint32_t p) -> uint64_t {
        if (kBin && in_lds) return lds_el[p];
        return glb_el[p];
    };
    unsigned long long fzt = 0;
    fz_mark(dbg, 0, fzt);
    // ---- 1 runs (blocks of kFzBlk elements over [h0, E))
    FAgg carry = fagg_id();
    uint32_t nf_carry = 0;
    for (uint32_t b0 = h0; b0 < E; b0 += kFzBlk) {
        const uint32_t e0 = b0 + threadIdx.x * kFzPer;
        uint64_t x[kFzPer];
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) x[k] = e0 + k < E ? EL(e0 + k) : 0ull;
        uint64_t px = e0 > h0 && e0 - 1 < E ? EL(e0 - 1) : 0ull;
        FAgg acc = fagg_id();
        uint32_t nfl = 0;
        bool hd[kFzPer], fh[kFzPer];
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) {
            const uint32_t p = e0 + k;
            const bool in = p < E;
            hd[k] = in && (p == h0 || el_runkey(x[k]) != el_runkey(px));
            fh[k] = in && (p == h0 || el_slot(x[k]) != el_slot(px));
            const uint32_t pr = in ? el_prio(x[k]) : 0u;
            const int32_t a = el_acq(x[k]);
            const FAgg v{hd[k] ? p + 1 : 0u, pr, 0u, hd[k] ? 1u : 0u, in ? a : INT32_MAX, in ? a : INT32_MIN};
            acc = fagg_combine(acc, v);
            nfl += fh[k] ? 1u : 0u;
            px = x[k];
        }
        FAgg tot;
        FAgg run = fagg_combine(carry, fagg_block_excl(acc, &tot, wtot));
        // rule heads: compacted in order (wave counts through LDS)
        uint32_t fx = nfl;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = shfl_up_u32(fx, o);
            if (lane >= o) fx += y;
        }
        if (lane == 63) s_wcnt[wave] = fx;
        __syncthreads();
        uint32_t fbase = nf_carry + fx - nfl, ftot = 0;
#pragma unroll
        for (int w = 0; w < kFzThreads / 64; ++w) {
            if (w < wave) fbase += s_wcnt[w];
            ftot += s_wcnt[w];
        }
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) {
            const uint32_t p = e0 + k;
            if (p >= E) break;
            const uint32_t pr = el_prio(x[k]);
            const FAgg v{hd[k] ? p + 1 : 0u, pr, 0u, hd[k] ? 1u : 0u, el_acq(x[k]), el_acq(x[k])};
            const uint32_t np_before = run.np;
            run = fagg_combine(run, v);
            if (fh[k]) {
                fslot[fbase] = el_slot(x[k]);
                fheads[fbase++] = p;
            }
            if (pr) sc.plist[h0 + np_before] = p;
            // run end: this is the last element of its run
            const bool last = p + 1 >= E || (k + 1 < kFzPer ? hd[k + 1] : (p + 1 < E && el_runkey(EL(p + 1)) != el_runkey(x[k])));
            if (last) {
                const uint32_t head = run.hpos - 1;
                const int32_t acq = run.mn == run.mx ? run.mn : 0;  // 0: mixed or escaped -> replay
                const uint32_t bd = (uint32_t)((x[k] >> kBdShift) & kBdEsc);
                if (head - h0 < rl_cap) {
                    rl_n[head - h0] = (RlT)(p + 1 - head);
                    rl_cp[head - h0] = (RlT)(run.np - run.hp);
                    rl_p0[head - h0] = (RlT)(h0 + run.hp - p0_rel);
                    rl_ab[head - h0] = (RlT)((uint32_t)acq | (bd << 8));
                } else {  // global run arrays, indexed by head position
                    sc.run_start[head] = p + 1 - head;
                    sc.run_cp[head] = run.np - run.hp;
                    sc.run_p0[head] = h0 + run.hp;
                    sc.run_acq[head] = acq;
                    sc.run_bd[head] = (uint8_t)bd;
                }
            }
        }
        carry = fagg_combine(carry, tot);
        nf_carry += ftot;
        __syncthreads();
    }
    const uint32_t nf = nf_carry;
    if (threadIdx.x == 0) {
        s_ncand = 0;
        s_next = kFzThreads;  // rules [0, kFzThreads) go to the lanes of the same index
        s_nlong = 0;
        s_huge = 0;
    }
    __syncthreads();  // run records and plist (global, this workgroup) before the flows read them
    // next-hot-set candidates: counts of at least the floor (half the last pick threshold) are
    // gathered in LDS and published with one global reservation per workgroup
    const uint32_t cand_floor = max(hot_min, sc.hot_ctl[7] >> 1);
    fz_mark(dbg, 1, fzt);
    // ---- 2 flows: every lane takes owned rules from a workgroup counter and walks each rule's runs
    // in time order, the rule's record in registers between its runs.  A lane that finishes a rule
    // takes the next one at once, so the wave's iterations follow the workgroup's total runs, not its
    // slowest lane's share of statically assigned rules.
    const uint32_t nfw = (dbg & 1) ? 0u : nf;
    uint32_t f = threadIdx.x, r = 0, r1 = 0, s = 0;
    SlotParam P;
    Rec R{nullptr, 0};
    double thr = 0;
    int64_t qbase = 0;
    RecCarry<10> rc;
    rc.have = false;
    const bool hdr_thr = st.uni_S && !simple;  // the closed form takes the threshold from the record header
    auto take_rule = [&]() {
        r = fheads[f];
        r1 = f + 1 < nf ? fheads[f + 1] : E;
        s = fslot[f];
        if (r1 - r >= cand_floor) {  // next batch's hot-set candidate
            const uint32_t k = atomicAdd(&s_ncand, 1u);
            if (k < (uint32_t)kFzThreads) {
                s_cand[2 * k] = s;
                s_cand[2 * k + 1] = r1 - r;
            }
        }
        if (st.uni_S) {
            // uniform geometry: the record address and the window geometry without the parameter
            // load; the threshold is the record header's copy (Rec::thr), which comes with the
            // header's loads (simple mode's threshold is a parameter load beside them)
            P.S = st.uni_S;
            P.W = st.uni_W;
            P.interval = st.uni_iv;
            P.isec = st.uni_iv / 1000.0;
            P.boff = s * rec_units(st.uni_S);
            P.thr = simple ? st.param[s].thr_simple : 0.0;
            P.thr_simple = P.thr;
            P.active = 1;
            P.ns = 0;
        } else {
            P = st.param[s];
        }
        R = rec_of(st, P);
        thr = simple ? P.thr_simple : P.thr;
        qbase = div_pos(ts_base, P.W);
        rc.have = false;
    };
    bool live = f < nfw;
    if (live) take_rule();
    while (live) {
        RunIn ri;
        ri.j0 = r;
        if (r - h0 < rl_cap) {
            ri.n = rl_n[r - h0];
            ri.cp_tot = rl_cp[r - h0];
            ri.p0 = (uint32_t)rl_p0[r - h0] + p0_rel;
            const uint32_t ab = rl_ab[r - h0];
            ri.a = (int32_t)(ab & 0xFFu);
            ri.bd = ab >> 8;
        } else {
            ri.n = sc.run_start[r];
            ri.cp_tot = sc.run_cp[r];
            ri.p0 = sc.run_p0[r];
            ri.a = sc.run_acq[r];
            ri.bd = sc.run_bd[r];
        }
        // prioritized requests among the run's first k: plist[p0 .. p0 + cp_tot) holds the
        // run's prioritized positions (ascending)
        auto prio_before = [&](uint32_t k) -> uint32_t {
            if (ri.cp_tot <= 4) {  // the usual case: the positions loaded together, no dependent search
                uint32_t pv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) pv[u] = sc.plist[ri.p0 + min((uint32_t)u, ri.cp_tot - 1)];
                uint32_t c = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u) c += ((uint32_t)u < ri.cp_tot && pv[u] < ri.j0 + k) ? 1u : 0u;
                return c;
            }
            uint32_t lo = 0, hi = ri.cp_tot;
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (sc.plist[ri.p0 + m] < ri.j0 + k) lo = m + 1;
                else hi = m;
            }
            return lo;
        };
        RunOut ro;
        // sampleCount <= 10 (the default, every C3 rule): ten pair registers carried between runs;
        // larger sampleCounts load the pairs every run
        bool fast;
        if (P.S <= 10) {
            fast = run_fast<decltype(prio_before), 10>(st, P, R, thr, hdr_thr, qbase, ri, prio_before, ro, rc);
        } else {
            RecCarry<0> rc0;
            rc0.have = false;
            fast = run_fast<decltype(prio_before), 0>(st, P, R, thr, hdr_thr, qbase, ri, prio_before, ro, rc0);
        }
        if (!fast) {
            for (uint32_t j = r; j < r + ri.n; ++j) {
                const uint32_t i = el_idx(EL(j));
                const int64_t t = ts_base + (int64_t)in.ts_at(i);
                const bool p = !simple && in.prio_at(i);
                out[i] = request_exact(st, s, t, in.acq_at(i), p, simple);
            }
            ro.mode = RUN_DONE;
            rc.have = false;  // the record changed in memory
        }
        // a closed-form run's TokenResults: from its flows lane when it is short (or the long-run list is
        // full), else from a whole wave in the results phase (s_long)
        bool direct = fast && ri.n <= (scan_results ? (uint32_t)kFzShortRun : (uint32_t)kFzDirect);
        if (fast && !direct && !scan_results) {
            const uint32_t k = atomicAdd(&s_nlong, 1u);
            if (k < (uint32_t)kFzLong) {
                s_long[k] = r;
                if (ri.n >= kFzHuge && ro.cw == 0) s_huge = 1u;
            } else {
                direct = true;
            }
        }
        if (direct) {
            // the run's elements in chunks of 8, loaded together at clamped positions, decided as the results
            // phase would (kp: prioritized requests of the run before the element)
            uint32_t kp = 0;
            for (uint32_t c0 = 0; c0 < ri.n; c0 += 8) {
                uint64_t x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = EL(r + min(c0 + (uint32_t)u, ri.n - 1));
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t loc = c0 + (uint32_t)u;
                    if (loc >= ri.n) break;
                    const uint32_t pr = el_prio(x[u]);
                    uint64_t res;
                    if (loc < ro.f) {
                        const int64_t sum = ro.s0 + (int64_t)loc * ri.a;
                        res = pack_result(TRS_OK, j_d2i(ro.thr - div_isec((double)sum, ro.isec) - (double)ri.a), 0);
                    } else if (pr && kp - ro.cpf < ro.cw) {
                        res = pack_result(TRS_SHOULD_WAIT, 0, (int32_t)ro.wait);
                    } else {
                        res = pack_result(TRS_BLOCKED, 0, 0);
                    }
                    if (!(dbg & 128)) out[el_idx(x[u])] = res;
                    kp += pr;
                }
            }
            ro.mode = RUN_DONE;
        }
        if (scan_results || (fast && !direct)) sc.run_out[r] = ro;  // read by the results phase
        r += ri.n;
        if (r >= r1) {
            f = atomicAdd(&s_next, 1u);
            live = f < nfw;
            if (live) take_rule();
        }
    }
    __syncthreads();  // run_out of every owned run
    fz_mark(dbg, 2, fzt);
    {
        const uint32_t nc = min(s_ncand, (uint32_t)kFzThreads);
        if (threadIdx.x == 0) s_cbase = nc ? atomicAdd(&sc.hot_ctl[6], nc) : 0u;
        __syncthreads();
        const uint32_t k = s_cbase + threadIdx.x;
        if (threadIdx.x < nc && k < (uint32_t)kHotCand) {
            sc.hot_cand[2 * k] = s_cand[2 * threadIdx.x];
            sc.hot_cand[2 * k + 1] = s_cand[2 * threadIdx.x + 1];
        }
    }
    // ---- 3 results
    if (!scan_results) {
        // the listed long runs, one wave per run: 64 elements per step, the prioritized requests before each
        // element from a ballot prefix
        const uint32_t nl = (dbg & 2) ? 0u : min(s_nlong, (uint32_t)kFzLong);
        const uint64_t lt = lanemask_lt64(lane);
        // huge runs without SHOULD_WAIT answers (no prioritized count needed): the whole workgroup over each
        // run's elements, eight loads in flight per thread (the sort path's hottest rule would otherwise be one
        // wave's serial walk: C5a 2.95 against 1.18 ms per step)
        auto run_len = [&](uint32_t hp) { return (hp - h0 < rl_cap) ? (uint32_t)rl_n[hp - h0] : sc.run_start[hp]; };
        for (uint32_t k = 0; k < (s_huge ? nl : 0u); ++k) {
            const uint32_t hp = s_long[k];
            const RunOut ro = sc.run_out[hp];
            const uint32_t n = run_len(hp);
            if (ro.cw != 0 || n < kFzHuge) continue;
            constexpr uint32_t kStep = kFzThreads * 8;
            for (uint32_t c0 = 0; c0 < n; c0 += kStep) {
                uint64_t x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = EL(hp + min(c0 + (uint32_t)u * kFzThreads + threadIdx.x, n - 1));
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t loc = c0 + (uint32_t)u * kFzThreads + threadIdx.x;
                    if (loc >= n) break;
                    const int32_t a = el_acq(x[u]);
                    uint64_t res;
                    if (loc < ro.f) {
                        const int64_t sum = ro.s0 + (int64_t)loc * a;
                        res = pack_result(TRS_OK, j_d2i(ro.thr - div_isec((double)sum, ro.isec) - (double)a), 0);
                    } else {
                        res = pack_result(TRS_BLOCKED, 0, 0);
                    }
                    if (!(dbg & 128)) out[el_idx(x[u])] = res;
                }
            }
        }
        // the other long runs: one wave per run, the prioritized requests before each element from a ballot prefix
        for (uint32_t k = (uint32_t)wave; k < nl; k += kFzThreads / 64) {
            const uint32_t hp = s_long[k];
            const RunOut ro = sc.run_out[hp];
            if (ro.cw == 0 && run_len(hp) >= kFzHuge) continue;
            const uint32_t n = (hp - h0 < rl_cap) ? (uint32_t)rl_n[hp - h0] : sc.run_start[hp];
            uint32_t kp0 = 0;
            for (uint32_t c0 = 0; c0 < n; c0 += 64) {
                const uint32_t loc = c0 + (uint32_t)lane;
                const uint64_t x = EL(hp + min(loc, n - 1));
                const bool pr = loc < n && el_prio(x);
                const uint64_t pb = __ballot(pr);
                const uint32_t kp = kp0 + (uint32_t)__popcll(pb & lt);
                kp0 += (uint32_t)__popcll(pb);
                if (loc >= n) continue;
                const int32_t a = el_acq(x);
                uint64_t res;
                if (loc < ro.f) {
                    const int64_t sum = ro.s0 + (int64_t)loc * a;
                    res = pack_result(TRS_OK, j_d2i(ro.thr - div_isec((double)sum, ro.isec) - (double)a), 0);
                } else if (pr && kp - ro.cpf < ro.cw) {
                    res = pack_result(TRS_SHOULD_WAIT, 0, (int32_t)ro.wait);
                } else {
                    res = pack_result(TRS_BLOCKED, 0, 0);
                }
                if (!(dbg & 128)) out[el_idx(x)] = res;
            }
        }
        fz_mark(dbg, 3, fzt);
        return;
    }
    // (A/B knob) the round-4 results scan over every element
    carry = fagg_id();
    for (uint32_t b0 = h0; b0 < ((dbg & 2) ? h0 : E); b0 += kFzBlk) {
        const uint32_t e0 = b0 + threadIdx.x * kFzPer;
        uint64_t x[kFzPer];
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) x[k] = e0 + k < E ? EL(e0 + k) : 0ull;
        uint64_t px = e0 > h0 && e0 - 1 < E ? EL(e0 - 1) : 0ull;
        FAgg acc = fagg_id();
        bool hd[kFzPer];
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) {
            const uint32_t p = e0 + k;
            const bool in = p < E;
            hd[k] = in && (p == h0 || el_runkey(x[k]) != el_runkey(px));
            const FAgg v{hd[k] ? p + 1 : 0u, in ? el_prio(x[k]) : 0u, 0u, hd[k] ? 1u : 0u, 0, 0};
            acc = fagg_combine(acc, v);
            px = x[k];
        }
        FAgg tot;
        FAgg run = fagg_combine(carry, fagg_block_excl(acc, &tot, wtot));
        uint32_t head[kFzPer], kp[kFzPer];
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) {
            const uint32_t p = e0 + k;
            const uint32_t pr = p < E ? el_prio(x[k]) : 0u;
            run = fagg_combine(run, FAgg{hd[k] ? p + 1 : 0u, pr, 0u, hd[k] ? 1u : 0u, 0, 0});
            head[k] = run.hpos - 1;
            kp[k] = run.np - pr - run.hp;  // prioritized requests of the run before this one
        }
        // run records of the 8 elements loaded together (one per run change; none for a short run its flows
        // lane answered)
        RunOut ro[kFzPer];
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) {
            if (e0 + k < E && (k == 0 || head[k] != head[k - 1])) ro[k] = sc.run_out[head[k]];
            else if (k > 0) ro[k] = ro[k - 1];
        }
#pragma unroll
        for (int k = 0; k < kFzPer; ++k) {
            const uint32_t p = e0 + k;
            if (p >= E || ro[k].mode != RUN_FAST) continue;
            const uint32_t local = p - head[k];
            const int32_t a = el_acq(x[k]);
            uint64_t res;
            if (local < ro[k].f) {
                const int64_t sum = ro[k].s0 + (int64_t)local * a;
                res = pack_result(TRS_OK, j_d2i(ro[k].thr - (double)sum / ro[k].isec - (double)a), 0);
            } else if (el_prio(x[k]) && kp[k] - ro[k].cpf < ro[k].cw) {
                res = pack_result(TRS_SHOULD_WAIT, 0, (int32_t)ro[k].wait);
            } else {
                res = pack_result(TRS_BLOCKED, 0, 0);
            }
            if (!(dbg & 128)) out[el_idx(x[k])] = res;
        }
        carry = fagg_combine(carry, tot);
        __syncthreads();
    }
    fz_mark(dbg, 3, fzt);
}
#define k_cold_fused k_cold_fused_t<kFzAll>

// ---------------------------------------------------------------- small batches (one call, few requests)
// A batch of at most kSmall requests (a single TokenService.requestToken, or the few a coalescing
// queue gathered) is classified and ordered by (rule, arrival) inside one workgroup -- a bitonic
// sort of the packed elements in LDS on the key slot << 32 | index -- and handed to k_cold_fused:
// two launches instead of the classify / three radix passes / runs pipeline.
constexpr int kSmall = 4096;
constexpr int kSmallThreads = 1024;
__device__ __forceinline__ uint64_t small_key(uint64_t e) { return ((uint64_t)el_slot(e) << 32) | el_idx(e); }
__global__ __launch_bounds__(kSmallThreads) void k_small_sort(ClusterState st, const int64_t *__restrict__ flow_id,
                                                              const int32_t *__restrict__ acquire,
                                                              const uint8_t *__restrict__ prio,
                                                              const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                              uint32_t n, uint32_t m, int simple, uint32_t invalid_key,
                                                              uint64_t *__restrict__ el, uint64_t *__restrict__ out) {
    __shared__ uint64_t e[kSmall];
    for (uint32_t i = threadIdx.x; i < m; i += kSmallThreads) {
        if (i >= n) {
            e[i] = ~0ull;  // padding: sorts last
            continue;
        }
        const int64_t f = flow_id[i];
        const int32_t a = acquire[i];
        int8_t status = TRS_OK;
        uint32_t slot = 0, W = 1;
        if (!simple && (f <= 0 || a <= 0)) {
            status = TRS_BAD_REQUEST;
        } else if (f <= 0) {
            status = TRS_NO_RULE_EXISTS;
        } else if (st.dense_n) {
            if (f <= (int64_t)st.dense_n) {
                const uint32_t d = (uint32_t)st.dense[f - 1];
                if (d == ~0u) status = TRS_NO_RULE_EXISTS;
                else {
                    slot = d & 0xFFFFFFu;
                    W = st.wtab[d >> 24];
                }
            } else {
                status = TRS_NO_RULE_EXISTS;
            }
        } else {
            uint32_t q = (uint32_t)hash_flow_id(f) & st.hmask;
            HashEntry he = st.htab[q];
            for (uint32_t probe = 1; probe <= st.hmask && he.key != f && he.key != 0; ++probe) {
                q = (q + 1) & st.hmask;
                he = st.htab[q];
            }
            if (he.key != f) status = TRS_NO_RULE_EXISTS;
            else {
                slot = he.slot;
                W = he.W;
            }
        }
        if (status != TRS_OK) {
            out[i] = pack_result(status, 0, 0);
            e[i] = ((uint64_t)invalid_key << kSlotShift) | i;
        } else {
            const uint32_t p = (!simple && prio && prio[i]) ? 1u : 0u;
            const int64_t bd = div_pos(ts_base + (int64_t)ts_off[i], (int64_t)W) - div_pos(ts_base, (int64_t)W);
            uint32_t a7 = (a >= 1 && a <= (int32_t)kAcqMax) ? (uint32_t)a : 0u;
            uint32_t bd6 = (uint32_t)bd;
            if (bd >= (int64_t)kBdEsc) {
                bd6 = kBdEsc;
                a7 = 0;
            }
            e[i] = el_pack(slot, bd6, p, a7, i);
        }
    }
    __syncthreads();
    // bitonic sort of m (a power of two) elements
    for (uint32_t k = 2; k <= m; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < m / 2; t += kSmallThreads) {
                const uint32_t i = 2 * t - (t & (j - 1));  // lower index of the pair (i, i + j)
                const uint32_t l = i + j;
                const uint64_t x = e[i], y = e[l];
                const bool up = (i & k) == 0;
                if ((small_key(x) > small_key(y)) == up) {
                    e[i] = y;
                    e[l] = x;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += kSmallThreads) el[i] = e[i];
}

// ---------------------------------------------------------------- hot path
// Under Zipf skew a few thousand rules carry most requests (C3: the 4096 hottest of 1M rules carry
// 77 % of them).  Those "hot" rules (hot id < kHot, picked from the previous batch's counts, all
// with one window length W) are decided without moving their requests:
//   k_hot_classify  one pass in input order.  Each wave owns kHotSeg consecutive requests and ranks
//                   every hot request among the segment's requests of its rule (12 ballots match
//                   equal hot ids, wave-private LDS counters keep arrival order); rank and bucket
//                   are stored as a 4-byte code per request, the per-rule counts as one row per
//                   segment.  Cold requests and prioritized hot ones are compacted into the sort
//                   input, 1024-request segments in arrival order.
//   k_hscan_*       column prefix of the count rows: rank of each segment's first request of each
//                   hot rule.  The position where each window bucket starts is recorded (segment,
//                   plus a snapshot of the counts before it when it falls inside a segment), so
//                   each run's first rank follows.
//   k_hot_flows     one wave per hot rule walks its runs (one per bucket of the batch) in time
//                   order with the closed form of the cold path (pass prefix, occupy count).
//   k_hot_final     each hot request's TokenResult from its rank, in input order (coalesced).
// Prioritized hot requests are sorted as key nslots + 1 + hot id, after every cold element, so
// each rule's prioritized ranks form one ascending list (the occupy decisions need the number of
// prioritized requests before a position); k_hot_final's first workgroups answer them.
// Preconditions, checked on the device before any rule state is touched (else the batch
// re-classifies every request as cold and takes the sort path): timestamps non-decreasing over the
// batch (then bucket order is arrival order for every rule), hot requests with acquireCount 1, at
// most kHotBuckets buckets, no hot rule window holding a bucket newer than the batch.
constexpr int kH1Waves = kThreads / 64;          // segments per workgroup
constexpr int kSubRounds = kSubSeg / 64;          // rounds per compaction segment (16)
constexpr int kSubPerSeg = kHotSeg / kSubSeg;     // 8
constexpr int kH1Chunk = 4;                       // rounds per pipeline chunk
static_assert(kSubRounds % kH1Chunk == 0, "chunks tile a compaction segment");
static_assert(kSubSeg * 4 == kRadix64Tile, "compaction segments are the sort's input segments");
constexpr uint32_t kNoCode = 0xFFFFFFFFu;

// Cross-lane moves that do not depend on which lanes are active (a __shfl is a ds_bpermute, and the
// compiler may sink one into a branch where its source lanes are masked off, which then read 0):
// DPP wave shifts and v_readlane.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t lane0) {  // lane i <- lane i - 1
    return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v, uint32_t lane63) {  // lane i <- lane i + 1
    return (uint32_t)__builtin_amdgcn_update_dpp((int)lane63, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ int64_t lane_i64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// In-order rank of a wave's hot lanes among its requests of their hot id so far: one LDS atomic
// add with return per round on per-wave counters packed two hot ids per word.  The lanes of one
// wave instruction that add to the same LDS word receive the old values in lane order on gfx950
// (probed once per process by lds_lane_order_ok(); the hot path stays off if it ever fails), so
// the returned count is the number of earlier requests of that hot id: arrival order.
__device__ __forceinline__ uint32_t rank_hot(uint32_t *cw, uint32_t hid) {
    const uint32_t sh = (hid & 1u) << 4;
    return (atomicAdd(&cw[hid >> 1], 1u << sh) >> sh) & 0xFFFFu;
}


__device__ __forceinline__ uint32_t hot_count(const BatchScratch &sc) {
    return min(sc.hot_ctl[0], (uint32_t)kHot);
}

// floor((ts_base + t) / W) - floor(ts_base / W) = floor((r0 + t) / W), r0 = ts_base mod W: one double
// multiply and an exact correction instead of two int64 divisions.
__device__ __forceinline__ uint32_t bucket_delta(uint32_t t, uint32_t W, uint32_t r0, double inv) {
    const uint64_t x = (uint64_t)r0 + t;
    int64_t q = (int64_t)((double)x * inv);
    const int64_t r = (int64_t)x - q * (int64_t)W;
    if (r < 0) --q;
    else if (r >= (int64_t)W) ++q;
    return (uint32_t)q;
}

// Per batch: r0 and 1/W of every window-length code (the dense flowId table's wcode), and the
// precheck: no hot rule's window may hold a bucket newer than the batch's first request (batches
// submitted out of time order), as the closed form needs each run's bucket to be the newest.
__global__ __launch_bounds__(kThreads) void k_hot_precheck(ClusterState st, BatchScratch sc, const ReqIn in,
                                                           int64_t ts_base, uint32_t n, int pipelined) {
    if (blockIdx.x == 0 && st.dense_n) {
        const uint32_t W = st.wtab[threadIdx.x];
        WConst wc;
        wc.W = W;
        wc.r0 = (uint32_t)(ts_base % (int64_t)W);
        wc.inv = 1.0 / (double)W;
        sc.wconst[threadIdx.x] = wc;
    }
    const uint32_t h = blockIdx.x * kThreads + threadIdx.x;
    if (h < (uint32_t)kHot) {  // the prioritized-range table of this batch (k_prio_rank fills it)
        sc.plo[h] = 0;
        sc.phi[h] = 0;
    }
    if (h >= hot_count(sc) || n == 0) return;
    const int64_t W = (int64_t)sc.hot_ctl[2];
    const int64_t t0 = ts_base + (int64_t)in.ts_at(0);
    // Pipelined batches: the window starts read here may still be written by the earlier batch being
    // decided.  That batch writes buckets at its own times only, so the answer is the same either way
    // when this batch starts no earlier than every earlier batch's latest time; otherwise no hot path.
    if (pipelined && h == 0 && t0 < (int64_t)*sc.tmax_all) atomicOr(&sc.counters[CTL_FLAGS], kFlagState);
    const int64_t ws0 = t0 - t0 % W;
    const uint32_t s = sc.hot_slot[h];
    const SlotParam P = st.param[s];
    bool bad = P.W != (int32_t)W || !P.active || P.S <= 1 || P.S > 64;
    const Rec R = rec_of(st, P);
    for (int j = 0; j < P.S && !bad; ++j) {
        const int64_t w = R.start(j);
        if (w != kAbsent && w > ws0) bad = true;
    }
    if (bad) atomicOr(&sc.counters[CTL_FLAGS], kFlagState);
}

// k_hot_key: one workgroup per kHotSeg-request rank segment, one wave per 1024-request compaction
// segment (sub).  Every request independently: validation (BAD_REQUEST / NO_RULE_EXISTS written
// directly), rule lookup, bucket deltas; cold requests become sort elements (compacted in arrival
// order).  Hot requests are ranked among the sub's requests of their rule in arrival order as they
// are classified (12 ballots match equal hot ids; wave-private LDS counters), the in-wave code
// (hot id | rank << 12 | bucket << 25, bit 31 prioritized) is stored, and once every wave of the
// segment is done the counters become per-wave prefixes (column scan over the 8 waves), the codes
// are re-read (L2) and fixed up to in-segment ranks, prioritized hot requests join their sub's
// elements (key nslots + 1 + hot id, rank in the bucket/acquire fields), and the segment's count
// row is written.  At a hot bucket boundary inside the segment the wave's counts before it are
// snapshot into a pre row (earlier waves' totals added after the scan); the boundary table records
// where every bucket of the batch starts.
// Pass 1 of the batch is this kernel again with no hot rules (launched always, returns at once
// unless a fallback flag is up): every valid request becomes a cold element.
// Software pipeline over chunks of kH1Chunk rounds with three register buffers used in rotation
// (the loop is unrolled three times, so no buffer is copied: copying a register a load is still
// writing waits for that load).  While chunk c is processed, the table lookups of chunk c + 1 and
// the field loads of chunk c + 2 are in flight; loads and lookups are unconditional (clamped
// indices, values masked when processed), so no branch stands around a load.
constexpr uint32_t kKeyHot = 1u << 19;
constexpr uint32_t kPsGroups = 256;  // the prioritized sort's groups of rank segments (k_psort_*)
constexpr int kKeyWaves = kHotSeg / kSubSeg;  // 8: one rank segment per workgroup
constexpr int kKeyThreads = kKeyWaves * 64;
static_assert(kKeyWaves == kSubPerSeg, "one wave per compaction segment");
struct KeyShared {
    WConst wcs[256];
    uint16_t cnt[kKeyWaves][kHot];  // per wave: hot requests so far per hot id
    uint32_t s_np[kKeyWaves], s_bd[kKeyWaves], s_tm[kKeyWaves];
    uint32_t s_bmin, s_bmax;  // hot buckets whose first request lies inside the segment (not at its start)
    union {
        uint32_t hist0[2][256];      // per sort tile of the segment: the first radix digit's counts
        uint32_t phist[kPartBins];   // partition mode: the segment's cold elements per slot bin
    };
};
// kPk: the requests are packed sga_token_request records (in.pk), else the four arrays of in.
template <int kPass, bool kDense, bool kNT = false, bool kPk = false>
__device__ __forceinline__ void hot_key(KeyShared &sh, const ClusterState &st, const BatchScratch &sc, const ReqIn in,
                                        int64_t ts_base, uint32_t n, uint64_t *__restrict__ out, int dbg,
                                        int d0, uint32_t *__restrict__ hist, uint32_t ntiles) {
    const int64_t *__restrict__ flow_id = in.flow;
    const int32_t *__restrict__ acquire = in.acq;
    const uint8_t *__restrict__ prio = in.prio;
    const uint32_t *__restrict__ ts_off = in.ts;
    const uint32_t *__restrict__ pk = in.pk;
    // d0 > 0: the LSD sort's first digit (d0 bits) counted per sort tile; d0 < 0: partition mode, the
    // cold elements counted per slot bin (slot >> -d0) into the segment's row of hist ([seg][kPartBins])
    WConst *wcs = sh.wcs;
    const int pl = d0 < 0 ? -d0 : 0;
    if (pl) d0 = 0;
    const uint32_t dmask = (1u << d0) - 1u;
    auto &cnt = sh.cnt;
    uint32_t *s_np = sh.s_np, *s_bd = sh.s_bd;
    const uint32_t flags0 = sc.counters[CTL_FLAGS];
    // pass 0 decides nothing when the precheck refused the hot path; pass 1 (re-classifying every request as
    // cold) runs after a refusal or a fallback flag of pass 0
    if (kPass == 0 && (flags0 & kFlagState)) return;
    if (kPass == 1 && !(flags0 & (kFlagRerun | kFlagState))) return;
    const uint32_t nhot = kPass == 0 ? hot_count(sc) : 0u;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt64(lane);
    if (kDense)
        for (int k = threadIdx.x; k < 256; k += kKeyThreads) wcs[k] = sc.wconst[k];  // window-length codes
    for (int k = threadIdx.x; k < (pl ? kPartBins : 2 * 256); k += kKeyThreads) sh.phist[k] = 0;
    if (nhot) {
        uint4 *cz = reinterpret_cast<uint4 *>(&cnt[0][0]);
        for (int k = threadIdx.x; k < (int)(sizeof(cnt) / 16); k += kKeyThreads) cz[k] = make_uint4(0, 0, 0, 0);
    }
    if (threadIdx.x == 0) {
        sh.s_bmin = 0xFFFFFFFFu;
        sh.s_bmax = 0u;
    }
    __syncthreads();
    const uint32_t seg = blockIdx.x;
    const uint32_t sub = seg * kKeyWaves + wave;
    const uint32_t ubase = sub * kSubSeg;
    const bool active = ubase < n;
    uint16_t *c = cnt[wave];
    const uint32_t Wh = nhot ? sc.hot_ctl[2] : 1u;
    const uint32_t r0h = (uint32_t)(ts_base % (int64_t)Wh);
    const double invh = 1.0 / (double)Wh;
    // a key-table entry may name a hot rule while this pass decides every request as cold (no hot path for
    // the batch, or the re-classifying pass): its slot from the hot set, its window length the hot rules' one
    const uint32_t Wc = (kDense && sc.hot_ctl[0]) ? sc.hot_ctl[2] : 1u;
    const uint32_t r0c = (uint32_t)(ts_base % (int64_t)Wc);
    const double invc = 1.0 / (double)Wc;
    uint32_t wflags = 0, nc = 0, np = 0, bdmax = 0, tmax_l = 0;
    const uint32_t send = min(n, ubase + (uint32_t)kSubSeg);
    // the sub's request codes stay in registers through the rank and fix-up passes (written once)
    uint32_t hc[kSubRounds];
#pragma unroll
    for (int r = 0; r < kSubRounds; ++r) hc[r] = kNoCode;
    if (active) {
        uint32_t ptso = ubase > 0 ? (kPk ? pk[3 * (size_t)(ubase - 1) + 1] : ts_off[ubase - 1]) : 0u;  // time order across the sub start
        // hot bucket of the previous request (bucket boundaries)
        uint32_t pbd = (nhot && ubase > 0) ? min(bucket_delta(ptso, Wh, r0h, invh), (uint32_t)kHotBuckets - 1) : 0u;
        const bool use_prio = kPk || prio != nullptr;
        constexpr int nchunks = kSubRounds / kH1Chunk;  // a short last sub runs masked rounds
        struct Buf {
            int64_t f[kH1Chunk];
            int32_t a[kH1Chunk];
            uint32_t t[kH1Chunk], p[kH1Chunk], d[kH1Chunk], m[kH1Chunk];
            HashEntry e[kH1Chunk];
        };
        Buf B0, B1, B2;
        // a missing prio array reads the acquire bytes instead, masked off when processed
        const uint8_t *pr_src = kPk ? nullptr : (use_prio ? prio : reinterpret_cast<const uint8_t *>(acquire));
        auto load = [&](int ch, Buf &B) {
#pragma unroll
            for (int u = 0; u < kH1Chunk; ++u) {
                const uint32_t i = min(ubase + (uint32_t)(ch * kH1Chunk + u) * 64 + lane, n - 1);
                if (kPk) {  // one 12-byte record: flowId, time offset, acquireCount | flags << 16
                    const uint32_t *r = pk + 3 * (size_t)i;
                    uint32_t w0, w1, w2;
                    if (kNT) {
                        w0 = __builtin_nontemporal_load(r);
                        w1 = __builtin_nontemporal_load(r + 1);
                        w2 = __builtin_nontemporal_load(r + 2);
                    } else {
                        w0 = r[0];
                        w1 = r[1];
                        w2 = r[2];
                    }
                    B.f[u] = (int64_t)w0;
                    B.t[u] = w1;
                    B.a[u] = (int32_t)(w2 & 0xFFFFu);
                    B.p[u] = w2 >> 16;  // the flags: bit 0 prioritized, other bits reserved (BAD_REQUEST)
                } else if (kNT) {  // streamed once: non-temporal, so the dense table keeps more of L2
                    B.f[u] = __builtin_nontemporal_load(&flow_id[i]);
                    B.a[u] = __builtin_nontemporal_load(&acquire[i]);
                    B.t[u] = __builtin_nontemporal_load(&ts_off[i]);
                    B.p[u] = __builtin_nontemporal_load(&pr_src[i]);
                } else {
                    B.f[u] = flow_id[i];
                    B.a[u] = acquire[i];
                    B.t[u] = ts_off[i];
                    B.p[u] = pr_src[i];
                }
            }
        };
        auto lookup = [&](Buf &B) {
#pragma unroll
            for (int u = 0; u < kH1Chunk; ++u) {
                // what processing needs of flowId / acquireCount / prioritized, in one register
                // (the 64-bit flowId and the acquire count are dead after this in the dense case)
                const int64_t f = B.f[u];
                const int32_t a = B.a[u];
                const bool pr = kPk ? (B.p[u] & 1u) != 0 : (use_prio && B.p[u]);
                const bool resv = kPk && (B.p[u] >> 1) != 0;  // reserved flag bits set: not a valid request
                B.m[u] = (pr ? 1u : 0u) | ((f <= 0 || a <= 0 || resv) ? 2u : 0u) |
                         ((uint64_t)(f - 1) < (uint64_t)st.dense_n ? 4u : 0u) | (a == 1 ? 8u : 0u) |
                         ((a >= 1 && a <= (int32_t)kAcqMax ? (uint32_t)a : 0u) << 8);
                if (kDense) {  // the hot path's key table: slot | wcode << 24, or kDkHot | hot id
                    const uint64_t k = (uint64_t)(B.f[u] - 1);
                    const uint32_t kk = k < (uint64_t)st.dense_n ? (uint32_t)k : 0u;
                    B.d[u] = st.dkey[kk];
                } else {
                    B.d[u] = (uint32_t)hash_flow_id(B.f[u]) & st.hmask;
                    B.e[u] = st.htab[B.d[u]];
                }
            }
        };
        auto process = [&](Buf &B, int ch) {
#pragma unroll
            for (int u = 0; u < kH1Chunk; ++u) {
                const uint32_t rbase = ubase + (uint32_t)(ch * kH1Chunk + u) * 64;
                const uint32_t i = rbase + lane;
                const bool valid = i < send;
                if (valid) tmax_l = max(tmax_l, B.t[u]);
                uint32_t d = B.d[u];
                const uint32_t m = B.m[u];
                if (kDense && !(m & 4u)) d = kDkNone;
                const uint32_t p = m & 1u;
                uint32_t kind = 0, hid = kColdId, slot = 0, bd6 = 0, a7 = 0;
                // hot bucket (window length of the hot rules) of every request: time order of the
                // buckets; the request's own bucket when its rule has that window length too
                const uint32_t q = (nhot && valid) ? bucket_delta(B.t[u], Wh, r0h, invh) : 0u;
                if (valid) {
                    int8_t status = TRS_OK;
                    uint32_t W = 0, r0 = 0;
                    double inv = 0;
                    if (m & 2u) {
                        status = TRS_BAD_REQUEST;
                    } else if (kDense) {
                        if (d == kDkNone) {
                            status = TRS_NO_RULE_EXISTS;
                        } else if (d & kDkHot) {  // a hot rule: its window length is the hot rules' one
                            hid = d & 0xFFFu;
                            W = Wc;
                            r0 = r0c;
                            inv = invc;
                            if (kPass == 1) {
                                // decided as cold in this pass: the slot and window length from the authoritative
                                // table (a key-table entry naming a hot id outside the hot set -- kFlagHotKey --
                                // would find a stale hot_slot)
                                const uint32_t dd = st.dense[(uint32_t)(B.f[u] - 1)];
                                slot = dd & 0xFFFFFFu;
                                const WConst wc = wcs[dd >> 24];
                                W = wc.W;
                                r0 = wc.r0;
                                inv = wc.inv;
                            } else if (hid >= nhot) {
                                wflags |= kFlagHotKey;
                            }
                        } else {
                            slot = d & 0xFFFFFFu;
                            const WConst wc = wcs[d >> 24];
                            W = wc.W;
                            r0 = wc.r0;
                            inv = wc.inv;
                        }
                    } else {
                        const int64_t f = B.f[u];
                        HashEntry he = B.e[u];
                        if (he.key != f && he.key != 0) {  // continue the linear probe
                            uint32_t q = d;
                            for (uint32_t probe = 1; probe <= st.hmask; ++probe) {
                                q = (q + 1) & st.hmask;
                                he = st.htab[q];
                                if (he.key == f || he.key == 0) break;
                            }
                        }
                        if (he.key != f) {
                            status = TRS_NO_RULE_EXISTS;
                        } else {
                            slot = he.slot;
                            W = he.W;
                            r0 = (uint32_t)(ts_base % (int64_t)W);
                            inv = 1.0 / (double)W;
                        }
                    }
                    if (status != TRS_OK) {
                        out[i] = pack_result(status, 0, 0);
                    } else {
                        uint32_t bd = q;
                        if (!nhot || W != Wh) bd = bucket_delta(B.t[u], W, r0, inv);
                        a7 = (m >> 8) & kAcqMax;
                        bd6 = bd;
                        if (bd >= kBdEsc) {
                            bd6 = kBdEsc;
                            a7 = 0;
                        }
                        kind = 1;
                        if (nhot) {
                            if (!kDense) hid = sc.hot_of[slot];
                            if (hid < nhot) {
                                kind = 2;
                                if (!(m & 8u)) wflags |= kFlagMixed;
                            }
                        }
                    }
                }
                if (nhot) {
                    // time order (every request with an index counts), hot bucket, in-wave rank
                    const uint32_t pt = wave_shr1(B.t[u], ptso);
                    const bool hp = lane ? true : i != 0;
                    if (valid && hp && B.t[u] < pt) wflags |= kFlagUnsorted;
                    ptso = lane_u32(B.t[u], 63);
                    if (valid && q >= (uint32_t)kHotBuckets) wflags |= kFlagBucket;
                    const uint32_t bdh = min(q, (uint32_t)kHotBuckets - 1);
                    if (valid) bdmax = max(bdmax, bdh);
                    if (i == 0) sc.counters[CTL_BDLO] = bdh;
                    const uint32_t pbk = wave_shr1(bdh, pbd);
                    if (valid && hp && bdh > pbk) {  // the first request of buckets pbk + 1 .. bdh
                        for (uint32_t qq = pbk + 1; qq <= bdh; ++qq) sc.hbnd[qq] = i;
                        if (i & (uint32_t)(kHotSeg - 1)) {  // inside the segment: its pre rows (below)
                            atomicMin(&sh.s_bmin, pbk + 1);
                            atomicMax(&sh.s_bmax, bdh);
                        }
                    }
                    pbd = lane_u32(bdh, 63);
                    if (valid) hc[ch * kH1Chunk + u] = (kind == 2 ? (kKeyHot | hid | (p << 12)) : 0u) | (bdh << 13);
                }
                // cold elements, compacted in arrival order
                const bool emit = kind == 1;
                const uint64_t em = __ballot(emit);
                if (emit) {
                    if (kNT)
                        __builtin_nontemporal_store(el_pack(slot, bd6, p, a7, i),
                                                    &sc.el_tile[(size_t)ubase + nc + (uint32_t)__popcll(em & lt)]);
                    else
                        sc.el_tile[(size_t)ubase + nc + (uint32_t)__popcll(em & lt)] = el_pack(slot, bd6, p, a7, i);
                    if (d0) atomicAdd(&sh.hist0[wave >> 2][slot & dmask], 1u);
                    if (pl) atomicAdd(&sh.phist[slot >> pl], 1u);
                }
                nc += (uint32_t)__popcll(em);
            }
        };
        load(0, B0);
        lookup(B0);
        load(1, B1);
#pragma unroll
        for (int ch = 0; ch < nchunks; ch += 3) {
            lookup(B1);
            load(ch + 2, B2);
            process(B0, ch);
            if (ch + 1 >= nchunks) break;
            lookup(B2);
            load(ch + 3, B0);
            process(B1, ch + 1);
            if (ch + 2 >= nchunks) break;
            lookup(B0);
            load(ch + 4, B1);
            process(B2, ch + 2);
        }
        if (nhot && !(dbg & 4)) {
            // rank pass over the sub's keys (just written: L2; all 16 loads in flight together, the
            // pipeline's registers are free), one round at a time
#pragma unroll
            for (int r = 0; r < kSubRounds; ++r) {
                const uint32_t i = ubase + (uint32_t)r * 64 + lane;
                const uint32_t kv = hc[r];
                const bool hot = i < send && (kv & kKeyHot);
                const uint32_t hid = kv & 0xFFFu, p = (kv >> 12) & 1u, bdh = (kv >> 13) & 63u;
                uint32_t r_in = 0;
                if (hot) r_in = rank_hot(reinterpret_cast<uint32_t *>(c), hid);
                np += (uint32_t)__popcll(__ballot(hot && p));
                hc[r] = hot ? ((p << 31) | hid | (r_in << 12) | (bdh << 25)) : kNoCode;
            }
        }
    }
    if (wflags) atomicOr(&sc.counters[CTL_FLAGS], wflags);
    if (nhot) {
bdmax = wave_max_u32(bdmax);
        if (lane == 0) {
            s_np[wave] = np;
            s_bd[wave] = bdmax;
        }
        __syncthreads();
        {  // per-wave counters -> exclusive prefixes over the waves (two hot ids per word: counts < 2^16)
            uint32_t *cw = reinterpret_cast<uint32_t *>(&cnt[0][0]);
            uint32_t *row = reinterpret_cast<uint32_t *>(sc.hcnt + (size_t)seg * kHot);
            for (uint32_t k = threadIdx.x; k < (nhot + 1) / 2; k += kKeyThreads) {
                uint32_t run = 0;
#pragma unroll
                for (int w = 0; w < kKeyWaves; ++w) {
                    const uint32_t v = cw[w * (kHot / 2) + k];
                    cw[w * (kHot / 2) + k] = run;
                    run += v;
                }
                row[k] = run;  // this segment's count row
            }
        }
        if (threadIdx.x == 0) {  // reduced by k_hot_mode: thousands of same-address atomics would serialize
            uint32_t a = 0, m = 0;
            for (int w = 0; w < kKeyWaves; ++w) {
                a += s_np[w];
                m = max(m, s_bd[w]);
            }
            sc.seg_stat[kSegStat * seg] = a;
            sc.seg_stat[kSegStat * seg + 1] = m;
        }
        __syncthreads();
        if (active) {
            // codes: in-wave ranks -> in-segment ranks; prioritized hot requests go to the segment's
            // prioritized buffer, compacted over the segment in arrival order (the waves' counts s_np give each
            // wave its offset; k_psort_* sort them by hot id)
            uint32_t npc = 0;
            for (int w = 0; w < wave; ++w) npc += s_np[w];
            const uint32_t pgper = (((n + kHotSeg - 1) / kHotSeg) + kPsGroups - 1) / kPsGroups;
#pragma unroll
            for (int r = 0; r < kSubRounds; ++r) {
                const uint32_t i = ubase + (uint32_t)r * 64 + lane;
                const uint32_t cd = hc[r];
                const bool hot = i < send && cd != kNoCode;
                const uint32_t hid = cd & 0xFFFu;
                const uint32_t r_seg = hot ? ((cd >> 12) & 0x1FFFu) + c[hid] : 0u;
                const bool pr = hot && (cd >> 31);
                if (i < send) sc.hcode[i] = hot ? ((cd & ~(0x1FFFu << 12)) | (r_seg << 12)) : kNoCode;
                const uint64_t em = __ballot(pr);
                if (pr) {
                    sc.pel_tile[(size_t)seg * kHotSeg + npc + (uint32_t)__popcll(em & lt)] = el_pack(hid, r_seg >> 7, 1u, r_seg & 127u, i);
                    atomicAdd(&sc.prow[(size_t)(seg / pgper) * kHot + hid], 1u);  // k_psort_cols
                }
                npc += (uint32_t)__popcll(em);
            }
        }
        // Per hot bucket whose first request P lies inside this segment (not at its start): the segment's hot
        // requests of each hot id before P (k_hot_flows adds them to the segment's base rank).  On the hot path
        // the times are sorted, so "before P" is "of an earlier bucket".  Rare (a few segments per batch).
        __syncthreads();  // the fix-up's reads of the wave prefixes are done: cnt is free
        const uint32_t b0 = sh.s_bmin, b1 = sh.s_bmax;
        uint32_t *pc = reinterpret_cast<uint32_t *>(&cnt[0][0]);
        for (uint32_t b = b0; b <= b1; ++b) {  // uniform; empty unless a boundary is inside
            for (uint32_t k = threadIdx.x; k < nhot; k += kKeyThreads) pc[k] = 0;
            __syncthreads();
#pragma unroll
            for (int r = 0; r < kSubRounds; ++r) {
                const uint32_t cd = hc[r];
                if (ubase + (uint32_t)r * 64 + lane < send && cd != kNoCode && ((cd >> 25) & 63u) < b)
                    atomicAdd(&pc[cd & 0xFFFu], 1u);
            }
            __syncthreads();
            for (uint32_t k = threadIdx.x; k < nhot; k += kKeyThreads) sc.hpre[(size_t)b * kHot + k] = (uint16_t)pc[k];
            if (threadIdx.x == 0) atomicAdd(&sc.counters[CTL_NPRE], 1u);
            __syncthreads();
        }
    }
    {  // the segment's latest request time (offset from ts_base): k_hot_mode keeps the maximum over batches
tmax_l = wave_max_u32(tmax_l);
        if (lane == 0) sh.s_tm[wave] = tmax_l;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t m = 0;
            for (int w = 0; w < kKeyWaves; ++w) m = max(m, sh.s_tm[w]);
            sc.seg_stat[kSegStat * seg + 2] = m;
        }
    }
    if (lane == 0) sc.tile_nc[sub] = active ? nc : 0u;  // totals: k_hot_mode
    if (pl) {  // the segment's bin counts (one contiguous row; k_part_colscan scans the columns)
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < (uint32_t)kPartBins; k += kKeyThreads)
            hist[(size_t)seg * kPartBins + k] = sh.phist[k];
    }
    if (d0) {  // the sort's first-pass histogram rows of this segment's two tiles
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < (2u << d0); k += kKeyThreads) {
            const uint32_t t = k >> d0, d = k & dmask, tile = seg * 2 + t;
            if (tile < ntiles) hist[(size_t)d * ntiles + tile] = sh.hist0[t][d];
        }
    }
}

// ---- cold partition (hot path; SURVEY hard part 4): the key kernels count each segment's cold elements
// per slot bin ([segment][bin], one contiguous row per segment), k_part_colscan turns each group of
// kPartGroup rows into exclusive prefixes down the columns (and the group sums), k_part_binscan scans
// the group sums per bin and the bin totals into bin starts, and k_part_scatter moves every cold element
// to bin start + its position among the bin's elements in arrival order: one pass over the elements
// instead of the LSD sort's three.  k_cold_fused then orders each bin inside its workgroup (bin_order).
__global__ __launch_bounds__(256) void k_part_colscan(BatchScratch sc, uint32_t nseg) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    const uint32_t t0 = blockIdx.y * kPartGroup, t1 = min(nseg, t0 + kPartGroup);
    uint32_t acc = 0;
    for (uint32_t t = t0; t < t1; t += 8) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = t + k < t1 ? sc.phist[(size_t)(t + k) * kPartBins + b] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (t + k < t1) sc.phist[(size_t)(t + k) * kPartBins + b] = acc;
            acc += v[k];
        }
    }
    sc.pgrp[(size_t)blockIdx.y * kPartBins + b] = acc;
}

// per bin: exclusive prefix of the group sums and the bin total (kPartBins / 256 workgroups); the last
// workgroup to finish turns the totals into the bin starts
__global__ __launch_bounds__(256) void k_part_binscan(BatchScratch sc, uint32_t ngroups) {
    __shared__ uint32_t ws[4];
    __shared__ uint32_t s_last;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t g = 0; g < ngroups; g += 8) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = g + k < ngroups ? sc.pgrp[(size_t)(g + k) * kPartBins + b] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (g + k < ngroups) sc.pgrp[(size_t)(g + k) * kPartBins + b] = acc;
            acc += v[k];
        }
    }
    sc.pstart[b] = acc;  // the bin's total for now
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&sc.pstart[kPartBins + 1], 1u) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    constexpr int kPer = kPartBins / 256;
    uint32_t tot[kPer], ts = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        tot[k] = __hip_atomic_load(&sc.pstart[threadIdx.x * kPer + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ts += tot[k];
    }
    uint32_t x = ts;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    uint32_t pre = x - ts;
    for (int w = 0; w < wave; ++w) pre += ws[w];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        sc.pstart[threadIdx.x * kPer + k] = pre;
        pre += tot[k];
    }
    if (threadIdx.x == 255) {
        sc.pstart[kPartBins] = pre;
        sc.pstart[kPartBins + 1] = 0;  // the done counter, for the next batch
    }
}

// One workgroup per key segment, one wave per compaction segment (sub): pass 1 counts each wave's
// elements per bin (ballot match, the lowest lane of a group adds it), the counts become prefixes
// over the waves, pass 2 places every element at its segment's base for the bin + the earlier waves'
// + the earlier lanes' elements of the bin.  Arrival order holds inside every bin.
__global__ __launch_bounds__(kKeyThreads) void k_part_scatter(BatchScratch sc, uint32_t nseg, int lb,
                                                              uint64_t *__restrict__ out, int dbg) {
    __shared__ uint32_t gb[kPartBins];               // this segment's first position in each bin
    __shared__ uint16_t wc[kKeyWaves][kPartBins];    // per wave: counts, then prefixes over the waves
    // XCD-aware: consecutive blocks round-robin over the 8 XCDs, so block b takes segment (b % 8) * per + b / 8:
    // each XCD's workgroups take consecutive segments, whose elements of one bin are neighbours in the
    // output, so a 128-byte line is completed in one XCD's L2 instead of written back in pieces from all 8
    const uint32_t per = (nseg + 7) / 8;
    const uint32_t seg = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (seg >= nseg) return;
    const uint32_t g = seg / kPartGroup;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt64(lane);
    for (uint32_t b = threadIdx.x; b < (uint32_t)kPartBins; b += kKeyThreads) {
        gb[b] = sc.pstart[b] + sc.pgrp[(size_t)g * kPartBins + b] + sc.phist[(size_t)seg * kPartBins + b];
#pragma unroll
        for (int w = 0; w < kKeyWaves; ++w) wc[w][b] = 0;
    }
    const uint32_t sub = seg * kKeyWaves + wave;
    const uint32_t nc = sc.tile_nc[sub];
    const uint64_t *src = sc.el_tile + (size_t)sub * kSubSeg;
    uint64_t x[kSubRounds];
#pragma unroll
    for (int r = 0; r < kSubRounds; ++r) {
        const uint32_t i = (uint32_t)r * 64 + lane;
        x[r] = src[i < nc ? i : 0u];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSubRounds; ++r) {
        if ((uint32_t)r * 64 >= nc) break;  // wave-uniform
        const bool valid = (uint32_t)r * 64 + lane < nc;
        const uint32_t b = el_slot(x[r]) >> lb;
        const uint64_t peers = match_lanes(b, kPartBits, valid);
        if (valid && (peers & lt) == 0) wc[wave][b] += (uint16_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < (uint32_t)kPartBins; b += kKeyThreads) {
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < kKeyWaves; ++w) {
            const uint32_t c = wc[w][b];
            wc[w][b] = (uint16_t)run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSubRounds; ++r) {
        if ((uint32_t)r * 64 >= nc) break;
        const bool valid = (uint32_t)r * 64 + lane < nc;
        const uint32_t b = el_slot(x[r]) >> lb;
        const uint64_t peers = match_lanes(b, kPartBits, valid);
        if (valid && !(dbg & 32)) out[gb[b] + wc[wave][b] + (uint32_t)__popcll(peers & lt)] = x[r];  // 32: profiling
        __builtin_amdgcn_wave_barrier();
        if (valid && (peers & lt) == 0) wc[wave][b] += (uint16_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
}

// Dense flowId table (the production layout): 4 waves per SIMD, two workgroups per CU.  kPk: packed requests.
template <int kPass, bool kNT = false, bool kPk = false>
__global__ __launch_bounds__(kKeyThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_hot_key_dense(
    ClusterState st, BatchScratch sc, ReqIn in, int64_t ts_base, uint32_t n, uint64_t *__restrict__ out, int dbg,
    int d0, uint32_t *__restrict__ hist, uint32_t ntiles) {
    __shared__ KeyShared sh;
    hot_key<kPass, true, kNT, kPk>(sh, st, sc, in, ts_base, n, out, dbg, d0, hist, ntiles);
}
// Hashed flowId table (sparse flowIds): the probe loop needs more registers.
template <int kPass, bool kPk = false>
__global__ __launch_bounds__(kKeyThreads) void k_hot_key_hash(
    ClusterState st, BatchScratch sc, ReqIn in, int64_t ts_base, uint32_t n, uint64_t *__restrict__ out, int dbg,
    int d0, uint32_t *__restrict__ hist, uint32_t ntiles) {
    __shared__ KeyShared sh;
    hot_key<kPass, false, false, kPk>(sh, st, sc, in, ts_base, n, out, dbg, d0, hist, ntiles);
}

// The batch's path and element counts: sums over the compaction segments and the rank segments
// (one workgroup).
__global__ __launch_bounds__(1024) void k_hot_mode(BatchScratch sc, uint32_t nsub, uint32_t nseg, int64_t ts_base) {
    __shared__ uint32_t red[4][16];
    const uint32_t f = sc.counters[CTL_FLAGS];
    const uint32_t nhot = (f & (kFlagRerun | kFlagState)) ? 0u : hot_count(sc);
    uint32_t ns = 0, np = 0, bd = 0, tm = 0;
    for (uint32_t k = threadIdx.x; k < nsub; k += 1024) ns += sc.tile_nc[k];
    for (uint32_t k = threadIdx.x; k < nseg; k += 1024) {
        if (nhot) {
            np += sc.seg_stat[kSegStat * k];
            bd = max(bd, sc.seg_stat[kSegStat * k + 1]);
        }
        tm = max(tm, sc.seg_stat[kSegStat * k + 2]);
    }
    ns = wave_sum_u32(ns);
    np = wave_sum_u32(np);
    bd = wave_max_u32(bd);
    tm = wave_max_u32(tm);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = ns;
        red[1][threadIdx.x >> 6] = np;
        red[2][threadIdx.x >> 6] = bd;
        red[3][threadIdx.x >> 6] = tm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0, m = 0, t = 0;
        for (int w = 0; w < 16; ++w) {
            a += red[0][w];
            b += red[1][w];
            m = max(m, red[2][w]);
            t = max(t, red[3][w]);
        }
        // the latest request time of every batch classified so far (pipelined prechecks)
        atomicMax(sc.tmax_all, (unsigned long long)(ts_base + (int64_t)t));
        sc.counters[CTL_NSORT] = a;  // the compaction segments hold the cold elements only
        sc.counters[CTL_NPRIO] = b;
        sc.counters[CTL_NCOLD] = a;
        sc.counters[CTL_BDHI] = m;
        sc.counters[CTL_MODE] = nhot ? 1u : 0u;
    }
}

// Column prefix of the count rows over segments, in groups of kHotGroupRows rows.
__global__ __launch_bounds__(kThreads) void k_hscan_group(BatchScratch sc, uint32_t nrows) {
    if (!sc.counters[CTL_MODE]) return;
    const uint32_t h = blockIdx.y * kThreads + threadIdx.x;
    if (h >= hot_count(sc)) return;
    const uint32_t r0 = blockIdx.x * kHotGroupRows;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kHotGroupRows; ++k)
        if (r0 + k < nrows) s += sc.hcnt[(size_t)(r0 + k) * kHot + h];
    sc.hgsum[(size_t)blockIdx.x * kHot + h] = s;
}

__device__ __forceinline__ void psort_cols_one(const BatchScratch &sc, uint32_t h, uint32_t ngroups);
// pgroups > 0: also the prioritized sort's column prefix (k_psort_cols) for hot id h, so the hot side's chain has
// one launch fewer
__global__ __launch_bounds__(kThreads) void k_hscan_mid(BatchScratch sc, uint32_t ngroups, uint32_t pgroups) {
    if (!sc.counters[CTL_MODE]) return;
    const uint32_t h = blockIdx.x * kThreads + threadIdx.x;
    if (pgroups) psort_cols_one(sc, h, pgroups);
    if (h >= hot_count(sc)) return;
    uint32_t acc = 0;
#pragma unroll 8
    for (uint32_t g = 0; g < ngroups; ++g) {
        const uint32_t v = sc.hgsum[(size_t)g * kHot + h];
        sc.hgsum[(size_t)g * kHot + h] = acc;
        acc += v;
    }
    sc.hot_tot[h] = acc;
}

__global__ __launch_bounds__(kThreads) void k_hscan_down(BatchScratch sc, uint32_t nrows) {
    if (!sc.counters[CTL_MODE]) return;
    const uint32_t h = blockIdx.y * kThreads + threadIdx.x;
    if (h >= hot_count(sc)) return;
    const uint32_t r0 = blockIdx.x * kHotGroupRows;
    uint32_t v[kHotGroupRows];
#pragma unroll
    for (int k = 0; k < kHotGroupRows; ++k) v[k] = r0 + k < nrows ? sc.hcnt[(size_t)(r0 + k) * kHot + h] : 0u;
    uint32_t run = sc.hgsum[(size_t)blockIdx.x * kHot + h];
#pragma unroll
    for (int k = 0; k < kHotGroupRows; ++k) {
        if (r0 + k < nrows) sc.hbase[(size_t)(r0 + k) * kHot + h] = run;
        run += v[k];
    }
}

// ---- the prioritized hot requests sorted by hot id, arrival order kept: a counting sort over kHot keys (the
// elements are about 1 % of the hot requests).  kPsGroups groups of consecutive rank segments, one wave each.
//   counts  the key kernel adds each element to prow[group][hot id] as it writes it (no-return atomics);
//   cols    k_psort_cols: per hot id, the groups' exclusive prefix (pstart) and the total (ptot);
//   scatter k_psort_scatter: per group, the hot ids' starts (prefix of ptot) + pstart; the group's elements in
//           arrival order, each to start + its rank so far (per round: the lanes of one hot id found by ballots,
//           one LDS add by the lowest, ranks in lane order); it zeroes its prow row for the next batch.
// Small workgroups (one wave, 16 KB LDS): they run beside the cold stage's wide workgroups.
__device__ __forceinline__ uint32_t ps_per_group(uint32_t nseg) { return (nseg + kPsGroups - 1) / kPsGroups; }

__global__ __launch_bounds__(256) void k_psort_cols(BatchScratch sc, uint32_t ngroups) {
    if (!sc.counters[CTL_MODE]) return;
    psort_cols_one(sc, blockIdx.x * 256 + threadIdx.x, ngroups);
}
__device__ __forceinline__ void psort_cols_one(const BatchScratch &sc, uint32_t h, uint32_t ngroups) {
    uint32_t acc = 0;
    constexpr int kChunk = 64;  // loads in flight per lane
    for (uint32_t g0 = 0; g0 < ngroups; g0 += kChunk) {
        uint32_t v[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) v[k] = g0 + k < ngroups ? sc.prow[(size_t)(g0 + k) * kHot + h] : 0u;
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            if (g0 + k < ngroups) sc.ppre[(size_t)(g0 + k) * kHot + h] = acc;
            acc += v[k];
        }
    }
    sc.ptot[h] = acc;
}

__global__ __launch_bounds__(64) void k_psort_scatter(BatchScratch sc, uint32_t nseg, uint64_t *__restrict__ out, int dbg) {
    __shared__ uint32_t base[kHot];
    const uint32_t g = blockIdx.x;
    const int lane = threadIdx.x;
    const bool mode = sc.counters[CTL_MODE] != 0;
    if (mode) {  // the hot ids' starts: exclusive prefix of ptot (64 consecutive ids per lane) + this group's
        constexpr int kPer = kHot / 64;
        uint32_t sum = 0;
        for (int k = 0; k < kPer; ++k) sum += sc.ptot[lane * kPer + k];
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= o) x += y;
        }
        uint32_t pre = x - sum;
        if ((dbg & 512) && g == 0 && lane == 63 && x != sc.counters[CTL_NPRIO])
            printf("psort: total %u != CTL_NPRIO %u\n", x, sc.counters[CTL_NPRIO]);
        if (dbg & 512) {  // the group's row total against the elements its segments hold
            uint32_t rs = 0;
            for (uint32_t h = lane; h < (uint32_t)kHot; h += 64) rs += sc.prow[(size_t)g * kHot + h];
            uint32_t ws = 0;
            const uint32_t per = ps_per_group(nseg);
            const uint32_t s0 = min(nseg, g * per), s1 = min(nseg, s0 + per);
            for (uint32_t k = s0 + lane; k < s1; k += 64) ws += sc.seg_stat[kSegStat * k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                rs += (uint32_t)__shfl_xor((int)rs, o, 64);
                ws += (uint32_t)__shfl_xor((int)ws, o, 64);
            }
            if (lane == 0 && rs != ws) printf("psort: group %u row %u segments %u (segs %u..%u)\n", g, rs, ws, s0, s1);
        }
        for (int k = 0; k < kPer; ++k) {
            const uint32_t h = lane * kPer + k, t = sc.ptot[h];
            base[h] = pre + sc.ppre[(size_t)g * kHot + h];
            if (g == 0) {  // each hot id's range in the sorted region (k_prio_rank, k_hot_final)
                sc.plo[h] = pre;
                sc.phi[h] = pre + t;
            }
            pre += t;
        }
    }
    for (uint32_t h = lane; h < (uint32_t)kHot; h += 64) sc.prow[(size_t)g * kHot + h] = 0u;  // the next batch's counts
    if (!mode) return;
    __syncthreads();
    const uint32_t per = ps_per_group(nseg);
    const uint32_t s0 = min(nseg, g * per), s1 = min(nseg, s0 + per);
    for (uint32_t k0 = s0; k0 < s1; k0 += 64) {
        const uint32_t kn = min(64u, s1 - k0);
        const uint32_t c = (uint32_t)lane < kn ? sc.seg_stat[kSegStat * (k0 + lane)] : 0u;
        uint32_t inc = c;  // inclusive prefix over the segments
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += y;
        }
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        constexpr int kPre = 4;  // element loads in flight per lane
        for (uint32_t j0 = 0; j0 < tot; j0 += 64 * kPre) {
            uint64_t e[kPre];
#pragma unroll
            for (int q = 0; q < kPre; ++q) {
                const uint32_t j = j0 + (uint32_t)(q * 64 + lane);
                // the element's segment: the first lane whose inclusive prefix exceeds j (binary search)
                uint32_t lo = 0;
#pragma unroll
                for (uint32_t st = 32; st > 0; st >>= 1) {
                    const uint32_t probe = lo + st - 1;
                    const uint32_t v = (uint32_t)__shfl((int)inc, (int)min(probe, 63u), 64);
                    if (probe < kn && v <= j) lo += st;
                }
                // every lane takes part in the permute (a lane outside the active mask reads as 0)
                const uint32_t bprev = (uint32_t)__shfl((int)inc, (int)(lo ? lo - 1 : 0), 64);
                const uint32_t before = lo ? bprev : 0u;
                e[q] = j < tot ? sc.pel_tile[(size_t)(k0 + min(lo, kn - 1)) * kHotSeg + (j - before)] : 0ull;
            }
#pragma unroll
            for (int q = 0; q < kPre; ++q) {
                const uint32_t j = j0 + (uint32_t)(q * 64 + lane);
                // one LDS add per distinct hot id of the instruction (its lowest lane), ranks in lane order by
                // ballots: no reliance on the order same-address atomics of one instruction return in
                const bool v = j < tot;
                const uint32_t hid = v ? el_slot(e[q]) : 0u;
                const uint64_t peers = match_lanes(hid, 12, v);
                const int lead = peers ? __ffsll((unsigned long long)peers) - 1 : lane;
                uint32_t old = 0;
                if (v && lead == lane) old = atomicAdd(&base[hid], (uint32_t)__popcll(peers));
                old = (uint32_t)__shfl((int)old, lead, 64);
                if (v) out[old + (uint32_t)__popcll(peers & lanemask_lt64(lane))] = e[q];
            }
        }
    }
}

// debug (SGA_FZ_DEBUG & 512): each segment's prioritized elements lie in the segment, in arrival order; each
// group's per-hot-id counts equal the key kernel's
__global__ __launch_bounds__(64) void k_psort_dbgcount(BatchScratch sc, uint32_t nseg) {
    __shared__ uint32_t cnt[kHot];
    if (!sc.counters[CTL_MODE]) return;
    const uint32_t g = blockIdx.x;
    const int lane = threadIdx.x;
    for (uint32_t h = lane; h < (uint32_t)kHot; h += 64) cnt[h] = 0;
    __syncthreads();
    const uint32_t per = ps_per_group(nseg);
    const uint32_t s0 = min(nseg, g * per), s1 = min(nseg, s0 + per);
    int bad = 0;
    for (uint32_t sg = s0; sg < s1; ++sg) {
        const uint32_t c = sc.seg_stat[kSegStat * sg];
        for (uint32_t j = lane; j < c; j += 64) {
            const uint64_t e = sc.pel_tile[(size_t)sg * kHotSeg + j];
            atomicAdd(&cnt[el_slot(e)], 1u);
            const uint32_t i = el_idx(e);
            const bool in_seg = i / kHotSeg == sg;
            const bool ordered = j == 0 || el_idx(sc.pel_tile[(size_t)sg * kHotSeg + j - 1]) < i;
            if ((!in_seg || !ordered) && bad++ < 2)
                printf("psort seg %u: j %u of %u: idx %u slot %u in_seg %d ordered %d\n", sg, j, c, i, el_slot(e), in_seg, ordered);
        }
    }
    __syncthreads();
    for (uint32_t h = lane; h < (uint32_t)kHot; h += 64)
        if (cnt[h] != sc.prow[(size_t)g * kHot + h] && bad++ < 4)
            printf("psort group %u hot id %u: walked %u key kernel %u\n", g, h, cnt[h], sc.prow[(size_t)g * kHot + h]);
}

// debug (SGA_FZ_DEBUG & 512): the sorted region is ordered by (hot id, arrival)
__global__ void k_psort_verify(BatchScratch sc, const uint64_t *__restrict__ el) {
    if (!sc.counters[CTL_MODE]) return;
    const uint32_t np = sc.counters[CTL_NPRIO];
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x + 1; j < np; j += gridDim.x * blockDim.x) {
        const uint64_t a = el[j - 1], b = el[j];
        const bool ok = el_slot(a) < el_slot(b) || (el_slot(a) == el_slot(b) && el_idx(a) < el_idx(b));
        if (!ok) printf("psort order: j %u: (%u,%u) then (%u,%u) of %u\n", j, el_slot(a), el_idx(a), el_slot(b), el_idx(b), np);
    }
}

// Rank of each prioritized hot request (sorted region: hot id major, arrival order within) and each
// hot id's range in the region.
__global__ __launch_bounds__(kThreads) void k_prio_rank(ClusterState st, BatchScratch sc,
                                                        const uint64_t *__restrict__ el) {
    if (!sc.counters[CTL_MODE]) return;
    const uint32_t np = sc.counters[CTL_NPRIO], base = 0;
    for (uint32_t j = blockIdx.x * kThreads + threadIdx.x; j < np; j += gridDim.x * kThreads) {
        const uint64_t e = el[base + j];
        const uint32_t h = el_slot(e);
        const uint32_t r_in = (((uint32_t)(e >> kBdShift) & kBdEsc) << 7) | (uint32_t)((e >> kAcqShift) & kAcqMax);
        const uint32_t seg = el_idx(e) / (uint32_t)kHotSeg;
        sc.prank[j] = sc.hbase[(size_t)seg * kHot + h] + r_in;
        if (j == 0 || el_slot(el[base + j - 1]) != el_slot(e)) sc.plo[h] = j;
        if (j + 1 == np || el_slot(el[base + j + 1]) != el_slot(e)) sc.phi[h] = j + 1;
    }
}

// First index in [lo, hi) with a[index] >= key (a ascending), the whole wave searching: 64 probes
// per step.
__device__ __forceinline__ uint32_t wave_lower_bound(const uint32_t *__restrict__ a, uint32_t lo, uint32_t hi,
                                                     uint32_t key, int lane) {
    while (hi - lo > 64) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t idx = lo + (uint32_t)lane * step;
        const bool below = idx < hi && a[idx] < key;
        const uint32_t k = (uint32_t)__popcll(__ballot(below));  // probes 0..k-1 are below the key
        if (k == 0) return lo;
        const uint32_t nlo = lo + (k - 1) * step + 1;
        hi = min(hi, lo + k * step);
        lo = nlo;
    }
    const uint32_t idx = lo + (uint32_t)lane;
    const bool below = idx < hi && a[idx] < key;
    return lo + (uint32_t)__popcll(__ballot(below));
}

// One wave per hot rule: its runs in bucket order, each with the closed form of run_fast (the S
// window buckets are read by S lanes, the sums are wave reductions, the decisions are uniform
// scalar arithmetic, lane 0 stores the bucket).
// Hot run records, bucket-major: a bucket's runs of consecutive hot ids are adjacent, so
// k_hot_final's cache fill (the hottest ids' runs of two buckets) reads contiguous records.
__device__ __forceinline__ HotRun *hrun_at(const BatchScratch &sc, uint32_t h, uint32_t b) {
    return sc.hrun + (size_t)b * kHot + h;
}

__global__ __launch_bounds__(kThreads) void k_hot_flows(ClusterState st, BatchScratch sc, int64_t ts_base) {
    // Beside the cold stage every dependent load waits the loaded latency, so the loads that do not
    // depend on each other are issued together, before any early exit, at clamped (valid) indices.
    const int lane = threadIdx.x & 63;
    const uint32_t h = blockIdx.x * kH1Waves + (threadIdx.x >> 6);  // < kHot
    const uint32_t mode = sc.counters[CTL_MODE], nhot = hot_count(sc);
    const uint32_t bd_lo = sc.counters[CTL_BDLO];
    const uint32_t bd_hi = min(sc.counters[CTL_BDHI], (uint32_t)kHotBuckets - 1);
    const uint32_t tot = sc.hot_tot[h];
    const uint32_t s_raw = sc.hot_slot[h];
    const uint32_t plo = sc.plo[h], phi = max(sc.phi[h], plo);
    const uint32_t s = s_raw < st.nslots ? s_raw : 0u;  // ids past the hot count hold stale slots
    SlotParam P;
    if (st.uni_S) {  // uniform geometry (ClusterState::uni_S): the record loads need no parameter load
        P.S = st.uni_S;
        P.W = st.uni_W;
        P.interval = st.uni_iv;
        P.isec = st.uni_iv / 1000.0;
        P.boff = s * rec_units(st.uni_S);
        P.thr = st.param[s].thr;
        P.thr_simple = P.thr;
        P.active = 1;
        P.ns = 0;
    } else {
        P = st.param[s];
    }
    if (!mode || h >= nhot) return;
    const uint32_t nb = bd_hi >= bd_lo ? bd_hi - bd_lo + 1 : 0;
    const bool bl = (uint32_t)lane < nb && lane > 0;
    const uint32_t bq = min(bd_lo + (uint32_t)lane, (uint32_t)kHotBuckets - 1);
    const uint32_t Pq = sc.hbnd[bq];  // the bucket's first request
    const uint32_t Pc = bl ? Pq : 0u;
    const uint32_t hb = sc.hbase[(size_t)(Pc / kHotSeg) * kHot + h];
    const uint32_t hp = sc.hpre[(size_t)bq * kHot + h];
    const uint32_t stb = bl ? hb + ((Pc % kHotSeg) ? hp : 0u) : 0u;
    uint32_t stn = wave_shl1(stb, 0u);
    if ((uint32_t)lane + 1 == nb) stn = tot;
    const uint32_t nrun = (uint32_t)lane < nb ? stn - stb : 0u;
    if ((uint32_t)lane < nb && nrun == 0) {
        HotRun z{};
        z.start = stb;
        *hrun_at(sc, h, bd_lo + lane) = z;
        sc.hfin[(size_t)(bd_lo + lane) * kHot + h] = make_uint4(0u, 0u, 0u, stb);
        sc.hfs[(size_t)(bd_lo + lane) * kHot + h] = make_uint2(0u, stb);
    }
    uint64_t rm = __ballot(nrun > 0);
    if (!rm) return;
    const Rec R = rec_of(st, P);
    const double thr = P.thr;
    if (lane == 0) sc.hthr[h] = make_double2(thr, P.isec);
    const int64_t qbase = div_pos(ts_base, P.W);
    const uint32_t *pr = sc.prank;
    const int jl = min(lane, P.S - 1);   // bucket lane (clamped: the loads stay unconditional)
    const int kl = min(lane, CEV_N - 1);  // counter lane
    while (rm) {
        const int lb = __builtin_ctzll(rm);
        rm &= rm - 1;
        const uint32_t j0 = lane_u32(stb, lb);
        const uint32_t n = lane_u32(nrun, lb);
        const uint32_t b = bd_lo + (uint32_t)lb;
        // window of the run's bucket (cluster rules: interval = S x W, so validity is the same for
        // any time in the bucket and the bucket start stands in for the request times)
        const int64_t q = qbase + (int64_t)b;
        const int64_t ws = q * P.W;
        const int64_t t0 = ws;
        const int64_t qs = div_pos(q, P.S);
        const int cj = (int)(q - qs * P.S);
        const int jh = cj + 1 == P.S ? 0 : cj + 1;
        const int64_t w_ld = R.start(jl), pv_ld = R.cnt(CEV_PASS, jl);
        const int64_t cl_ld = R.cnt(kl, cj);
        const SlotOcc o_ld = R.occ();
        const uint32_t p0 = plo < phi ? wave_lower_bound(pr, plo, phi, j0, lane) : plo;
        const uint32_t p1 = plo < phi ? wave_lower_bound(pr, p0, phi, j0 + n, lane) : plo;
        const uint32_t cp_tot = p1 - p0;
        const int64_t w = lane < P.S ? w_ld : kAbsent, pv = lane < P.S ? pv_ld : 0;
        const bool valid_b = lane < P.S && lane != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval);
        const int64_t bp = wave_sum_i64(valid_b ? pv : 0);
        const int64_t old = lane_i64(w, cj);
        const int64_t hstart = lane_i64(w, jh), hpass = lane_i64(pv, jh);
        bool ok = !(old != kAbsent && ws < old);
        const bool rot = old == kAbsent || ws > old;
        int64_t cl = 0;  // lane k < CEV_N: counter k of the current bucket after the rotation
        SlotOcc o{0, 0, 0, 0};
        bool occ_dirty = false;
        if (!rot && lane < CEV_N) cl = cl_ld;
        if (rot && old != kAbsent) {  // resetWindowTo + transferOccupyToBucket
            o = o_ld;
            if (o.has_occ) {
                if (lane == CEV_OCCUPIED_PASS || lane == CEV_PASS) cl += o.occ_pass;
                if (lane == CEV_PASS_REQUEST) cl += o.occ_preq;
                o.occ_pass = 0;
                o.occ_preq = 0;
                o.has_occ = 0;
                occ_dirty = true;
            }
        }
        const int64_t cpass = lane_i64(cl, CEV_PASS);
        const int64_t head = jh == cj ? cpass : ((hstart != kAbsent && !(t0 - hstart > (int64_t)P.interval)) ? hpass : 0);
        const int64_t s0 = bp + cpass;
        const uint32_t f = pass_prefix(thr, P.isec, s0, 1, n);
        uint32_t cpf = cp_tot;
        if (f < n && cp_tot > 0) cpf = wave_lower_bound(pr, p0, p1, j0 + f, lane) - p0;
        const uint32_t np_after = cp_tot - cpf;
        uint32_t cw = 0;
        if (np_after > 0) {
            const int64_t wt = (lane < P.S && valid_b) ? R.cnt(CEV_WAITING, lane) : 0;
            const int64_t w0 = lane_i64(cl, CEV_WAITING) + wave_sum_i64(wt);
            if (!(rot && old != kAbsent)) o = o_ld;  // not taken by the rotation above
            const double latest = div_isec((double)(s0 + (int64_t)f), P.isec);
            const double lim = st.max_occupy_ratio * thr;
            const int64_t occ0 = o.occ_pass;
            uint32_t l2 = 0, h2 = np_after;
            while (l2 < h2) {
                const uint32_t cc = l2 + ((h2 - l2) >> 1);
                const int64_t add = (int64_t)cc;
                const bool fits = (div_isec((double)(w0 + add), P.isec) <= lim) &&
                                  (latest + (double)(1 + occ0 + add) - (double)head <= thr);
                if (fits) l2 = cc + 1;
                else h2 = cc;
            }
            cw = l2;
            if (cw > 0) {
                o.occ_pass += (int64_t)cw;
                o.occ_preq += cw;
                o.has_occ = 1;
                occ_dirty = true;
            }
        }
        const uint32_t nblk = n - f - cw;
        if (lane == CEV_PASS) cl += (int64_t)f;
        if (lane == CEV_PASS_REQUEST) cl += f;
        if (lane == CEV_OCCUPIED_PASS) cl += (int64_t)cpf;
        if (lane == CEV_WAITING) cl += (int64_t)cw;
        if (lane == CEV_BLOCK) cl += (int64_t)nblk;
        if (lane == CEV_BLOCK_REQUEST) cl += nblk;
        if (lane == CEV_OCCUPIED_BLOCK) cl += (int64_t)(np_after - cw);
        if (ok) {
            if (lane < CEV_N) R.cnt(lane, cj) = cl;
            // the header's cached group follows (the cold closed form reads it when the rule turns cold)
            if (lane > 0 && lane < CEV_N) R.cache()[lane == CEV_WAITING ? 0 : lane] = cl;
            if (lane == 0) {
                if (rot) R.start(cj) = ws;
                if (occ_dirty) R.occ() = o;
                R.tag() = ws;
            }
        } else if (lane == 0) {
            atomicAdd(&sc.counters[CTL_HOTERR], 1u);
        }
        if (lane == 0) {
            HotRun r{};
            r.s0 = s0;
            r.thr = thr;
            r.isec = P.isec;
            r.f = f;
            r.start = j0;
            r.n = n;
            r.p0 = p0;
            r.cpf = cpf;
            r.cw = cw;
            r.wait = (uint16_t)(1000 / P.S);
            r.ok = ok ? 1 : 0;
            *hrun_at(sc, h, b) = r;
            sc.hfin[(size_t)b * kHot + h] = make_uint4((uint32_t)s0, (uint32_t)((uint64_t)s0 >> 32), f, j0);
            sc.hfs[(size_t)b * kHot + h] = make_uint2(f, j0);
        }
    }
}

// TokenResults of the prioritized hot requests (the sorted elements past the cold ones): the
// first workgroups of k_hot_final (no launch of its own on the hot side's critical path).
__device__ __forceinline__ void prio_results_range(const ClusterState &st, const BatchScratch &sc,
                                                   const uint64_t *__restrict__ el, uint64_t *__restrict__ out,
                                                   uint32_t j0, uint32_t stride) {
    const uint32_t np = sc.counters[CTL_NPRIO];
    const uint32_t bd_lo = sc.counters[CTL_BDLO];
    const uint32_t bd_hi = min(sc.counters[CTL_BDHI], (uint32_t)kHotBuckets - 1);
    for (uint32_t j = j0; j < np; j += stride) {
        const uint64_t e = el[j];
        const uint32_t h = el_slot(e);
        const uint32_t rank = sc.prank[j];
        uint32_t b = bd_lo;
        for (; b < bd_hi; ++b)
            if (rank - hrun_at(sc, h, b)->start < hrun_at(sc, h, b)->n) break;
        const HotRun hr = *hrun_at(sc, h, b);
        const uint32_t local = rank - hr.start;
        uint64_t res;
        if (local < hr.f) {
            const int64_t sum = hr.s0 + (int64_t)local;
            res = pack_result(TRS_OK, j_d2i(hr.thr - div_isec((double)sum, hr.isec) - 1.0), 0);
        } else if (j - hr.p0 - hr.cpf < hr.cw) {
            res = pack_result(TRS_SHOULD_WAIT, 0, (int32_t)hr.wait);
        } else {
            res = pack_result(TRS_BLOCKED, 0, 0);
        }
        out[el_idx(e)] = res;
    }
}


// TokenResults of the non-prioritized hot requests, in input order: one 16-wave workgroup per rank
// segment (its base row in LDS), kFinChunk rounds per wave.  The runs of the kFinCache hottest ids
// (k_hot_pick numbers them first) in the segment's first two buckets are staged in LDS; a lane whose
// run is staged still issues its gather, pointed at one shared line, so the loads stay unconditional.
constexpr int kFinChunk = 8;
#ifndef SGA_FIN_CACHE_N
#define SGA_FIN_CACHE_N 1024
#endif
constexpr uint32_t kFinCache = SGA_FIN_CACHE_N;
constexpr int kFinWgThreads = 1024;
constexpr int kFinWaves = kFinWgThreads / 64;
constexpr uint32_t kFinSpan = kHotSeg / kFinWaves;  // requests per wave
static_assert(kFinSpan == kFinChunk * 64, "one chunk per wave");
__device__ __forceinline__ int64_t i64_of(uint32_t lo, uint32_t hi) {
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double f64_of(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// The first kFinPrioWgs workgroups answer the prioritized hot requests, the rest one segment each.
constexpr uint32_t kFinPrioWgs = 32;
__global__ __launch_bounds__(kFinWgThreads) void k_hot_final(ClusterState st, BatchScratch sc, uint32_t n,
                                                             const uint64_t *__restrict__ el,
                                                             uint64_t *__restrict__ out, uint32_t cache_cap) {
    __shared__ uint32_t base[kHot];
    __shared__ double2 c_ti[kFinCache];      // thr, isec
    __shared__ int64_t c_s0[2][kFinCache];   // s0 of the runs in buckets b0, b0 + 1
    __shared__ uint2 c_fs[2][kFinCache];     // (f, start) of those runs
    __shared__ uint32_t s_b0;
    if (!sc.counters[CTL_MODE]) return;
    if (blockIdx.x < kFinPrioWgs) {  // dispatched first, so they overlap the segments
        prio_results_range(st, sc, el, out, blockIdx.x * kFinWgThreads + threadIdx.x, kFinPrioWgs * kFinWgThreads);
        return;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t seg = blockIdx.x - kFinPrioWgs;
    const uint32_t sbase = seg * kHotSeg;
    const uint32_t nhot = hot_count(sc);
    const uint32_t wbase = sbase + (uint32_t)wave * kFinSpan;
    uint32_t cn[kFinChunk];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) cn[u] = sc.hcode[min(wbase + (uint32_t)u * 64 + lane, n - 1)];
    if (wave == 0) {  // the segment's first bucket: the smallest among its first 64 codes
        uint32_t bk = (cn[0] >> 31) ? 0xFFu : (cn[0] >> 25);
        bk = wave_min_u32(bk);
        if (lane == 0) s_b0 = bk == 0xFFu ? sc.counters[CTL_BDLO] : bk;
    }
    for (uint32_t h = threadIdx.x; h < nhot; h += kFinWgThreads) base[h] = sc.hbase[(size_t)seg * kHot + h];
    __syncthreads();
    const uint32_t b0 = s_b0;
    const uint32_t ncache = min(nhot, cache_cap);
    for (uint32_t h = threadIdx.x; h < ncache; h += kFinWgThreads) {
        c_ti[h] = sc.hthr[h];
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
            const uint32_t b = min(b0 + k, (uint32_t)kHotBuckets - 1);
            const uint4 fr = sc.hfin[(size_t)b * kHot + h];  // contiguous over h
            c_s0[k][h] = i64_of(fr.x, fr.y);
            c_fs[k][h] = make_uint2(fr.z, fr.w);
        }
    }
    __syncthreads();
    const uint32_t wend = min(n, wbase + kFinSpan);
    if (wbase >= wend) return;
    uint32_t code[kFinChunk];
    bool hit[kFinChunk];
    uint4 ra[kFinChunk], rb[kFinChunk];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {
        const uint32_t i = wbase + u * 64 + lane;
        code[u] = (i < wend && !(cn[u] >> 31)) ? cn[u] : kNoCode;  // prioritized: prio_results_range
        const uint32_t cd = code[u];
        hit[u] = cd == kNoCode || ((cd & 0xFFFu) < cache_cap && (cd >> 25) - b0 < 2u);
        const uint4 *hp = reinterpret_cast<const uint4 *>(hit[u] ? sc.hrun : hrun_at(sc, cd & 0xFFFu, cd >> 25));
        ra[u] = hp[0];  // s0, thr
        rb[u] = hp[1];  // isec, f, start
    }
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {
        const uint32_t cd = code[u];
        if (cd == kNoCode) continue;
        const uint32_t h = cd & 0xFFFu, k = ((cd >> 25) - b0) & 1u;
        int64_t s0;
        double thr, isec;
        uint32_t f, st0;
        if (hit[u]) {
            s0 = c_s0[k][h];
            const double2 ti = c_ti[h];
            thr = ti.x;
            isec = ti.y;
            const uint2 fs = c_fs[k][h];
            f = fs.x;
            st0 = fs.y;
        } else {
            s0 = i64_of(ra[u].x, ra[u].y);
            thr = f64_of(ra[u].z, ra[u].w);
            isec = f64_of(rb[u].x, rb[u].y);
            f = rb[u].z;
            st0 = rb[u].w;
        }
        const uint32_t local = base[h] + ((cd >> 12) & 0x1FFFu) - st0;
        uint64_t res;
        if (local < f) {
            const int64_t sum = s0 + (int64_t)local;
            res = pack_result(TRS_OK, j_d2i(thr - div_isec((double)sum, isec) - 1.0), 0);
        } else {
            res = pack_result(TRS_BLOCKED, 0, 0);
        }
        out[wbase + u * 64 + lane] = res;
    }
}

// k_hot_final without LDS (the default; SGA_FIN_LDS=1 selects the LDS form above): every hot request
// gathers its rank base (hbase row of its segment) and its run record (hrun, a few hundred KB, L2-resident)
// directly.  Beside the cold stage, whose two workgroups per CU hold nearly all of the LDS, a kernel that
// needs no LDS still finds room on every CU.  Four waves of kFinChunk x 64 requests per workgroup; the
// first kFinPrioWgsG workgroups answer the prioritized hot requests.
constexpr uint32_t kFinPrioWgsG = 64;
constexpr int kFinGThreads = 256;
constexpr uint32_t kFinGSpan = kFinGThreads * kFinChunk;  // requests per workgroup
__global__ __launch_bounds__(kFinGThreads) void k_hot_final_g(ClusterState st, BatchScratch sc, uint32_t n,
                                                              const uint64_t *__restrict__ el,
                                                              uint64_t *__restrict__ out) {
    if (!sc.counters[CTL_MODE]) return;
    if (blockIdx.x < kFinPrioWgsG) {
        prio_results_range(st, sc, el, out, blockIdx.x * kFinGThreads + threadIdx.x, kFinPrioWgsG * kFinGThreads);
        return;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wbase = (blockIdx.x - kFinPrioWgsG) * kFinGSpan + (uint32_t)wave * (kFinChunk * 64);
    if (wbase >= n) return;
    uint32_t code[kFinChunk], bs[kFinChunk];
    uint4 ra[kFinChunk], rb[kFinChunk];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) code[u] = sc.hcode[min(wbase + (uint32_t)u * 64 + lane, n - 1)];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {  // unconditional gathers (a non-hot lane reads hot id 0's entries)
        const uint32_t i = min(wbase + (uint32_t)u * 64 + lane, n - 1);
        const uint32_t cd = code[u];
        const bool hot = cd != kNoCode && !(cd >> 31);
        const uint32_t h = hot ? (cd & 0xFFFu) : 0u, b = hot ? (cd >> 25) : 0u;
        bs[u] = sc.hbase[(size_t)(i / kHotSeg) * kHot + h];
        const uint4 *hp = reinterpret_cast<const uint4 *>(hrun_at(sc, h, b));
        ra[u] = hp[0];  // s0, thr
        rb[u] = hp[1];  // isec, f, start
    }
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {
        const uint32_t i = wbase + (uint32_t)u * 64 + lane;
        const uint32_t cd = code[u];
        if (i >= n || cd == kNoCode || (cd >> 31)) continue;  // cold, invalid or prioritized
        const int64_t s0 = i64_of(ra[u].x, ra[u].y);
        const double thr = f64_of(ra[u].z, ra[u].w), isec = f64_of(rb[u].x, rb[u].y);
        const uint32_t local = bs[u] + ((cd >> 12) & 0x1FFFu) - rb[u].w;
        uint64_t res;
        if (local < rb[u].z) {
            const int64_t sum = s0 + (int64_t)local;
            res = pack_result(TRS_OK, j_d2i(thr - div_isec((double)sum, isec) - 1.0), 0);
        } else {
            res = pack_result(TRS_BLOCKED, 0, 0);
        }
        out[i] = res;
    }
}

// k_hot_final_h (A/B knob SGA_FIN_H=1): as k_hot_final_g, with the segment's rank base row staged in LDS (16 KB, one
// coalesced fill per 2048 requests) and the fate of every hot request from its run's (f, start) alone (one 8-byte
// gather): most hot requests are blocked.  Only the passing ones read the run's window sum and the rule's
// threshold / interval, through buffer loads whose out-of-range offset (every other lane) returns 0 without a
// memory access, all issued together.
__global__ __launch_bounds__(kFinGThreads) void k_hot_final_h(ClusterState st, BatchScratch sc, uint32_t n,
                                                              const uint64_t *__restrict__ el,
                                                              uint64_t *__restrict__ out) {
    __shared__ uint32_t base[kHot];
    if (!sc.counters[CTL_MODE]) return;
    if (blockIdx.x < kFinPrioWgsG) {
        prio_results_range(st, sc, el, out, blockIdx.x * kFinGThreads + threadIdx.x, kFinPrioWgsG * kFinGThreads);
        return;
    }
    static_assert(kHotSeg % kFinGSpan == 0, "a workgroup's span lies in one rank segment");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wg0 = (blockIdx.x - kFinPrioWgsG) * kFinGSpan;
    if (wg0 >= n) return;
    const uint32_t nhot = hot_count(sc);
    {
        const uint32_t *row = sc.hbase + (size_t)(wg0 / kHotSeg) * kHot;
        for (uint32_t h = threadIdx.x; h < nhot; h += kFinGThreads) base[h] = row[h];
    }
    const uint32_t wbase = wg0 + (uint32_t)wave * (kFinChunk * 64);
    uint32_t code[kFinChunk];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) code[u] = sc.hcode[min(wbase + (uint32_t)u * 64 + lane, n - 1)];
    uint2 fs[kFinChunk];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {  // unconditional gathers (a non-hot lane reads hot id 0's)
        const uint32_t cd = code[u];
        const bool hot = cd != kNoCode && !(cd >> 31);
        fs[u] = sc.hfs[(size_t)(hot ? (cd >> 25) : 0u) * kHot + (hot ? (cd & 0xFFFu) : 0u)];
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        sc.hrun, 0, (int)((size_t)kHot * kHotBuckets * sizeof(HotRun)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(sc.hthr, 0, (int)(kHot * sizeof(double2)),
                                                                        0x00020000);
    constexpr uint32_t kOob = 0x80000000u;  // past both buffers: the load returns 0, touches nothing
    uint32_t local[kFinChunk];
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x2 s0v[kFinChunk];
    u32x4 tiv[kFinChunk];
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {
        const uint32_t i = wbase + (uint32_t)u * 64 + lane;
        const uint32_t cd = code[u];
        const bool hot = i < n && cd != kNoCode && !(cd >> 31);
        const uint32_t h = cd & 0xFFFu;
        local[u] = base[hot ? h : 0u] + ((cd >> 12) & 0x1FFFu) - fs[u].y;
        const bool pass = hot && local[u] < fs[u].x;
        const uint32_t ro = pass ? (uint32_t)(((cd >> 25) * (uint32_t)kHot + h) * sizeof(HotRun)) : kOob;
        const uint32_t to = pass ? h * (uint32_t)sizeof(double2) : kOob;
        s0v[u] = __builtin_amdgcn_raw_buffer_load_b64(rr, ro, 0, 0);
        tiv[u] = __builtin_amdgcn_raw_buffer_load_b128(rt, to, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kFinChunk; ++u) {
        const uint32_t i = wbase + (uint32_t)u * 64 + lane;
        const uint32_t cd = code[u];
        if (i >= n || cd == kNoCode || (cd >> 31)) continue;  // cold, invalid or prioritized
        uint64_t res;
        if (local[u] < fs[u].x) {
            const int64_t s0 = (int64_t)(((uint64_t)s0v[u].y << 32) | s0v[u].x);
            const double thr = __longlong_as_double((long long)(((uint64_t)tiv[u].y << 32) | tiv[u].x));
            const double isec = __longlong_as_double((long long)(((uint64_t)tiv[u].w << 32) | tiv[u].z));
            const int64_t sum = s0 + (int64_t)local[u];
            res = pack_result(TRS_OK, j_d2i(thr - div_isec((double)sum, isec) - 1.0), 0);
        } else {
            res = pack_result(TRS_BLOCKED, 0, 0);
        }
        out[i] = res;
    }
}

// k_hot_final_p (A/B knob SGA_FIN_P=1; measured slower than k_hot_final_g beside the cold stage, 0.78 against
// 0.74-0.76 ms per C3 batch): persistent workgroups over
// consecutive rank segments.  A workgroup stages (f, start) of every hot id's run in its first segment's bucket
// (hfs, 32 KB) once, and each segment's hbase row (16 KB) in LDS, so a hot request's fate -- pass (rank inside
// the run's pass prefix) or block -- costs two LDS reads; only the passing requests (and any request of another
// bucket) gather their run record, after the fate pass, all such gathers of a wave's 16 rounds in flight together.
constexpr int kFinPThreads = 512;
constexpr int kFinPRounds = kHotSeg / kFinPThreads;  // codes per thread per segment (16)
constexpr uint32_t kFinPrioWgsP = 32;
__global__ __launch_bounds__(kFinPThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_hot_final_p(ClusterState st, BatchScratch sc, uint32_t n,
                                                             const uint64_t *__restrict__ el,
                                                             uint64_t *__restrict__ out, uint32_t segs_per_wg) {
    __shared__ uint2 fs[kHot];       // (f, start) of each hot id's run in bucket b0
    __shared__ uint32_t base[kHot];  // the segment's rank base per hot id
    if (!sc.counters[CTL_MODE]) return;
    if (blockIdx.x < kFinPrioWgsP) {
        prio_results_range(st, sc, el, out, blockIdx.x * kFinPThreads + threadIdx.x, kFinPrioWgsP * kFinPThreads);
        return;
    }
    const uint32_t nseg = (n + kHotSeg - 1) / kHotSeg;
    const uint32_t seg0 = (blockIdx.x - kFinPrioWgsP) * segs_per_wg, seg1 = min(nseg, seg0 + segs_per_wg);
    if (seg0 >= seg1) return;
    const uint32_t nhot = hot_count(sc);
    // b0: the bucket holding the first request of seg0 (bucket starts hbnd[b], b in (bd_lo, bd_hi])
    const uint32_t bd_lo = sc.counters[CTL_BDLO];
    const uint32_t bd_hi = min(sc.counters[CTL_BDHI], (uint32_t)kHotBuckets - 1);
    uint32_t b0 = bd_lo;
    for (uint32_t b = bd_lo + 1; b <= bd_hi; ++b)
        if (sc.hbnd[b] <= seg0 * (uint32_t)kHotSeg) b0 = b;
    for (uint32_t h = threadIdx.x; h < nhot; h += kFinPThreads) fs[h] = sc.hfs[(size_t)b0 * kHot + h];
    uint32_t cn[kFinPRounds];
    auto load_codes = [&](uint32_t seg) {
#pragma unroll
        for (int u = 0; u < kFinPRounds; ++u)
            cn[u] = sc.hcode[min(seg * (uint32_t)kHotSeg + (uint32_t)u * kFinPThreads + threadIdx.x, n - 1)];
    };
    load_codes(seg0);
    for (uint32_t seg = seg0; seg < seg1; ++seg) {
        __syncthreads();  // the previous segment's base reads are done (and fs is in place)
        for (uint32_t h = threadIdx.x; h < nhot; h += kFinPThreads) base[h] = sc.hbase[(size_t)seg * kHot + h];
        __syncthreads();
        uint32_t code[kFinPRounds];
#pragma unroll
        for (int u = 0; u < kFinPRounds; ++u) code[u] = cn[u];
        if (seg + 1 < seg1) load_codes(seg + 1);  // the next segment's codes in flight during this one
        // per half of the rounds: the fate pass (blocked requests answered from LDS), then the gathers of the
        // passing requests (and of requests of another bucket), all in flight together, then their results
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            constexpr int kH = kFinPRounds / 2;
            uint32_t need = 0, loc[kH];
#pragma unroll
            for (int v = 0; v < kH; ++v) {
                const int u = hf * kH + v;
                const uint32_t i = seg * (uint32_t)kHotSeg + (uint32_t)u * kFinPThreads + threadIdx.x;
                const uint32_t cd = code[u];
                loc[v] = 0;
                if (i >= n || cd == kNoCode || (cd >> 31)) continue;  // cold, invalid, prioritized: answered elsewhere
                const uint32_t h = cd & 0xFFFu;
                const uint32_t r = base[h] + ((cd >> 12) & 0x1FFFu);
                if ((cd >> 25) != b0) {
                    need |= 1u << v;
                    loc[v] = r;
                    continue;
                }
                const uint2 w = fs[h];
                loc[v] = r - w.y;
                if (loc[v] < w.x) need |= 1u << v;
                else out[i] = pack_result(TRS_BLOCKED, 0, 0);
            }
            if (!__ballot(need != 0)) continue;  // wave-uniform: every hot request of these rounds blocked
            uint4 ra[kH], rb[kH];
#pragma unroll
            for (int v = 0; v < kH; ++v) {  // unconditional gathers (lanes without a need read one shared line)
                const uint32_t cd = code[hf * kH + v];
                const bool nd = (need >> v) & 1u;
                const uint4 *hp = reinterpret_cast<const uint4 *>(nd ? hrun_at(sc, cd & 0xFFFu, cd >> 25) : sc.hrun);
                ra[v] = hp[0];  // s0, thr
                rb[v] = hp[1];  // isec, f, start
            }
#pragma unroll
            for (int v = 0; v < kH; ++v) {
                if (!((need >> v) & 1u)) continue;
                const int u = hf * kH + v;
                const uint32_t i = seg * (uint32_t)kHotSeg + (uint32_t)u * kFinPThreads + threadIdx.x;
                const uint32_t cd = code[u];
                const uint32_t local = (cd >> 25) != b0 ? loc[v] - rb[v].w : loc[v];
                uint64_t res;
                if (local < rb[v].z) {
                    const int64_t sum = i64_of(ra[v].x, ra[v].y) + (int64_t)local;
                    res = pack_result(TRS_OK, j_d2i(f64_of(ra[v].z, ra[v].w) - (double)sum / f64_of(rb[v].x, rb[v].y) - 1.0),
                                      0);
                } else {
                    res = pack_result(TRS_BLOCKED, 0, 0);
                }
                out[i] = res;
            }
        }
    }
}

// ---- next batch's hot set: rules with at least T requests in this batch, T the smallest power of
// two (>= hot_min) that admits at most kHot rules; all of them with the window length of the
// busiest one, 1 < sampleCount <= 64 (the occupy path needs 1000 / sampleCount > 0).  Candidates:
// the cold rules k_cold_fused saw with at least hot_min requests, and (hot-path batches) the hot
// rules.
__device__ __forceinline__ bool hot_eligible(const SlotParam &P) { return P.S > 1 && P.S <= 64 && P.active; }

__device__ __forceinline__ uint32_t hot_ncand(const BatchScratch &sc, uint32_t &ncold) {
    ncold = min(sc.hot_ctl[6], (uint32_t)kHotCand);
    return ncold + (sc.counters[CTL_MODE] ? hot_count(sc) : 0u);
}

// (a rule's parameters are read only when its count can make it hot)
__device__ __forceinline__ bool hot_candidate(const ClusterState &st, const BatchScratch &sc, uint32_t i,
                                              uint32_t ncold, uint32_t hot_min, uint32_t &slot, uint32_t &count) {
    if (i < ncold) {
        slot = sc.hot_cand[2 * i];
        count = sc.hot_cand[2 * i + 1];
    } else {
        count = sc.hot_tot[i - ncold];
        slot = sc.hot_slot[i - ncold];
    }
    if (count < hot_min || count == 0) return false;
    return hot_eligible(st.param[slot]);
}

__device__ __forceinline__ void hot_hist_body(const ClusterState &st, const BatchScratch &sc, uint32_t hot_min) {
    __shared__ uint32_t bins[32];
    __shared__ unsigned long long best;
    if (threadIdx.x < 32) bins[threadIdx.x] = 0;
    if (threadIdx.x == 0) best = 0;
    __syncthreads();
    uint32_t ncold;
    const uint32_t ncand = hot_ncand(sc, ncold);
    unsigned long long mine = 0;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < ncand; i += gridDim.x * kThreads) {
        uint32_t slot, c;
        if (!hot_candidate(st, sc, i, ncold, hot_min, slot, c)) continue;
        atomicAdd(&bins[31 - __clz(c)], 1u);
        mine = max(mine, ((unsigned long long)c << 32) | slot);
    }
    if (mine) atomicMax(&best, mine);
    __syncthreads();
    if (threadIdx.x < 32 && bins[threadIdx.x]) atomicAdd(&sc.hot_ctl[8 + threadIdx.x], bins[threadIdx.x]);
    if (threadIdx.x == 0 && best) atomicMax(reinterpret_cast<unsigned long long *>(sc.hot_ctl + 4), best);
}

__global__ __launch_bounds__(kThreads) void k_hot_hist(ClusterState st, BatchScratch sc, uint32_t hot_min) {
    hot_hist_body(st, sc, hot_min);
}

// the key table entry of a rule entering (v = hot id) or leaving (kColdId) the hot set
__device__ __forceinline__ void hot_fid_set(const ClusterState &st, uint32_t slot, uint16_t v) {
    if (!st.dense_n || !st.dkey) return;
    const int64_t f = st.slot_fid[slot];
    if (f >= 1 && f <= (int64_t)st.dense_n) st.dkey[f - 1] = v == kColdId ? st.dense[f - 1] : (kDkHot | v);
}

__global__ __launch_bounds__(kThreads) void k_hot_clear(ClusterState st, BatchScratch sc) {
    const uint32_t h = blockIdx.x * kThreads + threadIdx.x;
    if (h < hot_count(sc)) {
        const uint32_t slot = sc.hot_slot[h];
        sc.hot_of[slot] = kColdId;
        hot_fid_set(st, slot, kColdId);
    }
}

// Hot ids go out in descending count-bin order (bin b holds counts in [2^b, 2^(b+1))): each bin
// owns a block of ids, so after k_hot_fin compacts the holes left by rules of another window
// length, the hottest rules have the smallest ids (k_hot_final caches the first kFinCache of them).
__device__ __forceinline__ void hot_pick_body(const ClusterState &st, const BatchScratch &sc, uint32_t hot_min) {
    __shared__ uint32_t thr, wbest, bcnt[32], bbase[32], lcnt[32], gbase[32];
    if (threadIdx.x < 32) bcnt[threadIdx.x] = sc.hot_ctl[8 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t cum = 0, t = 0xFFFFFFFFu;
        for (int b = 31; b >= 0; --b) {
            bbase[b] = cum;
            cum += bcnt[b];
            if (cum <= (uint32_t)kHot) t = 1u << b;
        }
        thr = max(t, max(hot_min, 1u));
        if (blockIdx.x == 0) sc.hot_ctl[7] = thr;  // next batch's candidate floor is half of it
        const unsigned long long best = *reinterpret_cast<const unsigned long long *>(sc.hot_ctl + 4);
        wbest = best ? (uint32_t)st.param[(uint32_t)best].W : 0u;
    }
    __syncthreads();
    if (!wbest) return;
    uint32_t ncold;
    const uint32_t ncand = hot_ncand(sc, ncold);
    for (uint32_t r0 = blockIdx.x * kThreads; r0 < ncand; r0 += gridDim.x * kThreads) {  // uniform per block
        if (threadIdx.x < 32) lcnt[threadIdx.x] = 0;
        __syncthreads();
        const uint32_t i = r0 + threadIdx.x;
        uint32_t slot = 0, c = 0, lo = 0;
        int b = -1;
        if (i < ncand && hot_candidate(st, sc, i, ncold, thr, slot, c) && (uint32_t)st.param[slot].W == wbest) {
            b = 31 - __clz(c);
            lo = atomicAdd(&lcnt[b], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 32 && lcnt[threadIdx.x]) gbase[threadIdx.x] = atomicAdd(&sc.hot_ctl[64 + threadIdx.x], lcnt[threadIdx.x]);
        __syncthreads();
        if (b >= 0) {
            const uint32_t hid = bbase[b] + gbase[b] + lo;
            if (hid < (uint32_t)kHot) {
                sc.hot_next[hid] = slot;
                sc.hot_of[slot] = (uint16_t)hid;
                hot_fid_set(st, slot, (uint16_t)hid);
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_hot_pick(ClusterState st, BatchScratch sc, uint32_t hot_min) {
    hot_pick_body(st, sc, hot_min);
}

// Compacts the picked ids (stable, so the count-bin order stays) and publishes them.  Holes are
// left only by candidates of another window length; a rule whose id moves is renamed here.
constexpr int kFinThreads = 1024;
template <int kNT>
__device__ __forceinline__ void hot_fin_body(const ClusterState &st, const BatchScratch &sc, uint32_t *wsum) {
    constexpr int kFinPer = kHot / kNT;
    constexpr int kFinThreads = kNT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t sl[kFinPer], cnt = 0;
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
        sl[k] = sc.hot_next[threadIdx.x * kFinPer + k];
        cnt += sl[k] != kNoSlot;
    }
    uint32_t inc = cnt;  // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(inc, d);
        if (lane >= d) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < kFinThreads / 64; ++w) {
        off += w < wave ? wsum[w] : 0u;
        tot += wsum[w];
    }
    uint32_t hid = off + inc - cnt;
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
        const uint32_t at = threadIdx.x * kFinPer + k;
        if (sl[k] == kNoSlot) continue;
        sc.hot_slot[hid] = sl[k];
        if (hid != at) {
            sc.hot_of[sl[k]] = (uint16_t)hid;
            hot_fid_set(st, sl[k], (uint16_t)hid);
        }
        sc.hot_next[at] = kNoSlot;
        ++hid;
    }
    if (threadIdx.x == 0) {
        const unsigned long long best = *reinterpret_cast<const unsigned long long *>(sc.hot_ctl + 4);
        sc.hot_ctl[2] = best ? (uint32_t)st.param[(uint32_t)best].W : 1u;
        sc.hot_ctl[0] = tot;
        sc.hot_ctl[4] = 0;
        sc.hot_ctl[5] = 0;
        sc.hot_ctl[6] = 0;  // the next batch's candidates
    }
    if (threadIdx.x < 32) {
        sc.hot_ctl[8 + threadIdx.x] = 0;
        sc.hot_ctl[64 + threadIdx.x] = 0;
    }
    if (threadIdx.x < CTL_WORDS) {  // the batch's control words for sga_cluster_batch_info; the next batch starts clear
        sc.counters_last[threadIdx.x] = sc.counters[threadIdx.x];
        sc.counters[threadIdx.x] = 0;
    }
}

__global__ __launch_bounds__(kFinThreads) void k_hot_fin(ClusterState st, BatchScratch sc) {
    __shared__ uint32_t wsum[kFinThreads / 64];
    hot_fin_body<kFinThreads>(st, sc, wsum);
}

// The next hot set in three launches (default: k_hot_next_a, k_hot_pick, k_hot_fin), or two (SGA_HOT_NEXT=2, an
// A/B knob; 4 keeps the four kernels above):
// k_hot_next_a = k_hot_hist + k_hot_clear (the clear only has to precede the picks); k_hot_next_b =
// k_hot_pick, then the last workgroup to finish runs k_hot_fin (a done counter in hot_ctl).
constexpr int kHotNextDone = 100;  // hot_ctl word: k_hot_next_b workgroups done
__global__ __launch_bounds__(kThreads) void k_hot_next_a(ClusterState st, BatchScratch sc, uint32_t hot_min) {
    const uint32_t nh = hot_count(sc);
    for (uint32_t h = blockIdx.x * kThreads + threadIdx.x; h < nh; h += gridDim.x * kThreads) {
        const uint32_t slot = sc.hot_slot[h];
        sc.hot_of[slot] = kColdId;
        hot_fid_set(st, slot, kColdId);
    }
    hot_hist_body(st, sc, hot_min);
}

__global__ __launch_bounds__(kThreads) void k_hot_next_b(ClusterState st, BatchScratch sc, uint32_t hot_min) {
    __shared__ uint32_t wsum[kThreads / 64];
    __shared__ uint32_t s_last;
    hot_pick_body(st, sc, hot_min);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&sc.hot_ctl[kHotNextDone], 1u) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    hot_fin_body<kThreads>(st, sc, wsum);
    if (threadIdx.x == 0) sc.hot_ctl[kHotNextDone] = 0;
}

__global__ void k_hot_reset(ClusterState st, BatchScratch sc, uint32_t nslots_cap) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nslots_cap; i += gridDim.x * blockDim.x)
        sc.hot_of[i] = kColdId;
    if (st.dkey)
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < st.dense_n; i += gridDim.x * blockDim.x)
            st.dkey[i] = st.dense[i] == ~0u ? kDkNone : st.dense[i];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)kHot; i += gridDim.x * blockDim.x)
        sc.hot_next[i] = kNoSlot;
    if (blockIdx.x == 0 && threadIdx.x < kHotCtlWords) sc.hot_ctl[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *sc.tmax_all = 0;  // no batch in flight (callers have joined)
        sc.pstart[kPartBins + 1] = 0;  // k_part_binscan's done counter
    }
}

__global__ void k_metric_sums(ClusterState st, uint32_t s, int64_t now, int64_t *out7) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const SlotParam P = st.param[s];
    cur_window(st, P, s, now);
    for (int k = 0; k < CEV_N; ++k) out7[k] = values_sum(st, P, now, k);
}

// ClusterMetricNodeGenerator.flowToMetricNode (CS/flow/statistic/ClusterMetricNodeGenerator.java:75-91):
// getAvg(BLOCK) then getAvg(PASS), each rotating the current window first.
__global__ __launch_bounds__(kThreads) void k_cluster_nodes(ClusterState st, const int64_t *__restrict__ slot_fid,
                                                            int64_t now, sga_cluster_metric_node *out, uint32_t cap,
                                                            uint32_t *count) {
    __shared__ uint32_t wbase[kThreads / 64];
    __shared__ uint32_t base;
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    const bool act = s < st.nslots && st.param[s].active;
    sga_cluster_metric_node m{};
    if (act) {
        const SlotParam P = st.param[s];
        m.flow_id = slot_fid[s];
        // getAvg(BLOCK) rotates the current window; getAvg(PASS)'s rotation at the same time is then
        // a no-op, so one rotation and one pass over the buckets give both sums
        cur_window(st, P, s, now);
        const Rec R = rec_of(st, P);
        int64_t sb = 0, sp = 0;
        if (P.S <= 10) {  // unconditional loads (clamped index), issued together
            int4 pr[10];
            int64_t bl[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                const int jj = min(j, P.S - 1);
                pr[j] = reinterpret_cast<const int4 *>(R.r)[jj];
                bl[j] = R.cnt(CEV_BLOCK, jj);
            }
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                const int64_t w = i64_lo(pr[j]);
                if (j < P.S && w != kAbsent && !(now - w > (int64_t)P.interval)) {
                    sp += i64_hi(pr[j]);
                    sb += bl[j];
                }
            }
        } else {
            sb = values_sum(st, P, now, CEV_BLOCK);
            sp = values_sum(st, P, now, CEV_PASS);
        }
        m.block_qps = (double)sb / P.isec;
        m.pass_qps = (double)sp / P.isec;
        m.timestamp = now;
    }
    // one reservation per workgroup (a same-address atomic per node would serialize the kernel)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t bm = __ballot(act);
    if (lane == 0) wbase[wave] = (uint32_t)__popcll(bm);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kThreads / 64; ++w) {
            const uint32_t c = wbase[w];
            wbase[w] = t;
            t += c;
        }
        base = t ? atomicAdd(count, t) : 0u;
    }
    __syncthreads();
    if (act) {
        const uint32_t k = base + wbase[wave] + (uint32_t)__popcll(bm & lanemask_lt64(lane));
        if (k < cap) out[k] = m;
    }
}

__global__ void k_init_slots(ClusterState st, const uint32_t *slots, uint32_t n) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slots[i];
    const SlotParam P = st.param[s];
    const Rec R = rec_of(st, P);
    for (int j = 0; j < P.S; ++j) {
        R.start(j) = kAbsent;
        bucket_zero(R, j);
    }
    R.occ() = SlotOcc{0, 0, 0, 0};
    R.tag() = kAbsent;
    R.thr() = P.thr;
}

__global__ void k_rec_thr(ClusterState st, uint32_t n) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= n) return;
    const SlotParam P = st.param[s];
    if (P.S <= 0) return;  // not allocated (its parameters are zero, its boff is no record)
    rec_of(st, P).thr() = P.thr;
}


// ---------------------------------------------------------------- namespace limiter (K9)
// ClusterFlowChecker.allowProceed -> GlobalRequestLimiter.tryPass(namespace) runs before the
// rule's metric is touched (CS/flow/ClusterFlowChecker.java:50-60), for every valid request
// whose rule lives in a limited namespace, in arrival order.  The limiter depends only on that
// arrival stream, so it is resolved as a pre-pass: the namespace's requests are compacted in
// arrival order and cut into runs of one 100 ms limiter bucket.  Inside a run the other nine
// buckets are fixed (the run rotates only its own bucket), so the passes of a run are a prefix
// whose length is found by binary search over the exact predicate
//   sum / 1.0 + 1 <= qpsAllowed     (RequestLimiter.canPass, :70-72)
// One thread walks the runs in order; rejected requests get TOO_MANY_REQUEST and leave the batch.
constexpr int kLimW = 100, kLimN = 10, kLimInterval = 1000;

template <class RuleParam>
__global__ __launch_bounds__(kThreads) void k_lim_flag(const RuleParam *param, const uint64_t *__restrict__ el,
                                                       uint32_t n, uint32_t invalid, int32_t ns,
                                                       uint32_t *__restrict__ flag) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = el_slot(el[i]);
    flag[i] = (k != invalid && param[k].ns == ns) ? 1u : 0u;
}

__global__ __launch_bounds__(kThreads) void k_lim_compact(const uint32_t *__restrict__ flag,
                                                          const uint32_t *__restrict__ pos, uint32_t n,
                                                          uint32_t *__restrict__ list, uint32_t *counters) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    if (flag[i]) list[pos[i]] = i;
    if (i == n - 1) counters[4] = pos[i] + flag[i];
}

__global__ __launch_bounds__(kThreads) void k_lim_heads(const uint32_t *__restrict__ list,
                                                        const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                        uint32_t n, const uint32_t *counters,
                                                        uint32_t *__restrict__ head) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= n) return;
    const uint32_t m = counters[4];
    uint32_t h = 0;
    if (j < m) {
        const int64_t b = (ts_base + (int64_t)ts_off[list[j]]) / kLimW;
        h = (j == 0 || b != (ts_base + (int64_t)ts_off[list[j - 1]]) / kLimW) ? 1u : 0u;
    }
    head[j] = h;
}

__global__ __launch_bounds__(kThreads) void k_lim_starts(const uint32_t *__restrict__ head,
                                                         const uint32_t *__restrict__ ridx, uint32_t n,
                                                         uint32_t *counters, uint32_t *__restrict__ rstart) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t m = counters[4];
    if (j >= m || j >= n) return;
    if (head[j]) rstart[ridx[j]] = j;
    if (j == m - 1) counters[5] = ridx[j] + head[j];
}

__global__ void k_lim_walk(NsLimiterDev *L, double qps_allowed, const uint32_t *__restrict__ list,
                           const uint32_t *__restrict__ rstart, const uint32_t *counters,
                           const uint32_t *__restrict__ ts_off, int64_t ts_base, uint32_t *__restrict__ rpass) {
    if (threadIdx.x || blockIdx.x) return;
    const uint32_t m = counters[4], R = counters[5];
    for (uint32_t r = 0; r < R && m; ++r) {
        const uint32_t j0 = rstart[r], j1 = r + 1 < R ? rstart[r + 1] : m;
        const int64_t nr = (int64_t)(j1 - j0);
        const int64_t t = ts_base + (int64_t)ts_off[list[j0]];
        const int idx = (int)((t / kLimW) % kLimN);
        const int64_t ws = t - t % kLimW;
        bool detached = false;
        if (L->start[idx] == kAbsent || ws > L->start[idx]) {  // new bucket / resetWindowTo
            L->start[idx] = ws;
            L->cnt[idx] = 0;
        } else if (ws < L->start[idx]) {
            detached = true;  // clock went back: a fresh detached bucket per call, adds lost
        }
        int64_t others = 0;
        for (int k = 0; k < kLimN; ++k) {
            if (!detached && k == idx) continue;
            if (L->start[k] != kAbsent && !(t - L->start[k] > kLimInterval)) others += L->cnt[k];
        }
        int64_t pass;
        if (detached) {
            pass = ((double)others / 1.0 + 1 <= qps_allowed) ? nr : 0;
        } else {
            const int64_t c0 = L->cnt[idx];
            int64_t lo = 0, hi = nr;
            while (lo < hi) {
                const int64_t mid = lo + ((hi - lo) >> 1);
                if ((double)(others + c0 + mid) / 1.0 + 1 <= qps_allowed) lo = mid + 1;
                else hi = mid;
            }
            pass = lo;
            L->cnt[idx] = c0 + pass;
        }
        rpass[r] = (uint32_t)pass;
    }
}

__global__ __launch_bounds__(kThreads) void k_lim_apply(const uint32_t *__restrict__ list,
                                                        const uint32_t *__restrict__ head,
                                                        const uint32_t *__restrict__ ridx,
                                                        const uint32_t *__restrict__ rstart,
                                                        const uint32_t *__restrict__ rpass, const uint32_t *counters,
                                                        uint32_t n, uint32_t invalid, uint64_t *__restrict__ el,
                                                        uint64_t *__restrict__ out) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t m = counters[4];
    if (j >= m || j >= n) return;
    const uint32_t r = ridx[j] + head[j] - 1;
    if (j - rstart[r] >= rpass[r]) {
        const uint32_t i = list[j];
        el[i] = (uint64_t)invalid << kSlotShift;
        out[i] = pack_result(TRS_TOO_MANY_REQUEST, 0, 0);
    }
}

__global__ void k_lim_init(NsLimiterDev *L) {
    const int k = threadIdx.x;
    if (k < kLimN) {
        L->start[k] = kAbsent;
        L->cnt[k] = 0;
    }
}

// ================================================================ cluster parameter flow (a26)
// DefaultTokenService.requestParamToken -> ClusterParamFlowChecker.acquireClusterToken over
// ClusterParamMetric (CS/flow/DefaultTokenService.java:52-64, CS/flow/ClusterParamFlowChecker.java:37-120,
// CS/flow/statistic/metric/ClusterParamMetric.java:52-88, ClusterParameterLeapArray.java:39-49).
//
// A key (rule, value) holds [stamp x S][count x S]; the rule holds the LeapArray starts.  When a
// rule's calls arrive in non-decreasing time (tmax before the batch <= every call, batch ascending)
// and every request names one value, the rule-level rotation by other values' calls never
// changes a key's sum (a stamp the rule start has moved past is already deprecated at the later
// call, LeapArray.isWindowDeprecated), so keys are independent and each (key, bucket) run is
// solved in closed form like a ClusterFlowChecker run.  Otherwise the rule's requests are
// replayed one by one against the rule-level starts (k_pslow), as are, from the batch their key count
// passes the bucket maps' capacity on, the rules whose maps may have to evict (cparam_exact.hpp, LRU mode).
// Both paths keep every key's last access stamp per bucket, which orders the maps when a rule switches.
// kErrKeys / kErrPool, prule_lookup, prule_threshold, vid_of, key_of: cparam_exact.hpp

// Stage 1a: validation (DefaultTokenService.notValidRequest || params empty -> BAD_REQUEST,
// :54-56), rule lookup (NO_RULE_EXISTS), sequential-path triggers.
__global__ __launch_bounds__(kThreads) void k_pcls(CParamState st, const int64_t *__restrict__ flow_id,
                                                   const int32_t *__restrict__ acquire,
                                                   const uint32_t *__restrict__ voff, int64_t ts_base,
                                                   const uint32_t *__restrict__ ts_off, uint32_t n,
                                                   uint32_t invalid_key, uint64_t *__restrict__ el,
                                                   uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const int64_t f = flow_id[i];
    const int32_t a = acquire[i];
    const uint32_t k = voff[i + 1] - voff[i];
    if (i > 0 && ts_off[i] < ts_off[i - 1]) st.ctl[3] = 1;  // not ascending: everything sequential
    if (f <= 0 || a <= 0 || k == 0) {
        out[i] = pack_result(TRS_BAD_REQUEST, 0, 0);
        el[i] = (uint64_t)invalid_key << kSlotShift;
        return;
    }
    const uint32_t slot = prule_lookup(st, f);
    if (slot == 0xFFFFFFFFu || !st.param[slot].active) {
        out[i] = pack_result(TRS_NO_RULE_EXISTS, 0, 0);
        el[i] = (uint64_t)invalid_key << kSlotShift;
        return;
    }
    // sequential path for the rule: several values, time before the rule's last call, or a
    // request the packed element cannot carry (acquire > 127, bucket delta >= 63)
    const int64_t t = ts_base + (int64_t)ts_off[i];
    const int32_t W = st.param[slot].W;
    if (k > 1 || t < st.tmax[slot] || a > (int32_t)kAcqMax || t / W - ts_base / W >= (int64_t)kBdEsc)
        st.coupled[slot] = 1;
    el[i] = ((uint64_t)slot << kSlotShift) | i;
}

// Stage 1b (after the limiter): every value of an admitted request gets its key.
__global__ __launch_bounds__(kThreads) void k_pkeys(CParamState st, const uint64_t *__restrict__ el,
                                                    const uint32_t *__restrict__ voff,
                                                    const int64_t *__restrict__ values, uint32_t n,
                                                    uint32_t invalid_key, uint32_t *__restrict__ vkey) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = el_slot(el[i]);
    if (slot == invalid_key) return;
    for (uint32_t v = voff[i]; v < voff[i + 1]; ++v) {
        const int64_t x = values[v];
        const uint32_t vid = vid_of(st, x, true);
        vkey[v] = vid == 0xFFFFFFFFu ? 0xFFFFFFFFu : key_of(st, slot, vid, x, true);
        if (vid == 0xFFFFFFFFu) atomicOr(&st.ctl[1], kErrKeys);
    }
}

// Stage 1c: path choice.  Key-parallel element (kidx in the slot field) or sequential element.
__global__ __launch_bounds__(kThreads) void k_ppath(CParamState st, uint64_t *__restrict__ el,
                                                    uint64_t *__restrict__ els, const uint32_t *__restrict__ voff,
                                                    const uint32_t *__restrict__ vkey, const int32_t *__restrict__ acquire,
                                                    int64_t ts_base, const uint32_t *__restrict__ ts_off, uint32_t n,
                                                    uint32_t invalid_key, uint32_t key_invalid) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = el_slot(el[i]);
    uint64_t fast = (uint64_t)key_invalid << kSlotShift, slow = (uint64_t)invalid_key << kSlotShift;
    if (slot != invalid_key) {
        const PRuleParam &Ps = st.param[slot];
        if (st.ctl[3] || st.coupled[slot] || st.pq[Ps.boff] != kPNoQueue || st.nkeys[slot] > Ps.cap) {
            slow = ((uint64_t)slot << kSlotShift) | i;
            atomicAdd(&st.ctl[2], 1u);
        } else {
            const uint32_t kidx = vkey[voff[i]];
            const PRuleParam &P = st.param[slot];
            const int32_t a = acquire[i];
            const int64_t bd = div_pos(ts_base + (int64_t)ts_off[i], P.W) - div_pos(ts_base, P.W);
            uint32_t a7 = (a >= 1 && a <= (int32_t)kAcqMax) ? (uint32_t)a : 0u;
            uint32_t bd6 = (uint32_t)bd;
            if (bd >= (int64_t)kBdEsc) {
                bd6 = kBdEsc;
                a7 = 0;
            }
            fast = el_pack(kidx, bd6, 0, a7, i);
        }
    }
    el[i] = fast;
    els[i] = slow;
}

// pm_window / pm_key_sum: cparam_exact.hpp

// Sequential path: one lane per rule replays its requests in arrival order.
__global__ __launch_bounds__(kThreads) void k_pslow(CParamState st, BatchScratch sc, const uint64_t *__restrict__ els,
                                                    const int32_t *__restrict__ acquire,
                                                    const uint32_t *__restrict__ voff,
                                                    const int64_t *__restrict__ values,
                                                    const uint32_t *__restrict__ vkey, int64_t ts_base,
                                                    const uint32_t *__restrict__ ts_off, uint64_t *__restrict__ out) {
    const uint32_t nflows = sc.counters[2];
    const uint32_t nruns = sc.counters[1];
    const uint32_t nvalid = sc.counters[0];
    for (uint32_t fl = blockIdx.x * kThreads + threadIdx.x; fl < nflows; fl += gridDim.x * kThreads) {
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t j0 = sc.run_start[r0], j1 = r1 < nruns ? sc.run_start[r1] : nvalid;
        const uint32_t slot = sc.run_slot[r0];
        const PRuleParam P = st.param[slot];
        int64_t tmax = st.tmax[slot];
        for (uint32_t j = j0; j < j1; ++j) {
            const uint32_t i = el_idx(els[j]);
            const int64_t t = ts_base + (int64_t)ts_off[i];
            const int32_t a = acquire[i];
            const uint32_t v0 = voff[i], v1 = voff[i + 1];
            double remaining = -1;
            bool passed = true;
            for (uint32_t v = v0; v < v1; ++v) {  // ClusterParamFlowChecker.java:61-71
                const uint32_t kidx = vkey[v];
                pm_window(st, P, t);
                const int64_t sum =
                    kidx == 0xFFFFFFFFu ? 0 : pm_key_sum_access(st, P, kidx, t, pstamp(st, i, min(v - v0, 0x7FFFu)));
                const double next = prule_threshold(st, P, values[v]) - (double)sum / P.isec - (double)a;
                remaining = next;
                if (next < 0) {
                    passed = false;
                    break;
                }
            }
            if (passed) {  // addValue for every value (:73-76)
                for (uint32_t v = v0; v < v1; ++v) {
                    const int idx = pm_window(st, P, t);
                    const uint32_t kidx = vkey[v];
                    if (idx < 0 || kidx == 0xFFFFFFFFu) continue;
                    pm_key_add(st, P, kidx, idx, a, pstamp(st, i, kPAddLow | min(v - v0, 0x7FFFu)));
                }
            }
            if (v1 - v0 > 1) remaining = -1;
            out[i] = passed ? pack_result(TRS_OK, j_d2i(remaining), 0) : pack_result(TRS_BLOCKED, 0, 0);
            tmax = t > tmax ? t : tmax;
        }
        st.tmax[slot] = tmax;
        st.coupled[slot] = 0;
    }
}

// Key-parallel path: one lane per key walks its (key, bucket) runs in time order.  Per run: the
// key's lazily rotated window sum, the pass prefix over the exact predicate
//   threshold - sum / intervalInSecond - count >= 0      (ClusterParamFlowChecker.java:62-66)
// (blocked requests add nothing, so the prefix is the whole answer), the bucket count, and the
// rule-level start / tmax raised to this run's bucket and time.
__global__ __launch_bounds__(kThreads) void k_pflows(CParamState st, BatchScratch sc, const uint64_t *__restrict__ el,
                                                     const int32_t *__restrict__ acquire, int64_t ts_base,
                                                     const uint32_t *__restrict__ ts_off, uint64_t *__restrict__ out) {
    const uint32_t nflows = sc.counters[2];
    const uint32_t nruns = sc.counters[1];
    const uint32_t nvalid = sc.counters[0];
    for (uint32_t fl = blockIdx.x * kThreads + threadIdx.x; fl < nflows; fl += gridDim.x * kThreads) {
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t kidx = sc.run_slot[r0];
        const uint32_t slot = st.kslot[kidx];
        const PRuleParam P = st.param[slot];
        const double thr = prule_threshold(st, P, st.kval[kidx]);
        int64_t *rec = st.krec + st.koff[kidx];
        uint32_t j0 = sc.run_start[r0];
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t j1 = r + 1 < nruns ? sc.run_start[r + 1] : nvalid;
            const uint32_t n = j1 - j0;
            const int32_t a = sc.run_acq[r];  // common acquire count, 0 = mixed
            RunOut ro;
            const int64_t t0 = ts_base + (int64_t)ts_off[sc.run_idx0[r]];
            const int64_t q = t0 / P.W;
            const int64_t ws = q * P.W;
            const int cj = (int)(q % P.S);
            int64_t s0 = 0;
            for (int j = 0; j < P.S; ++j) {
                const int64_t stp = rec[j];
                if (stp == kAbsent || t0 - stp > (int64_t)P.interval) continue;
                if (j == cj && stp != ws) continue;  // the current bucket was reset
                s0 += rec[P.S + j];
            }
            const bool held = rec[cj] == ws;  // the key is in the current bucket's map
            const int64_t cur = held ? rec[P.S + cj] : 0;
            uint32_t f = 0;
            int64_t added = 0;
            bool last_pass;
            if (a > 0) {
                f = pass_prefix(thr, P.isec, s0, a, n);
                added = (int64_t)f * a;
                last_pass = f == n;
            } else {  // mixed acquire counts: request by request on the same lazily rotated sum
                last_pass = false;
                for (uint32_t j = j0; j < j1; ++j) {
                    const uint32_t i = el_idx(el[j]);
                    const int32_t ai = acquire[i];
                    const double next = thr - (double)(s0 + added) / P.isec - (double)ai;
                    last_pass = next >= 0;
                    if (next >= 0) {
                        added += ai;
                        out[i] = pack_result(TRS_OK, j_d2i(next), 0);
                    } else {
                        out[i] = pack_result(TRS_BLOCKED, 0, 0);
                    }
                }
            }
            // last access stamps: every request's getSum reads the valid buckets holding the key, a pass
            // adds to the current one; per bucket the run's last such access
            const uint32_t il = el_idx(el[j1 - 1]);
            const int64_t tl = ts_base + (int64_t)ts_off[il];
            for (int j = 0; j < P.S; ++j) {
                if (j == cj) continue;
                const int64_t stp = rec[j];
                if (stp == kAbsent || t0 - stp > (int64_t)P.interval) continue;
                uint32_t ia = il;
                if (tl - stp > (int64_t)P.interval) {  // valid for a prefix of the run only
                    uint32_t lo = j0, hi = j1 - 1;     // last request with t - stp <= interval
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi + 1) >> 1;
                        if (ts_base + (int64_t)ts_off[el_idx(el[mid])] - stp <= (int64_t)P.interval) lo = mid;
                        else hi = mid - 1;
                    }
                    ia = el_idx(el[lo]);
                }
                rec[2 * P.S + j] = (int64_t)pstamp(st, ia, 0);
            }
            if (held || added > 0) {
                rec[cj] = ws;
                rec[P.S + cj] = cur + added;
                rec[2 * P.S + cj] = (int64_t)pstamp(st, il, last_pass ? kPAddLow : 0u);
            }
            atomicMax((long long *)&st.rstart[P.boff + cj], (long long)ws);
            atomicMax((long long *)&st.tmax[slot], (long long)tl);
            ro.s0 = s0;
            ro.thr = thr;
            ro.isec = P.isec;
            ro.f = f;
            ro.cpf = 0;
            ro.cw = 0;
            ro.wait = 0;
            ro.mode = a > 0 ? RUN_FAST : RUN_DONE;
            sc.run_out[r] = ro;
            j0 = j1;
        }
    }
}

__global__ void k_psum(CParamState st, uint32_t slot, int64_t value, int64_t now, int64_t *out) {
    if (threadIdx.x || blockIdx.x) return;
    const PRuleParam P = st.param[slot];
    pm_window(st, P, now);
    const uint32_t vid = vid_of(st, value, false);
    const uint32_t kidx = vid == 0xFFFFFFFFu ? 0xFFFFFFFFu : key_of(st, slot, vid, value, false);
    *out = kidx == 0xFFFFFFFFu ? 0 : pm_key_sum_access(st, P, kidx, now, pstamp(st, 0, 0));
}

// ClusterParamMetric.getTopValues(number), CS/flow/statistic/metric/ClusterParamMetric.java:90-133:
// currentWindow(), per value the sum over the valid buckets, the `number` largest (ties: smaller
// value key first -- the reference's order among equal counts is its HashMap's iteration order).
__global__ void k_pwindow(CParamState st, uint32_t slot, int64_t now) {
    if (threadIdx.x || blockIdx.x) return;
    pm_window(st, st.param[slot], now);
}

// every key of the rule with a positive sum -> (count, value) appended to `list`
__global__ __launch_bounds__(kThreads) void k_ptop_collect(CParamState st, uint32_t slot, int64_t now,
                                                           int64_t *list, uint32_t *count) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k > st.kmask || st.ktab[k] == 0 || st.kslot[k] != slot) return;
    const PRuleParam P = st.param[slot];
    const int64_t s = pm_key_sum(st, P, st.krec + st.koff[k], now);
    if (s <= 0) return;
    const uint32_t at = atomicAdd(count, 1u);
    list[2 * at] = s;
    list[2 * at + 1] = st.kval[k];
}

__device__ __forceinline__ bool top_before(int64_t c1, int64_t v1, int64_t c2, int64_t v2) {
    return c1 > c2 || (c1 == c2 && v1 < v2);
}

// `number` rounds of a block-wide arg-max over the collected list, each strictly after the last pick
__global__ __launch_bounds__(1024) void k_ptop_select(CParamState st, uint32_t slot, const int64_t *list,
                                                      const uint32_t *count, uint32_t number, int64_t *out_val,
                                                      double *out_qps, uint32_t *n_out) {
    __shared__ int64_t sc[1024], sv[1024];
    const uint32_t m = *count;
    const double isec = st.param[slot].isec;
    int64_t lc = INT64_MAX, lv = INT64_MIN;
    uint32_t got = 0;
    for (uint32_t r = 0; r < number; ++r) {
        int64_t bc = -1, bv = 0;
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
            const int64_t c = list[2 * i], v = list[2 * i + 1];
            if (top_before(lc, lv, c, v) && top_before(c, v, bc, bv)) {
                bc = c;
                bv = v;
            }
        }
        sc[threadIdx.x] = bc;
        sv[threadIdx.x] = bv;
        __syncthreads();
        for (uint32_t o = blockDim.x / 2; o > 0; o >>= 1) {
            if (threadIdx.x < o && top_before(sc[threadIdx.x + o], sv[threadIdx.x + o], sc[threadIdx.x], sv[threadIdx.x])) {
                sc[threadIdx.x] = sc[threadIdx.x + o];
                sv[threadIdx.x] = sv[threadIdx.x + o];
            }
            __syncthreads();
        }
        bc = sc[0];
        bv = sv[0];
        __syncthreads();
        if (bc <= 0) break;  // fewer values than `number`
        if (threadIdx.x == 0) {
            out_val[r] = bv;
            out_qps[r] = (double)bc / isec;
        }
        lc = bc;
        lv = bv;
        ++got;
    }
    if (threadIdx.x == 0) *n_out = got;
}

__global__ void k_pinit_rule(CParamState st, uint32_t slot) {
    const PRuleParam P = st.param[slot];
    for (int j = threadIdx.x; j < P.S; j += blockDim.x) {
        st.rstart[P.boff + j] = kAbsent;
        st.pq[P.boff + j] = kPNoQueue;
        st.psize[P.boff + j] = 0;
    }
    if (threadIdx.x == 0) {
        st.tmax[slot] = INT64_MIN;
        st.coupled[slot] = 0;
        st.nkeys[slot] = 0;
    }
}

// ---- CacheMap capacity: the switch to LRU mode (cparam_exact.hpp)
// 1. rules in free mode whose key count passed their capacity (only then can a bucket map overflow)
__global__ __launch_bounds__(kThreads) void k_plru_decide(CParamState st) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= st.nslots) return;
    const PRuleParam &P = st.param[s];
    if (P.S <= 0 || !P.active || st.pq[P.boff] != kPNoQueue || st.nkeys[s] <= P.cap) return;
    st.sw_list[atomicAdd(&st.ctl[4], 1u)] = s;
}

// 2. the host's areas: bucket j of listed rule w at qoff[w] + j (2 cap + 3), marked as filling
__global__ __launch_bounds__(kThreads) void k_plru_alloc(CParamState st, const uint64_t *qoff, uint32_t nsw) {
    const uint32_t w = blockIdx.x;
    if (w >= nsw) return;
    const PRuleParam &P = st.param[st.sw_list[w]];
    for (int j = threadIdx.x; j < P.S; j += kThreads) {
        const uint64_t q = qoff[w] + (uint64_t)j * (plru_qcap(P) + 1);
        st.pq[P.boff + j] = q;
        st.lpool[q] = PLruRec{kPLruBuilding, 0};
    }
}

// 3. every key of a switching rule held by a bucket's map -> (key, its access stamp there) into that
//    bucket's area
__global__ __launch_bounds__(kThreads) void k_plru_collect(CParamState st) {
    for (uint32_t k = blockIdx.x * kThreads + threadIdx.x; k <= st.kmask; k += gridDim.x * kThreads) {
        if (st.ktab[k] == 0) continue;
        const PRuleParam &P = st.param[st.kslot[k]];
        if (!P.active) continue;  // a dropped rule's keys stay in ktab; they never join a queue
        const uint64_t q0 = st.pq[P.boff];
        if (q0 == kPNoQueue || st.lpool[q0].kidx != kPLruBuilding) continue;
        const int64_t *rec = st.krec + st.koff[k];
        for (int j = 0; j < P.S; ++j) {
            const int64_t rs = st.rstart[P.boff + j];
            if (rs == kAbsent || rec[j] != rs) continue;
            const uint64_t q = st.pq[P.boff + j];
            const unsigned long long pos = atomicAdd((unsigned long long *)&st.lpool[q].stamp, 1ull);
            if (pos < plru_qcap(P)) st.lpool[q + 1 + pos] = PLruRec{k, (uint64_t)rec[2 * P.S + j]};
            else atomicOr(&st.ctl[1], 4u);
        }
    }
}

// 4. each area ordered by stamp (oldest first), head 0, tail n, size n: one workgroup per (rule, bucket),
//    bitonic in LDS up to kPLruLds records, else in the area (2 cap + 2 >= the padded count)
constexpr int kPLruSortThreads = 256, kPLruLds = 4096;
__global__ __launch_bounds__(kPLruSortThreads) void k_plru_sort(CParamState st, uint32_t nsw) {
    __shared__ uint64_t ks[kPLruLds], vs[kPLruLds];
    const uint32_t w = blockIdx.x, j = blockIdx.y;
    if (w >= nsw) return;
    const PRuleParam &P = st.param[st.sw_list[w]];
    if ((int)j >= P.S) return;
    const uint64_t q = st.pq[P.boff + j];
    PLruRec *rec = st.lpool + q + 1;
    const uint32_t n = (uint32_t)min<uint64_t>(st.lpool[q].stamp, plru_qcap(P));
    if (n > P.cap) {  // a free-mode map holds at most cap keys: never expected; the host fails the call
        if (threadIdx.x == 0) atomicOr(&st.ctl[1], 4u);
        return;  // (padding n past cap to a power of two could run past the area's 2 cap + 2 records)
    }
    uint32_t np2 = 1;
    while (np2 < n) np2 <<= 1;
    if (np2 <= (uint32_t)kPLruLds) {
        for (uint32_t k = threadIdx.x; k < np2; k += kPLruSortThreads) {
            ks[k] = k < n ? rec[k].stamp : ~0ull;
            vs[k] = k < n ? rec[k].kidx : 0ull;
        }
        __syncthreads();
        for (uint32_t kk = 2; kk <= np2; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                for (uint32_t a = threadIdx.x; a < np2; a += kPLruSortThreads) {
                    const uint32_t b = a ^ jj;
                    if (b > a && (ks[a] > ks[b]) == ((a & kk) == 0)) {
                        const uint64_t tk = ks[a], tv = vs[a];
                        ks[a] = ks[b];
                        vs[a] = vs[b];
                        ks[b] = tk;
                        vs[b] = tv;
                    }
                }
                __syncthreads();
            }
        for (uint32_t k = threadIdx.x; k < n; k += kPLruSortThreads) rec[k] = PLruRec{vs[k], ks[k]};
    } else {
        for (uint32_t k = n + threadIdx.x; k < np2; k += kPLruSortThreads) rec[k] = PLruRec{0, ~0ull};
        __syncthreads();
        for (uint32_t kk = 2; kk <= np2; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                for (uint32_t a = threadIdx.x; a < np2; a += kPLruSortThreads) {
                    const uint32_t b = a ^ jj;
                    if (b > a) {
                        const PLruRec x = rec[a], y = rec[b];
                        if ((x.stamp > y.stamp) == ((a & kk) == 0)) {
                            rec[a] = y;
                            rec[b] = x;
                        }
                    }
                }
                __syncthreads();
            }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        st.lpool[q] = PLruRec{0, n};
        st.psize[P.boff + j] = n;
    }
}

}  // namespace

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Namespace limiter pre-pass (K9) over the elements of a batch: rejected requests get
// TOO_MANY_REQUEST and the invalid key.  RuleParam: SlotParam or PRuleParam (both carry .ns).
template <class RuleParam>
static void apply_limiters(const RuleParam *param, BatchScratch &sc, uint64_t *el, uint32_t n, uint32_t invalid_key,
                           int64_t ts_base, const uint32_t *ts_off, uint64_t *out, const LimiterPass *lims, int nlims,
                           hipStream_t s) {
    const uint32_t nb = (n + kThreads - 1) / kThreads;
    for (int l = 0; l < nlims; ++l) {
        // scratch: the run arrays are free until the runs stage
        uint32_t *flag = sc.run_start, *pos = sc.run_slot, *list = sc.run_idx0, *rstart = sc.run_cp,
                 *rpass = sc.run_p0;
        hipLaunchKernelGGL(k_lim_flag<RuleParam>, dim3(nb), dim3(kThreads), 0, s, param, el, n, invalid_key,
                           lims[l].ns, flag);
        exclusive_scan_u32(flag, pos, n, sc.lim_partial, s);
        hipLaunchKernelGGL(k_lim_compact, dim3(nb), dim3(kThreads), 0, s, flag, pos, n, list, sc.counters);
        uint32_t *head = flag, *ridx = pos;
        hipLaunchKernelGGL(k_lim_heads, dim3(nb), dim3(kThreads), 0, s, list, ts_off, ts_base, n, sc.counters, head);
        exclusive_scan_u32(head, ridx, n, sc.lim_partial, s);
        hipLaunchKernelGGL(k_lim_starts, dim3(nb), dim3(kThreads), 0, s, head, ridx, n, sc.counters, rstart);
        hipLaunchKernelGGL(k_lim_walk, dim3(1), dim3(64), 0, s, lims[l].state, lims[l].qps_allowed, list, rstart,
                           sc.counters, ts_off, ts_base, rpass);
        hipLaunchKernelGGL(k_lim_apply, dim3(nb), dim3(kThreads), 0, s, list, head, ridx, rstart, rpass, sc.counters, n,
                           invalid_key, el, out);
    }
}

// the radix digit width depends on the live slot count: size for the widest
static size_t max_hist_entries(size_t cap, uint32_t nslots_cap) {
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)nslots_cap + kHot + 2) ++bits;
    size_t m = 0;
    for (int b = 1; b <= bits; ++b) m = std::max(m, ((size_t)1 << radix64_digit_bits(b)) * radix64_tiles(cap));
    return m;
}

// A/B knob for profiling only (results are wrong when set): 1 skips k_cold_fused's flows, 2 its results,
// 4 k_hot_key's rank pass, 8 its code fix-up, 32 k_part_scatter's stores (16: phase times, results exact)
static int fz_debug() {
    static const int v = getenv("SGA_FZ_DEBUG") ? atoi(getenv("SGA_FZ_DEBUG")) : 0;
    return v;
}

static uint32_t fin_cache() {  // profiling knob: SGA_FIN_CACHE=0 turns k_hot_final's LDS cache off
    static const uint32_t v = getenv("SGA_FIN_CACHE") ? std::min<uint32_t>(atoi(getenv("SGA_FIN_CACHE")), kFinCache) : kFinCache;
    return v;
}

// k_hot_final_g by default; SGA_FIN_LDS=1 (A/B knob) the LDS-cached k_hot_final
static bool fin_g() {  // A/B knob: SGA_FIN_H=1 takes k_hot_final_h (measured equal: 0.698-0.706 against
                       // 0.697-0.699 ms per C3 batch; the kernel is not bound by its gathers)
    static const bool v = !(getenv("SGA_FIN_H") && atoi(getenv("SGA_FIN_H")) == 1);
    return v;
}

static void launch_hot_final(const ClusterState &st, BatchScratch &sc, uint32_t n, const uint64_t *pel, uint64_t *out,
                             hipStream_t s) {
    static const bool lds = getenv("SGA_FIN_LDS") && atoi(getenv("SGA_FIN_LDS")) == 1;
    static const bool pers = getenv("SGA_FIN_P") && atoi(getenv("SGA_FIN_P")) == 1;
    if (pers) {  // persistent: about two workgroups per CU, consecutive segments each
        const uint32_t nseg = (n + kHotSeg - 1) / kHotSeg;
        const uint32_t wgs = std::min<uint32_t>(nseg, 512);
        const uint32_t per = (nseg + wgs - 1) / wgs;
        hipLaunchKernelGGL(k_hot_final_p, dim3((nseg + per - 1) / per + kFinPrioWgsP), dim3(kFinPThreads), 0, s, st, sc,
                           n, pel, out, per);
        return;
    }
    if (lds) {
        const uint32_t nseg = (n + kHotSeg - 1) / kHotSeg;
        hipLaunchKernelGGL(k_hot_final, dim3(nseg + kFinPrioWgs), dim3(kFinWgThreads), 0, s, st, sc, n, pel, out,
                           fin_cache());
    } else if (fin_g()) {
        hipLaunchKernelGGL(k_hot_final_g, dim3((n + kFinGSpan - 1) / kFinGSpan + kFinPrioWgsG), dim3(kFinGThreads), 0, s,
                           st, sc, n, pel, out);
    } else {
        hipLaunchKernelGGL(k_hot_final_h, dim3((n + kFinGSpan - 1) / kFinGSpan + kFinPrioWgsG), dim3(kFinGThreads), 0, s,
                           st, sc, n, pel, out);
    }
}

static int hot_overlap() {  // A/B knob: SGA_HOT_OVERLAP=0 runs the hot side after the cold stage
    static const int v = getenv("SGA_HOT_OVERLAP") ? atoi(getenv("SGA_HOT_OVERLAP")) : 1;
    return v;
}

// Stream schedule of a hot-path batch (A/B knob SGA_HOT_SCHED): 1 (default) -- the hot side (count scans,
// prioritized sort, hot runs, hot results) on side streams beside the cold partition and the cold stage; 2 -- the
// hot side's short kernels on the batch stream beside the cold partition (side stream), then the hot results (third
// stream) beside the cold stage.  Measured (C3, MI355X): 2 is slower, 0.83 against 0.76-0.78 ms per batch -- the hot
// results and the cold stage side by side slow each other down more than one after the other would.
static int hot_sched() {
    static const int v = getenv("SGA_HOT_SCHED") ? atoi(getenv("SGA_HOT_SCHED")) : 1;
    return v;
}

static int tail_early() {  // A/B knob: SGA_HOT_TAIL_EARLY=0 starts the next hot set after the hot results
    static const int v = getenv("SGA_HOT_TAIL_EARLY") ? atoi(getenv("SGA_HOT_TAIL_EARLY")) : 1;
    return v;
}

void batch_scratch_release(BatchScratch &sc) {
    if (sc.side) (void)hipStreamDestroy(sc.side);
    if (sc.ev_fork) (void)hipEventDestroy(sc.ev_fork);
    if (sc.ev_join) (void)hipEventDestroy(sc.ev_join);
    if (sc.ev_fork0) (void)hipEventDestroy(sc.ev_fork0);
    if (sc.ev_mid) (void)hipEventDestroy(sc.ev_mid);
    if (sc.side2) (void)hipStreamDestroy(sc.side2);
    if (sc.ev_prio) (void)hipEventDestroy(sc.ev_prio);
    sc.side = sc.side2 = nullptr;
    sc.ev_fork = sc.ev_join = sc.ev_fork0 = sc.ev_mid = sc.ev_prio = nullptr;
}


// Cold stage of a large batch over the sorted elements: runs, flows and results in one kernel.
// Partitioned (sc.part_lb > 0, hot path): one workgroup per slot bin, el = the partition output, each bin
// ordered into the other element buffer first.
static void cold_stage(const ClusterState &st, BatchScratch &sc, const uint64_t *el, uint32_t n, const uint32_t *dn,
                       uint32_t invalid_key, const ReqIn &in, int64_t ts_base, int simple, uint32_t hot_min,
                       uint64_t *out, hipStream_t s) {
    if (sc.part_lb) {
        uint64_t *es = el == sc.el[0] ? sc.el[1] : sc.el[0];
        hipLaunchKernelGGL(k_cold_fused_t<kFzBin>, dim3(kPartBins), dim3(kFzThreads), 0, s, st, sc, el, n, dn,
                           invalid_key, in, ts_base, simple, hot_min, out, fz_debug(), es, sc.part_lb);
        return;
    }
    hipLaunchKernelGGL(k_cold_fused, dim3((n + kFzChunk - 1) / kFzChunk), dim3(kFzThreads), 0, s, st, sc, el, n, dn,
                       invalid_key, in, ts_base, simple, hot_min, out, fz_debug(), nullptr, 0);
}

static size_t hot_rows(size_t cap) { return (cap + kHotSeg - 1) / kHotSeg; }
static size_t hot_groups(size_t cap) { return (hot_rows(cap) + kHotGroupRows - 1) / kHotGroupRows; }

size_t batch_scratch_bytes(size_t cap, uint32_t nslots_cap) {
    const size_t ntiles = (cap + kTileElems - 1) / kTileElems + 1;
    const size_t hist = max_hist_entries(cap, nslots_cap);
    const size_t nseg = hot_rows(cap) + 1;  // segments of k_hot_classify (whole workgroups: 4 per)
    const size_t segs_alloc = ((nseg + kH1Waves - 1) / kH1Waves) * kH1Waves;
    size_t b = 0;
    b += 2 * align_up(cap * 8);                 // elements (double buffer)
    b += 7 * align_up((cap + 1) * 4);           // run_start/slot/idx0/cp/p0/acq, flow_first_run
    b += align_up(cap + 1);                     // run_bd
    b += align_up(cap * 4);                     // plist
    b += align_up(cap * 8);                     // deferred (flow, run)
    b += align_up(cap * sizeof(RunOut));        // run_out
    b += align_up(ntiles * kRunWaves * sizeof(RAgg));
    b += 2 * align_up(ntiles * sizeof(Agg)) + align_up(ntiles * 4);
    b += 2 * align_up(CTL_WORDS * 4);  // counters, counters_last
    b += 2 * align_up(hist * 4) + align_up(scan_partials_needed(hist) * 4 + 64);
    b += align_up(scan_partials_needed(cap) * 4 + 64);
    b += align_up(kRadixGhistWords * 4) + align_up(64);  // look-back digit totals, error flag
    // hot path
    b += align_up((size_t)nslots_cap * 2) + 2 * align_up(kHot * 4) + align_up(kHotCtlWords * 4);  // hot_of/slot/next/ctl
    b += align_up(segs_alloc * kHotSeg * 8);                                       // el_tile
    b += align_up(segs_alloc * kSubPerSeg * 4);                                    // tile_nc
    b += align_up(segs_alloc * kHotSeg * 8) + 2 * align_up((size_t)kPsGroups * kHot * 4);  // pel_tile, prow, pstart
    b += align_up(kHot * 4);                                                               // ptot
    b += 2 * align_up(cap * 8);                                                    // pel (double buffer)
    b += 2 * align_up(hist * 4) + align_up(scan_partials_needed(hist) * 4 + 64);   // DEBUG pad
    b += align_up(kRadixGhistWords * 4) + align_up(64);                            // DEBUG pad
    b += align_up(segs_alloc * kHotSeg * 4);                                       // hcode
    b += align_up(segs_alloc * kHot * 2) + align_up(segs_alloc * kHot * 4);        // hcnt, hbase
    b += align_up(hot_groups(cap) * kHot * 4);                                     // hgsum
    b += align_up((size_t)kHotBuckets * kHot * 2) + align_up(kHotBuckets * 4);     // hpre, hbnd
    b += align_up((size_t)kHot * kHotBuckets * sizeof(HotRun));                   // hrun
    b += align_up((size_t)kHot * kHotBuckets * sizeof(uint4));                    // hfin
    b += align_up((size_t)kHot * kHotBuckets * sizeof(uint2));                    // hfs
    b += align_up(kHot * sizeof(double2));                                        // hthr
    b += align_up(cap * 4);                                                        // prank
    b += 3 * align_up(kHot * 4);                                                   // plo, phi, hot_tot
    b += align_up(256 * sizeof(WConst));
    b += align_up(segs_alloc * kSegStat * 4);                                      // seg_stat
    b += align_up(64);                                                             // tmax_all
    b += align_up((size_t)kHotCand * 2 * 4);                                       // hot_cand
    b += align_up(segs_alloc * kPartBins * 4);                                     // phist
    b += align_up(((segs_alloc + kPartGroup - 1) / kPartGroup) * kPartBins * 4);   // pgrp
    b += align_up((kPartBins + 2) * 4);                                            // pstart, done counter
    return b;
}

void batch_scratch_carve(BatchScratch &sc, void *base, size_t cap, uint32_t nslots_cap) {
    const size_t ntiles = (cap + kTileElems - 1) / kTileElems + 1;
    const size_t hist = max_hist_entries(cap, nslots_cap);
    const size_t nseg = hot_rows(cap) + 1;
    const size_t segs_alloc = ((nseg + kH1Waves - 1) / kH1Waves) * kH1Waves;
    char *p = (char *)base;
    auto take = [&](size_t bytes) {
        void *r = p;
        p += align_up(bytes);
        return r;
    };
    sc.el[0] = (uint64_t *)take(cap * 8);
    sc.el[1] = (uint64_t *)take(cap * 8);
    sc.run_start = (uint32_t *)take((cap + 1) * 4);
    sc.run_slot = (uint32_t *)take((cap + 1) * 4);
    sc.run_idx0 = (uint32_t *)take((cap + 1) * 4);
    sc.run_cp = (uint32_t *)take((cap + 1) * 4);
    sc.run_p0 = (uint32_t *)take((cap + 1) * 4);
    sc.run_acq = (int32_t *)take((cap + 1) * 4);
    sc.flow_first_run = (uint32_t *)take((cap + 1) * 4);
    sc.run_bd = (uint8_t *)take(cap + 1);
    sc.plist = (uint32_t *)take(cap * 4);
    sc.deferred = (uint32_t *)take(cap * 8);
    sc.run_out = (RunOut *)take(cap * sizeof(RunOut));
    sc.wave_carry = (RAgg *)take(ntiles * kRunWaves * sizeof(RAgg));
    sc.tile_agg = take(ntiles * sizeof(Agg));
    sc.tile_carry = take(ntiles * sizeof(Agg));
    sc.tile_valid = (uint32_t *)take(ntiles * 4);
    sc.counters = (uint32_t *)take(CTL_WORDS * 4);
    sc.counters_last = (uint32_t *)take(CTL_WORDS * 4);
    sc.counters_clean = 0;
    sc.radix.hist = (uint32_t *)take(hist * 4);
    sc.radix.hist_scan = (uint32_t *)take(hist * 4);
    sc.radix.partial = (uint32_t *)take(scan_partials_needed(hist) * 4 + 64);
    sc.lim_partial = (uint32_t *)take(scan_partials_needed(cap) * 4 + 64);
    sc.radix.ghist = (uint32_t *)take(kRadixGhistWords * 4);
    sc.radix.err = (uint32_t *)take(64);
    sc.hot_of = (uint16_t *)take((size_t)nslots_cap * 2);
    sc.hot_slot = (uint32_t *)take(kHot * 4);
    sc.hot_next = (uint32_t *)take(kHot * 4);
    sc.hot_ctl = (uint32_t *)take(kHotCtlWords * 4);
    sc.el_tile = (uint64_t *)take(segs_alloc * kHotSeg * 8);
    sc.tile_nc = (uint32_t *)take(segs_alloc * kSubPerSeg * 4);
    sc.pel_tile = (uint64_t *)take(segs_alloc * kHotSeg * 8);
    sc.prow = (uint32_t *)take((size_t)kPsGroups * kHot * 4);
    sc.ppre = (uint32_t *)take((size_t)kPsGroups * kHot * 4);
    sc.ptot = (uint32_t *)take(kHot * 4);
    SGA_HIP_CHECK(hipMemset(sc.prow, 0, (size_t)kPsGroups * kHot * 4));  // k_psort_scatter keeps it zero
    sc.pel[0] = (uint64_t *)take(cap * 8);
    sc.pel[1] = (uint64_t *)take(cap * 8);
    (void)take(hist * 4); (void)take(hist * 4); (void)take(scan_partials_needed(hist) * 4 + 64);  // DEBUG pad
    (void)take(kRadixGhistWords * 4); (void)take(64);
    sc.hcode = (uint32_t *)take(segs_alloc * kHotSeg * 4);
    sc.hcnt = (uint16_t *)take(segs_alloc * kHot * 2);
    sc.hbase = (uint32_t *)take(segs_alloc * kHot * 4);
    sc.hgsum = (uint32_t *)take(hot_groups(cap) * kHot * 4);
    sc.hpre = (uint16_t *)take((size_t)kHotBuckets * kHot * 2);
    sc.hbnd = (uint32_t *)take(kHotBuckets * 4);
    sc.hrun = (HotRun *)take((size_t)kHot * kHotBuckets * sizeof(HotRun));
    sc.hfin = (uint4 *)take((size_t)kHot * kHotBuckets * sizeof(uint4));
    sc.hfs = (uint2 *)take((size_t)kHot * kHotBuckets * sizeof(uint2));
    sc.hthr = (double2 *)take(kHot * sizeof(double2));
    sc.prank = (uint32_t *)take(cap * 4);
    sc.plo = (uint32_t *)take(kHot * 4);
    sc.phi = (uint32_t *)take(kHot * 4);
    sc.hot_tot = (uint32_t *)take(kHot * 4);
    sc.wconst = (WConst *)take(256 * sizeof(WConst));
    sc.seg_stat = (uint32_t *)take(segs_alloc * kSegStat * 4);
    sc.tmax_all = (unsigned long long *)take(64);
    sc.hot_cand = (uint32_t *)take((size_t)kHotCand * 2 * 4);
    sc.phist = (uint32_t *)take(segs_alloc * kPartBins * 4);
    sc.pgrp = (uint32_t *)take(((segs_alloc + kPartGroup - 1) / kPartGroup) * kPartBins * 4);
    sc.pstart = (uint32_t *)take((kPartBins + 2) * 4);
    sc.cap = cap;
}

// Probe of the LDS property rank_hot relies on: random hot ids (dense, skewed and sparse, all and
// half the lanes active) ranked by the packed atomic and by a ballot match of all 12 id bits;
// mismatches are counted.
__device__ __forceinline__ uint32_t probe_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__global__ __launch_bounds__(kThreads) void k_lds_order_probe(uint32_t *bad) {
    __shared__ uint32_t cw[kThreads / 64][kHot / 2];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t K = 1u << (blockIdx.x % 13);  // 1 .. 4096 distinct ids
    const int mode = (blockIdx.x / 13) % 3;
    for (int k = lane; k < kHot / 2; k += 64) cw[w][k] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint64_t lt = lanemask_lt64(lane);
    uint32_t nb = 0;
    for (uint32_t r = 0; r < 32; ++r) {
        const uint32_t x = probe_mix((blockIdx.x * 1315423911u) ^ (r * 2654435761u) ^ (threadIdx.x * 97u));
        uint32_t hid = x % K;
        if (mode == 1 && (x & 1u)) hid = 7 % K;
        const bool act = mode == 2 ? ((x >> 8) & 1u) : true;
        const uint32_t sh = (hid & 1u) << 4;
        const uint32_t before = (cw[w][hid >> 1] >> sh) & 0xFFFFu;
        __builtin_amdgcn_wave_barrier();
        uint64_t peers = __ballot(act);
        for (int b = 0; b < 12; ++b) {
            const bool bit = (hid >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t expect = before + (uint32_t)__popcll(peers & lt);
        __builtin_amdgcn_wave_barrier();
        uint32_t got = expect;
        if (act) got = rank_hot(cw[w], hid);
        __builtin_amdgcn_wave_barrier();
        if (got != expect) ++nb;
    }
    if (nb) atomicAdd(bad, nb);
}

bool lds_lane_order_ok(hipStream_t s) {
    uint32_t *d = nullptr, h = 1;
    if (hipMalloc(&d, 4) != hipSuccess) return false;
    bool ok = hipMemsetAsync(d, 0, 4, s) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_lds_order_probe, dim3(13 * 3 * 64), dim3(kThreads), 0, s, d);
        ok = hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess && h == 0;
    }
    (void)hipFree(d);
    return ok;
}

void hot_reset(const ClusterState &st, BatchScratch &sc, uint32_t nslots_cap, hipStream_t s) {
    const uint32_t m = std::max(nslots_cap, st.dkey ? st.dense_n : 0u);
    hipLaunchKernelGGL(k_hot_reset, dim3(std::max<uint32_t>(1, std::min<uint32_t>((m + 255) / 256, 4096))),
                       dim3(256), 0, s, st, sc, nslots_cap);
}

// Hot path batch (kernels above): precheck -> classify (+ fallback re-classification) -> count
// scan -> sort of the cold (and prioritized hot) elements -> cold runs / flows / results -> hot
// runs (k_hot_flows) -> hot results in input order -> prioritized hot results -> next hot set.
// Every kernel reads the batch's path from the control words, so no host synchronisation.
static void side_stream_init(BatchScratch &sc) {
    if (sc.side) return;
    static const int side_prio = getenv("SGA_SIDE_PRIO") ? atoi(getenv("SGA_SIDE_PRIO")) : 0;  // A/B knob
    if (side_prio) {
        int lo = 0, hi = 0;  // hi: the greatest priority (numerically lowest)
        SGA_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        SGA_HIP_CHECK(hipStreamCreateWithPriority(&sc.side, hipStreamNonBlocking, side_prio > 0 ? hi : lo));
    } else {
        SGA_HIP_CHECK(hipStreamCreateWithFlags(&sc.side, hipStreamNonBlocking));
    }
    // the fork / join events only order streams of this device: a device-scope release is enough (the default
    // system-scope one writes the L2s back at every record).  SGA_EV_SYSTEM=1 (A/B knob) keeps the default.
    static const bool ev_sys = getenv("SGA_EV_SYSTEM") && atoi(getenv("SGA_EV_SYSTEM")) == 1;
    const unsigned evf = hipEventDisableTiming | (ev_sys ? 0u : (unsigned)hipEventReleaseToDevice);
    SGA_HIP_CHECK(hipEventCreateWithFlags(&sc.ev_fork0, evf));
    SGA_HIP_CHECK(hipEventCreateWithFlags(&sc.ev_fork, evf));
    SGA_HIP_CHECK(hipEventCreateWithFlags(&sc.ev_join, evf));
    SGA_HIP_CHECK(hipEventCreateWithFlags(&sc.ev_mid, evf));
    SGA_HIP_CHECK(hipStreamCreateWithFlags(&sc.side2, hipStreamNonBlocking));
    SGA_HIP_CHECK(hipEventCreateWithFlags(&sc.ev_prio, evf));
}

// The cold partition's slot bits below the bin, or 0 (the LSD sort): bins of 2^lb slots need
// 5 <= lb <= kPartMaxLow (rule slot counts from 2^15 to about 2^21).  SGA_COLD_PART=0 (A/B knob) turns it off.
static int cold_part_lb(int bits) {
    static const bool off = getenv("SGA_COLD_PART") && atoi(getenv("SGA_COLD_PART")) == 0;
    const int lb = bits - kPartBits;
    return (!off && lb >= 5 && lb <= kPartMaxLow) ? lb : 0;
}

static int hot_key_bits(const ClusterState &st) {
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)st.nslots + kHot + 2) ++bits;
    return bits;
}

// Stage 1 of a hot-path batch (reads only its inputs, the dense table and -- the precheck -- the hot
// rules' window starts): the precheck, the key pass (in-segment ranks, cold elements), the count scans,
// the prioritized sort and the cold sort.  The result is in sc (CTL words, el[], pel[], hcode, hbase).
// pipelined: an earlier batch may still be deciding (sga_request_tokens_device_pipelined); the precheck
// then also refuses the hot path to a batch that starts before the latest time of any earlier batch.
// The hot side's runs and results (k_prio_rank, k_hot_flows, k_hot_final): once the count scans and the
// prioritized sort are done, on hs; ev_mid after the hot runs (the next hot set may start), ev_join after all.
static void hot_side(const ClusterState &st, BatchScratch &sc, int64_t ts_base, uint32_t n, uint64_t *out,
                     hipStream_t hs, bool ovl) {
    const uint32_t pgrid = std::max<uint32_t>(1, std::min<uint32_t>((n + kThreads - 1) / kThreads, 1024));
    hipLaunchKernelGGL(k_prio_rank, dim3(pgrid), dim3(kThreads), 0, hs, st, sc, sc.pel_sorted);
    hipLaunchKernelGGL(k_hot_flows, dim3(kHot / kH1Waves), dim3(kThreads), 0, hs, st, sc, ts_base);
    if (ovl) {
        SGA_HIP_CHECK(hipEventRecord(sc.ev_mid, hs));  // the hot runs read hot_slot; the next hot set may start
        launch_hot_final(st, sc, n, sc.pel_sorted, out, hs);
        SGA_HIP_CHECK(hipEventRecord(sc.ev_join, hs));
    }
}

// the prioritized hot requests sorted by hot id into pel[0] (k_psort_*; plo / phi per hot id)
static uint32_t ps_per_group_h(uint32_t nseg) { return std::max<uint32_t>(1, (nseg + kPsGroups - 1) / kPsGroups); }
static uint32_t ps_groups_h(uint32_t nseg) { return (nseg + ps_per_group_h(nseg) - 1) / ps_per_group_h(nseg); }
// cols_done: k_hscan_mid already made the column prefix (the one-stream hot side)
static void prio_sort(BatchScratch &sc, uint32_t nseg, hipStream_t s, bool cols_done = false) {
    const uint32_t ngroups = ps_groups_h(nseg);
    if (fz_debug() & 512) hipLaunchKernelGGL(k_psort_dbgcount, dim3(kPsGroups), dim3(64), 0, s, sc, nseg);
    if (!cols_done) hipLaunchKernelGGL(k_psort_cols, dim3(kHot / 256), dim3(256), 0, s, sc, ngroups);
    hipLaunchKernelGGL(k_psort_scatter, dim3(kPsGroups), dim3(64), 0, s, sc, nseg, sc.pel[0], fz_debug());
    if (fz_debug() & 512) hipLaunchKernelGGL(k_psort_verify, dim3(4), dim3(256), 0, s, sc, sc.pel[0]);
    sc.pel_sorted = sc.pel[0];
}

static void classify_hot(const ClusterState &st, BatchScratch &sc, const ReqIn &in, int64_t ts_base, uint32_t n,
                         uint64_t *out, hipStream_t s, bool clean, bool pipelined) {
    const int bits = hot_key_bits(st);
    const uint32_t nseg = (n + kHotSeg - 1) / kHotSeg;
    const uint32_t ngroups = (nseg + kHotGroupRows - 1) / kHotGroupRows;
    if (!clean) SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, CTL_WORDS * 4, s));
    hipLaunchKernelGGL(k_hot_precheck, dim3(kHot / kThreads), dim3(kThreads), 0, s, st, sc, in, ts_base, n,
                       pipelined ? 1 : 0);
    // the key pass streams its inputs and cold elements non-temporally, so the dense table keeps more of L2
    // (158 against 166 us on MI355X; SGA_KEY_NT=0, an A/B knob, turns it off)
    static const bool key_nt = !(getenv("SGA_KEY_NT") && atoi(getenv("SGA_KEY_NT")) == 0);
    const bool pk = in.pk != nullptr;
    auto hka = st.dense_n ? (pk ? (key_nt ? k_hot_key_dense<0, true, true> : k_hot_key_dense<0, false, true>)
                                : (key_nt ? k_hot_key_dense<0, true, false> : k_hot_key_dense<0, false, false>))
                          : (pk ? k_hot_key_hash<0, true> : k_hot_key_hash<0, false>);
    auto hkb = st.dense_n ? (pk ? k_hot_key_dense<1, false, true> : k_hot_key_dense<1, false, false>)
                          : (pk ? k_hot_key_hash<1, true> : k_hot_key_hash<1, false>);
    // the key kernels count the sort's first digit per tile as they write the elements
    // (their LDS counts hold 8-bit digits; a wider first digit is counted by the sort itself), or, with
    // the cold partition, each segment's elements per slot bin
    const int dsort = radix64_digit_bits(bits);
    sc.part_lb = cold_part_lb(bits);
    const int d0 = sc.part_lb ? -sc.part_lb : (dsort <= 8 ? dsort : 0);
    const uint32_t ntiles_sort = (uint32_t)radix64_tiles(n);
    uint32_t *khist = sc.part_lb ? sc.phist : sc.radix.hist;
    hipLaunchKernelGGL(hka, dim3(nseg), dim3(kKeyThreads), 0, s, st, sc, in, ts_base, n, out, fz_debug(), d0, khist,
                       ntiles_sort);
    hipLaunchKernelGGL(hkb, dim3(nseg), dim3(kKeyThreads), 0, s, st, sc, in, ts_base, n, out, fz_debug(), d0, khist,
                       ntiles_sort);
    hipLaunchKernelGGL(k_hot_mode, dim3(1), dim3(1024), 0, s, sc, nseg * kKeyWaves, nseg, ts_base);
    const bool ovl = hot_overlap() && !(fz_debug() & 16);
    sc.sched2 = ovl && !pipelined && hot_sched() == 2;
    if (sc.sched2) {
        // the cold partition (or sort) on the side stream; the hot side's short kernels on the batch stream
        // beside it; the hot results on the third stream once the hot runs are done (beside the cold stage,
        // which decide_hot queues on the batch stream after the partition)
        side_stream_init(sc);
        SGA_HIP_CHECK(hipEventRecord(sc.ev_fork0, s));
        SGA_HIP_CHECK(hipStreamWaitEvent(sc.side, sc.ev_fork0, 0));
        if (sc.part_lb) {
            const uint32_t pg = (nseg + kPartGroup - 1) / kPartGroup;
            hipLaunchKernelGGL(k_part_colscan, dim3(kPartBins / 256, pg), dim3(256), 0, sc.side, sc, nseg);
            hipLaunchKernelGGL(k_part_binscan, dim3(kPartBins / 256), dim3(256), 0, sc.side, sc, pg);
            hipLaunchKernelGGL(k_part_scatter, dim3(8 * ((nseg + 7) / 8)), dim3(kKeyThreads), 0, sc.side, sc, nseg,
                               sc.part_lb, sc.el[0], fz_debug());
            sc.el_sorted = sc.el[0];
        } else {
            const int np = radix_sort_u64_tiled(sc.el_tile, sc.tile_nc, sc.counters + CTL_NSORT, sc.el[0], sc.el[1], n,
                                                kSlotShift, bits, sc.radix, sc.side, d0 > 0);
            sc.el_sorted = (np & 1) ? sc.el[0] : sc.el[1];
        }
        SGA_HIP_CHECK(hipEventRecord(sc.ev_fork, sc.side));  // the cold elements ready (decide_hot waits)
        prio_sort(sc, nseg, s);
        hipLaunchKernelGGL(k_hscan_group, dim3(ngroups, kHot / kThreads), dim3(kThreads), 0, s, sc, nseg);
        hipLaunchKernelGGL(k_hscan_mid, dim3(kHot / kThreads), dim3(kThreads), 0, s, sc, ngroups, 0u);
        hipLaunchKernelGGL(k_hscan_down, dim3(ngroups, kHot / kThreads), dim3(kThreads), 0, s, sc, nseg);
        const uint32_t pgrid = std::max<uint32_t>(1, std::min<uint32_t>((n + kThreads - 1) / kThreads, 1024));
        hipLaunchKernelGGL(k_prio_rank, dim3(pgrid), dim3(kThreads), 0, s, st, sc, sc.pel_sorted);
        hipLaunchKernelGGL(k_hot_flows, dim3(kHot / kH1Waves), dim3(kThreads), 0, s, st, sc, ts_base);
        SGA_HIP_CHECK(hipEventRecord(sc.ev_mid, s));
        SGA_HIP_CHECK(hipStreamWaitEvent(sc.side2, sc.ev_mid, 0));
        launch_hot_final(st, sc, n, sc.pel_sorted, out, sc.side2);
        SGA_HIP_CHECK(hipEventRecord(sc.ev_join, sc.side2));
        sc.hot_early = true;
        return;
    }
    // the hot side's count scans and prioritized sort on the side stream, beside the cold sort; schedule 3
    // (SGA_HOT_SCHED=3): the count scans on the batch stream first, so the hot runs and results start beside
    // the partition instead of waiting for the scans' slots beside the cold stage
    const bool scans_first = ovl && !pipelined && hot_sched() == 3;
    // Round 6 (default, SGA_HOT_ONE=0 the round-5 form): the whole hot side on ONE side stream -- count scans
    // (k_hscan_mid also makes the prioritized sort's column prefix), the prioritized scatter, the hot runs and
    // results -- no second side stream and no cross-stream join inside the hot chain.  Beside the cold stage
    // every launch of the chain waits for free slots, so fewer launches shorten the chain.
    static const bool hot_one = !getenv("SGA_HOT_ONE") || atoi(getenv("SGA_HOT_ONE")) == 1;
    hipStream_t hs = s;
    if (ovl && !pipelined && !scans_first && hot_one) {
        side_stream_init(sc);
        SGA_HIP_CHECK(hipEventRecord(sc.ev_fork0, s));
        SGA_HIP_CHECK(hipStreamWaitEvent(sc.side, sc.ev_fork0, 0));
        hipStream_t hs1 = hs = sc.side;
        hipLaunchKernelGGL(k_hscan_group, dim3(ngroups, kHot / kThreads), dim3(kThreads), 0, hs1, sc, nseg);
        hipLaunchKernelGGL(k_hscan_mid, dim3(kHot / kThreads), dim3(kThreads), 0, hs1, sc, ngroups, ps_groups_h(nseg));
        hipLaunchKernelGGL(k_hscan_down, dim3(ngroups, kHot / kThreads), dim3(kThreads), 0, hs1, sc, nseg);
        sga::prio_sort(sc, nseg, hs1, true);
        sc.hot_early = true;
        hot_side(st, sc, ts_base, n, out, hs1, true);
    } else {
    if (ovl) {
        side_stream_init(sc);
        SGA_HIP_CHECK(hipEventRecord(sc.ev_fork0, s));
        if (!scans_first) {
            SGA_HIP_CHECK(hipStreamWaitEvent(sc.side, sc.ev_fork0, 0));
            hs = sc.side;
        }
    }
    // the prioritized hot requests, sorted by hot id on their own (12-bit key): on a third stream when the
    // hot side overlaps, so it and the count scans both run beside the cold sort / partition
    hipStream_t ps = hs;
    if (ovl) {
        SGA_HIP_CHECK(hipStreamWaitEvent(sc.side2, sc.ev_fork0, 0));
        ps = sc.side2;
    }
    // the count scans are queued before the prioritized sort (the two side streams may share a hardware queue,
    // where submission order is execution order): 0.70 against 0.71 ms per C3 batch (SGA_PRIO_LATE=0 the other
    // order)
    static const bool prio_late = !getenv("SGA_PRIO_LATE") || atoi(getenv("SGA_PRIO_LATE")) == 1;
    auto prio_sort = [&] { sga::prio_sort(sc, nseg, ps); };
    if (!prio_late) prio_sort();
    hipLaunchKernelGGL(k_hscan_group, dim3(ngroups, kHot / kThreads), dim3(kThreads), 0, hs, sc, nseg);
    hipLaunchKernelGGL(k_hscan_mid, dim3(kHot / kThreads), dim3(kThreads), 0, hs, sc, ngroups, 0u);
    hipLaunchKernelGGL(k_hscan_down, dim3(ngroups, kHot / kThreads), dim3(kThreads), 0, hs, sc, nseg);
    if (prio_late) prio_sort();
    if (scans_first) {  // the hot side forks after the scans and the prioritized sort
        SGA_HIP_CHECK(hipEventRecord(sc.ev_fork, s));
        SGA_HIP_CHECK(hipStreamWaitEvent(sc.side, sc.ev_fork, 0));
        hs = sc.side;
    }
    if (ovl) {  // the prioritized sort joins the side stream (k_prio_rank needs both)
        SGA_HIP_CHECK(hipEventRecord(sc.ev_prio, ps));
        SGA_HIP_CHECK(hipStreamWaitEvent(hs, sc.ev_prio, 0));
    }
    // Not pipelined: the hot side needs nothing of the cold sort (disjoint rules, disjoint results), so its runs
    // and results go on beside the sort and the cold stage waits for it only at the end of the batch.  Pipelined,
    // the hot runs write rule state and wait for stage 2 (after the earlier batch's decisions).
    sc.hot_early = ovl && !pipelined;
    if (sc.hot_early) hot_side(st, sc, ts_base, n, out, hs, true);
    }
    if (sc.part_lb) {  // the cold partition: one pass into slot bins, ordered per bin by k_cold_fused
        const uint32_t ngroups = (nseg + kPartGroup - 1) / kPartGroup;
        hipLaunchKernelGGL(k_part_colscan, dim3(kPartBins / 256, ngroups), dim3(256), 0, s, sc, nseg);
        hipLaunchKernelGGL(k_part_binscan, dim3(kPartBins / 256), dim3(256), 0, s, sc, ngroups);
        hipLaunchKernelGGL(k_part_scatter, dim3(8 * ((nseg + 7) / 8)), dim3(kKeyThreads), 0, s, sc, nseg, sc.part_lb,
                           sc.el[0], fz_debug());
        sc.el_sorted = sc.el[0];
    } else {
        const int np = radix_sort_u64_tiled(sc.el_tile, sc.tile_nc, sc.counters + CTL_NSORT, sc.el[0], sc.el[1], n,
                                            kSlotShift, bits, sc.radix, s, d0 > 0);
        sc.el_sorted = (np & 1) ? sc.el[0] : sc.el[1];
    }
    if (ovl && !sc.hot_early) {  // stage 1 ends on s
        SGA_HIP_CHECK(hipEventRecord(sc.ev_fork, hs));
        SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_fork, 0));
    }
}

// Stage 2 (the batch's decisions; batches' stage 2 run in order): the hot runs and results on the side
// stream beside the cold stage, then the next hot set.
static void decide_hot(const ClusterState &st, BatchScratch &sc, const ReqIn &in, int64_t ts_base, uint32_t n,
                       uint64_t *out, hipStream_t s) {
    const uint32_t invalid_key = st.nslots;
    const uint64_t *el = sc.el_sorted, *pel = sc.pel_sorted;
    const bool ovl = hot_overlap() && !(fz_debug() & 16);
    if (sc.sched2) SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_fork, 0));  // the cold partition (side stream)
    if (!sc.hot_early) {  // the hot side beside the cold stage
        hipStream_t hs = s;
        if (ovl) {
            side_stream_init(sc);
            SGA_HIP_CHECK(hipEventRecord(sc.ev_fork0, s));
            SGA_HIP_CHECK(hipStreamWaitEvent(sc.side, sc.ev_fork0, 0));
            hs = sc.side;
        }
        hot_side(st, sc, ts_base, n, out, hs, ovl);
    }
    cold_stage(st, sc, el, n, sc.counters + CTL_NCOLD, invalid_key, in, ts_base, 0, std::max<uint32_t>(sc.hot_min, 1),
               out, s);
    if (fz_debug() & 16) {  // profiling only: k_cold_fused phase cycles per workgroup
        unsigned long long ph[8];
        SGA_HIP_CHECK(hipMemcpyFromSymbolAsync(ph, HIP_SYMBOL(g_fz_phase), sizeof(ph), 0, hipMemcpyDeviceToHost, s));
        SGA_HIP_CHECK(hipStreamSynchronize(s));
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        SGA_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fz_phase), z, sizeof(z), 0, hipMemcpyHostToDevice, s));
        if (ph[7])
            fprintf(stderr, "fz phases (wall_clock64 ticks per workgroup, %llu wgs): order %.0f runs %.0f flows %.0f results %.0f\n",
                    ph[7], (double)ph[3] / ph[7], (double)ph[0] / ph[7], (double)ph[1] / ph[7], (double)ph[2] / ph[7]);
    }
    if (!ovl) {
        launch_hot_final(st, sc, n, pel, out, s);
    } else if (!tail_early()) {
        SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_join, 0));
    } else {
        // the next hot set needs the cold candidates (this stream) and the hot runs done (they read
        // hot_slot); it writes hot_of / hot_next / the dense hot ids, which the hot results do not
        // read, so it runs beside k_hot_final.  k_hot_fin (renames, control words) waits for both.
        SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_mid, 0));
    }
    const uint32_t sb = 64;  // few workgroups: their bins meet in global atomics
    static const int next = getenv("SGA_HOT_NEXT") ? atoi(getenv("SGA_HOT_NEXT")) : 3;  // A/B knob: 4, 3 or 2 launches
    if (next == 3) {  // the picks beside the hot results, k_hot_fin after both
        hipLaunchKernelGGL(k_hot_next_a, dim3(sb), dim3(kThreads), 0, s, st, sc, std::max<uint32_t>(sc.hot_min, 1));
        hipLaunchKernelGGL(k_hot_pick, dim3(sb), dim3(kThreads), 0, s, st, sc, sc.hot_min);
        if (ovl && tail_early()) SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_join, 0));
        hipLaunchKernelGGL(k_hot_fin, dim3(1), dim3(kFinThreads), 0, s, st, sc);
    } else if (next == 4) {
        hipLaunchKernelGGL(k_hot_hist, dim3(sb), dim3(kThreads), 0, s, st, sc, std::max<uint32_t>(sc.hot_min, 1));
        hipLaunchKernelGGL(k_hot_clear, dim3(kHot / kThreads), dim3(kThreads), 0, s, st, sc);
        hipLaunchKernelGGL(k_hot_pick, dim3(sb), dim3(kThreads), 0, s, st, sc, sc.hot_min);
        if (ovl && tail_early()) SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_join, 0));
        hipLaunchKernelGGL(k_hot_fin, dim3(1), dim3(kFinThreads), 0, s, st, sc);
    } else {
        // k_hot_fin clears the control words the hot results read: the pick launch (which ends in it) waits
        // for them
        hipLaunchKernelGGL(k_hot_next_a, dim3(sb), dim3(kThreads), 0, s, st, sc, std::max<uint32_t>(sc.hot_min, 1));
        if (ovl && tail_early()) SGA_HIP_CHECK(hipStreamWaitEvent(s, sc.ev_join, 0));
        hipLaunchKernelGGL(k_hot_next_b, dim3(sb), dim3(kThreads), 0, s, st, sc, sc.hot_min);
    }
    sc.counters_clean = 1;
}

bool cluster_hot_eligible(const ClusterState &st, const BatchScratch &sc, uint32_t n, int simple, int nlims) {
    const bool limited = nlims > 0 && !simple;
    if (n == 0 || (n <= std::min<uint32_t>(sc.small_max, kSmall) && !limited && !radix64_lookback())) return false;
    return sc.hot_enabled && sc.hot_lane_order && !simple && !limited && !radix64_lookback() &&
           st.nslots + (uint64_t)kHot + 2 < kMaxSlots;
}

void cluster_classify_hot(const ClusterState &st, BatchScratch &sc, const int64_t *flow_id, const int32_t *acquire,
                          const uint8_t *prio, int64_t ts_base, const uint32_t *ts_off, uint32_t n, void *out,
                          hipStream_t s) {
    const bool clean = sc.counters_clean != 0;
    sc.counters_clean = 0;
    ReqIn in;
    in.flow = flow_id;
    in.acq = acquire;
    in.prio = prio;
    in.ts = ts_off;
    classify_hot(st, sc, in, ts_base, n, (uint64_t *)out, s, clean, true);
}

void cluster_decide_hot(const ClusterState &st, BatchScratch &sc, const int32_t *acquire, const uint8_t *prio,
                        int64_t ts_base, const uint32_t *ts_off, uint32_t n, void *out, hipStream_t s) {
    ReqIn in;
    in.acq = acquire;
    in.prio = prio;
    in.ts = ts_off;
    decide_hot(st, sc, in, ts_base, n, (uint64_t *)out, s);
}

void cluster_decide_batch(const ClusterState &st, BatchScratch &sc, const int64_t *flow_id, const int32_t *acquire,
                          const uint8_t *prio, int64_t ts_base, const uint32_t *ts_off, uint32_t n, int simple,
                          void *out_v, hipStream_t s, const LimiterPass *lims, int nlims) {
    if (n == 0) return;
    ReqIn in;
    in.flow = flow_id;
    in.acq = acquire;
    in.prio = simple ? nullptr : prio;
    in.ts = ts_off;
    const bool clean = sc.counters_clean != 0;
    sc.counters_clean = 0;
    uint64_t *out = (uint64_t *)out_v;
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)st.nslots + 1) ++bits;
    const uint32_t invalid_key = st.nslots;
    const bool limited = nlims > 0 && !simple;
    const int d0 = radix64_digit_bits(bits);
    const uint32_t ntiles = (n + kTileElems - 1) / kTileElems;
    static_assert(kTileElems == kRadix64Tile, "classify tiles are sort tiles");
    const bool lb = radix64_lookback() != 0;
    const int npass = (bits + d0 - 1) / d0;
    if (lb && (npass << d0) > 1024)  // k_classify counts every pass's digits in 1024 LDS words
        throw HipError("look-back sort (SGA_RADIX_MODE=0) needs npass << digit bits <= 1024", __FILE__, __LINE__);
    static const int chunk = getenv("SGA_CLS_CHUNK") ? atoi(getenv("SGA_CLS_CHUNK")) : 2;  // A/B knob
    auto cls = chunk >= 16 ? k_classify<16>
                           : (chunk >= 8 ? k_classify<8> : (chunk >= 4 ? k_classify<4> : (chunk >= 2 ? k_classify<2> : k_classify<1>)));
    static const int nofuse = getenv("SGA_XP_NOFUSE") ? atoi(getenv("SGA_XP_NOFUSE")) : 0;  // A/B knob
    if (n <= std::min<uint32_t>(sc.small_max, kSmall) && !limited && !lb) {  // one call's worth of requests: two launches
        uint32_t m = 64;
        while (m < n) m <<= 1;
        hipLaunchKernelGGL(k_small_sort, dim3(1), dim3(kSmallThreads), 0, s, st, flow_id, acquire, prio, ts_off, ts_base,
                           n, m, simple, invalid_key, sc.el[0], out);
        hipLaunchKernelGGL(k_cold_fused, dim3((n + kFzChunk - 1) / kFzChunk), dim3(kFzThreads), 0, s, st, sc, sc.el[0],
                           n, nullptr, invalid_key, in, ts_base, simple, 0xFFFFFFFFu, out, 0, nullptr, 0);
        return;
    }
    if (cluster_hot_eligible(st, sc, n, simple, nlims)) {
        classify_hot(st, sc, in, ts_base, n, out, s, clean, false);
        decide_hot(st, sc, in, ts_base, n, out, s);
        return;
    }
    SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, CTL_WORDS * 4, s));
    if (lb) SGA_HIP_CHECK(hipMemsetAsync(sc.radix.ghist, 0, kRadixGhistWords * sizeof(uint32_t), s));
    if (lb) SGA_HIP_CHECK(hipMemsetAsync(sc.radix.err, 0, sizeof(uint32_t), s));
    // the sort's result buffer (radix_sort_u64 returns npass)
    const uint64_t *el = sc.el[npass & 1];
    hipLaunchKernelGGL(cls, dim3(ntiles), dim3(kThreads), 0, s, st, flow_id, acquire, prio, ts_off, ts_base, n, simple,
                       invalid_key, sc.el[0], out, (limited || nofuse) ? 0 : d0, ntiles, sc.radix.hist,
                       (lb && !limited) ? npass : 0, sc.radix.ghist);
    if (!simple) apply_limiters(st.param, sc, sc.el[0], n, invalid_key, ts_base, ts_off, out, lims, nlims, s);
    const int np = radix_sort_u64(sc.el[0], sc.el[1], n, kSlotShift, bits, sc.radix, s, !limited && !nofuse);
    if (np != npass) throw HipError("radix pass count mismatch", __FILE__, __LINE__);
    cold_stage(st, sc, el, n, nullptr, invalid_key, in, ts_base, simple, 0xFFFFFFFFu, out, s);
}

// packed requests -> the four arrays (the paths other than the hot one read those)
__global__ __launch_bounds__(kThreads) void k_unpack(const uint32_t *__restrict__ pk, uint32_t n, int64_t *__restrict__ f,
                                                     int32_t *__restrict__ a, uint8_t *__restrict__ p,
                                                     uint32_t *__restrict__ t) {
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const uint32_t *r = pk + 3 * (size_t)i;
        f[i] = (int64_t)r[0];
        t[i] = r[1];
        // reserved flag bits set: acquireCount 0, so the request answers BAD_REQUEST like the hot path's
        a[i] = (r[2] >> 17) ? 0 : (int32_t)(r[2] & 0xFFFFu);
        p[i] = (uint8_t)((r[2] >> 16) & 1u);
    }
}

void cluster_decide_batch_packed(const ClusterState &st, BatchScratch &sc, const uint32_t *pk, int64_t ts_base,
                                 uint32_t n, void *out_v, hipStream_t s, const LimiterPass *lims, int nlims) {
    if (n == 0) return;
    const bool small = n <= std::min<uint32_t>(sc.small_max, kSmall) && nlims == 0 && !radix64_lookback();
    if (!small && cluster_hot_eligible(st, sc, n, 0, nlims)) {
        const bool clean = sc.counters_clean != 0;
        sc.counters_clean = 0;
        ReqIn in;
        in.pk = pk;
        classify_hot(st, sc, in, ts_base, n, (uint64_t *)out_v, s, clean, false);
        decide_hot(st, sc, in, ts_base, n, (uint64_t *)out_v, s);
        return;
    }
    // the hot path's scratch holds the arrays: flowIds in pel[0], acquire counts and time offsets in pel[1],
    // prioritized flags in prank (none of them is used off the hot path)
    int64_t *f = reinterpret_cast<int64_t *>(sc.pel[0]);
    int32_t *a = reinterpret_cast<int32_t *>(sc.pel[1]);
    uint32_t *t = reinterpret_cast<uint32_t *>(sc.pel[1]) + sc.cap;
    uint8_t *p = reinterpret_cast<uint8_t *>(sc.prank);
    const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>((n + kThreads - 1) / kThreads, 4096));
    hipLaunchKernelGGL(k_unpack, dim3(nb), dim3(kThreads), 0, s, pk, n, f, a, p, t);
    cluster_decide_batch(st, sc, f, a, p, ts_base, t, n, 0, out_v, s, lims, nlims);
}

// ---------------------------------------------------------------- cluster parameter flow (host)
size_t cparam_scratch_bytes(size_t cap) { return 2 * align_up(cap * 8) + align_up(cap * 4); }

void cparam_scratch_carve(CParamScratch &ps, void *base, size_t cap) {
    char *p = (char *)base;
    ps.els[0] = (uint64_t *)p;
    p += align_up(cap * 8);
    ps.els[1] = (uint64_t *)p;
    p += align_up(cap * 8);
    ps.vkey = (uint32_t *)p;
}

void cparam_stage1(const CParamState &st, BatchScratch &sc, CParamScratch &ps, const int64_t *flow_id,
                   const int32_t *acquire, const uint32_t *voff, const int64_t *values, int64_t ts_base,
                   const uint32_t *ts_off, uint32_t n, void *out_v, hipStream_t s, const LimiterPass *lims,
                   int nlims) {
    sc.counters_clean = 0;  // the stages use the control words
    if (n == 0) return;
    uint64_t *out = (uint64_t *)out_v;
    const uint32_t invalid_key = st.nslots;
    const uint32_t nb = (n + kThreads - 1) / kThreads;
    SGA_HIP_CHECK(hipMemsetAsync(st.ctl + 1, 0, 3 * sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_pcls, dim3(nb), dim3(kThreads), 0, s, st, flow_id, acquire, voff, ts_base, ts_off, n,
                       invalid_key, sc.el[0], out);
    SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, 64, s));
    apply_limiters(st.param, sc, sc.el[0], n, invalid_key, ts_base, ts_off, out, lims, nlims, s);
    hipLaunchKernelGGL(k_pkeys, dim3(nb), dim3(kThreads), 0, s, st, sc.el[0], voff, values, n, invalid_key, ps.vkey);
    hipLaunchKernelGGL(k_ppath, dim3(nb), dim3(kThreads), 0, s, st, sc.el[0], ps.els[0], voff, ps.vkey, acquire,
                       ts_base, ts_off, n, invalid_key, st.kmask + 1);
    cparam_lru_decide(st, s);
}

void cparam_lru_decide(const CParamState &st, hipStream_t s) {
    if (st.nslots == 0) return;
    SGA_HIP_CHECK(hipMemsetAsync(st.ctl + 4, 0, 4, s));
    hipLaunchKernelGGL(k_plru_decide, dim3((st.nslots + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st);
}

void cparam_lru_switch(const CParamState &st, const uint64_t *d_qoff, uint32_t nsw, uint32_t max_s, hipStream_t s) {
    if (nsw == 0) return;
    hipLaunchKernelGGL(k_plru_alloc, dim3(nsw), dim3(kThreads), 0, s, st, d_qoff, nsw);
    const uint32_t nk = st.kmask + 1;
    hipLaunchKernelGGL(k_plru_collect, dim3(std::min<uint32_t>((nk + kThreads - 1) / kThreads, 4096)), dim3(kThreads),
                       0, s, st);
    hipLaunchKernelGGL(k_plru_sort, dim3(nsw, max_s), dim3(kPLruSortThreads), 0, s, st, nsw);
}

void cparam_stage2(const CParamState &st, BatchScratch &sc, CParamScratch &ps, const int32_t *acquire,
                   const uint32_t *voff, const int64_t *values, int64_t ts_base, const uint32_t *ts_off, uint32_t n,
                   uint32_t nslow, void *out_v, hipStream_t s) {
    sc.counters_clean = 0;  // the stages use the control words
    if (n == 0) return;
    uint64_t *out = (uint64_t *)out_v;
    const uint32_t ntiles = (n + kTileElems - 1) / kTileElems;
    const uint32_t fb = std::max<uint32_t>(1, std::min<uint32_t>((n + kThreads - 1) / kThreads, 16384));
    auto runs = [&](const uint64_t *el, uint32_t invalid_key) {
        SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, 64, s));
        hipLaunchKernelGGL(k_runs_up, dim3(ntiles), dim3(kRunThreads), 0, s, el, n, invalid_key, (Agg *)sc.tile_agg,
                           sc.tile_valid, nullptr);
        hipLaunchKernelGGL(k_runs_tiles, dim3(1), dim3(kTileScanThreads), 0, s, (const Agg *)sc.tile_agg, sc.tile_valid,
                           ntiles, (Agg *)sc.tile_carry, sc.counters, nullptr);
        hipLaunchKernelGGL(k_runs_down, dim3(ntiles), dim3(kRunThreads), 0, s, el, invalid_key,
                           (const Agg *)sc.tile_carry, sc);
    };
    if (nslow < n) {  // key-parallel path (elements keyed by kidx, invalid = kmask + 1)
        const uint32_t kinv = st.kmask + 1;
        int bits = 1;
        while (((uint64_t)1 << bits) < (uint64_t)kinv + 1) ++bits;
        const int np = radix_sort_u64(sc.el[0], sc.el[1], n, kSlotShift, bits, sc.radix, s, false);
        const uint64_t *el = sc.el[np & 1];
        runs(el, kinv);
        hipLaunchKernelGGL(k_pflows, dim3(fb), dim3(kThreads), 0, s, st, sc, el, acquire, ts_base, ts_off, out);
        hipLaunchKernelGGL(k_results, dim3(ntiles), dim3(kRunThreads), 0, s, sc, el, kinv, out);
    }
    if (nslow > 0) {  // sequential path, one lane per rule
        int bits = 1;
        while (((uint64_t)1 << bits) < (uint64_t)st.nslots + 1) ++bits;
        const int np = radix_sort_u64(ps.els[0], ps.els[1], n, kSlotShift, bits, sc.radix, s, false);
        const uint64_t *els = ps.els[np & 1];
        runs(els, st.nslots);
        hipLaunchKernelGGL(k_pslow, dim3(fb), dim3(kThreads), 0, s, st, sc, els, acquire, voff, values, ps.vkey,
                           ts_base, ts_off, out);
    }
}

void cparam_sum(const CParamState &st, uint32_t slot, int64_t value, int64_t now, int64_t *d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_psum, dim3(1), dim3(64), 0, s, st, slot, value, now, d_out);
}

void cparam_top_values(const CParamState &st, uint32_t slot, int64_t now, uint32_t number, int64_t *d_list,
                       uint32_t *d_count, int64_t *d_val, double *d_qps, uint32_t *d_n, hipStream_t s) {
    hipLaunchKernelGGL(k_pwindow, dim3(1), dim3(64), 0, s, st, slot, now);
    SGA_HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(uint32_t), s));
    const uint32_t nk = st.kmask + 1;
    hipLaunchKernelGGL(k_ptop_collect, dim3((nk + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st, slot, now,
                       d_list, d_count);
    hipLaunchKernelGGL(k_ptop_select, dim3(1), dim3(1024), 0, s, st, slot, d_list, d_count, number, d_val, d_qps,
                       d_n);
}

void cparam_init_rule(const CParamState &st, uint32_t slot, hipStream_t s) {
    hipLaunchKernelGGL(k_pinit_rule, dim3(1), dim3(64), 0, s, st, slot);
}

void cluster_metric_nodes(const ClusterState &st, const int64_t *slot_fid, int64_t now, void *out, uint32_t cap,
                          uint32_t *count, hipStream_t s) {
    SGA_HIP_CHECK(hipMemsetAsync(count, 0, 4, s));
    if (st.nslots == 0) return;
    hipLaunchKernelGGL(k_cluster_nodes, dim3((st.nslots + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st,
                       slot_fid, now, (sga_cluster_metric_node *)out, cap, count);
}

__global__ __launch_bounds__(kThreads) void k_ts_offsets(const int32_t *__restrict__ ts, int64_t lo,
                                                         uint32_t *__restrict__ off, uint32_t n) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) off[i] = (uint32_t)((int64_t)ts[i] - lo);
}

void cluster_ts_offsets(const int32_t *ts, int64_t lo, uint32_t *off, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_ts_offsets, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, ts, lo, off, n);
}

__global__ __launch_bounds__(kThreads) void k_ts_minmax(const int64_t *__restrict__ ts, uint32_t n, int64_t *mm) {
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const int64_t t = ts[i];
        lo = min(lo, t);
        hi = max(hi, t);
    }
    lo = wave_min_i64(lo);
    hi = wave_max_i64(hi);
    if ((threadIdx.x & 63) == 0) {
        atomicMin((long long *)&mm[0], (long long)lo);
        atomicMax((long long *)&mm[1], (long long)hi);
    }
}

__global__ void k_ts_minmax_init(int64_t *mm) {
    if (threadIdx.x == 0) {
        mm[0] = INT64_MAX;
        mm[1] = INT64_MIN;
    }
}

void cluster_ts_minmax(const int64_t *ts, uint32_t n, int64_t *minmax, hipStream_t s) {
    hipLaunchKernelGGL(k_ts_minmax_init, dim3(1), dim3(64), 0, s, minmax);
    if (n) hipLaunchKernelGGL(k_ts_minmax, dim3(std::min<uint32_t>((n + kThreads - 1) / kThreads, 2048)), dim3(kThreads), 0, s,
                              ts, n, minmax);
}

__global__ __launch_bounds__(kThreads) void k_ts_offsets64(const int64_t *__restrict__ ts, int64_t lo,
                                                           uint32_t *__restrict__ off, uint32_t n) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) off[i] = (uint32_t)(ts[i] - lo);
}

void cluster_ts_offsets64(const int64_t *ts, int64_t lo, uint32_t *off, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_ts_offsets64, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, ts, lo, off, n);
}

void cluster_init_limiter(NsLimiterDev *d, hipStream_t s) {
    hipLaunchKernelGGL(k_lim_init, dim3(1), dim3(64), 0, s, d);
}

// ---- Envoy RLS over device buffers (SentinelEnvoyRlsServiceImpl.shouldRateLimit,
// envoy/rls/SentinelEnvoyRlsServiceImpl.java:52-90): every descriptor of a request is one
// SimpleClusterFlowChecker request at the request's time with acquire = hitsAddend (0 -> 1).
// A request with hitsAddend < 0 checks nothing: its descriptors take flowId 0, which no rule can
// hold (cluster rules need flowId > 0), so they answer NO_RULE_EXISTS without touching a window.
__global__ __launch_bounds__(kThreads) void k_rls_expand(const uint32_t *__restrict__ off, uint32_t nreq,
                                                         const int64_t *__restrict__ dfid,
                                                         const int32_t *__restrict__ hits,
                                                         const uint32_t *__restrict__ ts_off, int64_t *fid_out,
                                                         int32_t *acq_out, uint32_t *ts_out) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= nreq) return;
    const int32_t h = hits[r];
    const int32_t a = h <= 0 ? 1 : h;
    const uint32_t t = ts_off[r];
    for (uint32_t d = off[r]; d < off[r + 1]; ++d) {
        fid_out[d] = h < 0 ? 0 : dfid[d];
        acq_out[d] = a;
        ts_out[d] = t;
    }
}

// Code.OVER_LIMIT (2) when a descriptor is neither OK nor NO_RULE_EXISTS, Code.OK (1) otherwise,
// -1 for hitsAddend < 0 (onError); per descriptor the TokenResult status and remaining.
__global__ __launch_bounds__(kThreads) void k_rls_finish(const uint32_t *__restrict__ off, uint32_t nreq,
                                                         const int32_t *__restrict__ hits,
                                                         const uint64_t *__restrict__ res, int8_t *desc_status,
                                                         int32_t *desc_rem, int32_t *code) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= nreq) return;
    const bool skip = hits[r] < 0;
    bool blocked = false;
    for (uint32_t d = off[r]; d < off[r + 1]; ++d) {
        const int8_t stt = skip ? (int8_t)TRS_NO_RULE_EXISTS : (int8_t)(res[d] >> 48);
        blocked |= stt != TRS_OK && stt != TRS_NO_RULE_EXISTS;
        if (desc_status) desc_status[d] = stt;
        if (desc_rem) desc_rem[d] = skip ? 0 : (int32_t)(uint32_t)res[d];
    }
    code[r] = skip ? -1 : (blocked ? 2 : 1);
}

void rls_expand(const uint32_t *off, uint32_t nreq, const int64_t *dfid, const int32_t *hits, const uint32_t *ts_off,
                int64_t *fid_out, int32_t *acq_out, uint32_t *ts_out, hipStream_t s) {
    if (!nreq) return;
    hipLaunchKernelGGL(k_rls_expand, dim3((nreq + kThreads - 1) / kThreads), dim3(kThreads), 0, s, off, nreq, dfid,
                       hits, ts_off, fid_out, acq_out, ts_out);
}

void rls_finish(const uint32_t *off, uint32_t nreq, const int32_t *hits, const uint64_t *res, int8_t *desc_status,
                int32_t *desc_rem, int32_t *code, hipStream_t s) {
    if (!nreq) return;
    hipLaunchKernelGGL(k_rls_finish, dim3((nreq + kThreads - 1) / kThreads), dim3(kThreads), 0, s, off, nreq, hits,
                       res, desc_status, desc_rem, code);
}

void cluster_metric_sums(const ClusterState &st, uint32_t slot, int64_t now, int64_t *d_out7, hipStream_t s) {
    hipLaunchKernelGGL(k_metric_sums, dim3(1), dim3(64), 0, s, st, slot, now, d_out7);
}

void cluster_init_slots(const ClusterState &st, const uint32_t *d_slots, uint32_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_init_slots, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st, d_slots, n);
}

void cluster_sync_rec_thr(const ClusterState &st, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_rec_thr, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st, n);
}

}  // namespace sga
