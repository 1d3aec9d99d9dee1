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

#include <cstdlib>

#include <algorithm>

namespace sga {

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTileElems = kThreads * kItems;  // 4096

enum : int8_t { TRS_BAD_REQUEST = -4, TRS_TOO_MANY_REQUEST = -2, TRS_FAIL = -1, TRS_OK = 0, TRS_BLOCKED = 1,
                TRS_SHOULD_WAIT = 2, TRS_NO_RULE_EXISTS = 3 };
enum : uint8_t { RUN_FAST = 0, RUN_DONE = 1 };

__device__ __forceinline__ uint64_t pack_result(int8_t status, int32_t remaining, int32_t wait) {
    return (uint64_t)(uint32_t)remaining | ((uint64_t)(uint16_t)(int16_t)wait << 32) |
           ((uint64_t)(uint8_t)status << 48);
}

__device__ __forceinline__ HashEntry slot_lookup(const ClusterState &st, int64_t fid) {
    uint32_t h = (uint32_t)hash_flow_id(fid) & st.hmask;
    for (uint32_t probe = 0; probe <= st.hmask; ++probe) {
        const HashEntry e = st.htab[h];
        if (e.key == fid || e.key == 0) return e;
        h = (h + 1) & st.hmask;
    }
    return HashEntry{0, 0, 0};
}

// ---------------------------------------------------------------- classify
// kClassifyItems requests per thread (strided by the block size, so every load stays coalesced);
// the first hash probes of all of them are issued before any is resolved.
constexpr int kClassifyItems = 4;

__global__ __launch_bounds__(kThreads) void k_classify(ClusterState st, const int64_t *__restrict__ flow_id,
                                                       const int32_t *__restrict__ acquire,
                                                       const uint8_t *__restrict__ prio,
                                                       const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                       uint32_t n, int simple, uint32_t invalid_key, uint32_t *__restrict__ keys,
                                                       Payload *__restrict__ pay, uint64_t *__restrict__ out,
                                                       uint32_t *__restrict__ counters) {
    const uint32_t base = blockIdx.x * (kThreads * kClassifyItems) + threadIdx.x;
    int64_t fid[kClassifyItems];
    int32_t acq[kClassifyItems];
    uint32_t h[kClassifyItems];
    HashEntry e[kClassifyItems];
#pragma unroll
    for (int u = 0; u < kClassifyItems; ++u) {
        const uint32_t i = base + u * kThreads;
        fid[u] = i < n ? flow_id[i] : 0;
        acq[u] = i < n ? acquire[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kClassifyItems; ++u) {
        h[u] = (uint32_t)hash_flow_id(fid[u]) & st.hmask;
        e[u] = fid[u] > 0 ? st.htab[h[u]] : HashEntry{0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < kClassifyItems; ++u) {
        const uint32_t i = base + u * kThreads;
        if (i >= n) continue;
        const int64_t f = fid[u];
        const int32_t a = acq[u];
        int8_t status = TRS_OK;
        HashEntry he = e[u];
        if (!simple && (f <= 0 || a <= 0)) {
            status = TRS_BAD_REQUEST;  // DefaultTokenService.notValidRequest, :87-89
        } else {
            // ClusterFlowRuleManager.getFlowRuleById: validId(id > 0) && FLOW_RULES.get(id)
            if (f > 0 && he.key != f && he.key != 0) {  // continue the linear probe
                uint32_t hh = h[u];
                for (uint32_t probe = 1; probe <= st.hmask; ++probe) {
                    hh = (hh + 1) & st.hmask;
                    he = st.htab[hh];
                    if (he.key == f || he.key == 0) break;
                }
            }
            if (he.key != f || f <= 0) status = TRS_NO_RULE_EXISTS;
        }
        if (status != TRS_OK) {
            out[i] = pack_result(status, 0, 0);
            keys[i] = invalid_key;
            pay[i] = Payload{i, 0u, 0u, 0u};
        } else {
            keys[i] = he.slot;
            const uint32_t p = (!simple && prio && prio[i]) ? 0x80000000u : 0u;
            const uint32_t off = ts_off[i];
            const int64_t t = ts_base + (int64_t)off;
            pay[i] = Payload{i, off, (uint32_t)a | p, (uint32_t)(t / (int64_t)he.W)};
        }
    }
    (void)counters;  // the valid count is derived after the sort (invalid keys sort last)
}

// ---------------------------------------------------------------- runs (segmented scan)
// A run = maximal group of sorted requests with the same (rule, window bucket).
// Segmented scan value: run/flow head counts (plain sums) and, since the last
// run head, the number of prioritized requests and the min/max acquire count.
struct Agg {
    uint32_t nh, nf;  // run heads, flow heads
    uint32_t flag;    // segment (run) head seen
    uint32_t cnt;     // prioritized events since last run head
    int32_t mn, mx;   // min / max acquire since last run head
};

__device__ __forceinline__ Agg agg_identity() { return Agg{0, 0, 0, 0, INT32_MAX, INT32_MIN}; }

__device__ __forceinline__ Agg agg_combine(const Agg &a, const Agg &b) {
    Agg r;
    r.nh = a.nh + b.nh;
    r.nf = a.nf + b.nf;
    r.flag = a.flag | b.flag;
    r.cnt = b.flag ? b.cnt : a.cnt + b.cnt;
    r.mn = b.flag ? b.mn : min(a.mn, b.mn);
    r.mx = b.flag ? b.mx : max(a.mx, b.mx);
    return r;
}

__device__ __forceinline__ Agg agg_shfl_up(const Agg &v, int o) {
    return Agg{(uint32_t)__shfl_up((int)v.nh, o, 64), (uint32_t)__shfl_up((int)v.nf, o, 64),
               (uint32_t)__shfl_up((int)v.flag, o, 64), (uint32_t)__shfl_up((int)v.cnt, o, 64),
               __shfl_up(v.mn, o, 64), __shfl_up(v.mx, o, 64)};
}

__device__ __forceinline__ Agg agg_shfl(const Agg &v, int src) {
    return Agg{(uint32_t)__shfl((int)v.nh, src, 64), (uint32_t)__shfl((int)v.nf, src, 64),
               (uint32_t)__shfl((int)v.flag, src, 64), (uint32_t)__shfl((int)v.cnt, src, 64),
               __shfl(v.mn, src, 64), __shfl(v.mx, src, 64)};
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

constexpr int kRunThreads = 512;
constexpr int kRunRounds = 8;                       // rounds of 64 per wave
constexpr int kRunWaves = kRunThreads / 64;         // 8
constexpr int kWaveElems = kRunRounds * 64;         // 512
static_assert(kWaveElems * kRunWaves == kTileElems, "tile geometry");

struct RunIn {
    uint32_t key;
    Payload q;
};

__device__ __forceinline__ RunIn run_load(const uint32_t *keys, const Payload *pay, uint32_t e, uint32_t nlim,
                                          uint32_t invalid_key) {
    RunIn x;
    if (e < nlim) {
        x.key = keys[e];
        x.q = pay[e];
    } else {
        x.key = invalid_key;
        x.q = Payload{0, 0, 0, 0};
    }
    return x;
}

__device__ __forceinline__ RunIn run_shfl_up1(const RunIn &x) {
    RunIn y;
    y.key = (uint32_t)__shfl_up((int)x.key, 1, 64);
    y.q.idx = (uint32_t)__shfl_up((int)x.q.idx, 1, 64);
    y.q.ts_off = (uint32_t)__shfl_up((int)x.q.ts_off, 1, 64);
    y.q.acq_prio = (uint32_t)__shfl_up((int)x.q.acq_prio, 1, 64);
    y.q.bucket = (uint32_t)__shfl_up((int)x.q.bucket, 1, 64);
    return y;
}

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }

// Agg contribution of element x with predecessor px (has_prev = x is not element 0)
__device__ __forceinline__ Agg run_value(const RunIn &x, const RunIn &px, bool has_prev, bool valid) {
    if (!valid) return agg_identity();
    const bool fh = !has_prev || x.key != px.key;
    const bool h = fh || x.q.bucket != px.q.bucket;
    const int32_t a = (int32_t)(x.q.acq_prio & 0x7FFFFFFFu);
    return Agg{h ? 1u : 0u, fh ? 1u : 0u, h ? 1u : 0u, x.q.acq_prio >> 31, a, a};
}

// Per tile: aggregate over its valid elements + count of valid elements.
__global__ __launch_bounds__(kRunThreads) void k_runs_up(const uint32_t *__restrict__ keys,
                                                      const Payload *__restrict__ pay, uint32_t n,
                                                      uint32_t invalid_key, Agg *__restrict__ tile_agg,
                                                      uint32_t *__restrict__ tile_valid) {
    __shared__ Agg wagg[kRunWaves];
    __shared__ uint32_t wval[kRunWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wb = blockIdx.x * kTileElems + wave * kWaveElems;
    RunIn last = run_load(keys, pay, wb - 1, wb > 0 ? min(wb, n) : 0, invalid_key);  // element wb-1 (if any)
    Agg acc = agg_identity();
    uint32_t nval = 0;
    for (int r = 0; r < kRunRounds; ++r) {
        const uint32_t e = wb + r * 64 + lane;
        const RunIn x = run_load(keys, pay, e, n, invalid_key);
        const bool valid = x.key != invalid_key;
        RunIn px = run_shfl_up1(x);
        if (lane == 0) px = last;
        Agg v = run_value(x, px, e > 0, valid);
        // ordered tree reduction: lane 0 ends with lanes 0..63 combined in order
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const Agg y = agg_shfl(v, (lane + o) & 63);
            if (lane + o < 64 && (lane & (2 * o - 1)) == 0) v = agg_combine(v, y);
        }
        acc = agg_combine(acc, agg_shfl(v, 0));
        nval += (uint32_t)__popcll(__ballot(valid));
        last.key = shfl_u32(x.key, 63);
        last.q.bucket = shfl_u32(x.q.bucket, 63);
    }
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

// Single workgroup: tile carries, nvalid / nruns / nflows.
__global__ __launch_bounds__(kTileScanThreads) void k_runs_tiles(const Agg *__restrict__ tile_agg,
                                                                 const uint32_t *__restrict__ tile_valid,
                                                                 uint32_t ntiles, Agg *__restrict__ tile_carry,
                                                                 uint32_t *__restrict__ counters) {
    Agg carry = agg_identity();
    uint32_t nvalid = 0;
    for (uint32_t b = 0; b < ntiles; b += kTileScanThreads) {
        const uint32_t t = b + threadIdx.x;
        const Agg v = t < ntiles ? tile_agg[t] : agg_identity();
        const uint32_t c = t < ntiles ? tile_valid[t] : 0;
        Agg total;
        const Agg ex = block_excl_scan_1024(v, &total);
        if (t < ntiles) tile_carry[t] = agg_combine(carry, ex);
        carry = agg_combine(carry, total);
        // valid counts: plain block sum
        uint32_t s = c;
        for (int o = 32; o > 0; o >>= 1) s += (uint32_t)__shfl_down((int)s, o, 64);
        __shared__ uint32_t ws[kTileScanThreads / 64];
        if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 0; w < kTileScanThreads / 64; ++w) nvalid += ws[w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counters[0] = nvalid;
        counters[1] = carry.nh;
        counters[2] = carry.nf;
    }
}

// Per tile: per-event run id and prioritized prefix; run and flow records.
__global__ __launch_bounds__(kRunThreads) void k_runs_down(const uint32_t *__restrict__ keys,
                                                        const Payload *__restrict__ pay, uint32_t invalid_key,
                                                        const Agg *__restrict__ tile_carry, BatchScratch sc) {
    __shared__ Agg wagg[kRunWaves];
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wb = base + wave * kWaveElems;
    RunIn x[kRunRounds];
    const RunIn first_prev = run_load(keys, pay, wb - 1, wb > 0 ? min(wb, nvalid) : 0, invalid_key);
    RunIn last = first_prev;
    Agg acc = agg_identity();
    // pass 1: ordered wave reduction per round (elements stay in registers)
#pragma unroll
    for (int r = 0; r < kRunRounds; ++r) {
        const uint32_t e = wb + r * 64 + lane;
        x[r] = run_load(keys, pay, e, nvalid, invalid_key);
        RunIn px = run_shfl_up1(x[r]);
        if (lane == 0) px = last;
        Agg v = run_value(x[r], px, e > 0, e < nvalid);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const Agg y = agg_shfl(v, (lane + o) & 63);
            if (lane + o < 64 && (lane & (2 * o - 1)) == 0) v = agg_combine(v, y);
        }
        acc = agg_combine(acc, agg_shfl(v, 0));
        last.key = shfl_u32(x[r].key, 63);
        last.q.bucket = shfl_u32(x[r].q.bucket, 63);
    }
    if (lane == 0) wagg[wave] = acc;
    __syncthreads();
    Agg carry = tile_carry[blockIdx.x];
    for (int w = 0; w < wave; ++w) carry = agg_combine(carry, wagg[w]);
    // element after this wave's sub-tile (for the last element of the last round)
    const uint32_t enext = wb + kWaveElems;
    const RunIn after = run_load(keys, pay, enext, nvalid, invalid_key);
    // pass 2: inclusive scan per round with the running carry
#pragma unroll
    for (int r = 0; r < kRunRounds; ++r) {
        const uint32_t e = wb + r * 64 + lane;
        // cross-lane reads are done by every lane (a shuffle from an inactive lane is undefined)
        RunIn px = run_shfl_up1(x[r]);
        const uint32_t prev_key = r == 0 ? first_prev.key : shfl_u32(x[r > 0 ? r - 1 : 0].key, 63);
        const uint32_t prev_bucket = r == 0 ? first_prev.q.bucket : shfl_u32(x[r > 0 ? r - 1 : 0].q.bucket, 63);
        uint32_t nkey = (uint32_t)__shfl_down((int)x[r].key, 1, 64);
        uint32_t nbucket = (uint32_t)__shfl_down((int)x[r].q.bucket, 1, 64);
        const uint32_t next_key = r + 1 < kRunRounds ? shfl_u32(x[r + 1 < kRunRounds ? r + 1 : r].key, 0) : after.key;
        const uint32_t next_bucket =
            r + 1 < kRunRounds ? shfl_u32(x[r + 1 < kRunRounds ? r + 1 : r].q.bucket, 0) : after.q.bucket;
        if (lane == 0) {
            px.key = prev_key;
            px.q.bucket = prev_bucket;
        }
        if (lane == 63) {
            nkey = next_key;
            nbucket = next_bucket;
        }
        const Agg vr = wave_incl_scan(run_value(x[r], px, e > 0, e < nvalid), lane);
        const Agg run = agg_combine(carry, vr);  // inclusive up to e
        carry = agg_combine(carry, agg_shfl(vr, 63));
        if (e >= nvalid) continue;
        const uint32_t rid = run.nh - 1;
        const uint32_t p = x[r].q.acq_prio >> 31;
        sc.ev_run[e] = rid;
        sc.ev_cp[e] = run.cnt - p;
        const bool fh = e == 0 || x[r].key != px.key;
        const bool h = fh || x[r].q.bucket != px.q.bucket;
        if (h) {
            sc.run_start[rid] = e;
            sc.run_slot[rid] = x[r].key;
            sc.run_t0off[rid] = x[r].q.ts_off;
        }
        if (fh) sc.flow_first_run[run.nf - 1] = rid;
        const bool last_of_run = (e + 1 >= nvalid) || nkey != x[r].key || nbucket != x[r].q.bucket;
        if (last_of_run) {
            sc.run_end[rid] = e + 1;
            sc.run_cp[rid] = run.cnt;
            sc.run_amin[rid] = run.mn;
            sc.run_amax[rid] = run.mx;
        }
    }
}

// ---------------------------------------------------------------- exact per-request replay (device)
// Window state of a rule lives in one contiguous record of 8 x S int64:
//   [start x S][PASS x S][WAITING x S][per bucket j: BLOCK, PASS_REQUEST, BLOCK_REQUEST,
//   OCCUPIED_PASS, OCCUPIED_BLOCK]
// so the window sums read 3 dense vectors and a run's update writes the current bucket's
// PASS, WAITING and one 40-byte group.
struct Rec {
    int64_t *r;
    int S;
    __device__ __forceinline__ int64_t &start(int j) const { return r[j]; }
    __device__ __forceinline__ int64_t &cnt(int ev, int j) const {
        if (ev == CEV_PASS) return r[S + j];
        if (ev == CEV_WAITING) return r[2 * S + j];
        return r[3 * S + 5 * j + (ev - 1)];  // BLOCK..OCCUPIED_BLOCK = ordinals 1..5
    }
};

__device__ __forceinline__ Rec rec_of(const ClusterState &st, const SlotParam &P) {
    return Rec{st.rec + (size_t)P.boff * 8, P.S};
}

struct WinRef {
    int j;
    bool detached;
};

__device__ __forceinline__ void bucket_zero(const Rec &R, int j) {
#pragma unroll
    for (int k = 0; k < CEV_N; ++k) R.cnt(k, j) = 0;
}

// LeapArray.currentWindow(t) on a ClusterMetricLeapArray (t >= 0)
__device__ WinRef cur_window(const ClusterState &st, const SlotParam &P, uint32_t s, int64_t t) {
    const Rec R = rec_of(st, P);
    const int j = (int)((t / P.W) % P.S);
    const int64_t ws = t - t % P.W;
    const int64_t old = R.start(j);
    if (old == kAbsent) {  // newEmptyBucket: no occupy transfer
        R.start(j) = ws;
        bucket_zero(R, j);
        return WinRef{j, false};
    }
    if (ws == old) return WinRef{j, false};
    if (ws > old) {  // resetWindowTo + transferOccupyToBucket
        R.start(j) = ws;
        bucket_zero(R, j);
        SlotOcc &o = st.occ[s];
        if (o.has_occ) {
            R.cnt(CEV_OCCUPIED_PASS, j) += o.occ_pass;
            R.cnt(CEV_PASS, j) += o.occ_pass;
            o.occ_pass = 0;
            R.cnt(CEV_PASS_REQUEST, j) += o.occ_preq;
            o.occ_preq = 0;
            o.has_occ = 0;
        }
        return WinRef{j, false};
    }
    return WinRef{j, true};  // time went backwards: detached bucket, adds lost
}

__device__ int64_t values_sum(const ClusterState &st, const SlotParam &P, int64_t t, int ev) {
    const Rec R = rec_of(st, P);
    int64_t s = 0;
    for (int j = 0; j < P.S; ++j) {
        const int64_t w = R.start(j);
        if (w != kAbsent && !(t - w > (int64_t)P.interval)) s += R.cnt(ev, j);
    }
    return s;
}

__device__ __forceinline__ double get_avg(const ClusterState &st, const SlotParam &P, uint32_t s, int64_t t, int ev) {
    cur_window(st, P, s, t);
    return (double)values_sum(st, P, t, ev) / P.isec;
}

__device__ __forceinline__ void metric_add(const ClusterState &st, const SlotParam &P, uint32_t s, int64_t t, int ev,
                                           int64_t n) {
    const WinRef w = cur_window(st, P, s, t);
    if (!w.detached) rec_of(st, P).cnt(ev, w.j) += n;
}

// ClusterMetricLeapArray.getFirstCountOfWindow(PASS) = getValidHead(now).value().get(PASS)
__device__ __forceinline__ int64_t head_pass(const ClusterState &st, const SlotParam &P, int64_t t) {
    const Rec R = rec_of(st, P);
    const int j = (int)(((t + P.W) / P.W) % P.S);
    const int64_t w = R.start(j);
    return (w != kAbsent && !(t - w > (int64_t)P.interval)) ? R.cnt(CEV_PASS, j) : 0;
}

// ClusterFlowChecker.acquireClusterToken / SimpleClusterFlowChecker.acquireClusterToken for one request
__device__ uint64_t request_exact(const ClusterState &st, uint32_t s, int64_t t, int32_t a, bool p, int simple) {
    const SlotParam P = st.param[s];
    const double thr = simple ? P.thr_simple : P.thr;
    const double latest = get_avg(st, P, s, t, CEV_PASS);
    const double rem = thr - latest - (double)a;
    if (rem >= 0) {
        metric_add(st, P, s, t, CEV_PASS, a);
        metric_add(st, P, s, t, CEV_PASS_REQUEST, 1);
        if (p) metric_add(st, P, s, t, CEV_OCCUPIED_PASS, a);
        return pack_result(TRS_OK, j_d2i(rem), 0);
    }
    if (p) {
        const double occupy_avg = get_avg(st, P, s, t, CEV_WAITING);
        if (occupy_avg <= st.max_occupy_ratio * thr) {
            // ClusterMetric.tryOccupyNext(PASS, a, thr)
            const double latest2 = get_avg(st, P, s, t, CEV_PASS);
            const int64_t head = head_pass(st, P, t);
            SlotOcc &o = st.occ[s];
            if (latest2 + (double)((int64_t)a + o.occ_pass) - (double)head <= thr) {
                o.occ_pass += a;
                o.occ_preq += 1;
                o.has_occ = 1;
                metric_add(st, P, s, t, CEV_WAITING, a);
                const int32_t wait = 1000 / P.S;
                if (wait > 0) return pack_result(TRS_SHOULD_WAIT, 0, wait);
            }
        }
    }
    metric_add(st, P, s, t, CEV_BLOCK, a);
    metric_add(st, P, s, t, CEV_BLOCK_REQUEST, 1);
    if (p) metric_add(st, P, s, t, CEV_OCCUPIED_BLOCK, a);
    return pack_result(TRS_BLOCKED, 0, 0);
}

// ---------------------------------------------------------------- flows: resolve runs per rule
__device__ __forceinline__ bool pass_cond(double thr, double isec, int64_t sum, int32_t a) {
    // nextRemaining = globalThreshold - latestQps - acquireCount >= 0   ClusterFlowChecker.java:67-71
    return thr - (double)sum / isec - (double)a >= 0;
}

// G lanes per rule: lanes load the record's start/PASS/WAITING vectors in parallel, lane 0
// of the group resolves the runs.  G = 1 (one rule per lane) keeps the most rules in flight.
template <int G>
__device__ __forceinline__ int64_t group_sum(int64_t v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
        const int lo = __shfl_xor((int)(uint32_t)v, o, G);
        const int hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), o, G);
        v += (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    }
    return v;
}

// First k in [0, n] with !pass_cond(s0 + k*a): a closed-form guess corrected against the
// exact predicate (monotone in k), so the result equals the sequential one.
__device__ __forceinline__ uint32_t pass_prefix(double thr, double isec, int64_t s0, int32_t a, uint32_t n) {
    if (n == 0) return 0;
    if (a <= 0) return pass_cond(thr, isec, s0, a) ? n : 0u;
    const double g = floor(((thr - (double)a) * isec - (double)s0) / (double)a) + 1.0;
    uint32_t k = 0;
    if (g >= (double)n) k = n;
    else if (g > 0) k = (uint32_t)g;
    while (k > 0 && !pass_cond(thr, isec, s0 + (int64_t)(k - 1) * a, a)) --k;
    while (k < n && pass_cond(thr, isec, s0 + (int64_t)k * a, a)) ++k;
    return k;
}

__device__ __forceinline__ int64_t i64_lo(const int4 &v) {
    return (int64_t)(((uint64_t)(uint32_t)v.y << 32) | (uint32_t)v.x);
}
__device__ __forceinline__ int64_t i64_hi(const int4 &v) {
    return (int64_t)(((uint64_t)(uint32_t)v.w << 32) | (uint32_t)v.z);
}

// One rule per lane, fused window update: the current bucket's seven counters are
// loaded once (or start from zero when LeapArray.currentWindow rotates it), updated in
// registers and stored once; the head bucket (LeapArray.getValidHead) is read from the
// same vector loads as the window sums.  Same decisions as k_flows<G>.
__global__ __launch_bounds__(kThreads) void k_flows1(ClusterState st, BatchScratch sc, const Payload *__restrict__ pay,
                                                     int64_t ts_base, int simple, uint64_t *__restrict__ out) {
    const uint32_t nflows = sc.counters[2];
    const uint32_t nruns = sc.counters[1];
    for (uint32_t fl = blockIdx.x * kThreads + threadIdx.x; fl < nflows; fl += gridDim.x * kThreads) {
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t s = sc.run_slot[r];
            const SlotParam P = st.param[s];
            const Rec R = rec_of(st, P);
            const uint32_t j0 = sc.run_start[r], j1 = sc.run_end[r];
            const uint32_t n = j1 - j0;
            const int64_t t0 = ts_base + (int64_t)sc.run_t0off[r];
            const uint32_t cp_tot = sc.run_cp[r];
            const int32_t a = sc.run_amin[r];
            const double thr = simple ? P.thr_simple : P.thr;
            const int64_t ws = t0 - t0 % P.W;
            const int cj = (int)((t0 / P.W) % P.S);
            const int64_t old = R.start(cj);
            bool fast = (a == sc.run_amax[r]) && !(old != kAbsent && ws < old);
            if (cp_tot > 0 && (P.S <= 1 || 1000 / P.S <= 0)) fast = false;
            if (!fast) {  // exact replay of every request of the run, in order
                for (uint32_t j = j0; j < j1; ++j) {
                    const Payload q = pay[j];
                    const int64_t t = ts_base + (int64_t)q.ts_off;
                    out[q.idx] = request_exact(st, s, t, (int32_t)(q.acq_prio & 0x7FFFFFFFu), (q.acq_prio >> 31) != 0,
                                               simple);
                }
                sc.run_mode[r] = RUN_DONE;
                continue;
            }
            const int jh = (int)(((t0 + P.W) / P.W) % P.S);  // LeapArray.getValidHead index
            int64_t bp = 0, bw = 0, hstart = kAbsent, hpass = 0;
            if ((P.S & 1) == 0) {
                const int4 *v = reinterpret_cast<const int4 *>(R.r);
                const int hs = P.S >> 1;
                for (int q = 0; q < hs; ++q) {
                    const int4 st2 = v[q], ps2 = v[hs + q], wt2 = v[2 * hs + q];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int jj = 2 * q + h;
                        const int64_t w = h ? i64_hi(st2) : i64_lo(st2);
                        const int64_t pv = h ? i64_hi(ps2) : i64_lo(ps2);
                        if (jj == jh) {
                            hstart = w;
                            hpass = pv;
                        }
                        if (jj != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval)) {
                            bp += pv;
                            bw += h ? i64_hi(wt2) : i64_lo(wt2);
                        }
                    }
                }
            } else {
                for (int jj = 0; jj < P.S; ++jj) {
                    const int64_t w = R.start(jj);
                    const int64_t pv = R.cnt(CEV_PASS, jj);
                    if (jj == jh) {
                        hstart = w;
                        hpass = pv;
                    }
                    if (jj != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval)) {
                        bp += pv;
                        bw += R.cnt(CEV_WAITING, jj);
                    }
                }
            }
            // ---- LeapArray.currentWindow(t0) on the current bucket, in registers
            const bool rot = old == kAbsent || ws > old;
            int64_t c[CEV_N];
            SlotOcc o{0, 0, 0};
            bool occ_dirty = false;
            if (rot) {
#pragma unroll
                for (int k = 0; k < CEV_N; ++k) c[k] = 0;
                if (old != kAbsent) {  // resetWindowTo + transferOccupyToBucket
                    o = st.occ[s];
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
#pragma unroll
                for (int k = 0; k < CEV_N; ++k) c[k] = R.cnt(k, cj);
            }
            // getValidHead after the rotation (the head is the current bucket when S == 1)
            int64_t head;
            if (jh == cj) head = c[CEV_PASS];
            else head = (hstart != kAbsent && !(t0 - hstart > (int64_t)P.interval)) ? hpass : 0;
            const int64_t s0 = bp + c[CEV_PASS];
            const int64_t w0 = bw + c[CEV_WAITING];
            const uint32_t f = pass_prefix(thr, P.isec, s0, a, n);
            const uint32_t cpf = (f >= n) ? cp_tot : (cp_tot ? sc.ev_cp[j0 + f] : 0u);
            const uint32_t np_after = cp_tot - cpf;
            uint32_t cw = 0;
            if (np_after > 0) {
                if (!occ_dirty && !rot) o = st.occ[s];
                else if (!occ_dirty) o = st.occ[s];
                const double latest = (double)(s0 + (int64_t)f * a) / P.isec;
                const double lim = st.max_occupy_ratio * thr;
                const int64_t occ0 = o.occ_pass;
                uint32_t l2 = 0, h2 = np_after;
                while (l2 < h2) {
                    const uint32_t cc = l2 + ((h2 - l2) >> 1);
                    const int64_t add = (int64_t)cc * a;
                    const bool ok = ((double)(w0 + add) / P.isec <= lim) &&
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
            const int64_t wa = (int64_t)cw * a;
            const uint32_t nblk = n - f - cw;
            c[CEV_PASS] += (int64_t)f * a;
            c[CEV_PASS_REQUEST] += f;
            c[CEV_OCCUPIED_PASS] += (int64_t)cpf * a;
            c[CEV_WAITING] += wa;
            c[CEV_BLOCK] += (int64_t)nblk * a;
            c[CEV_BLOCK_REQUEST] += nblk;
            c[CEV_OCCUPIED_BLOCK] += (int64_t)(np_after - cw) * a;
            if (rot) R.start(cj) = ws;
#pragma unroll
            for (int k = 0; k < CEV_N; ++k) R.cnt(k, cj) = c[k];
            if (occ_dirty) st.occ[s] = o;
            sc.run_s0[r] = s0;
            sc.run_f[r] = f;
            sc.run_cpf[r] = cpf;
            sc.run_cw[r] = cw;
            sc.run_thr[r] = thr;
            sc.run_isec[r] = P.isec;
            sc.run_wait[r] = 1000 / P.S;
            sc.run_mode[r] = RUN_FAST;
        }
    }
}

template <int G>
__global__ __launch_bounds__(kThreads) void k_flows(ClusterState st, BatchScratch sc, const Payload *__restrict__ pay,
                                                    int64_t ts_base, int simple, uint64_t *__restrict__ out) {
    const uint32_t nflows = sc.counters[2];
    const uint32_t nruns = sc.counters[1];
    const int gl = threadIdx.x & (G - 1);
    const uint32_t groups_per_block = kThreads / G;
    const uint32_t stride = gridDim.x * groups_per_block;
    for (uint32_t fl = blockIdx.x * groups_per_block + threadIdx.x / G; fl < nflows; fl += stride) {
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t s = sc.run_slot[r];
            const SlotParam P = st.param[s];
            const Rec R = rec_of(st, P);
            const uint32_t j0 = sc.run_start[r], j1 = sc.run_end[r];
            const uint32_t n = j1 - j0;
            const int64_t t0 = ts_base + (int64_t)sc.run_t0off[r];
            const uint32_t cp_tot = sc.run_cp[r];
            const int32_t a = sc.run_amin[r];
            const double thr = simple ? P.thr_simple : P.thr;
            // ---- fast path eligibility: equal acquire counts, no clock regression,
            //      prioritized requests only where the occupy path is regular
            const int64_t ws = t0 - t0 % P.W;
            const int cj = (int)((t0 / P.W) % P.S);
            const int64_t old = R.start(cj);
            bool fast = (a == sc.run_amax[r]) && !(old != kAbsent && ws < old);
            if (cp_tot > 0 && (P.S <= 1 || 1000 / P.S <= 0)) fast = false;
            if (!fast) {
                if (gl == 0) {  // exact replay of every request of the run, in order
                    for (uint32_t j = j0; j < j1; ++j) {
                        const Payload q = pay[j];
                        const int64_t t = ts_base + (int64_t)q.ts_off;
                        out[q.idx] = request_exact(st, s, t, (int32_t)(q.acq_prio & 0x7FFFFFFFu),
                                                   (q.acq_prio >> 31) != 0, simple);
                    }
                    sc.run_mode[r] = RUN_DONE;
                    __threadfence_block();
                }
                continue;
            }
            // ---- window sums over the valid buckets other than the current one (rotation of the
            //      current bucket does not touch them); lanes split the buckets
            int64_t bp = 0, bw = 0;
            if (G == 1 && (P.S & 1) == 0) {
                // start / PASS / WAITING vectors are contiguous and 16-B aligned: pairwise loads
                const int4 *v = reinterpret_cast<const int4 *>(R.r);
                const int hs = P.S >> 1;
                for (int q = 0; q < hs; ++q) {
                    const int4 st2 = v[q], ps2 = v[hs + q], wt2 = v[2 * hs + q];
                    const int64_t w0 = (int64_t)(((uint64_t)(uint32_t)st2.y << 32) | (uint32_t)st2.x);
                    const int64_t w1 = (int64_t)(((uint64_t)(uint32_t)st2.w << 32) | (uint32_t)st2.z);
                    const int j0 = 2 * q, j1 = 2 * q + 1;
                    if (j0 != cj && w0 != kAbsent && !(t0 - w0 > (int64_t)P.interval)) {
                        bp += (int64_t)(((uint64_t)(uint32_t)ps2.y << 32) | (uint32_t)ps2.x);
                        bw += (int64_t)(((uint64_t)(uint32_t)wt2.y << 32) | (uint32_t)wt2.x);
                    }
                    if (j1 != cj && w1 != kAbsent && !(t0 - w1 > (int64_t)P.interval)) {
                        bp += (int64_t)(((uint64_t)(uint32_t)ps2.w << 32) | (uint32_t)ps2.z);
                        bw += (int64_t)(((uint64_t)(uint32_t)wt2.w << 32) | (uint32_t)wt2.z);
                    }
                }
            } else {
                for (int jj = gl; jj < P.S; jj += G) {
                    const int64_t w = R.start(jj);
                    if (jj != cj && w != kAbsent && !(t0 - w > (int64_t)P.interval)) {
                        bp += R.cnt(CEV_PASS, jj);
                        bw += R.cnt(CEV_WAITING, jj);
                    }
                }
            }
            const int64_t base_pass = group_sum<G>(bp);
            const int64_t base_wait = group_sum<G>(bw);
            if (gl != 0) continue;
            // ---- lane 0: rotate the current window (LeapArray.currentWindow(t0)), then resolve
            cur_window(st, P, s, t0);
            const int64_t head = head_pass(st, P, t0);
            const int64_t s0 = base_pass + R.cnt(CEV_PASS, cj);
            const int64_t w0 = base_wait + R.cnt(CEV_WAITING, cj);
            // pass prefix: first i with !cond(s0 + i*a, a)   (monotone in i)
            const uint32_t f = pass_prefix(thr, P.isec, s0, a, n);
            const uint32_t cpf = (f >= n) ? cp_tot : (cp_tot ? sc.ev_cp[j0 + f] : 0u);
            const uint32_t np_after = cp_tot - cpf;
            // occupied prefix among prioritized blocked requests (monotone in the count)
            uint32_t cw = 0;
            if (np_after > 0) {
                const double latest = (double)(s0 + (int64_t)f * a) / P.isec;
                const double lim = st.max_occupy_ratio * thr;
                const int64_t occ0 = st.occ[s].occ_pass;
                uint32_t l2 = 0, h2 = np_after;
                while (l2 < h2) {
                    const uint32_t c = l2 + ((h2 - l2) >> 1);
                    const int64_t add = (int64_t)c * a;
                    const bool ok = ((double)(w0 + add) / P.isec <= lim) &&
                                    (latest + (double)((int64_t)a + occ0 + add) - (double)head <= thr);
                    if (ok) l2 = c + 1;
                    else h2 = c;
                }
                cw = l2;
            }
            // counters of the current bucket
            const int64_t wa = (int64_t)cw * a;
            const uint32_t nblk = n - f - cw;
            R.cnt(CEV_PASS, cj) += (int64_t)f * a;
            R.cnt(CEV_PASS_REQUEST, cj) += f;
            R.cnt(CEV_OCCUPIED_PASS, cj) += (int64_t)cpf * a;
            R.cnt(CEV_WAITING, cj) += wa;
            R.cnt(CEV_BLOCK, cj) += (int64_t)nblk * a;
            R.cnt(CEV_BLOCK_REQUEST, cj) += nblk;
            R.cnt(CEV_OCCUPIED_BLOCK, cj) += (int64_t)(np_after - cw) * a;
            if (cw > 0) {
                SlotOcc &o = st.occ[s];
                o.occ_pass += wa;
                o.occ_preq += cw;
                o.has_occ = 1;
            }
            sc.run_s0[r] = s0;
            sc.run_f[r] = f;
            sc.run_cpf[r] = cpf;
            sc.run_cw[r] = cw;
            sc.run_thr[r] = thr;
            sc.run_isec[r] = P.isec;
            sc.run_wait[r] = 1000 / P.S;
            sc.run_mode[r] = RUN_FAST;
            __threadfence_block();  // the group's lanes re-read this record for the rule's next run
        }
    }
}

// ---------------------------------------------------------------- results
__global__ __launch_bounds__(kThreads) void k_results(ClusterState st, BatchScratch sc, const uint32_t *__restrict__ keys,
                                                      const Payload *__restrict__ pay, int simple,
                                                      uint64_t *__restrict__ out) {
    const uint32_t nvalid = sc.counters[0];
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= nvalid) return;
    const uint32_t r = sc.ev_run[j];
    if (sc.run_mode[r] != RUN_FAST) return;
    const Payload q = pay[j];
    const uint32_t local = j - sc.run_start[r];
    const uint32_t f = sc.run_f[r];
    const int32_t a = (int32_t)(q.acq_prio & 0x7FFFFFFFu);
    uint64_t res;
    if (local < f) {
        const int64_t sum = sc.run_s0[r] + (int64_t)local * a;
        res = pack_result(TRS_OK, j_d2i(sc.run_thr[r] - (double)sum / sc.run_isec[r] - (double)a), 0);
    } else if ((q.acq_prio >> 31) && sc.ev_cp[j] - sc.run_cpf[r] < sc.run_cw[r]) {
        res = pack_result(TRS_SHOULD_WAIT, 0, (int32_t)sc.run_wait[r]);
    } else {
        res = pack_result(TRS_BLOCKED, 0, 0);
    }
    out[q.idx] = res;
}

__global__ void k_metric_sums(ClusterState st, uint32_t s, int64_t now, int64_t *out7) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const SlotParam P = st.param[s];
    cur_window(st, P, s, now);
    for (int k = 0; k < CEV_N; ++k) out7[k] = values_sum(st, P, now, k);
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
    st.occ[s] = SlotOcc{0, 0, 0, 0};
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

__global__ __launch_bounds__(kThreads) void k_lim_flag(ClusterState st, const uint32_t *__restrict__ keys, uint32_t n,
                                                       uint32_t invalid, int32_t ns, uint32_t *__restrict__ flag) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    flag[i] = (k != invalid && st.param[k].ns == ns) ? 1u : 0u;
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
                                                        uint32_t n, uint32_t invalid, uint32_t *__restrict__ keys,
                                                        uint64_t *__restrict__ out) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t m = counters[4];
    if (j >= m || j >= n) return;
    const uint32_t r = ridx[j] + head[j] - 1;
    if (j - rstart[r] >= rpass[r]) {
        const uint32_t i = list[j];
        keys[i] = invalid;
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

}  // namespace

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// the radix digit width depends on the live slot count: size for the worst width
static size_t max_hist_entries(size_t cap, uint32_t nslots_cap) {
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)nslots_cap + 1) ++bits;
    size_t m = 0;
    for (int b = 1; b <= bits; ++b) m = std::max(m, radix_hist_entries(cap, b));
    return m;
}

size_t batch_scratch_bytes(size_t cap, uint32_t nslots_cap) {
    const size_t ntiles = (cap + kTileElems - 1) / kTileElems + 1;
    const size_t hist = max_hist_entries(cap, nslots_cap);
    size_t b = 0;
    b += 2 * align_up(cap * 4) + 2 * align_up(cap * sizeof(Payload));
    b += 2 * align_up(cap * 4);                 // ev_run, ev_cp
    b += 8 * align_up(cap * 4);                 // run_* u32/i32
    b += align_up(cap * 8);                     // run_s0
    b += 4 * align_up(cap * 4);                 // run_f, run_cpf, run_cw, run_wait
    b += 2 * align_up(cap * 8);                 // run_thr, run_isec
    b += align_up(cap);                         // run_mode
    b += align_up(cap * 4);                     // flow_first_run
    b += 2 * align_up(ntiles * sizeof(Agg)) + align_up(ntiles * 4);
    b += align_up(64);
    b += 2 * align_up(hist * 4) + align_up(scan_partials_needed(hist) * 4 + 64);
    b += align_up(scan_partials_needed(cap) * 4 + 64);
    return b;
}

void batch_scratch_carve(BatchScratch &sc, void *base, size_t cap, uint32_t nslots_cap) {
    const size_t ntiles = (cap + kTileElems - 1) / kTileElems + 1;
    const size_t hist = max_hist_entries(cap, nslots_cap);
    char *p = (char *)base;
    auto take = [&](size_t bytes) {
        void *r = p;
        p += align_up(bytes);
        return r;
    };
    sc.keys[0] = (uint32_t *)take(cap * 4);
    sc.keys[1] = (uint32_t *)take(cap * 4);
    sc.pay[0] = (Payload *)take(cap * sizeof(Payload));
    sc.pay[1] = (Payload *)take(cap * sizeof(Payload));
    sc.ev_run = (uint32_t *)take(cap * 4);
    sc.ev_cp = (uint32_t *)take(cap * 4);
    sc.run_start = (uint32_t *)take(cap * 4);
    sc.run_end = (uint32_t *)take(cap * 4);
    sc.run_slot = (uint32_t *)take(cap * 4);
    sc.run_t0off = (uint32_t *)take(cap * 4);
    sc.run_cp = (uint32_t *)take(cap * 4);
    sc.run_amin = (int32_t *)take(cap * 4);
    sc.run_amax = (int32_t *)take(cap * 4);
    (void)take(cap * 4);
    sc.run_s0 = (int64_t *)take(cap * 8);
    sc.run_f = (uint32_t *)take(cap * 4);
    sc.run_cpf = (uint32_t *)take(cap * 4);
    sc.run_cw = (uint32_t *)take(cap * 4);
    sc.run_wait = (uint32_t *)take(cap * 4);
    sc.run_thr = (double *)take(cap * 8);
    sc.run_isec = (double *)take(cap * 8);
    sc.run_mode = (uint8_t *)take(cap);
    sc.flow_first_run = (uint32_t *)take(cap * 4);
    sc.tile_agg = take(ntiles * sizeof(Agg));
    sc.tile_carry = take(ntiles * sizeof(Agg));
    sc.tile_valid = (uint32_t *)take(ntiles * 4);
    sc.counters = (uint32_t *)take(64);
    sc.radix.hist = (uint32_t *)take(hist * 4);
    sc.radix.hist_scan = (uint32_t *)take(hist * 4);
    sc.radix.partial = (uint32_t *)take(scan_partials_needed(hist) * 4 + 64);
    sc.lim_partial = (uint32_t *)take(scan_partials_needed(cap) * 4 + 64);
    sc.cap = cap;
}

void cluster_decide_batch(const ClusterState &st, BatchScratch &sc, const int64_t *flow_id, const int32_t *acquire,
                          const uint8_t *prio, int64_t ts_base, const uint32_t *ts_off, uint32_t n, int simple,
                          void *out_v, hipStream_t s, const LimiterPass *lims, int nlims) {
    if (n == 0) return;
    uint64_t *out = (uint64_t *)out_v;
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)st.nslots + 1) ++bits;
    const uint32_t invalid_key = st.nslots;
    SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, 64, s));
    const uint32_t nb = (n + kThreads - 1) / kThreads;
    const uint32_t ncb = (n + kThreads * kClassifyItems - 1) / (kThreads * kClassifyItems);
    hipLaunchKernelGGL(k_classify, dim3(ncb), dim3(kThreads), 0, s, st, flow_id, acquire, prio, ts_off, ts_base, n,
                       simple, invalid_key, sc.keys[0], sc.pay[0], out, sc.counters);
    for (int l = 0; l < nlims && !simple; ++l) {
        // scratch: the sort's alternate buffers are free until the sort starts
        uint32_t *flag = sc.keys[1];
        uint32_t *u = (uint32_t *)sc.pay[1];
        uint32_t *pos = u, *list = u + n, *rstart = u + 2 * (size_t)n, *rpass = u + 3 * (size_t)n;
        hipLaunchKernelGGL(k_lim_flag, dim3(nb), dim3(kThreads), 0, s, st, sc.keys[0], n, invalid_key, lims[l].ns, flag);
        exclusive_scan_u32(flag, pos, n, sc.lim_partial, s);
        hipLaunchKernelGGL(k_lim_compact, dim3(nb), dim3(kThreads), 0, s, flag, pos, n, list, sc.counters);
        uint32_t *head = flag, *ridx = pos;
        hipLaunchKernelGGL(k_lim_heads, dim3(nb), dim3(kThreads), 0, s, list, ts_off, ts_base, n, sc.counters, head);
        exclusive_scan_u32(head, ridx, n, sc.lim_partial, s);
        hipLaunchKernelGGL(k_lim_starts, dim3(nb), dim3(kThreads), 0, s, head, ridx, n, sc.counters, rstart);
        hipLaunchKernelGGL(k_lim_walk, dim3(1), dim3(64), 0, s, lims[l].state, lims[l].qps_allowed, list, rstart,
                           sc.counters, ts_off, ts_base, rpass);
        hipLaunchKernelGGL(k_lim_apply, dim3(nb), dim3(kThreads), 0, s, list, head, ridx, rstart, rpass, sc.counters, n,
                           invalid_key, sc.keys[0], out);
    }
    const int npass = radix_sort_pairs(sc.keys[0], sc.pay[0], sc.keys[1], sc.pay[1], n, bits, sc.radix, s);
    const uint32_t *keys = sc.keys[npass & 1];
    const Payload *pay = sc.pay[npass & 1];
    const uint32_t ntiles = (n + kTileElems - 1) / kTileElems;
    hipLaunchKernelGGL(k_runs_up, dim3(ntiles), dim3(kRunThreads), 0, s, keys, pay, n, invalid_key, (Agg *)sc.tile_agg,
                       sc.tile_valid);
    hipLaunchKernelGGL(k_runs_tiles, dim3(1), dim3(kTileScanThreads), 0, s, (const Agg *)sc.tile_agg, sc.tile_valid,
                       ntiles, (Agg *)sc.tile_carry, sc.counters);
    hipLaunchKernelGGL(k_runs_down, dim3(ntiles), dim3(kRunThreads), 0, s, keys, pay, invalid_key,
                       (const Agg *)sc.tile_carry, sc);
    const uint64_t max_flows = n < st.nslots ? n : st.nslots;
    static const int lanes = [] {
        const char *e = getenv("SGA_FLOWS_LANES");  // A/B knob: lanes per rule in k_flows (1 or 16)
        const int v = e ? atoi(e) : 0;
        return (v == 16 || v == 4 || v == 1) ? v : 0;  // 0: k_flows1
    }();
    uint32_t fb = (uint32_t)std::min<uint64_t>((max_flows * (lanes ? lanes : 1) + kThreads - 1) / kThreads, 16384);
    if (fb == 0) fb = 1;
    if (lanes == 16) hipLaunchKernelGGL(k_flows<16>, dim3(fb), dim3(kThreads), 0, s, st, sc, pay, ts_base, simple, out);
    else if (lanes == 4) hipLaunchKernelGGL(k_flows<4>, dim3(fb), dim3(kThreads), 0, s, st, sc, pay, ts_base, simple, out);
    else if (lanes == 1) hipLaunchKernelGGL(k_flows<1>, dim3(fb), dim3(kThreads), 0, s, st, sc, pay, ts_base, simple, out);
    else hipLaunchKernelGGL(k_flows1, dim3(fb), dim3(kThreads), 0, s, st, sc, pay, ts_base, simple, out);
    hipLaunchKernelGGL(k_results, dim3(nb), dim3(kThreads), 0, s, st, sc, keys, pay, simple, out);
}

void cluster_init_limiter(NsLimiterDev *d, hipStream_t s) {
    hipLaunchKernelGGL(k_lim_init, dim3(1), dim3(64), 0, s, d);
}

void cluster_metric_sums(const ClusterState &st, uint32_t slot, int64_t now, int64_t *d_out7, hipStream_t s) {
    hipLaunchKernelGGL(k_metric_sums, dim3(1), dim3(64), 0, s, st, slot, now, d_out7);
}

void cluster_init_slots(const ClusterState &st, const uint32_t *d_slots, uint32_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_init_slots, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st, d_slots, n);
}

}  // namespace sga
