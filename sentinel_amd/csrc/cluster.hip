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

__device__ __forceinline__ int64_t slot_lookup(const ClusterState &st, int64_t fid) {
    uint32_t h = (uint32_t)hash_flow_id(fid) & st.hmask;
    for (uint32_t probe = 0; probe <= st.hmask; ++probe) {
        const int64_t k = st.hkeys[h];
        if (k == fid) return st.hvals[h];
        if (k == 0) return -1;
        h = (h + 1) & st.hmask;
    }
    return -1;
}

// ---------------------------------------------------------------- classify
__global__ __launch_bounds__(kThreads) void k_classify(ClusterState st, const int64_t *__restrict__ flow_id,
                                                       const int32_t *__restrict__ acquire,
                                                       const uint8_t *__restrict__ prio,
                                                       const uint32_t *__restrict__ ts_off, uint32_t n, int simple,
                                                       uint32_t invalid_key, uint32_t *__restrict__ keys,
                                                       Payload *__restrict__ pay, uint64_t *__restrict__ out,
                                                       uint32_t *__restrict__ counters) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    bool valid = false;
    if (i < n) {
        const int64_t fid = flow_id[i];
        const int32_t a = acquire[i];
        int8_t status = TRS_OK;
        int64_t slot = -1;
        if (!simple && (fid <= 0 || a <= 0)) {
            status = TRS_BAD_REQUEST;  // DefaultTokenService.notValidRequest, :87-89
        } else {
            // ClusterFlowRuleManager.getFlowRuleById: validId(id > 0) && FLOW_RULES.get(id)
            slot = fid > 0 ? slot_lookup(st, fid) : -1;
            if (slot < 0 || !st.param[slot].active) status = TRS_NO_RULE_EXISTS;
        }
        if (status != TRS_OK) {
            out[i] = pack_result(status, 0, 0);
            keys[i] = invalid_key;
            pay[i] = Payload{i, 0u, 0u};
        } else {
            valid = true;
            keys[i] = (uint32_t)slot;
            const uint32_t p = (!simple && prio && prio[i]) ? 0x80000000u : 0u;
            pay[i] = Payload{i, ts_off[i], (uint32_t)a | p};
        }
    }
    const uint64_t m = __ballot(valid);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&counters[0], (uint32_t)__popcll(m));
}

// ---------------------------------------------------------------- runs (segmented scan)
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
    if (b.flag) {
        r.flag = 1;
        r.cnt = b.cnt;
        r.mn = b.mn;
        r.mx = b.mx;
    } else {
        r.flag = a.flag;
        r.cnt = a.cnt + b.cnt;
        r.mn = min(a.mn, b.mn);
        r.mx = max(a.mx, b.mx);
    }
    return r;
}

__device__ __forceinline__ Agg agg_shfl_up(const Agg &v, int o) {
    Agg r;
    r.nh = __shfl_up(v.nh, o, 64);
    r.nf = __shfl_up(v.nf, o, 64);
    r.flag = __shfl_up(v.flag, o, 64);
    r.cnt = __shfl_up(v.cnt, o, 64);
    r.mn = __shfl_up(v.mn, o, 64);
    r.mx = __shfl_up(v.mx, o, 64);
    return r;
}

// exclusive scan of one Agg per thread over the workgroup (NT threads)
template <int NT>
__device__ Agg block_excl_scan(const Agg &v, Agg *total) {
    constexpr int NW = NT / 64;
    __shared__ Agg wtot[NW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Agg x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        Agg y = agg_shfl_up(x, o);
        if (lane >= o) x = agg_combine(y, x);
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    Agg wpre = agg_identity();
    for (int w = 0; w < wave; ++w) wpre = agg_combine(wpre, wtot[w]);
    Agg lane_excl = agg_shfl_up(x, 1);
    if (lane == 0) lane_excl = agg_identity();
    if (total) {
        Agg t = agg_identity();
        for (int w = 0; w < NW; ++w) t = agg_combine(t, wtot[w]);
        *total = t;
    }
    __syncthreads();
    return agg_combine(wpre, lane_excl);
}

struct Elem {
    uint32_t key;
    uint32_t ts_off;
    int32_t a;
    uint32_t p;
    int64_t bucket;
};

__device__ __forceinline__ Elem load_elem(const ClusterState &st, const uint32_t *keys, const Payload *pay,
                                          int64_t ts_base, uint32_t e) {
    Elem x;
    x.key = keys[e];
    const Payload q = pay[e];
    x.ts_off = q.ts_off;
    x.a = (int32_t)(q.acq_prio & 0x7FFFFFFFu);
    x.p = q.acq_prio >> 31;
    const int64_t t = ts_base + (int64_t)q.ts_off;
    x.bucket = t / (int64_t)st.param[x.key].W;
    return x;
}

__global__ __launch_bounds__(kThreads) void k_runs_up(ClusterState st, const uint32_t *__restrict__ keys,
                                                      const Payload *__restrict__ pay, int64_t ts_base,
                                                      const uint32_t *__restrict__ counters, Agg *__restrict__ tile_agg) {
    const uint32_t nvalid = counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;
    const uint32_t e0 = base + threadIdx.x * kItems;
    Agg acc = agg_identity();
    if (e0 < nvalid) {
        Elem prev;
        if (e0 > 0) prev = load_elem(st, keys, pay, ts_base, e0 - 1);
        for (int i = 0; i < kItems; ++i) {
            const uint32_t e = e0 + i;
            if (e >= nvalid) break;
            const Elem x = load_elem(st, keys, pay, ts_base, e);
            const bool fh = e == 0 || x.key != prev.key;
            const bool h = fh || x.bucket != prev.bucket;
            Agg v{h ? 1u : 0u, fh ? 1u : 0u, h ? 1u : 0u, x.p, x.a, x.a};
            acc = agg_combine(acc, v);
            prev = x;
        }
    }
    Agg total;
    block_excl_scan<kThreads>(acc, &total);
    if (threadIdx.x == 0) tile_agg[blockIdx.x] = total;
}

constexpr int kTileScanThreads = 1024;

__global__ __launch_bounds__(kTileScanThreads) void k_runs_tiles(const Agg *__restrict__ tile_agg,
                                                                 const uint32_t *__restrict__ counters,
                                                                 Agg *__restrict__ tile_carry) {
    const uint32_t nvalid = counters[0];
    const uint32_t ntiles = (nvalid + kTileElems - 1) / kTileElems;
    Agg carry = agg_identity();
    for (uint32_t b = 0; b < ntiles; b += kTileScanThreads) {
        const uint32_t t = b + threadIdx.x;
        const Agg v = t < ntiles ? tile_agg[t] : agg_identity();
        Agg total;
        const Agg ex = block_excl_scan<kTileScanThreads>(v, &total);
        if (t < ntiles) tile_carry[t] = agg_combine(carry, ex);
        carry = agg_combine(carry, total);
    }
}

__global__ __launch_bounds__(kThreads) void k_runs_down(ClusterState st, const uint32_t *__restrict__ keys,
                                                        const Payload *__restrict__ pay, int64_t ts_base,
                                                        const Agg *__restrict__ tile_carry, BatchScratch sc) {
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;
    const uint32_t e0 = base + threadIdx.x * kItems;
    // pass 1: thread aggregate
    Agg acc = agg_identity();
    Elem prev;
    const bool any = e0 < nvalid;
    if (any) {
        if (e0 > 0) prev = load_elem(st, keys, pay, ts_base, e0 - 1);
        Elem pv = prev;
        for (int i = 0; i < kItems; ++i) {
            const uint32_t e = e0 + i;
            if (e >= nvalid) break;
            const Elem x = load_elem(st, keys, pay, ts_base, e);
            const bool fh = e == 0 || x.key != pv.key;
            const bool h = fh || x.bucket != pv.bucket;
            acc = agg_combine(acc, Agg{h ? 1u : 0u, fh ? 1u : 0u, h ? 1u : 0u, x.p, x.a, x.a});
            pv = x;
        }
    }
    const Agg ex = block_excl_scan<kThreads>(acc, nullptr);
    if (!any) return;
    Agg run = agg_combine(tile_carry[blockIdx.x], ex);  // everything before e0
    Elem x = load_elem(st, keys, pay, ts_base, e0);
    for (int i = 0; i < kItems; ++i) {
        const uint32_t e = e0 + i;
        if (e >= nvalid) break;
        const bool fh = e == 0 || x.key != prev.key;
        const bool h = fh || x.bucket != prev.bucket;
        run = agg_combine(run, Agg{h ? 1u : 0u, fh ? 1u : 0u, h ? 1u : 0u, x.p, x.a, x.a});
        const uint32_t r = run.nh - 1;
        sc.ev_run[e] = r;
        sc.ev_cp[e] = run.cnt - x.p;
        if (h) {
            sc.run_start[r] = e;
            sc.run_slot[r] = x.key;
            sc.run_t0off[r] = x.ts_off;
        }
        if (fh) sc.flow_first_run[run.nf - 1] = r;
        // is e the last event of its run?
        bool last = (e + 1 >= nvalid);
        Elem nx;
        if (!last) {
            nx = load_elem(st, keys, pay, ts_base, e + 1);
            last = nx.key != x.key || nx.bucket != x.bucket;
        }
        if (last) {
            sc.run_end[r] = e + 1;
            sc.run_cp[r] = run.cnt;
            sc.run_amin[r] = run.mn;
            sc.run_amax[r] = run.mx;
        }
        if (e + 1 == nvalid) {
            sc.counters[1] = run.nh;
            sc.counters[2] = run.nf;
        }
        prev = x;
        if (e + 1 < nvalid) x = nx;
    }
}

// ---------------------------------------------------------------- exact per-request replay (device)
struct WinRef {
    uint32_t b;
    bool detached;
};

__device__ __forceinline__ void bucket_zero(const ClusterState &st, uint32_t b) {
#pragma unroll
    for (int k = 0; k < CEV_N; ++k) st.cnt[k][b] = 0;
}

// LeapArray.currentWindow(t) on a ClusterMetricLeapArray (t >= 0)
__device__ WinRef cur_window(const ClusterState &st, const SlotParam &P, uint32_t s, int64_t t) {
    const int64_t tid = t / P.W;
    const uint32_t b = P.boff + (uint32_t)(tid % P.S);
    const int64_t ws = t - t % P.W;
    const int64_t old = st.bstart[b];
    if (old == kAbsent) {  // newEmptyBucket: no occupy transfer
        st.bstart[b] = ws;
        bucket_zero(st, b);
        return WinRef{b, false};
    }
    if (ws == old) return WinRef{b, false};
    if (ws > old) {  // resetWindowTo + transferOccupyToBucket
        st.bstart[b] = ws;
        bucket_zero(st, b);
        SlotOcc &o = st.occ[s];
        if (o.has_occ) {
            st.cnt[CEV_OCCUPIED_PASS][b] += o.occ_pass;
            st.cnt[CEV_PASS][b] += o.occ_pass;
            o.occ_pass = 0;
            st.cnt[CEV_PASS_REQUEST][b] += o.occ_preq;
            o.occ_preq = 0;
            o.has_occ = 0;
        }
        return WinRef{b, false};
    }
    return WinRef{b, true};  // time went backwards: detached bucket, adds lost
}

__device__ int64_t values_sum(const ClusterState &st, const SlotParam &P, int64_t t, int ev) {
    int64_t s = 0;
    for (int j = 0; j < P.S; ++j) {
        const uint32_t b = P.boff + j;
        const int64_t w = st.bstart[b];
        if (w != kAbsent && !(t - w > (int64_t)P.interval)) s += st.cnt[ev][b];
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
    if (!w.detached) st.cnt[ev][w.b] += n;
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
            int64_t head = 0;
            {
                const uint32_t hb = P.boff + (uint32_t)(((t + P.W) / P.W) % P.S);
                const int64_t w = st.bstart[hb];
                if (w != kAbsent && !(t - w > (int64_t)P.interval)) head = st.cnt[CEV_PASS][hb];
            }
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

__global__ __launch_bounds__(kThreads) void k_flows(ClusterState st, BatchScratch sc, const Payload *__restrict__ pay,
                                                    int64_t ts_base, int simple, uint64_t *__restrict__ out) {
    const uint32_t nflows = sc.counters[2];
    const uint32_t nruns = sc.counters[1];
    for (uint32_t fl = blockIdx.x * kThreads + threadIdx.x; fl < nflows; fl += gridDim.x * kThreads) {
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t s = sc.run_slot[r];
            const SlotParam P = st.param[s];
            const uint32_t j0 = sc.run_start[r], j1 = sc.run_end[r];
            const uint32_t n = j1 - j0;
            const int64_t t0 = ts_base + (int64_t)sc.run_t0off[r];
            const uint32_t cp_tot = sc.run_cp[r];
            const int32_t a = sc.run_amin[r];
            const double thr = simple ? P.thr_simple : P.thr;
            // ---- decide fast path eligibility
            const int64_t ws = t0 - t0 % P.W;
            const uint32_t cb = P.boff + (uint32_t)((t0 / P.W) % P.S);
            const int64_t old = st.bstart[cb];
            bool fast = (a == sc.run_amax[r]) && !(old != kAbsent && ws < old);
            if (cp_tot > 0 && (P.S <= 1 || 1000 / P.S <= 0)) fast = false;
            if (!fast) {
                // exact replay of every request of the run, in order
                for (uint32_t j = j0; j < j1; ++j) {
                    const Payload q = pay[j];
                    const int64_t t = ts_base + (int64_t)q.ts_off;
                    out[q.idx] = request_exact(st, s, t, (int32_t)(q.acq_prio & 0x7FFFFFFFu), (q.acq_prio >> 31) != 0,
                                               simple);
                }
                sc.run_mode[r] = RUN_DONE;
                continue;
            }
            // ---- rotate the current window once (LeapArray.currentWindow(t0))
            cur_window(st, P, s, t0);
            int64_t base_pass = 0, base_wait = 0;
            for (int jj = 0; jj < P.S; ++jj) {
                const uint32_t b = P.boff + jj;
                if (b == cb) continue;
                const int64_t w = st.bstart[b];
                if (w != kAbsent && !(t0 - w > (int64_t)P.interval)) {
                    base_pass += st.cnt[CEV_PASS][b];
                    base_wait += st.cnt[CEV_WAITING][b];
                }
            }
            int64_t head = 0;
            {
                const uint32_t hb = P.boff + (uint32_t)(((t0 + P.W) / P.W) % P.S);
                const int64_t w = st.bstart[hb];
                if (w != kAbsent && !(t0 - w > (int64_t)P.interval)) head = st.cnt[CEV_PASS][hb];
            }
            const int64_t s0 = base_pass + st.cnt[CEV_PASS][cb];
            const int64_t w0 = base_wait + st.cnt[CEV_WAITING][cb];
            // ---- pass prefix: first i with !cond(s0 + i*a, a)   (monotone in i)
            uint32_t lo = 0, hi = n;
            while (lo < hi) {
                const uint32_t mid = lo + ((hi - lo) >> 1);
                if (pass_cond(thr, P.isec, s0 + (int64_t)mid * a, a)) lo = mid + 1;
                else hi = mid;
            }
            const uint32_t f = lo;
            const uint32_t cpf = (f >= n) ? cp_tot : (cp_tot ? sc.ev_cp[j0 + f] : 0u);
            const uint32_t np_after = cp_tot - cpf;
            // ---- occupied prefix among prioritized blocked requests (monotone in count)
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
            // ---- counters of the current bucket
            const int64_t fa = (int64_t)f * a;
            const int64_t wa = (int64_t)cw * a;
            const uint32_t nblk = n - f - cw;
            st.cnt[CEV_PASS][cb] += fa;
            st.cnt[CEV_PASS_REQUEST][cb] += f;
            st.cnt[CEV_OCCUPIED_PASS][cb] += (int64_t)cpf * a;
            st.cnt[CEV_WAITING][cb] += wa;
            st.cnt[CEV_BLOCK][cb] += (int64_t)nblk * a;
            st.cnt[CEV_BLOCK_REQUEST][cb] += nblk;
            st.cnt[CEV_OCCUPIED_BLOCK][cb] += (int64_t)(np_after - cw) * a;
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
            sc.run_mode[r] = RUN_FAST;
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
        const SlotParam &P = st.param[keys[j]];
        const double thr = simple ? P.thr_simple : P.thr;
        const int64_t sum = sc.run_s0[r] + (int64_t)local * a;
        res = pack_result(TRS_OK, j_d2i(thr - (double)sum / P.isec - (double)a), 0);
    } else if ((q.acq_prio >> 31) && sc.ev_cp[j] - sc.run_cpf[r] < sc.run_cw[r]) {
        res = pack_result(TRS_SHOULD_WAIT, 0, 1000 / st.param[keys[j]].S);
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

__global__ void k_init_buckets(ClusterState st, uint32_t b0, uint32_t b1) {
    const uint32_t b = b0 + blockIdx.x * kThreads + threadIdx.x;
    if (b >= b1) return;
    st.bstart[b] = kAbsent;
#pragma unroll
    for (int k = 0; k < CEV_N; ++k) st.cnt[k][b] = 0;
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
    b += 3 * align_up(cap * 4);                 // run_f, run_cpf, run_cw
    b += align_up(cap);                         // run_mode
    b += align_up(cap * 4);                     // flow_first_run
    b += 2 * align_up(ntiles * sizeof(Agg));
    b += align_up(64);
    b += 2 * align_up(hist * 4) + align_up(scan_partials_needed(hist) * 4 + 64);
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
    sc.run_mode = (uint8_t *)take(cap);
    sc.flow_first_run = (uint32_t *)take(cap * 4);
    sc.tile_agg = take(ntiles * sizeof(Agg));
    sc.tile_carry = take(ntiles * sizeof(Agg));
    sc.counters = (uint32_t *)take(64);
    sc.radix.hist = (uint32_t *)take(hist * 4);
    sc.radix.hist_scan = (uint32_t *)take(hist * 4);
    sc.radix.partial = (uint32_t *)take(scan_partials_needed(hist) * 4 + 64);
    sc.cap = cap;
}

void cluster_decide_batch(const ClusterState &st, BatchScratch &sc, const int64_t *flow_id, const int32_t *acquire,
                          const uint8_t *prio, int64_t ts_base, const uint32_t *ts_off, uint32_t n, int simple,
                          void *out_v, hipStream_t s) {
    if (n == 0) return;
    uint64_t *out = (uint64_t *)out_v;
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)st.nslots + 1) ++bits;
    const uint32_t invalid_key = st.nslots;
    SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, 64, s));
    const uint32_t nb = (n + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(k_classify, dim3(nb), dim3(kThreads), 0, s, st, flow_id, acquire, prio, ts_off, n, simple,
                       invalid_key, sc.keys[0], sc.pay[0], out, sc.counters);
    const int npass = radix_sort_pairs(sc.keys[0], sc.pay[0], sc.keys[1], sc.pay[1], n, bits, sc.radix, s);
    const uint32_t *keys = sc.keys[npass & 1];
    const Payload *pay = sc.pay[npass & 1];
    const uint32_t ntiles = (n + kTileElems - 1) / kTileElems;
    hipLaunchKernelGGL(k_runs_up, dim3(ntiles), dim3(kThreads), 0, s, st, keys, pay, ts_base, sc.counters,
                       (Agg *)sc.tile_agg);
    hipLaunchKernelGGL(k_runs_tiles, dim3(1), dim3(kTileScanThreads), 0, s, (const Agg *)sc.tile_agg, sc.counters,
                       (Agg *)sc.tile_carry);
    hipLaunchKernelGGL(k_runs_down, dim3(ntiles), dim3(kThreads), 0, s, st, keys, pay, ts_base,
                       (const Agg *)sc.tile_carry, sc);
    uint32_t flow_threads = n < st.nslots ? n : st.nslots;
    uint32_t fb = (flow_threads + kThreads - 1) / kThreads;
    if (fb == 0) fb = 1;
    hipLaunchKernelGGL(k_flows, dim3(fb), dim3(kThreads), 0, s, st, sc, pay, ts_base, simple, out);
    hipLaunchKernelGGL(k_results, dim3(nb), dim3(kThreads), 0, s, st, sc, keys, pay, simple, out);
}

void cluster_metric_sums(const ClusterState &st, uint32_t slot, int64_t now, int64_t *d_out7, hipStream_t s) {
    hipLaunchKernelGGL(k_metric_sums, dim3(1), dim3(64), 0, s, st, slot, now, d_out7);
}

void cluster_init_buckets(const ClusterState &st, uint32_t b0, uint32_t b1, hipStream_t s) {
    if (b1 <= b0) return;
    const uint32_t nb = (b1 - b0 + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(k_init_buckets, dim3(nb), dim3(kThreads), 0, s, st, b0, b1);
}

}  // namespace sga
