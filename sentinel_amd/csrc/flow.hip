// Local path on gfx950: StatisticSlot + ParamFlowSlot + FlowSlot + DegradeSlot over batches of
// entry/exit events (kernels K1-K5, K8 of DESIGN.md).
//
// Semantics restated from the reference (aliases as in SURVEY.md):
//   StatisticNode / ArrayMetric / Occupiable+Future+BucketLeapArray  CORE/node/StatisticNode.java:99-350,
//       CORE/slots/statistic/metric/ArrayMetric.java:37-350, .../occupy/OccupiableBucketLeapArray.java:33-82
//   StatisticSlot.entry/exit  CORE/slots/statistic/StatisticSlot.java:64-187
//   DefaultController / RateLimiterController / WarmUpController / WarmUpRateLimiterController
//       CORE/slots/block/flow/controller/*.java
//   ParamFlowChecker / ParameterMetric  PF/slots/block/flow/param/ParamFlowChecker.java:48-281, ParameterMetric.java
//   Exception/ResponseTimeCircuitBreaker + DegradeSlot  CORE/slots/block/degrade/**
//
// Batch algorithm: events are sorted by resource (stable: arrival order kept per resource) and
// segmented into runs = (resource, 500 ms second-window bucket).  One lane per resource walks its
// runs in time order.  A run of a resource whose only rule is a QPS DefaultController or
// WarmUpController, without prioritized entries and with equal acquire counts, is resolved in
// closed form: the window sums after one rotation, the pass prefix by binary search over the exact
// Java predicate, all exits of the run applied as one segmented reduction.  Every other run is
// replayed event by event with a device restatement of the whole slot chain.
#include "flow.hpp"
#include "cluster_exact.hpp"
#include "cparam_exact.hpp"

#include <algorithm>
#include <type_traits>
#include <cstring>
#include <new>

namespace sga {

namespace {

constexpr int kT = 256;
constexpr int kItems = 16;
constexpr int kTileElems = kT * kItems;  // 4096
constexpr int kSecW = 500, kSecInterval = 1000;   // SampleCountProperty.SAMPLE_COUNT = 2, INTERVAL = 1000
constexpr int kMinW = 1000, kMinInterval = 60000;
constexpr int kOccupyTimeout = 500;               // OccupyTimeoutProperty
enum : int8_t { D_PASS = 0, D_BLOCK_FLOW = 1, D_BLOCK_PARAM = 2, D_BLOCK_DEGRADE = 3, D_PASS_WAIT = 4,
                D_BLOCK_SYSTEM = 5 };
// F_SPECIAL: the event is replayed with its original kind, flags and arguments by the per-resource replay
// (replay_event): a kind 2 / 3 event, or arguments k_lclassify could not restate as one value
enum : uint32_t { F_SPECIAL = 1u << 31, F_EXIT = 1u << 30, F_ERROR = 1u << 29, F_PARAM = 1u << 28,
                  F_IDX = (1u << 28) - 1 };
constexpr uint32_t kHeavyEvents = 1024;  // per batch: replayed by k_lheavy instead of one k_lflows lane
#ifndef SGA_WAVE_EVENTS
#define SGA_WAVE_EVENTS 128
#endif
// per batch: a single-rule fast-path resource decided by one k_lwave wave instead of one k_lflows lane
// (1024 until round 5; C2 28.0 / 23.0 / 22.3 ms per step at 1024 / 256 / 128: its lanes of 128..1023 events
// were the k_lflows tail; round 6: 8.59 / 9.22 ms at 64 / 32 against 8.65 at 128, C5b unchanged -- kept)
constexpr uint32_t kWaveEvents = SGA_WAVE_EVENTS;
// RUN_POS: k_lwave left each entry's decision and wait in ev_eidx (wait << 1 | blocked; ~0: written
// already), k_lresults scatters them in parallel
// RUN_PSEG: a parameter-only resource's run, decided per (rule, value) segment (k_pseg_*)
// RUN_WRL: a RateLimiter run k_lflows sent to k_lwave (k_lwsum summarizes its windows); k_lwave turns it
// into RUN_POS or RUN_WIN
// RUN_WIN: as RUN_POS, except the run's interior windows k_lwave skipped (wstate: latestPassedTime - ts_base
// while it held; kWinWalked: walked, in ev_eidx), whose entries k_lresults decides from that state
enum : uint8_t { RUN_FAST = 0, RUN_DONE = 1, RUN_POS = 2, RUN_PSEG = 3, RUN_WIN = 4, RUN_WRL = 5 };
constexpr int64_t kWinWalked = INT64_MIN;

struct Ctx {
    FlowState st;
    int64_t max_rt;  // csp.sentinel.statistic.max.rt
    PEntry *pentry;  // k_lheavy: the current event's entry of the resource's only parameter rule, an
                     // LDS copy of the map entry (null: look the entry up in the map)
    int8_t pre_param;   // k_lheavy: that rule's check already decided by the value's lane (1 pass, 2 block)
    int64_t pre_wait;   // its wait
    const ResDev *res;  // k_lheavy: the resource's record, held by the replaying lane (null: st.res)
    uint64_t *pstamp_ref;  // k_lheavy: the LDS stamp of pentry (its last access)
};

// ------------------------------------------------------------------ MetricBucket windows
__device__ __forceinline__ void mb_zero(int64_t *b, int64_t max_rt) {
#pragma unroll
    for (int k = 1; k < MB_MINRT; ++k) b[k] = 0;
    b[MB_MINRT] = max_rt;
}

// FutureBucketLeapArray (borrow) getWindowValue(t): bucket whose [start, start+500) contains t
__device__ __forceinline__ int64_t *bor_value(int64_t *node, int64_t t) {
    if (t < 0) return nullptr;
    int64_t *b = node + kNodeBor + 2 * (int)((t / kSecW) % 2);
    if (b[0] == kAbsent || !(b[0] <= t && t < b[0] + kSecW)) return nullptr;
    return b;
}

// LeapArray.currentWindow(t) on the borrow array (newEmpty / reset both give an empty bucket)
__device__ int64_t *bor_current(int64_t *node, int64_t t, bool *detached) {
    int64_t *b = node + kNodeBor + 2 * (int)((t / kSecW) % 2);
    const int64_t ws = t - t % kSecW;
    *detached = false;
    if (b[0] == kAbsent || ws > b[0]) {
        b[0] = ws;
        b[1] = 0;
        return b;
    }
    if (ws == b[0]) return b;
    *detached = true;
    return nullptr;
}

// OccupiableBucketLeapArray.currentWindow(t): new bucket copies the borrowed bucket,
// a reset bucket takes only its PASS ((int) cast), OccupiableBucketLeapArray.java:40-64
__device__ int64_t *sec_current(int64_t *node, int64_t t, int64_t max_rt) {
    int64_t *b = node + kNodeSec + kMB * (int)((t / kSecW) % 2);
    const int64_t ws = t - t % kSecW;
    if (b[0] == kAbsent) {
        mb_zero(b, max_rt);
        const int64_t *bb = bor_value(node, t);
        if (bb) b[MB_PASS] = bb[1];  // MetricBucket.reset(borrow): every counter (only PASS is ever borrowed)
        b[0] = ws;
        return b;
    }
    if (ws == b[0]) return b;
    if (ws > b[0]) {
        b[0] = ws;
        mb_zero(b, max_rt);
        const int64_t *bb = bor_value(node, ws);
        if (bb) b[MB_PASS] += (int64_t)(int32_t)bb[1];
        return b;
    }
    return nullptr;  // clock went backwards: detached bucket, adds lost
}

__device__ int64_t *min_current(int64_t *node, int64_t t, int64_t max_rt) {
    int64_t *b = node + kNodeMin + kMB * (int)((t / kMinW) % 60);
    const int64_t ws = t - t % kMinW;
    if (b[0] == kAbsent || ws > b[0]) {
        b[0] = ws;
        mb_zero(b, max_rt);
        return b;
    }
    if (ws == b[0]) return b;
    return nullptr;
}

__device__ __forceinline__ int64_t sec_sum(int64_t *node, int64_t t, int f) {
    int64_t s = 0;
    for (int j = 0; j < 2; ++j) {
        const int64_t *b = node + kNodeSec + kMB * j;
        if (b[0] != kAbsent && !(t - b[0] > kSecInterval)) s += b[f];
    }
    return s;
}

__device__ __forceinline__ int64_t min_sum(int64_t *node, int64_t t, int f) {
    int64_t s = 0;
    for (int j = 0; j < 60; ++j) {
        const int64_t *b = node + kNodeMin + kMB * j;
        if (b[0] != kAbsent && !(t - b[0] > kMinInterval)) s += b[f];
    }
    return s;
}

// ------------------------------------------------------------------ StatisticNode
__device__ __forceinline__ double node_pass_qps(const Ctx &c, int64_t *node, int64_t t) {
    sec_current(node, t, c.max_rt);
    return (double)sec_sum(node, t, MB_PASS) / 1.0;
}

// minute.previousWindowPass() / previousWindowBlock(): currentWindow(now) then getPreviousWindow(now),
// LeapArray.java:230-248, ArrayMetric.java:283-297
__device__ double node_prev_qps(const Ctx &c, int64_t *node, int64_t t, int f) {
    min_current(node, t, c.max_rt);
    const int64_t tp = t - kMinW;
    if (t < 0) return 0;
    const int64_t *b = node + kNodeMin + kMB * (int)((tp / kMinW) % 60);
    if (b[0] == kAbsent || t - b[0] > kMinInterval) return 0;
    if (b[0] + kMinW < tp) return 0;
    return (double)b[f];
}
__device__ double node_prev_pass_qps(const Ctx &c, int64_t *node, int64_t t) { return node_prev_qps(c, node, t, MB_PASS); }

__device__ __forceinline__ void node_add(const Ctx &c, int64_t *node, int64_t t, int f, int64_t n) {
    int64_t *b = sec_current(node, t, c.max_rt);
    if (b) b[f] += n;
    b = min_current(node, t, c.max_rt);
    if (b) b[f] += n;
}

__device__ void node_add_rt_success(const Ctx &c, int64_t *node, int64_t t, int64_t rt, int count) {
    int64_t *b = sec_current(node, t, c.max_rt);
    if (b) b[MB_SUCC] += count;
    b = sec_current(node, t, c.max_rt);
    if (b) {
        b[MB_RT] += rt;
        if (rt < b[MB_MINRT]) b[MB_MINRT] = rt;
    }
    b = min_current(node, t, c.max_rt);
    if (b) b[MB_SUCC] += count;
    b = min_current(node, t, c.max_rt);
    if (b) {
        b[MB_RT] += rt;
        if (rt < b[MB_MINRT]) b[MB_MINRT] = rt;
    }
}

__device__ int64_t node_waiting(int64_t *node, int64_t t) {
    bool det;
    bor_current(node, t, &det);
    int64_t s = 0;
    for (int j = 0; j < 2; ++j) {
        const int64_t *b = node + kNodeBor + 2 * j;
        if (b[0] != kAbsent && !(t >= b[0])) s += b[1];  // FutureBucketLeapArray deprecation
    }
    return s;
}

// StatisticNode.tryOccupyNext, StatisticNode.java:302-334
__device__ int64_t node_try_occupy_next(const Ctx &c, int64_t *node, int64_t t, int acquire, double threshold) {
    const double max_count = threshold * kSecInterval / 1000;
    const int64_t current_borrow = node_waiting(node, t);
    if ((double)current_borrow >= max_count) return kOccupyTimeout;
    const int window_length = kSecInterval / 2;
    int64_t earliest = t - t % window_length + window_length - kSecInterval;
    int idx = 0;
    sec_current(node, t, c.max_rt);
    int64_t current_pass = sec_sum(node, t, MB_PASS);
    while (earliest < t) {
        const int64_t wait = (int64_t)idx * window_length + window_length - t % window_length;
        if (wait >= kOccupyTimeout) break;
        int64_t window_pass = 0;
        {  // ArrayMetric.getWindowPass(earliest) = data.getWindowValue(earliest)
            const int64_t *b = node + kNodeSec + kMB * (int)((earliest / kSecW) % 2);
            if (earliest >= 0 && b[0] != kAbsent && b[0] <= earliest && earliest < b[0] + kSecW) window_pass = b[MB_PASS];
        }
        if ((double)(current_pass + current_borrow + acquire - window_pass) <= max_count) return wait;
        earliest += window_length;
        current_pass -= window_pass;
        idx++;
    }
    return kOccupyTimeout;
}

// ------------------------------------------------------------------ controllers
__device__ void warmup_sync(FlowRuleDev &r, int64_t t, int64_t pass_qps) {  // WarmUpController.java:140-175
    const int64_t current_time = t - t % 1000;
    if (current_time <= r.last_filled) return;
    const int64_t old_value = r.stored_tokens;
    int64_t new_value = old_value;
    if (old_value < r.warning_token) {
        new_value = j_d2l((double)old_value + (double)(current_time - r.last_filled) * r.count / 1000);
    } else if (old_value > r.warning_token) {
        if (pass_qps < (int64_t)(j_d2i(r.count) / r.cold_factor))
            new_value = j_d2l((double)old_value + (double)(current_time - r.last_filled) * r.count / 1000);
    }
    if (new_value > (int64_t)r.max_token) new_value = r.max_token;
    r.stored_tokens = new_value - pass_qps;
    if (r.stored_tokens < 0) r.stored_tokens = 0;
    r.last_filled = current_time;
}

__device__ int8_t pace_tail(FlowRuleDev &r, int64_t t, int64_t cost, int64_t *wait_ms) {
    const int64_t expected = cost + r.latest_passed;
    if (expected <= t) {
        r.latest_passed = t;
        return D_PASS;
    }
    int64_t wait = cost + r.latest_passed - t;
    if (wait > r.max_queue) return D_BLOCK_FLOW;
    r.latest_passed += cost;
    wait = r.latest_passed - t;
    if (wait > r.max_queue) {
        r.latest_passed -= cost;
        return D_BLOCK_FLOW;
    }
    *wait_ms = wait > 0 ? wait : 0;
    return D_PASS;
}

__device__ int8_t rater_can_pass(const Ctx &c, FlowRuleDev &r, int64_t *node, int64_t t, int acquire, bool prio,
                                 int64_t *wait_ms) {
    *wait_ms = 0;
    switch (r.behavior) {
    case 2: {  // RateLimiterController.canPass, :46-91
        if (acquire <= 0) return D_PASS;
        if (r.count <= 0) return D_BLOCK_FLOW;
        return pace_tail(r, t, j_round(1.0 * acquire / r.count * 1000), wait_ms);
    }
    case 1: {  // WarmUpController.canPass, :113-138
        const int64_t pass_qps = j_d2l(node_pass_qps(c, node, t));
        const int64_t previous_qps = j_d2l(node_prev_pass_qps(c, node, t));
        warmup_sync(r, t, previous_qps);
        const int64_t rest = r.stored_tokens;
        if (rest >= r.warning_token) {
            const int64_t above = rest - r.warning_token;
            const double warning_qps = j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
            if ((double)(pass_qps + acquire) <= warning_qps) return D_PASS;
        } else if ((double)(pass_qps + acquire) <= r.count) {
            return D_PASS;
        }
        return D_BLOCK_FLOW;
    }
    case 3: {  // WarmUpRateLimiterController.canPass, :43-87
        const int64_t previous_qps = j_d2l(node_prev_pass_qps(c, node, t));
        warmup_sync(r, t, previous_qps);
        const int64_t rest = r.stored_tokens;
        int64_t cost;
        if (rest >= r.warning_token) {
            const int64_t above = rest - r.warning_token;
            const double warming_qps = j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
            cost = j_round(1.0 * acquire / warming_qps * 1000);
        } else {
            cost = j_round(1.0 * acquire / r.count * 1000);
        }
        return pace_tail(r, t, cost, wait_ms);
    }
    default: {  // DefaultController.canPass, DefaultController.java:49-78
        int32_t cur = r.grade == 0 ? (int32_t)node[kNodeThreads] : j_d2i(node_pass_qps(c, node, t));
        const int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)acquire);
        if ((double)sum > r.count) {
            if (prio && r.grade == 1) {
                const int64_t wait = node_try_occupy_next(c, node, t, acquire, r.count);
                if (wait < kOccupyTimeout) {
                    bool det;
                    int64_t *bb = bor_current(node, t + wait, &det);  // addWaitingRequest(now + wait)
                    if (bb) bb[1] += acquire;
                    int64_t *m = min_current(node, t, c.max_rt);      // addOccupiedPass
                    if (m) m[MB_OPASS] += acquire;
                    m = min_current(node, t, c.max_rt);
                    if (m) m[MB_PASS] += acquire;
                    *wait_ms = wait;
                    return D_PASS_WAIT;
                }
            }
            return D_BLOCK_FLOW;
        }
        return D_PASS;
    }
    }
}

// ------------------------------------------------------------------ parameter maps
// Concurrency contract: the entries of one owner (a parameter rule, or a resource for thread
// counts) are touched by one lane at a time (k_lflows, k_lseq, lane 0 of k_lheavy) or through
// k_lheavy's dedupe / find / insert phases.  Lanes of other owners only need a slot's owner to skip
// it, and the claiming CAS publishes the owner itself, so no fence is needed.  (An agent-scope
// release per insert writes back the XCD's L2 and made C4's 10M-value maps crawl.)
__device__ __forceinline__ uint32_t ptab_home(uint32_t mask, uint32_t owner, uint64_t value) {
    return (uint32_t)splitmix64(value ^ ((uint64_t)owner << 40) ^ 0xA5A5ULL) & mask;
}

// Claimed-slot counters: kClaimHdr entries in front of each table's slot 0 (never probed), their `a` words
// counting every slot claim (64 shards against same-address contention).  The host reads them to bound the
// table's load without scanning it (FlowEngine::grow_map).
constexpr uint32_t kClaimHdr = 64;
__device__ __forceinline__ void claim_note(PEntry *tab, uint32_t h) {
    atomicAdd(reinterpret_cast<unsigned long long *>(&tab[-1 - (int)(h & (kClaimHdr - 1))].a), 1ull);
}

__device__ PEntry *ptab_get(PEntry *tab, uint32_t mask, uint32_t owner, uint64_t value, bool create,
                            uint32_t *overflow) {
    uint32_t h = (uint32_t)splitmix64(value ^ ((uint64_t)owner << 40) ^ 0xA5A5ULL) & mask;
    // the maps stay at most a quarter full (FlowEngine::ensure_maps), so a long probe sequence means a
    // broken invariant: fail the batch (overflow -> -ENOMEM) instead of walking the whole table
    const uint32_t max_probe = mask < 4096u ? mask : 4096u;
    for (uint32_t probe = 0; probe <= max_probe; ++probe) {
        PEntry *e = &tab[h];
        uint32_t o = __hip_atomic_load(&e->owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o == 0) {
            if (!create) return nullptr;
            const uint32_t prev = atomicCAS(&e->owner, 0u, owner);  // the claim publishes the owner
            if (prev == 0) {
                claim_note(tab, h);
                e->value = value;
                e->a = kPAbsent;
                e->b = kPAbsent;
                return e;
            }
            o = prev;
        }
        if (o == owner && e->value == value) return e;
        h = (h + 1) & mask;
    }
    atomicOr(overflow, 1u);
    return nullptr;
}

// Insert of a key known to be absent (k_lheavy, after a find): the first free slot of the probe
// sequence, no value comparisons (so no read of an entry another lane is still filling).
__device__ PEntry *ptab_insert_absent(PEntry *tab, uint32_t mask, uint32_t owner, uint64_t value,
                                      uint32_t *overflow) {
    uint32_t h = (uint32_t)splitmix64(value ^ ((uint64_t)owner << 40) ^ 0xA5A5ULL) & mask;
    const uint32_t max_probe = mask < 4096u ? mask : 4096u;
    for (uint32_t probe = 0; probe <= max_probe; ++probe) {
        PEntry *e = &tab[h];
        if (__hip_atomic_load(&e->owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
            atomicCAS(&e->owner, 0u, owner) == 0u) {
            claim_note(tab, h);
            e->value = value;
            e->a = kPAbsent;
            e->b = kPAbsent;
            return e;
        }
        h = (h + 1) & mask;
    }
    atomicOr(overflow, 1u);
    return nullptr;
}

__device__ __forceinline__ int64_t lwrap_mul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
__device__ __forceinline__ int64_t lwrap_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

// thread-count map owner of (resource r, argument index k): resource + 1 for index 0
__device__ __forceinline__ uint32_t tmap_owner(uint32_t r, uint32_t k) { return (r + 1) | (k << 24); }

// ------------------------------------------------------------------ CacheMap capacity (strict LRU)
// ParameterMetric's maps (ParameterMetric.java:37-39,95-121) are ConcurrentLinkedHashMapWrappers of a fixed
// capacity (CLHM 1.4.2, not vendored: restated as strict LRU, oracle/oracle_ext.c lru_*).  flow.hpp LruRec
// describes the free / LRU modes.  A key access = CacheMap.get / putIfAbsent / put of a present key; an
// insert = putIfAbsent / put of an absent one; a remove = the thread-count map's remove at zero.
__device__ __forceinline__ uint64_t lru_stamp(const FlowState &st, uint32_t eidx, uint32_t q) {
    return ((st.seq_base + eidx) << 16) | (uint64_t)min(q, 0xFFFFu);
}

struct MapRef {  // one owner's map
    PEntry *tab;
    uint64_t *stamp;
    uint32_t mask, owner;
    uint32_t *size;
    uint64_t *q;
    uint32_t cap;
    uint32_t *overflow;
};
__device__ __forceinline__ MapRef map_ref_p(const FlowState &st, const ParamRuleDev &p) {
    return MapRef{st.ptab, st.pstamp, st.pmask, p.id + 1, st.psize + p.id, st.pq + p.id, p.cap, st.overflow};
}
__device__ __forceinline__ MapRef map_ref_t(const FlowState &st, uint32_t r, uint32_t k) {
    const uint32_t j = st.tbase[r] + k;
    return MapRef{st.ttab, st.tstamp, st.tmask, tmap_owner(r, k), st.tsize + j, st.tq + j, kThreadMapCap, st.overflow};
}
__device__ __forceinline__ bool lru_on_p(const FlowState &st) { return st.pstamp != nullptr; }
__device__ __forceinline__ bool lru_on_t(const FlowState &st, uint32_t r) {
    return st.tstamp != nullptr && st.tbase != nullptr && st.tbase[r] != kNoTBase;
}

// LRU-mode queues: the owner is decided by one lane, plain loads and stores.  The area is
// [meta {head, tail}][2 cap + 2 records]; a record is live while its key is present with its stamp.
__device__ __forceinline__ uint64_t lru_qcap(const MapRef &m) { return 2ull * m.cap + 2; }
__device__ __forceinline__ bool lru_live(const MapRef &m, const LruRec &rec, PEntry **pe) {
    PEntry *e = ptab_get(m.tab, m.mask, m.owner, rec.value, false, m.overflow);
    if (!e || e->a == kPAbsent || m.stamp[e - m.tab] != rec.stamp) return false;
    *pe = e;
    return true;
}
// SGA_LRU_PROF=1 (diagnostics only): [0] pushes [1] compactions [2] records scanned by them [3] their ticks
// [4] evictions [5] records popped [6] k_llru entry ticks [7] k_llru exit ticks
__device__ unsigned long long g_lru_prof[8];
__device__ int g_lru_prof_on;
__device__ void lru_compact(const MapRef &m, LruRec *area) {
    const bool prof = g_lru_prof_on != 0;
    const uint64_t t0 = prof ? wall_clock64() : 0;
    const uint64_t qcap = lru_qcap(m);
    uint64_t w = area[0].value;
    for (uint64_t i = area[0].value; i < area[0].stamp; ++i) {
        const LruRec rec = area[1 + i % qcap];
        PEntry *e;
        if (lru_live(m, rec, &e)) area[1 + (w++) % qcap] = rec;
    }
    if (prof) {
        atomicAdd(&g_lru_prof[1], 1ull);
        atomicAdd(&g_lru_prof[2], (unsigned long long)(area[0].stamp - area[0].value));
        atomicAdd(&g_lru_prof[3], (unsigned long long)(wall_clock64() - t0));
    }
    area[0].stamp = w;
}
__device__ void lru_push(const FlowState &st, const MapRef &m, uint64_t value, uint64_t stamp) {
    LruRec *area = st.lpool + *m.q;
    const uint64_t qcap = lru_qcap(m);
    if (area[0].stamp - area[0].value >= qcap) lru_compact(m, area);  // live records <= cap + 1
    if (area[0].stamp - area[0].value >= qcap) {
        atomicOr(&st.lru_ctl[1], 2u);
        atomicOr(st.overflow, 1u);
        return;
    }
    area[1 + area[0].stamp % qcap] = LruRec{value, stamp};
    area[0].stamp += 1;
    if (g_lru_prof_on) atomicAdd(&g_lru_prof[0], 1ull);
}
// a full map's least recently used key (CLHM evicts after the insert that overflows it)
__device__ void lru_evict(const FlowState &st, const MapRef &m) {
    LruRec *area = st.lpool + *m.q;
    const uint64_t qcap = lru_qcap(m);
    if (g_lru_prof_on) atomicAdd(&g_lru_prof[4], 1ull);
    while (area[0].value < area[0].stamp) {
        const LruRec rec = area[1 + area[0].value % qcap];
        area[0].value += 1;
        if (g_lru_prof_on) atomicAdd(&g_lru_prof[5], 1ull);
        PEntry *e;
        if (lru_live(m, rec, &e)) {
            e->a = kPAbsent;
            e->b = kPAbsent;
            *m.size -= 1;
            return;
        }
    }
    atomicOr(&st.lru_ctl[1], 2u);  // a full map without a live record: never expected
    atomicOr(st.overflow, 1u);
}
// kLru: the caller may hold owners in LRU mode (k_llru, k_lseq: one lane per owner); the parallel kernels
// only ever see free-mode owners (the count pass routes the others away) and compile without the queues
template <bool kLru>
__device__ __forceinline__ void lru_touch(const FlowState &st, const MapRef &m, PEntry *e, uint64_t stamp) {
    m.stamp[e - m.tab] = stamp;
    if (kLru && *m.q != kNoQueue) lru_push(st, m, e->value, stamp);
}
// e absent (a == kPAbsent) and about to be set present by the caller
template <bool kLru>
__device__ __forceinline__ void lru_insert(const FlowState &st, const MapRef &m, PEntry *e, uint64_t stamp) {
    m.stamp[e - m.tab] = stamp;
    if (!kLru || *m.q == kNoQueue) {  // free mode: the count pass guarantees room; lanes of one owner may add together
        atomicAdd(m.size, 1u);
        return;
    }
    *m.size += 1;
    lru_push(st, m, e->value, stamp);
    if (*m.size > m.cap) lru_evict(st, m);
}
template <bool kLru>
__device__ __forceinline__ void lru_remove(const MapRef &m) {
    if (!kLru || *m.q == kNoQueue) atomicSub(m.size, 1u);
    else *m.size -= 1;
}

__device__ bool hot_lookup(const Ctx &c, const ParamRuleDev &p, uint64_t v, int64_t *thr) {
    for (int i = 0; i < p.n_hot; ++i)
        if (c.st.hot_v[p.hot_off + i] == v) {
            *thr = c.st.hot_t[p.hot_off + i];
            return true;
        }
    return false;
}

// ParamFlowChecker.passSingleValueCheck / passDefaultLocalCheck / passThrottleLocalCheck
// QPS grade against the value's (lastAddTokenTime, tokens) or throttle-time entry e.  The check's constants for
// (rule, value, acquireCount) come first (param_pre: the token count with the value's hot item, then the
// throttle cost or the bucket's maxCount), so a caller checking many events of one value computes them once.
struct ParamPre {
    int64_t tc;  // token count (0: every check fails)
    int64_t k2;  // throttle: cost of the acquire in ms; token bucket: maxCount
};
__device__ __forceinline__ ParamPre param_pre(const Ctx &c, const ParamRuleDev &p, uint64_t v, int acquire) {
    int64_t tc = j_d2l(p.count), hot;
    if (hot_lookup(c, p, v, &hot)) tc = hot;
    if (tc == 0) return {0, 0};
    if (p.behavior == 2)  // ParamFlowChecker.java:224-281
        return {tc, j_round(1.0 * 1000 * (double)acquire * (double)p.duration / (double)tc)};
    return {tc, lwrap_add(tc, p.burst)};  // ParamFlowChecker.java:132-222
}
template <class E>
__device__ __forceinline__ bool param_pass_pre(const ParamRuleDev &p, E &e, ParamPre q, int acquire, int64_t t,
                                               int64_t *wait_ms) {
    *wait_ms = 0;
    const int64_t token_count = q.tc;
    if (token_count == 0) return false;
    if (p.behavior == 2) {  // throttle
        const int64_t cost = q.k2;
        if (e.a == kPAbsent) {
            e.a = t;
            return true;
        }
        const int64_t expected = e.a + cost;
        if (expected <= t || expected - t < p.max_queue) {
            e.a = t;
            const int64_t wait = expected - t;
            if (wait > 0) {
                e.a = expected;
                *wait_ms = wait;
            }
            return true;
        }
        return false;
    }
    // token bucket
    const int64_t max_count = q.k2;
    if ((int64_t)acquire > max_count) return false;
    if (e.a == kPAbsent) {
        e.a = t;
        if (e.b == kPAbsent) e.b = max_count - acquire;
        return true;
    }
    const int64_t pass_time = t - e.a;
    const int64_t dur_ms = lwrap_mul(p.duration, 1000);
    if (pass_time > dur_ms) {
        if (e.b == kPAbsent) {
            e.b = max_count - acquire;
            e.a = t;
            return true;
        }
        const int64_t rest = e.b;
        const int64_t to_add = lwrap_mul(pass_time, token_count) / dur_ms;
        const int64_t nq = lwrap_add(to_add, rest) > max_count ? max_count - acquire
                                                               : lwrap_add(rest, to_add) - acquire;
        if (nq < 0) return false;
        e.b = nq;
        e.a = t;
        return true;
    }
    if (e.b != kPAbsent) {
        if (e.b - acquire >= 0) {
            e.b -= acquire;
            return true;
        }
        return false;
    }
    return false;
}
template <class E>
__device__ __forceinline__ bool param_pass_qps(const Ctx &c, const ParamRuleDev &p, E &e, uint64_t v, int acquire,
                                               int64_t t, int64_t *wait_ms) {
    return param_pass_pre(p, e, param_pre(c, p, v, acquire), acquire, t, wait_ms);
}

// whether a QPS check of value v reaches the rule's maps: not for a zero threshold, nor (token bucket)
// for acquireCount > maxCount (ParamFlowChecker.java:137-154, 230-234)
__device__ __forceinline__ bool param_pre_access(const ParamRuleDev &p, ParamPre q, int acquire) {
    return q.tc != 0 && (p.behavior == 2 || (int64_t)acquire <= q.k2);
}
__device__ __forceinline__ bool param_map_access(const Ctx &c, const ParamRuleDev &p, uint64_t v, int acquire) {
    return param_pre_access(p, param_pre(c, p, v, acquire), acquire);
}

template <bool kLru>
__device__ bool param_pass(const Ctx &c, const ParamRuleDev &p, uint64_t v, int acquire, int64_t t,
                           int64_t thread_count, int64_t *wait_ms, uint64_t stamp) {
    *wait_ms = 0;
    int64_t hot;
    if (p.grade == 1) {
        int64_t token_count = j_d2l(p.count);
        if (hot_lookup(c, p, v, &hot)) token_count = hot;
        if (token_count == 0) return false;  // before any map access, as the reference
        const bool access = p.behavior == 2 || (int64_t)acquire <= lwrap_add(token_count, p.burst);
        if (c.pentry) {  // k_lheavy's LDS copy (free mode): its stamp beside it, its count at the write-back
            if (access && c.pstamp_ref) *c.pstamp_ref = stamp;
            return param_pass_qps(c, p, *c.pentry, v, acquire, t, wait_ms);
        }
        PEntry *e = ptab_get(c.st.ptab, c.st.pmask, p.id + 1, v, true, c.st.overflow);
        if (!e) return false;
        if (access && lru_on_p(c.st)) {  // time map then token map: the same key sequence, one recency order
            const MapRef m = map_ref_p(c.st, p);
            if (e->a == kPAbsent) lru_insert<kLru>(c.st, m, e, stamp);
            else lru_touch<kLru>(c.st, m, e, stamp);
        }
        return param_pass_qps(c, p, *e, v, acquire, t, wait_ms);
    }
    if (p.grade == 0) {
        if (hot_lookup(c, p, v, &hot)) return ++thread_count <= hot;
        return ++thread_count <= j_d2l(p.count);
    }
    return true;
}

// ------------------------------------------------------------------ circuit breakers
__device__ void cb_to_open(CbDev &b, int64_t t) {
    if (b.state == 0 || b.state == 2) {
        b.state = 1;
        b.next_retry = t + b.recovery_ms;
    }
}

__device__ void cb_stat_at(CbDev &b, int64_t ws) {  // LeapArray(1, statIntervalMs).currentWindow(t), ws = its start
    if (b.st_start == kAbsent || ws > b.st_start) {
        b.st_start = ws;
        b.st_bad = 0;
        b.st_total = 0;
    }
}

// DegradeSlot.entry over the resource's breakers (DegradeSlot.java:52-66): tryPass of each in order;
// a breaker moved to HALF_OPEN goes back to OPEN when a later one blocks (whenTerminate, blockError)
__device__ int degrade_block_index(CbDev *cbs, uint32_t n, int64_t t) {  // -1: every breaker passes
    uint64_t half_mask = 0;
    for (uint32_t k = 0; k < n; ++k) {
        CbDev &b = cbs[k];
        bool ok = false;
        if (b.state == 0) ok = true;
        else if (b.state == 1 && t >= b.next_retry) {
            b.state = 2;
            b.probe_t = t;
            if (k < 64) half_mask |= 1ULL << k;
            ok = true;
        }
        if (!ok) {
            for (uint32_t q = 0; q < k && q < 64; ++q) {
                CbDev &bq = cbs[q];
                if (((half_mask >> q) & 1) && bq.state == 2) bq.state = 1;
            }
            return (int)k;
        }
    }
    return -1;
}
__device__ __forceinline__ bool degrade_pass(CbDev *cbs, uint32_t n, int64_t t) {
    return degrade_block_index(cbs, n, t) < 0;
}

// handleStateChangeWhenThresholdExceeded of a CLOSED breaker over its current window's counts
// (ResponseTimeCircuitBreaker.java:88-106, ExceptionCircuitBreaker.java:75-94)
__device__ __forceinline__ bool cb_trips(const CbDev &b, int64_t badc, int64_t total) {
    if (total < b.min_req) return false;
    if (b.grade == 0) {
        const double ratio = (double)badc * 1.0 / (double)total;
        return ratio > b.slow_ratio || (ratio == b.slow_ratio && b.slow_ratio == 1.0);
    }
    double cur = (double)badc;
    if (b.grade == 1) cur = (double)badc * 1.0 / (double)total;
    return cur > b.count;
}

// AbstractCircuitBreaker.onRequestComplete with the stat window start ws = t - t % statIntervalMs
// given (k_lheavy computes it for a chunk on all lanes)
__device__ void cb_on_complete_ws(CbDev &b, int64_t t, int64_t ws, int64_t rt, bool error) {
    const bool is_rt = b.grade == 0;
    const bool bad = is_rt ? rt > b.max_allowed_rt : error;
    const bool detached = b.st_start != kAbsent && ws < b.st_start;
    cb_stat_at(b, ws);
    if (!detached) {
        if (bad) b.st_bad += 1;
        b.st_total += 1;
    }
    if (b.state == 1) return;
    if (b.state == 2) {
        if (bad) cb_to_open(b, t);
        else {
            b.state = 0;  // fromHalfOpenToClose -> resetStat on currentWindow()
            cb_stat_at(b, ws);
            if (!(b.st_start != kAbsent && ws < b.st_start)) {
                b.st_bad = 0;
                b.st_total = 0;
            }
        }
        return;
    }
    int64_t badc = 0, total = 0;
    if (b.st_start != kAbsent && !(t - b.st_start > b.stat_interval)) {
        badc = b.st_bad;
        total = b.st_total;
    }
    if (cb_trips(b, badc, total)) cb_to_open(b, t);
}

__device__ __forceinline__ void cb_on_complete(CbDev &b, int64_t t, int64_t rt, bool error) {
    cb_on_complete_ws(b, t, t - t % b.stat_interval, rt, error);
}

// ------------------------------------------------------------------ slot chain (one event)
// Where a resource's mutable state lives during a replay: global memory, or the LDS copy a
// heavy resource's workgroup works on (k_lheavy).
struct ResMem {
    int64_t *node;
    FlowRuleDev *rules;  // the resource's rules (st.rules + rule_off)
    CbDev *cbs;          // its circuit breakers (st.cbs + cb_off)
};

__device__ __forceinline__ ResMem res_global(const Ctx &c, uint32_t r, const ResDev &R) {
    return ResMem{c.st.node + (size_t)r * kNodeWords, c.st.rules + R.rule_off, c.st.cbs + R.cb_off};
}

// The event's arguments (SphU.entry(..., Object... args)).  args = [param] (SGA_EV_HAS_PARAM), [] (none),
// args[0] a Collection / array (SGA_EV_PARAM_LIST: v0 / n0), or a whole argument vector (SGA_EV_ARGS:
// word pairs at args, kind << 62 | list length, then the key or the list's offset into pvals).
struct PArgs {
    const uint64_t *v;  // SGA_EV_PARAM_LIST: args[0]'s elements
    uint32_t n;
    const uint64_t *args = nullptr;   // SGA_EV_ARGS
    const uint64_t *pvals = nullptr;
    uint32_t nargs = 0;
};
enum : int { ARG_SCALAR = 0, ARG_NULL = 1, ARG_LIST = 2 };

__device__ __forceinline__ uint32_t ev_nargs(const PArgs &pa, bool has_param) {
    return pa.args ? pa.nargs : (has_param ? 1u : 0u);
}

// args[k]: its kind and values (a scalar is one value); `one` holds a scalar for the legacy forms
__device__ __forceinline__ int ev_arg(const PArgs &pa, uint32_t k, const uint64_t &param, const uint64_t **vals,
                                      uint32_t *n) {
    if (pa.args) {
        const uint64_t h = pa.args[2 * k];
        const int kind = (int)(h >> 62);
        if (kind == ARG_LIST) {
            *vals = pa.pvals + pa.args[2 * k + 1];
            *n = (uint32_t)(h & 0xFFFFFFFFu);
        } else {
            *vals = &pa.args[2 * k + 1];
            *n = 1;
        }
        return kind;
    }
    if (k == 0 && pa.v) {
        *vals = pa.v;
        *n = pa.n;
        return ARG_LIST;
    }
    *vals = &param;
    *n = 1;
    return ARG_SCALAR;
}

// ParameterMetric.addThreadCount / decreaseThreadCount (ParameterMetric.java:125-230): every argument
// index with a thread-count map, every element of a Collection / array, null arguments skipped
template <bool kLru>
__device__ void param_threads(const Ctx &c, uint32_t r, const PArgs &pa, bool has_param, const uint64_t &param,
                              int delta, uint32_t eidx) {
    const uint64_t mask = c.st.tmapmask ? c.st.tmapmask[r] : 0ull;
    if (!mask) return;
    const uint32_t na = min(ev_nargs(pa, has_param), (uint32_t)kMaxParamIdx);
    for (uint32_t k = 0; k < na; ++k) {
        if (!((mask >> k) & 1ull)) continue;
        const uint64_t *vals;
        uint32_t nv;
        if (ev_arg(pa, k, param, &vals, &nv) == ARG_NULL) continue;
        for (uint32_t q = 0; q < nv; ++q) {
            PEntry *te = ptab_get(c.st.ttab, c.st.tmask, tmap_owner(r, k), vals[q], true, c.st.overflow);
            if (!te) continue;
            const bool lru = lru_on_t(c.st, r);
            MapRef m{};
            if (lru) m = map_ref_t(c.st, r, k);
            const uint64_t stamp = lru_stamp(c.st, eidx, q);
            if (te->a == kPAbsent) {  // putIfAbsent(value, new AtomicInteger()) inserts
                if (lru) lru_insert<kLru>(c.st, m, te, stamp);
                te->a = delta > 0 ? 1 : 0;  // then put(value, new AtomicInteger(1)); a decrease leaves 0
            } else {
                if (lru) lru_touch<kLru>(c.st, m, te, stamp);
                if (delta > 0) {
                    te->a += 1;
                } else if (--te->a <= 0) {
                    te->a = kPAbsent;  // remove(value)
                    if (lru) lru_remove<kLru>(m);
                }
            }
        }
    }
}

// ParamFlowSlot.applyRealParamIdx (ParamFlowSlot.java:56-66): a negative index is rewritten on the rule
// at its first check (the reference mutates the rule object), so the first event's arity fixes it
__device__ __forceinline__ int32_t param_idx_of(ParamRuleDev &p, uint32_t nargs) {
    if (p.idx_res == kIdxUnresolved) {
        int32_t idx = p.param_idx;
        if (idx < 0) idx = (-idx <= (int32_t)nargs) ? (int32_t)nargs + idx : -idx;
        p.idx_res = idx;
    }
    return p.idx_res;
}

// ParamFlowChecker.passLocalCheck (ParamFlowChecker.java:79-106): every element must pass, in order
// (elements before a failing one keep their token updates)
template <bool kLru>
__device__ bool param_local_check(const Ctx &c, uint32_t r, ParamRuleDev &p, int32_t idx, const uint64_t *vals,
                                  uint32_t nv, int acquire, int64_t t, int64_t *total_wait, uint32_t eidx) {
    for (uint32_t q = 0; q < nv; ++q) {
        const uint64_t v = vals[q];
        const uint64_t stamp = lru_stamp(c.st, eidx, q);
        int64_t tc = 0;
        if (p.grade == 0 && idx < kMaxParamIdx) {  // getThreadCount(rule.getParamIdx(), value): CacheMap.get
            PEntry *te = ptab_get(c.st.ttab, c.st.tmask, tmap_owner(r, (uint32_t)idx), v, false, c.st.overflow);
            if (te && te->a != kPAbsent) {
                tc = te->a;
                if (lru_on_t(c.st, r)) lru_touch<kLru>(c.st, map_ref_t(c.st, r, (uint32_t)idx), te, stamp);
            }
        }
        int64_t w = 0;
        const bool ok = c.pre_param ? (w = c.pre_wait, c.pre_param == 1) : param_pass<kLru>(c, p, v, acquire, t, tc, &w, stamp);
        if (!ok) return false;
        *total_wait += w;
    }
    return true;
}

template <bool kLru = false>
__device__ int8_t chain_entry(const Ctx &c, uint32_t r, const ResMem &m, int64_t t, int acquire, bool prio,
                              bool has_param, uint64_t param, int64_t *wait_ms, PArgs pa, uint32_t eidx) {
    const ResDev R = c.res ? *c.res : c.st.res[r];
    int64_t *node = m.node;
    *wait_ms = 0;
    int64_t total_wait = 0;
    // ParamFlowSlot.checkFlow (ParamFlowSlot.java:65-92): args is never null (SphU.entry passes [])
    const uint32_t nargs = ev_nargs(pa, has_param);
    for (uint32_t k = 0; k < R.n_prules; ++k) {
        ParamRuleDev &p = c.st.prules[R.prule_off + k];
        const int32_t idx = param_idx_of(p, nargs);
        // ParameterMetricStorage.initParamMetricsFor: the rule's thread-count map exists from now on
        if (idx < kMaxParamIdx && c.st.tmapmask) c.st.tmapmask[r] |= 1ull << idx;
        if ((int64_t)nargs <= (int64_t)idx) continue;  // ParamFlowChecker.passCheck: args.length <= paramIdx
        const uint64_t *vals;
        uint32_t nv;
        if (ev_arg(pa, (uint32_t)idx, param, &vals, &nv) == ARG_NULL) continue;  // a null value passes
        bool ok;
        if (p.cluster && p.grade == 1) {
            // passClusterCheck (ParamFlowChecker.java:305-333): requestParamToken(flowId, count,
            // toCollection(value)) to the embedded server, in event order; OK passes, BLOCKED blocks,
            // anything else -- or no token service -- falls back (fallbackToLocalOrPass, :335-343)
            int8_t ts = TRS_FAIL;
            if (c.st.cluster_on)
                ts = (int8_t)(cparam_request_exact(c.st.cpst, p.cflow, acquire, vals, nv, t, eidx) >> 48);
            if (ts == TRS_OK) ok = true;
            else if (ts == TRS_BLOCKED) ok = false;
            else ok = p.cfallback ? param_local_check<kLru>(c, r, p, idx, vals, nv, acquire, t, &total_wait, eidx) : true;
        } else {
            ok = param_local_check<kLru>(c, r, p, idx, vals, nv, acquire, t, &total_wait, eidx);
        }
        if (!ok) {
            node_add(c, node, t, MB_BLOCK, acquire);
            *wait_ms = (int64_t)k;  // block detail: the ParamFlowRule's index in the resource's list
            return D_BLOCK_PARAM;
        }
    }
    // FlowSlot
    for (uint32_t k = 0; k < R.n_rules; ++k) {
        int64_t w = 0;
        FlowRuleDev &fr = m.rules[k];
        if (fr.cluster) {
            // FlowRuleChecker.passClusterCheck (:168-188): the token service decides; the embedded
            // server is this engine's cluster path (DefaultTokenService.requestToken), in event order
            int8_t ts = TRS_FAIL;  // no service: fallbackToLocalOrPass
            int32_t tw = 0;
            if (c.st.cluster_on) {
                if (acquire <= 0) {
                    ts = TRS_BAD_REQUEST;
                } else if (fr.cslot < 0) {
                    ts = TRS_NO_RULE_EXISTS;
                } else {
                    const uint64_t res = request_exact(c.st.cst, (uint32_t)fr.cslot, t, acquire, prio, 0);
                    ts = (int8_t)(res >> 48);
                    tw = (int16_t)(res >> 32);
                }
            }
            if (ts == TRS_OK) continue;  // applyTokenResult (:203-230)
            if (ts == TRS_SHOULD_WAIT) {  // Thread.sleep(waitInMs), then pass
                total_wait += tw;
                continue;
            }
            if (ts == TRS_BLOCKED) {
                node_add(c, node, t, MB_BLOCK, acquire);
                *wait_ms = (int64_t)k;  // block detail: the FlowRule's index (FlowRuleComparator order)
                return D_BLOCK_FLOW;
            }
            if (!fr.cfallback) continue;  // fallbackToLocalOrPass: the rule is not activated
        }
        const int8_t d = rater_can_pass(c, fr, node, t, acquire, prio, &w);
        if (d == D_BLOCK_FLOW) {
            node_add(c, node, t, MB_BLOCK, acquire);
            *wait_ms = (int64_t)k;
            return D_BLOCK_FLOW;
        }
        if (d == D_PASS_WAIT) {
            node[kNodeThreads] += 1;
            param_threads<kLru>(c, r, pa, has_param, param, 1, eidx);
            *wait_ms = w;
            return D_PASS_WAIT;
        }
        total_wait += w;
    }
    // DegradeSlot
    if (const int kb = degrade_block_index(m.cbs, R.n_cbs, t); kb >= 0) {
        node_add(c, node, t, MB_BLOCK, acquire);
        *wait_ms = kb;  // block detail: the breaker's index (DegradeRuleManager list order)
        return D_BLOCK_DEGRADE;
    }
    node[kNodeThreads] += 1;
    node_add(c, node, t, MB_PASS, acquire);
    param_threads<kLru>(c, r, pa, has_param, param, 1, eidx);
    *wait_ms = total_wait;
    return D_PASS;
}

template <bool kLru = false>
__device__ void chain_exit(const Ctx &c, uint32_t r, const ResMem &m, int64_t t, int64_t rt, int count, bool error,
                           bool has_param, uint64_t param, PArgs pa, uint32_t eidx) {
    const ResDev R = c.res ? *c.res : c.st.res[r];
    int64_t *node = m.node;
    node_add_rt_success(c, node, t, rt, count);
    node[kNodeThreads] -= 1;
    if (error) node_add(c, node, t, MB_EXC, count);
    param_threads<kLru>(c, r, pa, has_param, param, -1, eidx);  // ParameterMetric.decreaseThreadCount
    for (uint32_t k = 0; k < R.n_cbs; ++k) cb_on_complete(m.cbs[k], t, rt, error);
}

// eidx: the event's index in the batch (CacheMap access stamps)
template <bool kLru = false>
__device__ __forceinline__ int8_t chain_entry(const Ctx &c, uint32_t r, int64_t t, int acquire, bool prio,
                                              bool has_param, uint64_t param, int64_t *wait_ms, PArgs pa,
                                              uint32_t eidx) {
    return chain_entry<kLru>(c, r, res_global(c, r, c.st.res[r]), t, acquire, prio, has_param, param, wait_ms, pa,
                             eidx);
}

template <bool kLru = false>
__device__ __forceinline__ void chain_exit(const Ctx &c, uint32_t r, int64_t t, int64_t rt, int count, bool error,
                                           bool has_param, uint64_t param, PArgs pa, uint32_t eidx) {
    chain_exit<kLru>(c, r, res_global(c, r, c.st.res[r]), t, rt, count, error, has_param, param, pa, eidx);
}

// StatisticSlot's BlockException branch for a block thrown by a slot outside the engine (SGA_KIND_BLOCKED,
// StatisticSlot.java:121-135): the resource's node counts the block (ENTRY_NODE: the caller)
__device__ __forceinline__ void blocked_event(const Ctx &c, uint32_t r, int64_t t, int a) {
    node_add(c, c.st.node + (size_t)r * kNodeWords, t, MB_BLOCK, a);
}

// SGA_KIND_REVOKE: a slot after the engine's checks blocked an entry the engine passed.  StatisticSlot never
// reached its pass accounting (StatisticSlot.java:77-84 follow fireEntry), only the block branch (:121-135):
// the pass and the thread are taken back, the block counted, the parameter thread counts released; a breaker
// this entry moved to HALF_OPEN falls back to OPEN, next retry kept (the probe's whenTerminate hook,
// AbstractCircuitBreaker.java:117-139, issue 1638) -- the entry is identified by its time, which the revoke
// carries.  ENTRY_NODE: the caller.
template <bool kLru = false>
__device__ void revoke_event(const Ctx &c, uint32_t r, int64_t t, int a, const PArgs &pa, bool hp, const uint64_t &pv,
                             uint32_t eidx) {
    int64_t *nd = c.st.node + (size_t)r * kNodeWords;
    nd[kNodeThreads] -= 1;
    node_add(c, nd, t, MB_PASS, -(int64_t)a);
    node_add(c, nd, t, MB_BLOCK, a);
    param_threads<kLru>(c, r, pa, hp, pv, -1, eidx);
    CbDev *cbs = c.st.cbs + c.st.res[r].cb_off;
    for (uint32_t k = 0; k < c.st.res[r].n_cbs; ++k)
        if (cbs[k].state == 2 && cbs[k].probe_t == t) cbs[k].state = 1;
}

// ------------------------------------------------------------------ SystemSlot / ENTRY_NODE
// Constants.ENTRY_NODE is node record nres.  StatisticSlot (StatisticSlot.java:54-137) updates it
// for inbound (EntryType.IN) entries and their exits.
__device__ __forceinline__ int64_t *entry_node(const Ctx &c) { return c.st.node + (size_t)c.st.nres * kNodeWords; }

// SystemRuleManager.checkSystem + checkBbr (SystemRuleManager.java:298-353) for an inbound entry
// returns the check that blocks (SystemBlockException's limitType: 0 "qps", 1 "thread", 2 "rt",
// 3 "load", 4 "cpu") or -1
__device__ int system_block_type(const Ctx &c, const SysDev &s, int64_t t, int count) {
    if (!s.check) return -1;
    int64_t *e = entry_node(c);
    if (node_pass_qps(c, e, t) + (double)count > s.qps) return 0;  // ENTRY_NODE.passQps()
    const int32_t thr = (int32_t)e[kNodeThreads];                  // curThreadNum()
    if ((int64_t)thr > s.max_thread) return 1;
    sec_current(e, t, c.max_rt);                                      // avgRt(): success(), rt()
    const int64_t succ = sec_sum(e, t, MB_SUCC);
    const double rt = succ == 0 ? 0.0 : (double)sec_sum(e, t, MB_RT) * 1.0 / (double)succ;
    if (rt > (double)s.max_rt) return 2;
    if (s.load_set && s.cur_load > s.load) {
        if (thr > 1) {
            // maxSuccessQps() = maxSuccess * sampleCount / intervalInSec; minRt() = max(1, min bucket minRt)
            int64_t ms = 0, mr = c.max_rt;
            for (int j = 0; j < 2; ++j) {
                const int64_t *b = e + kNodeSec + kMB * j;
                if (b[0] == kAbsent || t - b[0] > kSecInterval) continue;
                if (b[MB_SUCC] > ms) ms = b[MB_SUCC];
                if (b[MB_MINRT] < mr) mr = b[MB_MINRT];
            }
            if (ms < 1) ms = 1;
            if (mr < 1) mr = 1;
            const double cap = (double)ms * 2.0 / 1.0 * (double)mr / 1000;
            if ((double)thr > cap) return 3;
        }
    }
    if (s.cpu_set && s.cur_cpu > s.cpu) return 4;
    return -1;
}

__device__ __forceinline__ void entry_node_after_entry(const Ctx &c, int64_t t, int a, int8_t d) {
    int64_t *e = entry_node(c);
    if (d == D_PASS) {
        e[kNodeThreads] += 1;
        node_add(c, e, t, MB_PASS, a);
    } else if (d == D_PASS_WAIT) {
        e[kNodeThreads] += 1;
    } else {
        node_add(c, e, t, MB_BLOCK, a);
    }
}

__device__ __forceinline__ void entry_node_after_exit(const Ctx &c, int64_t t, int64_t rt, int a, bool error) {
    int64_t *e = entry_node(c);
    node_add_rt_success(c, e, t, rt, a);
    e[kNodeThreads] -= 1;
    if (error) node_add(c, e, t, MB_EXC, a);
}

// System-rule mode: the whole batch by one lane in arrival order (checkSystem reads ENTRY_NODE,
// which every earlier inbound decision of every resource changed).
// Device entry gate (FlowEngine::submit_device): k_lgate sets kGateSeq when the chunk must be replayed
// in arrival order (inbound events under a SystemRule, or Collection arguments), kGateIn when it holds
// inbound events, kGateBad on invalid input (the chunk is not applied).  A null gate (host entry)
// lets every kernel run; the host launches only the ones the chunk needs.
constexpr uint32_t kGateSeq = 1, kGateIn = 2, kGateBad = 4;
__device__ __forceinline__ bool gate_is(const uint32_t *g, uint32_t mask, uint32_t want) {
    return !g || (*g & mask) == want;
}

__global__ __launch_bounds__(kT) void k_lgate(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ resource,
                                              const int32_t *__restrict__ acquire, const uint8_t *__restrict__ flags,
                                              const uint64_t *__restrict__ param_in, uint32_t n, uint32_t nres,
                                              int sys_check, uint64_t npvals, uint32_t *gate,
                                              const uint64_t *__restrict__ pvals) {
    uint32_t g = 0;
    for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
        const uint8_t fl = flags ? flags[i] : 0;
        if (acquire[i] < 0 || kind[i] > SGA_KIND_REVOKE) g |= kGateBad;
        // kind 2 / 3 events and argument lists take the parallel pipeline (their resources are replayed per
        // resource, in arrival order); only SystemRules couple resources (one lane for the whole chunk)
        if ((fl & SGA_EV_INBOUND) && resource[i] < nres) g |= sys_check ? (kGateIn | kGateSeq) : kGateIn;
        if (fl & SGA_EV_ARGS) {  // the argument vector's word pairs and every list inside npvals
            const uint64_t pv = param_in ? param_in[i] : 0;
            const uint64_t off = pv >> 32, na = pv & 0xFFFFFFFFu;
            if (!pvals || off + 2 * na > npvals) {
                g |= kGateBad;
            } else {
                for (uint64_t k = 0; k < na; ++k) {
                    const uint64_t h = pvals[off + 2 * k], w = pvals[off + 2 * k + 1];
                    if ((h >> 62) > 2 || ((h >> 62) == ARG_LIST && w + (h & 0xFFFFFFFFu) > npvals)) g |= kGateBad;
                }
            }
        } else if ((fl & (SGA_EV_PARAM_LIST | SGA_EV_HAS_PARAM)) == (SGA_EV_PARAM_LIST | SGA_EV_HAS_PARAM)) {
            const uint64_t pv = param_in ? param_in[i] : 0;
            if ((pv >> 32) + (pv & 0xFFFFFFFFu) > npvals) g |= kGateBad;
        }
    }
    g = wave_or_u32(g);
    if ((threadIdx.x & 63) == 0 && g) atomicOr(gate, g);
}

// Last kernel of a device chunk: an invalid chunk answers -1 for every event; the sticky word
// (device_status) collects invalid chunks (bit 0) and full parameter maps (bit 1).
__global__ __launch_bounds__(kT) void k_lfail(const uint32_t *gate, const uint32_t *overflow, uint32_t *sticky,
                                              uint32_t n, int8_t *decision, int32_t *wait_ms) {
    const uint32_t g = *gate;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint32_t o = *overflow;
        const uint32_t e = ((g & kGateBad) ? 1u : 0u) | ((o & ~kOvfMissingEntry) ? 2u : 0u) |
                           ((o & kOvfMissingEntry) ? 4u : 0u);
        if (e) atomicOr(sticky, e);
    }
    if (!(g & kGateBad) && !(*overflow & kOvfMissingEntry)) return;  // else every decision answers -1
    for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
        decision[i] = -1;
        wait_ms[i] = 0;
    }
}

__global__ void k_lseq(FlowState st, int64_t max_rt, SysDev sys, const uint8_t *__restrict__ kind,
                       const uint32_t *__restrict__ resource, const uint32_t *__restrict__ ts_off, int64_t ts_base,
                       const int32_t *__restrict__ acquire, const uint8_t *__restrict__ flags,
                       const int64_t *__restrict__ rt_in, const uint64_t *__restrict__ param_in, uint32_t n,
                       int8_t *decision, int32_t *wait_ms, const uint64_t *__restrict__ pvals) {
    if (threadIdx.x || blockIdx.x || !gate_is(st.gate, kGateSeq | kGateBad, kGateSeq)) return;
    const Ctx c{st, max_rt};
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r = resource[i];
        decision[i] = D_PASS;
        wait_ms[i] = 0;
        if (r >= st.nres) continue;  // unknown resource: no node, no rules
        const int64_t t = ts_base + (int64_t)ts_off[i];
        const uint8_t fl = flags[i];
        const bool in = (fl & SGA_EV_INBOUND) != 0, hp = (fl & SGA_EV_HAS_PARAM) != 0;
        const int a = (int)((uint32_t)acquire[i] & 0x7FFFFFFFu);
        PArgs pa{nullptr, 0};
        if ((fl & SGA_EV_ARGS) && pvals) {
            pa.args = pvals + (param_in[i] >> 32);
            pa.pvals = pvals;
            pa.nargs = (uint32_t)param_in[i];
        } else if (hp && (fl & SGA_EV_PARAM_LIST) && pvals) {
            pa = PArgs{pvals + (param_in[i] >> 32), (uint32_t)param_in[i]};
        }
        if (kind[i] == 1) {
            chain_exit<true>(c, r, t, rt_in[i], a, (fl & SGA_EV_ERROR) != 0, hp, param_in[i], pa, i);
            if (in) entry_node_after_exit(c, t, rt_in[i], a, (fl & SGA_EV_ERROR) != 0);
            continue;
        }
        if (kind[i] == SGA_KIND_BLOCKED) {  // StatisticSlot's BlockException branch for a block thrown outside the engine
            blocked_event(c, r, t, a);
            if (in) node_add(c, entry_node(c), t, MB_BLOCK, a);
            continue;
        }
        if (kind[i] == SGA_KIND_REVOKE) {
            revoke_event<true>(c, r, t, a, pa, hp, param_in[i], i);
            if (in) {
                int64_t *e = entry_node(c);
                e[kNodeThreads] -= 1;
                node_add(c, e, t, MB_PASS, -(int64_t)a);
                node_add(c, e, t, MB_BLOCK, a);
            }
            continue;
        }
        int8_t d;
        int64_t w = 0;
        if (const int sb = in ? system_block_type(c, sys, t, a) : -1; sb >= 0) {
            node_add(c, st.node + (size_t)r * kNodeWords, t, MB_BLOCK, a);  // StatisticSlot: increaseBlockQps
            d = D_BLOCK_SYSTEM;
            w = sb;  // block detail: the SystemRule check
        } else {
            d = chain_entry<true>(c, r, t, a, (fl & SGA_EV_PRIORITIZED) != 0, hp, param_in[i], &w, pa, i);
        }
        if (in) entry_node_after_entry(c, t, a, d);
        decision[i] = d;
        wait_ms[i] = (int32_t)w;
    }
}

// ENTRY_NODE statistics after a parallel batch (no system check): one workgroup walks the batch
// in tiles.  A tile whose times do not decrease (and do not go below the previous tile's last
// time) is reduced per 500 ms second-window bucket and applied bucket by bucket -- the same
// window rotations as event by event, since a 500 ms bucket lies inside one 1 s minute bucket;
// any other tile is applied event by event by one lane.
constexpr int kEnTile = 1024, kEnBuckets = 64;
__global__ __launch_bounds__(kEnTile) void k_entry_stats(FlowState st, int64_t max_rt,
                                                         const uint8_t *__restrict__ kind,
                                                         const uint32_t *__restrict__ resource,
                                                         const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                         const int32_t *__restrict__ acquire,
                                                         const uint8_t *__restrict__ flags,
                                                         const int64_t *__restrict__ rt_in,
                                                         const int8_t *__restrict__ decision, uint32_t n) {
    __shared__ unsigned long long bs[kEnBuckets][5];  // pass, block, success, rt, exception (two's complement)
    __shared__ long long bmin[kEnBuckets];            // min rt
    __shared__ unsigned long long thr_delta;
    __shared__ int mono, any;
    __shared__ int64_t prev_last;
    if (!gate_is(st.gate, kGateSeq | kGateIn | kGateBad, kGateIn)) return;
    const Ctx c{st, max_rt};
    if (threadIdx.x == 0) prev_last = INT64_MIN;
    for (uint32_t base = 0; base < n; base += kEnTile) {
        const uint32_t i = base + threadIdx.x;
        const bool live = i < n && resource[i] < st.nres && (flags[i] & SGA_EV_INBOUND);
        const int64_t t = i < n ? ts_base + (int64_t)ts_off[i] : INT64_MAX;
        for (int k = threadIdx.x; k < kEnBuckets * 5; k += kEnTile) bs[k / 5][k % 5] = 0;
        for (int k = threadIdx.x; k < kEnBuckets; k += kEnTile) bmin[k] = max_rt;
        if (threadIdx.x == 0) {
            mono = 1;
            any = 0;
            thr_delta = 0;
        }
        __syncthreads();
        const int64_t t0 = ts_base + (int64_t)ts_off[base];
        if (i < n) {
            const int64_t tp = threadIdx.x == 0 ? prev_last : ts_base + (int64_t)ts_off[i - 1];
            if (t < tp || t / kSecW - t0 / kSecW >= kEnBuckets) mono = 0;
        }
        if (live) any = 1;
        __syncthreads();
        if (any && mono) {
            if (live) {
                const int bk = (int)(t / kSecW - t0 / kSecW);
                const int a = (int)((uint32_t)acquire[i] & 0x7FFFFFFFu);
                typedef unsigned long long u64;
                if (kind[i] == 1) {
                    atomicAdd(&bs[bk][2], (u64)a);
                    atomicAdd(&bs[bk][3], (u64)rt_in[i]);
                    if (flags[i] & SGA_EV_ERROR) atomicAdd(&bs[bk][4], (u64)a);
                    atomicMin(&bmin[bk], (long long)rt_in[i]);
                    atomicAdd(&thr_delta, ~0ull);  // -1
                } else if (kind[i] == SGA_KIND_BLOCKED) {  // StatisticSlot's block branch on ENTRY_NODE
                    atomicAdd(&bs[bk][1], (u64)a);
                } else if (kind[i] == SGA_KIND_REVOKE) {  // the pass and the thread taken back, the block counted
                    atomicAdd(&bs[bk][0], (u64)(-(int64_t)a));
                    atomicAdd(&bs[bk][1], (u64)a);
                    atomicAdd(&thr_delta, ~0ull);
                } else {
                    const int8_t d = decision[i];
                    if (d == D_PASS) {
                        atomicAdd(&bs[bk][0], (u64)a);
                        atomicAdd(&thr_delta, 1ull);
                    } else if (d == D_PASS_WAIT) {
                        atomicAdd(&thr_delta, 1ull);
                    } else {
                        atomicAdd(&bs[bk][1], (u64)a);
                    }
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int64_t *e = entry_node(c);
                const int64_t last_t = ts_base + (int64_t)ts_off[min(base + kEnTile, n) - 1];
                const int nb = (int)(last_t / kSecW - t0 / kSecW) + 1;
                for (int b = 0; b < nb; ++b) {
                    int64_t v[6];
                    for (int q = 0; q < 5; ++q) v[q] = (int64_t)bs[b][q];
                    v[5] = bmin[b];
                    const bool has_sec = v[0] || v[1] || v[2] || v[3] || v[4] || v[5] != max_rt;
                    if (!has_sec) continue;
                    const int64_t tb = (t0 / kSecW + b) * kSecW;
                    int64_t *w2[2] = {sec_current(e, tb, max_rt), min_current(e, tb, max_rt)};
                    for (int q = 0; q < 2; ++q) {
                        int64_t *w = w2[q];
                        if (!w) continue;
                        w[MB_PASS] += v[0];
                        w[MB_BLOCK] += v[1];
                        w[MB_SUCC] += v[2];
                        w[MB_RT] += v[3];
                        w[MB_EXC] += v[4];
                        if (v[5] < w[MB_MINRT]) w[MB_MINRT] = v[5];
                    }
                }
                e[kNodeThreads] += (int64_t)thr_delta;
            }
        } else if (any && threadIdx.x == 0) {  // out of order: event by event
            for (uint32_t j = base; j < min(base + kEnTile, n); ++j) {
                if (resource[j] >= st.nres || !(flags[j] & SGA_EV_INBOUND)) continue;
                const int64_t tj = ts_base + (int64_t)ts_off[j];
                const int a = (int)((uint32_t)acquire[j] & 0x7FFFFFFFu);
                if (kind[j] == 1) {
                    entry_node_after_exit(c, tj, rt_in[j], a, (flags[j] & SGA_EV_ERROR) != 0);
                } else if (kind[j] == SGA_KIND_BLOCKED) {
                    node_add(c, entry_node(c), tj, MB_BLOCK, a);
                } else if (kind[j] == SGA_KIND_REVOKE) {
                    int64_t *e = entry_node(c);
                    e[kNodeThreads] -= 1;
                    node_add(c, e, tj, MB_PASS, -(int64_t)a);
                    node_add(c, e, tj, MB_BLOCK, a);
                } else {
                    entry_node_after_entry(c, tj, a, decision[j]);
                }
            }
        }
        if (threadIdx.x == 0) prev_last = ts_base + (int64_t)ts_off[min(base + kEnTile, n) - 1];
        __syncthreads();
    }
}

// ------------------------------------------------------------------ classify
// An argument vector (SGA_EV_ARGS) restated as the one-value form (args = [param] or []) when that decides
// and counts the same: every parameter rule of the resource reads argument 0 (its index resolved, or fixed at
// 0), no thread-count map of another index exists (only rules create them), and argument 0 is a scalar or
// null (a null or absent argument passes every rule and counts no thread: the no-parameter form).  A
// Collection at 0, or another index, keeps the vector (F_SPECIAL).
__device__ __forceinline__ bool args_one_value(const FlowState &st, uint32_t r, uint64_t pv,
                                               const uint64_t *__restrict__ pvals, bool *hp, uint64_t *v) {
    const ResDev R = st.res[r];
    for (uint32_t k = 0; k < R.n_prules; ++k) {
        const ParamRuleDev &p = st.prules[R.prule_off + k];
        const int32_t idx = p.idx_res != kIdxUnresolved ? p.idx_res : (p.param_idx >= 0 ? p.param_idx : -1);
        if (idx != 0) return false;
    }
    if (st.tmapmask && (st.tmapmask[r] & ~1ull)) return false;
    const uint32_t na = (uint32_t)pv;
    if (na == 0) {
        *hp = false;
        *v = 0;
        return true;
    }
    const uint64_t h = pvals[pv >> 32];
    const int k0 = (int)(h >> 62);
    if (k0 == ARG_LIST) return false;
    *hp = k0 == ARG_SCALAR;
    *v = *hp ? pvals[(pv >> 32) + 1] : 0;
    return true;
}

__global__ __launch_bounds__(kT) void k_lclassify(FlowState st, FlowScratch sc, const uint8_t *__restrict__ kind,
                                                  const uint32_t *__restrict__ resource,
                                                  const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                  const int32_t *__restrict__ acquire,
                                                  const uint8_t *__restrict__ flags,
                                                  const uint64_t *__restrict__ param_in, uint32_t n, uint32_t *keys,
                                                  Payload *pay, int8_t *decision, int32_t *wait_ms) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) {  // k_lseq or k_lfail answers: every event a no-op here
        keys[i] = st.nres;
        pay[i] = Payload{i, 0, 0, 0};
        return;
    }
    const uint32_t r = resource[i];
    const uint8_t fl = flags ? flags[i] : 0;
    const uint8_t kd = kind[i];
    const bool ex = kd == 1;
    wait_ms[i] = 0;
    if (r >= st.nres) {  // unknown resource: no node, no rules (documented)
        decision[i] = D_PASS;
        keys[i] = st.nres;
        pay[i] = Payload{i, 0, 0, 0};
        return;
    }
    keys[i] = r;
    const uint32_t off = ts_off[i];
    const int64_t t = ts_base + (int64_t)off;
    // the parameter the parallel kernels read (ev_param): the event's own, or its argument vector's one value
    bool hp = (fl & SGA_EV_HAS_PARAM) != 0, kept = false;  // kept: the arguments stay whole (the replay reads them)
    uint64_t pv = param_in ? param_in[i] : 0;
    if (fl & SGA_EV_ARGS) {
        kept = !args_one_value(st, r, pv, sc.pvals, &hp, &pv);
    } else if (hp && (fl & SGA_EV_PARAM_LIST)) {
        kept = true;
    }
    const bool spec = kept || kd >= SGA_KIND_BLOCKED;
    // the resource's level this chunk (res_special = epoch << 2 | level, the highest wins): 1 -- kind 2 / 3 events
    // only, which the per-value segments of a parameter-only resource also take (a revoke is an exit there
    // that takes its pass back); 2 -- arguments kept whole: the per-resource replay
    const uint32_t lvl = kept ? 2u : (spec ? 1u : 0u);
    if (spec && sc.res_special) {
        const uint32_t mark = (sc.epoch << 2) | lvl;
        if (sc.res_special[r] < mark) atomicMax(&sc.res_special[r], mark);
    }
    if (sc.ev_param) sc.ev_param[i] = pv;
    // a revoke is an exit (thread counts) that takes its pass back; a block is neither entry nor exit
    // (its parameter bit: a block outside the engine touches no parameter map)
    uint32_t idx = i | ((ex || kd == SGA_KIND_REVOKE) ? F_EXIT : 0u) | ((fl & SGA_EV_ERROR) ? F_ERROR : 0u) |
                   ((hp && kd != SGA_KIND_BLOCKED) ? F_PARAM : 0u) | (spec ? F_SPECIAL : 0u);
    const uint32_t a = (uint32_t)acquire[i] & 0x7FFFFFFFu;
    pay[i] = Payload{idx, off, a | ((!ex && !spec && (fl & SGA_EV_PRIORITIZED)) ? 0x80000000u : 0u),
                     (uint32_t)(t / kSecW)};
    // the default decision: PASS; a parameter entry of a resource with parameter rules starts as a parameter
    // block, so k_pseg_long writes only its passes (coalesced here instead of a scattered fill of the long
    // segments' blocks).  Every other path that decides such an entry writes its decision explicitly
    // (lane_run / k_lheavy / k_llru_ps / k_lseq / k_pseg_solve).
    decision[i] = (kd == 0 && hp && !spec && st.res[r].n_prules) ? (int8_t)D_BLOCK_PARAM : (int8_t)D_PASS;
}

// ------------------------------------------------------------------ runs (segmented scan)
struct LAgg {
    uint32_t nh, nf, flag;
    uint32_t nent, nexit, cp;   // entries, exits, prioritized entries since the run head
    int32_t mn, mx;             // entry acquire min / max
    int64_t asum;               // entry acquire sum
};

__device__ __forceinline__ LAgg lagg_id() { return LAgg{0, 0, 0, 0, 0, 0, INT32_MAX, INT32_MIN, 0}; }

__device__ __forceinline__ LAgg lagg_combine(const LAgg &a, const LAgg &b) {
    LAgg r;
    r.nh = a.nh + b.nh;
    r.nf = a.nf + b.nf;
    r.flag = a.flag | b.flag;
    r.nent = b.flag ? b.nent : a.nent + b.nent;
    r.nexit = b.flag ? b.nexit : a.nexit + b.nexit;
    r.cp = b.flag ? b.cp : a.cp + b.cp;
    r.mn = b.flag ? b.mn : min(a.mn, b.mn);
    r.mx = b.flag ? b.mx : max(a.mx, b.mx);
    r.asum = b.flag ? b.asum : a.asum + b.asum;
    return r;
}

// staged run-scan element: key with the exit flag in bit 31 (kKeyExit), bucket, acq_prio
constexpr uint32_t kKeyExit = 0x80000000u;
__device__ __forceinline__ LAgg lagg_value(uint32_t kx, uint32_t pkx, uint32_t b, uint32_t pb, uint32_t acq_prio,
                                           bool has_prev, bool valid) {
    if (!valid) return lagg_id();
    const bool fh = !has_prev || ((kx ^ pkx) & ~kKeyExit) != 0;
    const bool h = fh || b != pb;
    const bool ex = (kx & kKeyExit) != 0;
    const int32_t a = (int32_t)(acq_prio & 0x7FFFFFFFu);
    return LAgg{h ? 1u : 0u, fh ? 1u : 0u, h ? 1u : 0u, ex ? 0u : 1u, ex ? 1u : 0u,
                ex ? 0u : (acq_prio >> 31), ex ? INT32_MAX : a, ex ? INT32_MIN : a, ex ? 0 : (int64_t)a};
}

// blocked arrangement per thread (kItems consecutive events), block scan of thread aggregates
template <int NT>
__device__ LAgg lblock_excl(const LAgg &v, LAgg *total) {
    __shared__ LAgg sh[NT];
    sh[threadIdx.x] = v;
    __syncthreads();
    // Hillis-Steele in LDS (NT = 256: 8 steps)
    for (int o = 1; o < NT; o <<= 1) {
        LAgg x = sh[threadIdx.x];
        if ((int)threadIdx.x >= o) x = lagg_combine(sh[threadIdx.x - o], x);
        __syncthreads();
        sh[threadIdx.x] = x;
        __syncthreads();
    }
    const LAgg incl = sh[threadIdx.x];
    if (total) *total = sh[NT - 1];
    const LAgg ex = threadIdx.x ? sh[threadIdx.x - 1] : lagg_id();
    __syncthreads();
    (void)incl;
    return ex;
}

// The blocked arrangement (thread t: the tile's elements t * kItems .. + kItems) read through LDS: one
// thread's consecutive elements are kItems x 16 bytes apart, so direct loads put every lane of a wave on
// its own cache lines and the lines are fetched again for each element (10x the bytes, PMC).  The tile
// and its neighbours ([base - 1, base + kTileElems + 1), kStage elements) are loaded with coalesced
// (striped) loads instead; an LDS slot per kItems elements of padding keeps the strided reads of the
// compute loops off one bank.
constexpr int kStage = kTileElems + 2;
constexpr int kStagePad = kStage + kStage / kItems + 1;
__device__ __forceinline__ uint32_t spad(uint32_t i) { return i + i / kItems; }
// LDS slot of element e of the tile at base (e in [base - 1, base + kTileElems + 1))
__device__ __forceinline__ uint32_t sslot(uint32_t base, uint32_t e) { return spad(e + 1 - base); }
template <class T>
__device__ __forceinline__ void stage_tile(T *lds, const T *__restrict__ g, uint32_t base, uint32_t lim, T none) {
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < (uint32_t)kStage; i += kT) {
        const uint32_t e = base + i - 1;  // base 0: e wraps for i = 0, and lim excludes it
        lds[spad(i)] = (base + i >= 1 && e < lim) ? g[e] : none;
    }
}

// the run scans stage only what they read of an element (12 of its 20 bytes: key + exit flag, bucket,
// acquire): 52 KB of LDS per tile instead of 87, so that more than one tile is resident per CU
__device__ __forceinline__ void stage_runs(uint32_t *skey, uint32_t *sbk, uint32_t *sacq, const uint32_t *__restrict__ keys,
                                           const Payload *__restrict__ pay, uint32_t base, uint32_t lim,
                                           uint32_t invalid) {
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < (uint32_t)kStage; i += kT) {
        const uint32_t e = base + i - 1;  // base 0: e wraps for i = 0, and lim excludes it
        uint32_t k = invalid, b = 0, a = 0;
        if (base + i >= 1 && e < lim) {
            const Payload q = pay[e];
            k = keys[e] | ((q.idx & F_EXIT) ? kKeyExit : 0u);
            b = q.bucket;
            a = q.acq_prio;
        }
        skey[spad(i)] = k;
        sbk[spad(i)] = b;
        sacq[spad(i)] = a;
    }
}

__global__ __launch_bounds__(kT) void k_lruns_up(const uint32_t *__restrict__ keys, const Payload *__restrict__ pay,
                                                 uint32_t n, uint32_t invalid, LAgg *tile_agg, uint32_t *tile_valid) {
    __shared__ uint32_t skey[kStagePad], sbk[kStagePad], sacq[kStagePad];
    const uint32_t base = blockIdx.x * kTileElems;
    stage_runs(skey, sbk, sacq, keys, pay, base, n, invalid);
    __syncthreads();
    const uint32_t e0 = base + threadIdx.x * kItems;
    LAgg acc = lagg_id();
    uint32_t nv = 0;
    if (e0 < n) {
        uint32_t pk = e0 > 0 ? skey[sslot(base, e0 - 1)] : invalid;
        uint32_t pb = e0 > 0 ? sbk[sslot(base, e0 - 1)] : 0u;
        for (int i = 0; i < kItems && e0 + i < n; ++i) {
            const uint32_t e = e0 + i;
            const uint32_t k = skey[sslot(base, e)], b = sbk[sslot(base, e)];
            const bool valid = (k & ~kKeyExit) != invalid;
            acc = lagg_combine(acc, lagg_value(k, pk, b, pb, sacq[sslot(base, e)], e > 0, valid));
            nv += valid ? 1 : 0;
            pk = k;
            pb = b;
        }
    }
    LAgg total;
    lblock_excl<kT>(acc, &total);
    __shared__ uint32_t cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    atomicAdd(&cnt, nv);
    __syncthreads();
    if (threadIdx.x == 0) {
        tile_agg[blockIdx.x] = total;
        tile_valid[blockIdx.x] = cnt;
    }
}

__global__ __launch_bounds__(kT) void k_lruns_tiles(const LAgg *__restrict__ tile_agg,
                                                    const uint32_t *__restrict__ tile_valid, uint32_t ntiles,
                                                    LAgg *tile_carry, uint32_t *counters) {
    LAgg carry = lagg_id();
    uint32_t nvalid = 0;
    for (uint32_t b = 0; b < ntiles; b += kT) {
        const uint32_t t = b + threadIdx.x;
        const LAgg v = t < ntiles ? tile_agg[t] : lagg_id();
        LAgg total;
        const LAgg ex = lblock_excl<kT>(v, &total);
        if (t < ntiles) tile_carry[t] = lagg_combine(carry, ex);
        carry = lagg_combine(carry, total);
        __shared__ uint32_t s;
        if (threadIdx.x == 0) s = 0;
        __syncthreads();
        if (t < ntiles) atomicAdd(&s, tile_valid[t]);
        __syncthreads();
        nvalid += s;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counters[0] = nvalid;
        counters[1] = carry.nh;
        counters[2] = carry.nf;
    }
}

__global__ __launch_bounds__(kT) void k_lruns_down(const uint32_t *__restrict__ keys, const Payload *__restrict__ pay,
                                                   const int64_t *__restrict__ rt_in, uint32_t invalid,
                                                   const LAgg *__restrict__ tile_carry, FlowScratch sc) {
    __shared__ uint32_t skey[kStagePad], sbk[kStagePad], sacq[kStagePad];
    // the per-event outputs, stored coalesced below: run ids less the tile's first (they fit 16 bits), and
    // entry indices over the element's own acquire slot (each thread reads only its own elements' sacq, and
    // reads each before it writes it)
    __shared__ uint16_t srun[kTileElems];
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;
    stage_runs(skey, sbk, sacq, keys, pay, base, nvalid, invalid);
    __syncthreads();
    const uint32_t e0 = base + threadIdx.x * kItems;
    LAgg acc = lagg_id();
    uint32_t pk0 = e0 > 0 && e0 - 1 < nvalid ? skey[sslot(base, e0 - 1)] : invalid;
    uint32_t pb0 = e0 > 0 && e0 - 1 < nvalid ? sbk[sslot(base, e0 - 1)] : 0u;
    {
        uint32_t pk = pk0, pb = pb0;
        for (int i = 0; i < kItems && e0 + i < nvalid; ++i) {
            const uint32_t e = e0 + i;
            const uint32_t k = skey[sslot(base, e)], b = sbk[sslot(base, e)];
            acc = lagg_combine(acc, lagg_value(k, pk, b, pb, sacq[sslot(base, e)], e > 0, true));
            pk = k;
            pb = b;
        }
    }
    const LAgg ex = lblock_excl<kT>(acc, nullptr);
    const LAgg carry = tile_carry[blockIdx.x];
    const uint32_t rid0 = carry.nh - 1;  // the run before the tile's first element (wraps for tile 0)
    LAgg run = lagg_combine(carry, ex);
    uint32_t pk = pk0, pb = pb0;
    for (int i = 0; i < kItems && e0 + i < nvalid; ++i) {
        const uint32_t e = e0 + i;
        const uint32_t kx = skey[sslot(base, e)], b = sbk[sslot(base, e)];
        const LAgg v = lagg_value(kx, pk, b, pb, sacq[sslot(base, e)], e > 0, true);
        run = lagg_combine(run, v);
        const uint32_t rid = run.nh - 1;
        const bool ex_ev = (kx & kKeyExit) != 0;
        const uint32_t k = kx & ~kKeyExit;
        srun[e - base] = (uint16_t)(rid - rid0);
        sacq[sslot(base, e)] = ex_ev ? 0xFFFFFFFFu : run.nent - 1;  // entry index within the run
        if (v.flag) {
            sc.run_start[rid] = e;
            sc.run_slot[rid] = k;
            sc.run_t0off[rid] = pay[e].ts_off;
            sc.run_exc[rid] = 0;
            sc.run_exerr[rid] = 0;
            sc.run_exrt[rid] = 0;
            sc.run_exmin[rid] = INT64_MAX;
        }
        if (v.nf) sc.flow_first_run[run.nf - 1] = rid;
        bool last = e + 1 >= nvalid;
        if (!last) last = (skey[sslot(base, e + 1)] & ~kKeyExit) != k || sbk[sslot(base, e + 1)] != b;
        if (last) {
            sc.run_end[rid] = e + 1;
            sc.run_nent[rid] = run.nent;
            sc.run_nexit[rid] = run.nexit;
            sc.run_cp[rid] = run.cp;
            sc.run_amin[rid] = run.mn;
            sc.run_amax[rid] = run.mx;
            sc.run_asum[rid] = run.asum;
        }
        pk = kx;
        pb = b;
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < (uint32_t)kTileElems; i += kT) {
        if (base + i >= nvalid) break;
        sc.ev_run[base + i] = rid0 + (uint32_t)srun[i];
        sc.ev_eidx[base + i] = sacq[spad(i + 1)];
    }
}

// exit aggregates per run (SUCCESS count, exceptions, RT sum, min RT): atomics per run
// pre-reduced inside each thread's consecutive events.
// a tile's (idx | acq_prio << 32) per element, staged like stage_tile (8 of a payload's 16 bytes)
__device__ __forceinline__ void stage_idx_acq(uint64_t *sia, const Payload *__restrict__ pay, uint32_t base,
                                              uint32_t lim) {
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < (uint32_t)kStage; i += kT) {
        const uint32_t e = base + i - 1;
        uint64_t v = 0;
        if (base + i >= 1 && e < lim) {
            const Payload q = pay[e];
            v = (uint64_t)q.idx | ((uint64_t)q.acq_prio << 32);
        }
        sia[spad(i)] = v;
    }
}

__global__ __launch_bounds__(kT) void k_lexits(const Payload *__restrict__ pay, const int64_t *__restrict__ rt_in,
                                               FlowScratch sc) {
    // staged: run ids, and (idx | acq_prio << 32) per element, whose slot an exit then overwrites with its RT
    // (each thread reads and writes only its own elements): 56 KB of LDS, two tiles per CU
    __shared__ uint32_t srun[kStagePad];
    __shared__ uint64_t sia[kStagePad];
    __shared__ uint8_t sex[kTileElems];  // an exit's RT is in sia
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;  // the whole block
    stage_tile(srun, sc.ev_run, base, nvalid, 0xFFFFFFFFu);
    stage_idx_acq(sia, pay, base, nvalid);
    for (uint32_t i = threadIdx.x; i < (uint32_t)kTileElems; i += kT) sex[i] = 0;
    __syncthreads();
    const uint32_t e0 = (blockIdx.x * kT + threadIdx.x) * kItems;  // no early return: the wave reduction below
    uint32_t cur = 0xFFFFFFFFu;
    uint64_t c = 0, er = 0;
    int64_t rs = 0, mn = INT64_MAX;
    auto flush = [&]() {
        if (cur == 0xFFFFFFFFu || (c == 0 && mn == INT64_MAX)) return;
        atomicAdd((unsigned long long *)&sc.run_exc[cur], (unsigned long long)c);
        atomicAdd((unsigned long long *)&sc.run_exerr[cur], (unsigned long long)er);
        atomicAdd((unsigned long long *)&sc.run_exrt[cur], (unsigned long long)rs);
        atomicMin((long long *)&sc.run_exmin[cur], (long long)mn);
    };
    for (int i = 0; i < kItems && e0 + i < nvalid; ++i) {
        const uint32_t e = e0 + i;
        const uint64_t qv = sia[sslot(base, e)];
        const uint32_t qidx = (uint32_t)qv, qacq = (uint32_t)(qv >> 32);
        if (!(qidx & F_EXIT) || (qidx & F_SPECIAL)) continue;  // a revoke completes nothing (no success, no RT)
        const uint32_t r = srun[sslot(base, e)];
        if (r != cur) {
            flush();
            cur = r;
            c = er = 0;
            rs = 0;
            mn = INT64_MAX;
        }
        const uint64_t cnt = qacq & 0x7FFFFFFFu;
        const int64_t rt = rt_in[qidx & F_IDX];
        sia[sslot(base, e)] = (uint64_t)rt;
        sex[e - base] = 1;
        c += cnt;
        if (qidx & F_ERROR) er += cnt;
        rs += rt;
        if (rt < mn) mn = rt;
    }
    // a long run covers whole waves: one set of atomics per wave
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur);
    if (__all(cur == c0) && c0 != 0xFFFFFFFFu) {
        c = (uint64_t)readlane_i64(wave_incl_sum_i64((int64_t)c), 63);
        er = (uint64_t)readlane_i64(wave_incl_sum_i64((int64_t)er), 63);
        rs = readlane_i64(wave_incl_sum_i64(rs), 63);
        mn = readlane_i64(wave_incl_min_i64(mn), 63);
        if ((threadIdx.x & 63) != 0) cur = 0xFFFFFFFFu;
    }
    flush();
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (uint32_t)kTileElems; i += kT) {  // the exits' RTs, coalesced
        if (base + i >= nvalid) break;
        if (sex[i]) sc.rt_sorted[base + i] = (int64_t)sia[spad(i + 1)];
    }
}

// ------------------------------------------------------------------ per-resource resolve
__device__ __forceinline__ bool default_cond(double count, int64_t sum, int32_t a) {
    // curCount + acquireCount > count ? block : pass, curCount = (int) passQps, DefaultController.java:77
    const int32_t cur = j_d2i((double)sum / 1.0);
    return !((double)(int32_t)((uint32_t)cur + (uint32_t)a) > count);
}

// One event of the per-resource replay in arrival order (lane_run's event-by-event runs, k_llru): the slot
// chain, or -- F_SPECIAL -- the event's original kind and arguments, as k_lseq takes them (ENTRY_NODE is
// k_entry_stats').
template <bool kLru>
__device__ __forceinline__ void replay_event(const Ctx &c, const FlowScratch &sc, uint32_t res, const Payload &q,
                                             int64_t ts_base, const int64_t *__restrict__ rt_in,
                                             const uint64_t *__restrict__ param_in, int8_t *decision,
                                             int32_t *wait_ms) {
    const int64_t t = ts_base + (int64_t)q.ts_off;
    const uint32_t idx = q.idx & F_IDX;
    const int a = (int)(q.acq_prio & 0x7FFFFFFFu);
    if (q.idx & F_SPECIAL) {
        const uint8_t kd = sc.in_kind[idx];
        const uint8_t fl = sc.in_flags ? sc.in_flags[idx] : 0;
        const uint64_t pv = sc.in_param ? sc.in_param[idx] : 0;
        const bool hp = (fl & SGA_EV_HAS_PARAM) != 0;
        PArgs pa{nullptr, 0};
        if ((fl & SGA_EV_ARGS) && sc.pvals) {
            pa.args = sc.pvals + (pv >> 32);
            pa.pvals = sc.pvals;
            pa.nargs = (uint32_t)pv;
        } else if (hp && (fl & SGA_EV_PARAM_LIST) && sc.pvals) {
            pa = PArgs{sc.pvals + (pv >> 32), (uint32_t)pv};
        }
        if (kd == SGA_KIND_BLOCKED) {
            blocked_event(c, res, t, a);
        } else if (kd == SGA_KIND_REVOKE) {
            revoke_event<kLru>(c, res, t, a, pa, hp, pv, idx);
        } else if (kd == 1) {
            chain_exit<kLru>(c, res, t, rt_in[idx], a, (fl & SGA_EV_ERROR) != 0, hp, pv, pa, idx);
        } else {
            int64_t w = 0;
            decision[idx] = chain_entry<kLru>(c, res, t, a, (fl & SGA_EV_PRIORITIZED) != 0, hp, pv, &w, pa, idx);
            wait_ms[idx] = (int32_t)w;
        }
        return;
    }
    const bool hp = (q.idx & F_PARAM) != 0;
    const uint64_t pv = hp ? param_in[idx] : 0;
    if (q.idx & F_EXIT) {
        chain_exit<kLru>(c, res, t, rt_in[idx], a, (q.idx & F_ERROR) != 0, hp, pv, PArgs{nullptr, 0}, idx);
    } else {
        int64_t w = 0;
        decision[idx] = chain_entry<kLru>(c, res, t, a, (q.acq_prio >> 31) != 0, hp, pv, &w, PArgs{nullptr, 0}, idx);
        wait_ms[idx] = (int32_t)w;
    }
}

// Small batches (the coalescing event queue's rounds, a single SphU.entry): one workgroup.  The first event of
// each resource in the batch leads: its lane replays the resource's events in arrival order with the whole slot
// chain (replay_event, as lane_run does for a resource with F_SPECIAL events), the resources side by side; then
// one lane adds the inbound events to ENTRY_NODE in arrival order (no SystemRule check on this path).
#ifndef SGA_LSMALL_THREADS
#define SGA_LSMALL_THREADS 512
#endif
// threads of k_lsmall: fewer than the chunk's events, so each lane holds the slot chain in registers (at 1024
// threads a lane gets 128 VGPRs and the chain spills to scratch, a memory round trip per spilled value)
constexpr int kLSmall = SGA_LSMALL_THREADS;
__global__ __launch_bounds__(kLSmall) void k_lsmall(FlowState st, int64_t max_rt, FlowScratch fs,
                                                    const uint32_t *__restrict__ resource,
                                                    const uint32_t *__restrict__ ts_off, int64_t ts_base,
                                                    const int32_t *__restrict__ acquire,
                                                    const int64_t *__restrict__ rt_in, uint32_t n, int8_t *decision,
                                                    int32_t *wait_ms, uint32_t *ovf_out, int zero_ovf) {
    __shared__ uint32_t sres[FlowEngine::kSmallEvents];
    const uint32_t i = threadIdx.x;
    const Ctx c{st, max_rt};
    if (zero_ovf && i == 0) *st.overflow = 0;  // no lru_prepare ahead of this kernel: the batch's overflow word
    for (uint32_t k = i; k < n; k += kLSmall) {
        sres[k] = resource[k];
        decision[k] = D_PASS;
        wait_ms[k] = 0;
    }
    __syncthreads();
    for (uint32_t k = i; k < n; k += kLSmall) {  // each resource's first event leads: its lane replays them in order
        const uint32_t r = sres[k];
        bool lead = r < st.nres;
        for (uint32_t j = 0; j < k && lead; ++j) lead = sres[j] != r;
        if (lead)
            for (uint32_t j = k; j < n; ++j) {
                if (sres[j] != r) continue;
                const Payload q{j | F_SPECIAL, ts_off[j], (uint32_t)acquire[j] & 0x7FFFFFFFu, 0u};
                replay_event<true>(c, fs, r, q, ts_base, rt_in, fs.in_param, decision, wait_ms);
            }
    }
    __syncthreads();
    if (i == 0) {
        for (uint32_t j = 0; j < n; ++j) {
            const uint8_t fl = fs.in_flags ? fs.in_flags[j] : 0;
            if (sres[j] >= st.nres || !(fl & SGA_EV_INBOUND)) continue;
            const int64_t t = ts_base + (int64_t)ts_off[j];
            const int a = (int)((uint32_t)acquire[j] & 0x7FFFFFFFu);
            const uint8_t kd = fs.in_kind[j];
            if (kd == 1) {
                entry_node_after_exit(c, t, rt_in[j], a, (fl & SGA_EV_ERROR) != 0);
            } else if (kd == SGA_KIND_BLOCKED) {
                node_add(c, entry_node(c), t, MB_BLOCK, a);
            } else if (kd == SGA_KIND_REVOKE) {
                int64_t *e = entry_node(c);
                e[kNodeThreads] -= 1;
                node_add(c, e, t, MB_PASS, -(int64_t)a);
                node_add(c, e, t, MB_BLOCK, a);
            } else {
                entry_node_after_entry(c, t, a, decision[j]);
            }
        }
        *ovf_out = *st.overflow;
    }
}

// One run of a resource decided by one lane (k_lflows; k_lwave's lane 0 for runs it cannot split):
// RateLimiter pacing in registers, the per-event slot chain, or the closed form (RUN_FAST: k_lresults
// writes the decisions from run_f).
__device__ __noinline__ void lane_run(const Ctx &c, int64_t max_rt, FlowScratch &sc, const Payload *__restrict__ pay,
                         int64_t ts_base, const int64_t *__restrict__ rt_in, const uint64_t *__restrict__ param_in,
                         int8_t *decision, int32_t *wait_ms, uint32_t r, bool special = false) {
    const FlowState &st = c.st;
    const uint32_t res = sc.run_slot[r];
    const ResDev R = st.res[res];
    int64_t *node = st.node + (size_t)res * kNodeWords;
    const uint32_t j0 = sc.run_start[r], j1 = sc.run_end[r];
    const uint32_t nent = sc.run_nent[r];
    const int32_t a = sc.run_amin[r];
    const int64_t t0 = ts_base + (int64_t)sc.run_t0off[r];
    if (special) {  // a resource with F_SPECIAL events this chunk: every run event by event
        for (uint32_t j = j0; j < j1; ++j) replay_event<false>(c, sc, res, pay[j], ts_base, rt_in, param_in, decision, wait_ms);
        sc.run_mode[r] = RUN_DONE;
        return;
    }
    if (nent == 0 && (R.fast & 5u)) {
        // An exit-only run of a single-rule resource (no parameter rules, no breakers: an exit only
        // adds to the node).  Its exits share one second bucket and one minute bucket, so each
        // window either takes all of the run's adds (the bucket is current, or older and rotated at
        // the first exit) or none (the window already holds a newer bucket: LeapArray.currentWindow
        // returns a detached bucket, LeapArray.java:216-220) -- also when exits are submitted after
        // later entries.  curThreadNum drops in every case (StatisticNode.decreaseThreadNum).
        const int64_t *sb0 = node + kNodeSec + kMB * (int)((t0 / kSecW) % 2);
        const int64_t *mb0 = node + kNodeMin + kMB * (int)((t0 / kMinW) % 60);
        const bool sdet = sb0[0] != kAbsent && t0 - t0 % kSecW < sb0[0];
        const bool mdet = mb0[0] != kAbsent && t0 - t0 % kMinW < mb0[0];
        const int64_t exc = (int64_t)sc.run_exc[r], exerr = (int64_t)sc.run_exerr[r];
        const int64_t exrt = sc.run_exrt[r], exmin = sc.run_exmin[r];
        for (int k = 0; k < 2; ++k) {
            if (k == 0 ? sdet : mdet) continue;
            int64_t *b = k == 0 ? sec_current(node, t0, max_rt) : min_current(node, t0, max_rt);
            b[MB_SUCC] += exc;
            b[MB_RT] += exrt;
            b[MB_EXC] += exerr;
            if (exmin < b[MB_MINRT]) b[MB_MINRT] = exmin;
        }
        node[kNodeThreads] -= (int64_t)sc.run_nexit[r];
        sc.run_mode[r] = RUN_DONE;
        return;
    }
    bool fast = (R.fast & 1u) && sc.run_cp[r] == 0 && (nent == 0 || a == sc.run_amax[r]) && a >= 0;
    bool pace = (R.fast & 4u) != 0;
    if (fast || pace) {  // no clock regression in this resource's windows
        const int64_t *sb = node + kNodeSec + kMB * (int)((t0 / kSecW) % 2);
        const int64_t *mb = node + kNodeMin + kMB * (int)((t0 / kMinW) % 60);
        if ((sb[0] != kAbsent && t0 - t0 % kSecW < sb[0]) || (mb[0] != kAbsent && t0 - t0 % kMinW < mb[0]))
            fast = pace = false;
    }
    if (pace) {
        // RateLimiterController alone (RateLimiterController.java:46-91): the decisions depend on
        // latestPassedTime only, so the run's entries are paced in registers, in order; the run's
        // statistics (one 500 ms bucket) are added once, like the closed form below.
        FlowRuleDev &rule = st.rules[R.rule_off];
        int64_t latest = rule.latest_passed;
        // the rule fields in registers: the decision stores could alias them otherwise, and
        // every reload would wait behind the previous stores
        const double rcount = rule.count;
        const int64_t rqueue = rule.max_queue;
        int64_t pa = 0, ba = 0, npass = 0;
        int last_aq = -1;  // Math.round(1.0 * acquire / count * 1000) of the last acquire count
        int64_t last_cost = 0;
        // decide one event in registers; returns its (index, decision, wait) for the store
        auto pace_one = [&](const Payload &q, uint32_t &idx, int8_t &d, int32_t &wo) {
            idx = q.idx & F_IDX;
            d = D_PASS;
            wo = 0;
            if (q.idx & F_EXIT) return false;
            const int64_t t = ts_base + (int64_t)q.ts_off;
            const int aq = (int)(q.acq_prio & 0x7FFFFFFFu);
            int64_t w = 0;
            if (aq > 0) {
                if (rcount <= 0) {
                    d = D_BLOCK_FLOW;
                } else {
                    if (aq != last_aq) {
                        last_aq = aq;
                        last_cost = j_round(1.0 * aq / rcount * 1000);
                    }
                    const int64_t cost = last_cost;
                    if (cost + latest <= t) {
                        latest = t;
                    } else if (cost + latest - t > rqueue) {
                        d = D_BLOCK_FLOW;
                    } else {
                        latest += cost;
                        w = latest - t;
                        if (w > rqueue) {
                            latest -= cost;
                            d = D_BLOCK_FLOW;
                            w = 0;
                        } else if (w < 0) {
                            w = 0;
                        }
                    }
                }
            }
            wo = (int32_t)w;
            if (d == D_PASS) {
                pa += aq;
                ++npass;
            } else {
                ba += aq;
            }
            return true;
        };
        // software pipeline: the next 4 payloads are loaded before this group's stores are
        // issued, so a load never waits behind the previous group's scattered stores
        constexpr uint32_t kG = 4;
        const Payload none{F_EXIT, 0, 0, 0};
        // loads at clamped indices, the out-of-run ones replaced after the load (a load under a
        // branch is waited for before the branch closes)
        auto ld = [&](uint32_t j) {
            Payload q = pay[min(j, j1 - 1)];
            if (j >= j1) q = none;
            return q;
        };
        Payload c0 = ld(j0), c1 = ld(j0 + 1), c2 = ld(j0 + 2), c3 = ld(j0 + 3);
        for (uint32_t g = j0; g < j1; g += kG) {
            const uint32_t nx = g + kG;
            const Payload n0 = ld(nx), n1 = ld(nx + 1), n2 = ld(nx + 2), n3 = ld(nx + 3);
            uint32_t i0, i1, i2, i3;
            int8_t d0, d1, d2, d3;
            int32_t w0, w1, w2, w3;
            const bool v0 = pace_one(c0, i0, d0, w0), v1 = pace_one(c1, i1, d1, w1);
            const bool v2 = pace_one(c2, i2, d2, w2), v3 = pace_one(c3, i3, d3, w3);
            if (v0) { decision[i0] = d0; wait_ms[i0] = w0; }
            if (v1) { decision[i1] = d1; wait_ms[i1] = w1; }
            if (v2) { decision[i2] = d2; wait_ms[i2] = w2; }
            if (v3) { decision[i3] = d3; wait_ms[i3] = w3; }
            c0 = n0;
            c1 = n1;
            c2 = n2;
            c3 = n3;
        }
        rule.latest_passed = latest;
        int64_t *sb = sec_current(node, t0, max_rt);
        int64_t *mb = min_current(node, t0, max_rt);
        const int64_t exc = (int64_t)sc.run_exc[r], exerr = (int64_t)sc.run_exerr[r];
        const int64_t exrt = sc.run_exrt[r], exmin = sc.run_exmin[r];
        int64_t *w2[2] = {sb, mb};
        for (int k = 0; k < 2; ++k) {
            int64_t *b = w2[k];
            b[MB_PASS] += pa;
            b[MB_BLOCK] += ba;
            b[MB_SUCC] += exc;
            b[MB_RT] += exrt;
            b[MB_EXC] += exerr;
            if (exmin < b[MB_MINRT]) b[MB_MINRT] = exmin;
        }
        node[kNodeThreads] += npass - (int64_t)sc.run_nexit[r];
        sc.run_mode[r] = RUN_DONE;
        return;
    }
    if (fast && nent) {  // WarmUp sync must only see entries in one second (true: run is inside one 500 ms bucket)
        const int64_t s0 = sec_sum(node, t0, MB_PASS);
        if (s0 + (int64_t)nent * a + a >= (int64_t)INT32_MAX) fast = false;
    }
    if (!fast) {
        for (uint32_t j = j0; j < j1; ++j) replay_event<false>(c, sc, res, pay[j], ts_base, rt_in, param_in, decision, wait_ms);
        sc.run_mode[r] = RUN_DONE;
        return;
    }
    // ---- closed form: rotate both windows once at the run's first event
    int64_t *sb = sec_current(node, t0, max_rt);
    int64_t *mb = min_current(node, t0, max_rt);
    uint32_t f = 0;
    if (nent) {
        FlowRuleDev &rule = st.rules[R.rule_off];
        const int64_t s0 = sec_sum(node, t0, MB_PASS);
        if (rule.behavior == 1) {
            // WarmUpController: sync once (the run is inside one second), then a fixed threshold
            const int64_t previous_qps = j_d2l(node_prev_pass_qps(c, node, t0));
            warmup_sync(rule, t0, previous_qps);
            const int64_t rest = rule.stored_tokens;
            double lim;
            if (rest >= rule.warning_token) {
                const int64_t above = rest - rule.warning_token;
                lim = j_next_up(1.0 / ((double)above * rule.slope + 1.0 / rule.count));
            } else {
                lim = rule.count;
            }
            uint32_t lo = 0, hi = nent;
            while (lo < hi) {
                const uint32_t mid = lo + ((hi - lo) >> 1);
                const int64_t pq = j_d2l((double)(s0 + (int64_t)mid * a) / 1.0);
                if ((double)(pq + a) <= lim) lo = mid + 1;
                else hi = mid;
            }
            f = lo;
        } else {
            uint32_t lo = 0, hi = nent;
            while (lo < hi) {
                const uint32_t mid = lo + ((hi - lo) >> 1);
                if (default_cond(rule.count, s0 + (int64_t)mid * a, a)) lo = mid + 1;
                else hi = mid;
            }
            f = lo;
        }
    }
    const int64_t pa = (int64_t)f * a, ba = (int64_t)(nent - f) * a;
    const int64_t exc = (int64_t)sc.run_exc[r], exerr = (int64_t)sc.run_exerr[r];
    const int64_t exrt = sc.run_exrt[r], exmin = sc.run_exmin[r];
    sb[MB_PASS] += pa;
    sb[MB_BLOCK] += ba;
    sb[MB_SUCC] += exc;
    sb[MB_RT] += exrt;
    sb[MB_EXC] += exerr;
    if (exmin < sb[MB_MINRT]) sb[MB_MINRT] = exmin;
    mb[MB_PASS] += pa;
    mb[MB_BLOCK] += ba;
    mb[MB_SUCC] += exc;
    mb[MB_RT] += exrt;
    mb[MB_EXC] += exerr;
    if (exmin < mb[MB_MINRT]) mb[MB_MINRT] = exmin;
    node[kNodeThreads] += (int64_t)f - (int64_t)sc.run_nexit[r];
    sc.run_f[r] = f;
    sc.run_mode[r] = RUN_FAST;
}

// A parameter-only resource (one QPS-grade ParamFlowRule of index 0, no FlowRule, no breaker, its maps in
// free mode) is decided per (rule, value) segment (k_pseg_*): a value's token bucket / throttle time and its
// thread count see only that value's events, and its node statistics never feed a decision.  Taken here,
// in k_lflows, on the flow's lane: ParamFlowSlot.applyRealParamIdx fixes an unresolved index at the first
// entry (as chain_entry would), and the first entry creates the thread-count map of index 0
// (ParameterMetricStorage.initParamMetricsFor) -- a flow whose parameter exits come before that entry
// while the map does not exist yet stays with the event-by-event replay.
__device__ bool pseg_take(const FlowState &st, const FlowScratch &sc, const Payload *__restrict__ pay, uint32_t res,
                          uint32_t r0, uint32_t r1) {
    const ResDev R = st.res[res];
    if (R.n_rules || R.n_cbs || R.n_prules != 1 || !st.tmapmask) return false;
    ParamRuleDev &p = st.prules[R.prule_off];
    if (p.grade != 1 || p.cluster) return false;
    const uint32_t jb = sc.run_start[r0], je = sc.run_end[r1 - 1];
    bool ent = false;
    for (uint32_t r = r0; r < r1 && !ent; ++r) ent = sc.run_nent[r] != 0;
    if (!ent) {  // exits only: nothing to resolve, the map exists or is never touched
        return p.idx_res == 0;
    }
    uint32_t j = jb;
    bool pexit = false;  // a parameter exit (or revoke) before the first entry
    for (; j < je; ++j) {
        const uint32_t f = pay[j].idx;
        if (!(f & F_EXIT)) {
            if (f & F_SPECIAL) continue;  // a block outside the engine checks nothing (not the first entry)
            break;
        }
        pexit |= (f & F_PARAM) != 0;
    }
    int32_t idx = p.idx_res;
    if (idx == kIdxUnresolved) {
        if (j == je) return false;
        idx = param_idx_of(p, (pay[j].idx & F_PARAM) ? 1u : 0u);
    }
    if (idx != 0) return false;
    const uint64_t mask = st.tmapmask[res];
    if (!(mask & 1ull) && j < je) {
        if (pexit) return false;
        st.tmapmask[res] = mask | 1ull;
    }
    return true;
}

// A breaker-only resource (one DegradeRule, no FlowRule, no ParamFlowRule) whose batch holds only entries or
// only exits: its entries move the breaker only OPEN -> HALF_OPEN (the first entry at or after the retry
// time, AbstractCircuitBreaker.tryPass), its exits only feed the breaker (onRequestComplete); k_cb_flows
// decides it, the node statistics go in aggregate as for the parameter-only resources.  Returns 0 (not
// taken), 1 (taken, no breaker work: a CLOSED breaker passes every entry) or 2 (taken, k_cb_flows).
__device__ int cb_take(const FlowState &st, const FlowScratch &sc, uint32_t res, uint32_t r0, uint32_t r1) {
    const ResDev R = st.res[res];
    if (R.n_rules || R.n_prules || R.n_cbs != 1) return 0;
    bool ent = false, ex = false;
    for (uint32_t r = r0; r < r1; ++r) {
        ent |= sc.run_nent[r] != 0;
        ex |= sc.run_nexit[r] != 0;
    }
    if (ent && ex) return 0;
    return (ent && st.cbs[R.cb_off].state == 0) ? 1 : 2;
}

// k_llru_ps (below): LRU-mode parameter-only resources, chunked through LDS
constexpr uint32_t kLruPs = 0x80000000u;
constexpr int kPsPre = 128;
__device__ __forceinline__ int64_t ps_ld(const int64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ps_ldu(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// k_llru_ps's resources (called on the flow's lane in k_lflows): as pseg_take, the flow's first entry resolves
// the rule's index (ParamFlowSlot.applyRealParamIdx) and creates the index-0 thread-count map when it does not
// exist yet (the first batch of a fresh engine); a parameter exit before that entry stays with k_llru
__device__ bool lru_ps_take(const FlowState &st, const FlowScratch &sc, const Payload *__restrict__ pay, uint32_t res,
                            uint32_t r0, uint32_t r1) {
    const ResDev R = st.res[res];
    if (R.n_rules || R.n_cbs || R.n_prules != 1 || !st.tmapmask || (st.tmapmask[res] & ~1ull)) return false;
    ParamRuleDev &p = st.prules[R.prule_off];
    if (!(p.grade == 1 && !p.cluster && st.pstamp && st.tstamp && st.tbase && st.tbase[res] != kNoTBase))
        return false;
    const bool has_map = (st.tmapmask[res] & 1ull) != 0;
    if (p.idx_res == 0 && has_map) return true;
    if (p.idx_res != 0 && p.idx_res != kIdxUnresolved) return false;
    const uint32_t je = sc.run_end[r1 - 1];
    uint32_t j = sc.run_start[r0];
    for (; j < je; ++j) {
        const uint32_t f = pay[j].idx;
        if (!(f & F_EXIT)) break;
        if ((f & F_PARAM) && !has_map) return false;  // a parameter exit before the map exists
    }
    if (j == je) return p.idx_res == 0 && has_map;  // exits only
    if (param_idx_of(p, (pay[j].idx & F_PARAM) ? 1u : 0u) != 0) return false;
    st.tmapmask[res] = 1ull;  // the first entry creates the map
    return true;
}

// a list append from divergent lanes: one counter atomic per wave and list (its lowest active lane)
__device__ __forceinline__ uint32_t wave_append(uint32_t *ctr) {
    const uint64_t act = __ballot(1);
    const int lane = (int)(threadIdx.x & 63), lead = __ffsll((unsigned long long)act) - 1;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(ctr, (uint32_t)__popcll(act));
    base = (uint32_t)__shfl((int)base, lead, 64);
    return base + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
}

__global__ __launch_bounds__(kT) void k_lflows(FlowState st, int64_t max_rt, FlowScratch sc,
                                               const Payload *__restrict__ pay, const uint32_t *__restrict__ keys,
                                               int64_t ts_base, const int64_t *__restrict__ rt_in,
                                               const uint64_t *__restrict__ param_in, int8_t *decision,
                                               int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const Ctx c{st, max_rt};
    const uint32_t nflows = sc.counters[2], nruns = sc.counters[1];
    for (uint32_t fl = blockIdx.x * kT + threadIdx.x; fl < nflows; fl += gridDim.x * kT) {
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        {  // a long event-by-event replay goes to k_lheavy (its state in LDS)
            const uint32_t res = sc.run_slot[r0];
            const uint32_t nev = sc.run_end[r1 - 1] - sc.run_start[r0];
            // events replayed with their original kind / arguments (F_SPECIAL) this chunk: this resource's events
            // in arrival order on this lane (k_llru in LRU mode); the other resources keep every parallel form
            const uint32_t rs = sc.res_special ? sc.res_special[res] : 0u;
            const uint32_t special = (rs >> 2) == sc.epoch ? (rs & 3u) : 0u;  // level (k_lclassify)
            if (st.lru_res && st.lru_res[res]) {  // a CacheMap in LRU mode: arrival order, one lane (k_llru)
                // parameter-only: the chunked replay (k_llru_ps, SGA_LRU_PS=0 turns it off: an A/B knob)
                const bool ps = !special && st.lru_ps && lru_ps_take(st, sc, pay, res, r0, r1);
                sc.lru[wave_append(&sc.counters[10])] = fl | (ps ? 0x80000000u : 0u);
                continue;
            }
            if (special) {
                // kind 2 / 3 events of a parameter-only resource: its per-value segments (the revokes are exits
                // there, the node statistics in aggregate); anything else event by event on this lane
                if (special == 1 && sc.pseg && pseg_take(st, sc, pay, res, r0, r1)) {
                    for (uint32_t r = r0; r < r1; ++r) {
                        sc.run_mode[r] = RUN_PSEG;
                        sc.run_pa[r] = 0;
                        sc.run_ba[r] = 0;
                        sc.run_np[r] = 0;
                    }
                    sc.pseg[wave_append(&sc.counters[11])] = fl;
                    continue;
                }
                for (uint32_t r = r0; r < r1; ++r)
                    lane_run(c, max_rt, sc, pay, ts_base, rt_in, param_in, decision, wait_ms, r, true);
                continue;
            }
            int cbk = 0;
            if (sc.pseg && ((cbk = cb_take(st, sc, res, r0, r1)) != 0 ||
                            pseg_take(st, sc, pay, res, r0, r1))) {
                if (cbk == 2) sc.cbf[wave_append(&sc.counters[13])] = fl;
                for (uint32_t r = r0; r < r1; ++r) {
                    sc.run_mode[r] = RUN_PSEG;
                    sc.run_pa[r] = 0;
                    sc.run_ba[r] = 0;
                    sc.run_np[r] = 0;
                }
                sc.pseg[wave_append(&sc.counters[11])] = fl;
                continue;
            }
            if ((st.res[res].fast & 5u) == 0 && nev >= kHeavyEvents) {
                sc.heavy[wave_append(&sc.counters[8])] = fl;
                continue;
            }
            if ((st.res[res].fast & 5u) && nev >= kWaveEvents) {  // a long single-rule fast path: k_lwave
                if (st.res[res].fast & 4u)
                    for (uint32_t r = r0; r < r1; ++r) sc.run_mode[r] = RUN_WRL;  // k_lwsum's windows
                sc.pace[wave_append(&sc.counters[9])] = fl;
                continue;
            }
        }
        for (uint32_t r = r0; r < r1; ++r)
            lane_run(c, max_rt, sc, pay, ts_base, rt_in, param_in, decision, wait_ms, r);
    }
}

// Heavy resources (many events, no closed form): one workgroup each; its node record, rules and
// breakers are copied to LDS, lane 0 replays every event in order against the LDS copy (an LDS
// round trip instead of a global one per state access), and the state is written back.
constexpr int kHeavyRules = 16, kHeavyCbs = 16, kHeavyChunk = 512, kHeavySlots = 1024;
// Resources with a long batch and a single-rule fast path (k_lflows sends them here), one wave each.
// Both fast controllers decide an entry by a monotone test against state that only passing entries
// move, so a window of 64 entries is decided by finding its first passing lane (a ballot), blocking
// every open lane before it, applying that pass and repeating from the next lane:
//   RateLimiterController alone (RateLimiterController.java:46-91): an entry passes iff
//     cost + latest <= t or cost + latest - t <= maxQueueingTimeMs; a pass moves latestPassedTime;
//   DefaultController / WarmUpController with mixed acquire counts (DefaultController.java:47-77,
//     WarmUpController.java:115-138): an entry passes iff curCount(S) + acquire fits the run's fixed
//     threshold, S the passed count so far; before the first block a window is one prefix sum.
// A window costs one iteration per pass after its first block, instead of one dependent step per entry.
// Runs with a uniform acquire keep the closed form, and runs that go back in time or hold prioritized
// entries take lane_run on lane 0, exactly as in k_lflows.
// A RateLimiter run's windows (RUN_WRL): the summary of every 64-event window (j / 64) that lies inside one
// such run, one wave each over the whole GPU, so that k_lwave<1> walks a saturated run by the summaries
// alone.  Blocked entries and zero-cost passes behind the queue leave latestPassedTime alone
// (RateLimiterController.java:56-89), so such a window's decisions follow from the state it starts at.
__global__ __launch_bounds__(256) void k_lwsum(FlowState st, FlowScratch sc, const Payload *__restrict__ pay) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0) || sc.counters[9] == 0) return;
    const uint32_t nvalid = sc.counters[0];
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t jb = w * 64;
    if (jb + 64 > nvalid) return;  // wave-uniform
    const uint32_t r = sc.ev_run[jb];
    if (sc.ev_run[jb + 63] != r || sc.run_mode[r] != RUN_WRL) return;  // wave-uniform
    const double rcount = st.rules[st.res[sc.run_slot[r]].rule_off].count;
    const Payload q = pay[jb + lane];
    const bool ent = !(q.idx & F_EXIT);
    const int aq = ent ? (int)(q.acq_prio & 0x7FFFFFFFu) : 0;
    const int64_t cost = (ent && aq > 0 && rcount > 0) ? j_round(1.0 * aq / rcount * 1000) : 0;
    const bool zero = ent && cost == 0;
    // a cost past 2^40 ms takes the exact walk (Java's long sums)
    const int64_t key = cost == 0 ? INT64_MIN : cost > ((int64_t)1 << 40) ? INT64_MAX : (int64_t)q.ts_off - cost;
    const bool zt = zero && aq > 0;
    const int64_t kmax = wave_max_i64(key);
    const int64_t a0 = wave_sum_i64(zero ? (int64_t)aq : 0);
    const uint32_t t0min = wave_min_u32(zt ? q.ts_off : 0xFFFFFFFFu), t0max = wave_max_u32(zt ? q.ts_off : 0u);
    const uint32_t n0 = (uint32_t)__builtin_popcountll(__ballot(zero));
    const uint32_t has0 = (uint32_t)(__ballot(zt) != 0);
    if (lane == 0) sc.wsum[w] = WinSum{kmax, a0, t0min, t0max, n0, has0};
}

#ifndef SGA_WAVE_PF
#define SGA_WAVE_PF 8
#endif
#ifndef SGA_WIN_MIN
#define SGA_WIN_MIN 512
#endif
#ifndef SGA_WIN_STEPS
#define SGA_WIN_STEPS 4
#endif
constexpr uint32_t kWinMin = SGA_WIN_MIN;
constexpr int kWinSteps = SGA_WIN_STEPS;  // k_lwave<1> window(): movers of latestPassedTime stepped one by one, beyond that a scan  // k_lwave<1>: RateLimiter runs of this many events walk window summaries
constexpr int kWavePf = SGA_WAVE_PF;  // k_lwave: windows loaded ahead (even: RateLimiter runs take them in pairs)
// kRl: 1 = the RateLimiter resources only, 0 = the others (two launches, each compiled without the other's
// window code: one kernel holding both spilled registers and waited on its own stores)
template <int kRl>
__global__ __launch_bounds__(64) void k_lwave(FlowState st, int64_t max_rt, FlowScratch sc,
                                              const Payload *__restrict__ pay, int64_t ts_base,
                                              const int64_t *__restrict__ rt_in, const uint64_t *__restrict__ param_in,
                                              int8_t *decision, int32_t *wait_ms, uint64_t *prof) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const Ctx c{st, max_rt};
    const int lane = threadIdx.x;
    const uint32_t nwave = sc.counters[9], nflows = sc.counters[2], nruns = sc.counters[1];
    uint64_t pr_iter = 0, pr_lr = 0, pr_lrt = 0;  // profiling (SGA_LWAVE_PROF=1)
    constexpr bool pace_pairs = true;  // RateLimiter windows two at a time (pace2)
    for (uint32_t h = blockIdx.x; h < nwave; h += gridDim.x) {
        const uint32_t fl = sc.pace[h];
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        if (((st.res[sc.run_slot[r0]].fast & 4u) != 0) != (kRl != 0)) continue;  // the other launch's
        const uint64_t pt0 = prof ? wall_clock64() : 0;
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t res = sc.run_slot[r];
            const ResDev R = st.res[res];
            int64_t *node = st.node + (size_t)res * kNodeWords;
            const uint32_t j0 = sc.run_start[r], j1 = sc.run_end[r];
            const uint32_t nent = sc.run_nent[r];
            const int32_t amin = sc.run_amin[r], amax = sc.run_amax[r];
            const int64_t t0 = ts_base + (int64_t)sc.run_t0off[r];
            bool regress;
            {
                const int64_t *sb = node + kNodeSec + kMB * (int)((t0 / kSecW) % 2);
                const int64_t *mb = node + kNodeMin + kMB * (int)((t0 / kMinW) % 60);
                regress = (sb[0] != kAbsent && t0 - t0 % kSecW < sb[0]) || (mb[0] != kAbsent && t0 - t0 % kMinW < mb[0]);
            }
            const bool pace = kRl && (R.fast & 4u) && !regress;
            bool greedy = !kRl && (R.fast & 1u) && !regress && sc.run_cp[r] == 0 && amin >= 0 && nent > 0 && amin != amax;
            FlowRuleDev &rule = st.rules[R.rule_off];
            int64_t s0 = 0;
            double lim = 0;
            if (greedy) {  // the closed form's prologue: rotate once, the run's fixed threshold
                if (lane == 0) {
                    sec_current(node, t0, max_rt);
                    min_current(node, t0, max_rt);
                    s0 = sec_sum(node, t0, MB_PASS);
                    if (rule.behavior == 1 && s0 + (int64_t)nent * amax + amax >= (int64_t)INT32_MAX) {
                        lim = -1;  // the int passQps could overflow: per-event chain
                    } else if (rule.behavior == 1) {
                        warmup_sync(rule, t0, j_d2l(node_prev_pass_qps(c, node, t0)));
                        const int64_t rest = rule.stored_tokens;
                        lim = rest >= rule.warning_token
                                  ? j_next_up(1.0 / ((double)(rest - rule.warning_token) * rule.slope + 1.0 / rule.count))
                                  : rule.count;
                    } else {
                        lim = rule.count;
                    }
                }
                s0 = __shfl(s0, 0);
                lim = __shfl(lim, 0);
                if (rule.behavior == 1 && lim == -1) greedy = false;
            }
            if (!pace && !greedy) {  // closed form, prioritized entries or a clock regression: one lane
                const uint64_t lt0 = prof ? wall_clock64() : 0;
                if (lane == 0) lane_run(c, max_rt, sc, pay, ts_base, rt_in, param_in, decision, wait_ms, r);
                __syncthreads();
                if (prof) {
                    pr_lrt += wall_clock64() - lt0;
                    ++pr_lr;
                }
                continue;
            }
            const bool warm = rule.behavior == 1;
            const double rcount = rule.count;
            const int64_t rqueue = rule.max_queue;
            int64_t latest = pace ? rule.latest_passed : 0;
            int64_t S = s0;
            // entry passes against the current state
            auto passes = [&](int64_t tt, int64_t cost, int aq) -> bool {
                if (pace) return aq <= 0 || (rcount > 0 && (cost + latest <= tt || cost + latest - tt <= rqueue));
                return warm ? (double)(j_d2l((double)S / 1.0) + aq) <= lim : default_cond(rcount, S, aq);
            };
            int64_t pa = 0, ba = 0, npass = 0;  // this lane's share
            // windows of 64 entries, kWavePf of them loaded ahead in a register ring (unconditional
            // loads at a clamped index, so no load waits at a branch): the state chain between
            // windows is a few ballots, the payload load latency is paid once per ring
            Payload ring[kWavePf];
#pragma unroll
            for (int k = 0; k < kWavePf; ++k) ring[k] = pay[min(j0 + (uint32_t)(k * 64 + lane), j1 - 1)];
            bool pred_c = true;  // pacing: the last decision of an entry with a nonzero cost
            auto window = [&](uint32_t g, Payload q) {
                const uint32_t j = g + (uint32_t)lane;
                if (j >= j1 || j < j0) q.idx = F_EXIT;
                const bool ent = !(q.idx & F_EXIT);
                const int64_t t = ts_base + (int64_t)q.ts_off;
                const int aq = ent ? (int)(q.acq_prio & 0x7FFFFFFFu) : 0;
                const int64_t cost = (pace && ent && aq > 0 && rcount > 0) ? j_round(1.0 * aq / rcount * 1000) : 0;
                int8_t d = D_PASS;
                int64_t w = 0;
                uint64_t rem = __ballot(ent);
                if (pace) {
                    // RateLimiterController (RateLimiterController.java:46-91) by speculation: every open
                    // entry gets a predicted decision (acquireCount <= 0: pass; count <= 0: block;
                    // cost 0: pass; otherwise the last decision of a costly entry), latestPassedTime
                    // follows the predicted passes as a max-plus scan (a pass sets it to
                    // max(latest + cost, now)), and every prediction is checked against the state
                    // before it.  Lanes up to the first wrong prediction are decided; that lane takes
                    // its true decision, and the rest of the window goes round again.
                    // When few open entries would move latestPassedTime at the current state (a saturated
                    // queue: costly entries block, zero-cost ones pass behind it), the step is exact
                    // without a scan: every entry before the first mover is decided at the current
                    // state, the mover passes and moves it.
                    while (rem) {
                        if (prof) ++pr_iter;
                        const bool open = (rem >> lane) & 1ull;
                        {
                            const bool act = aq <= 0 || (rcount > 0 && (cost + latest <= t || cost + latest - t <= rqueue));
                            const uint64_t mvm = __ballot(open && act && aq > 0 && (cost > 0 || t > latest));
                            if (__builtin_popcountll(mvm) <= kWinSteps) {
                                const int f = mvm ? __builtin_ctzll(mvm) : 64;
                                if (open && lane < f) {
                                    d = act ? D_PASS : D_BLOCK_FLOW;
                                    if (act && aq > 0) w = latest - t;  // a zero-cost pass behind the queue
                                }
                                const uint64_t before = f == 64 ? rem : rem & ((1ull << f) - 1);
                                if (__ballot(cost > 0) & before) pred_c = false;  // costly entries before f blocked
                                if (f == 64) break;
                                const int64_t tf = readlane_i64(t, f), cf = readlane_i64(cost, f);
                                const int64_t lf = max(latest + cf, tf);
                                if (lane == f) w = lf - tf;  // d: D_PASS
                                latest = lf;
                                if (cf > 0) pred_c = true;
                                rem &= (f == 63) ? 0ull : (~0ull << (f + 1));
                                continue;
                            }
                        }
                        const bool mv = open && aq > 0 && rcount > 0;
                        const bool spec = aq <= 0 || (rcount > 0 && (cost == 0 || pred_c));
                        int64_t A = (mv && spec) ? cost : 0, B = (mv && spec) ? t : kMaxPlusNegInf;
                        wave_incl_maxplus(A, B);
                        const int64_t Lk = max(latest + A, B);
                        const int64_t Lprev = wave_shr1_i64(Lk, latest);
                        const bool actual = aq <= 0 || (rcount > 0 && (cost + Lprev <= t || cost + Lprev - t <= rqueue));
                        const uint64_t mis = __ballot(open && actual != spec);
                        const int m = mis ? __builtin_ctzll(mis) : 64;
                        if (open && lane < m) {
                            d = spec ? D_PASS : D_BLOCK_FLOW;
                            if (spec && mv) w = Lk - t;
                        }
                        if (m == 64) {
                            latest = readlane_i64(Lk, 63);
                            break;
                        }
                        if (m > 0) latest = readlane_i64(Lk, m - 1);
                        // lane m: its true decision (the state before it is now exact)
                        const int am = __builtin_amdgcn_readlane(aq, m);
                        const int64_t tm = readlane_i64(t, m), cm = readlane_i64(cost, m);
                        const bool pm = (__ballot(actual) >> m) & 1ull;
                        if (lane == m) d = pm ? D_PASS : D_BLOCK_FLOW;
                        if (pm && am > 0) {
                            const int64_t lm = max(latest + cm, tm);
                            if (lane == m) w = lm - tm;
                            latest = lm;
                        }
                        if (am > 0 && cm > 0) pred_c = pm;
                        rem &= (m == 63) ? 0ull : (~0ull << (m + 1));
                    }
                    rem = 0;
                }
                if (!pace && !passes(0, 0, amin)) {
                    // saturated: not even the run's smallest acquireCount fits, and blocked entries
                    // leave the pass count alone, so the rest of the run blocks without a scan
                    if (ent) d = D_BLOCK_FLOW;
                    rem = 0;
                }
                if (!pace && rem) {  // before the window's first block every entry passes: one prefix sum
                    const int64_t incl = wave_incl_sum_i64(aq);
                    const int64_t before = S + incl - aq;
                    const bool ok_pre = warm ? (double)(j_d2l((double)before / 1.0) + aq) <= lim
                                             : default_cond(rcount, before, aq);
                    const uint64_t bad = __ballot(ent && !ok_pre);
                    const int b = bad ? __builtin_ctzll(bad) : 64;
                    const int64_t upto = b == 0 ? 0 : readlane_i64(incl, b - 1);  // entries' acquire before lane b
                    S += upto;
                    rem &= b >= 64 ? 0ull : (~0ull << b);
                }
                while (rem) {
                    if (prof) ++pr_iter;
                    bool open = (rem >> lane) & 1ull;
                    const uint64_t pm = __ballot(open && passes(t, cost, aq));
                    const int first = pm ? __builtin_ctzll(pm) : 64;
                    if (open && lane < first && (pace ? aq > 0 : true)) d = D_BLOCK_FLOW;
                    if (first == 64) break;
                    const int af = __builtin_amdgcn_readlane(aq, first);
                    if (pace) {
                        const int64_t tf = readlane_i64(t, first), cf = readlane_i64(cost, first);
                        if (af > 0) {
                            int64_t wf = 0;
                            if (cf + latest <= tf) {
                                latest = tf;
                            } else {
                                latest += cf;
                                wf = latest - tf;
                            }
                            if (lane == first) w = wf;
                        }
                    } else {
                        S += af;
                    }
                    rem &= (first == 63) ? 0ull : (~0ull << (first + 1));
                }
                if (ent && j < j1) {
                    // sorted-order (coalesced) store; k_lresults scatters it by request index
                    if (w < ((int64_t)1 << 30)) {
                        sc.ev_eidx[j] = ((uint32_t)w << 1) | (d != D_PASS ? 1u : 0u);
                    } else {
                        const uint32_t idx = q.idx & F_IDX;
                        decision[idx] = d;
                        wait_ms[idx] = (int32_t)w;
                        sc.ev_eidx[j] = ~0u;
                    }
                    if (d == D_PASS) {
                        pa += aq;
                        ++npass;
                    } else {
                        ba += aq;
                    }
                }
            };
            // the decided entry's store (sorted order, coalesced; k_lresults scatters it by request index) and
            // this lane's share of the statistics
            auto store_ev = [&](uint32_t j, const Payload &q, bool ent, int aq, int8_t d, int64_t w) {
                if (!(ent && j < j1)) return;
                if (w < ((int64_t)1 << 30)) {
                    sc.ev_eidx[j] = ((uint32_t)w << 1) | (d != D_PASS ? 1u : 0u);
                } else {
                    const uint32_t idx = q.idx & F_IDX;
                    decision[idx] = d;
                    wait_ms[idx] = (int32_t)w;
                    sc.ev_eidx[j] = ~0u;
                }
                if (d == D_PASS) {
                    pa += aq;
                    ++npass;
                } else {
                    ba += aq;
                }
            };
            // RateLimiter, two windows (128 entries) per step: the same speculation as window(), the two
            // halves' max-plus scans independent (the second composed with the first's total), so their
            // dependent DPP chains interleave -- one wave's window walk is bound by that latency
            auto pace2 = [&](uint32_t g, Payload q0, Payload q1) {
                const uint32_t ja = g + (uint32_t)lane, jb = g + 64u + (uint32_t)lane;
                if (ja >= j1) q0.idx = F_EXIT;
                if (jb >= j1) q1.idx = F_EXIT;
                const bool ea = !(q0.idx & F_EXIT), eb = !(q1.idx & F_EXIT);
                const int64_t ta = ts_base + (int64_t)q0.ts_off, tb = ts_base + (int64_t)q1.ts_off;
                const int aa = ea ? (int)(q0.acq_prio & 0x7FFFFFFFu) : 0, ab = eb ? (int)(q1.acq_prio & 0x7FFFFFFFu) : 0;
                const int64_t ca = (ea && aa > 0 && rcount > 0) ? j_round(1.0 * aa / rcount * 1000) : 0;
                const int64_t cb = (eb && ab > 0 && rcount > 0) ? j_round(1.0 * ab / rcount * 1000) : 0;
                int8_t da = D_PASS, db = D_PASS;
                int64_t wa = 0, wb = 0;
                uint64_t ra = __ballot(ea), rb = __ballot(eb);
                while (ra | rb) {
                    if (prof) ++pr_iter;
                    const bool oa = (ra >> lane) & 1ull, ob = (rb >> lane) & 1ull;
                    const bool mva = oa && aa > 0 && rcount > 0, mvb = ob && ab > 0 && rcount > 0;
                    const bool spa = aa <= 0 || (rcount > 0 && (ca == 0 || pred_c));
                    const bool spb = ab <= 0 || (rcount > 0 && (cb == 0 || pred_c));
                    int64_t Aa = (mva && spa) ? ca : 0, Ba = (mva && spa) ? ta : kMaxPlusNegInf;
                    int64_t Ab = (mvb && spb) ? cb : 0, Bb = (mvb && spb) ? tb : kMaxPlusNegInf;
                    wave_incl_maxplus(Aa, Ba);
                    wave_incl_maxplus(Ab, Bb);
                    const int64_t Lka = max(latest + Aa, Ba);
                    const int64_t Lenda = readlane_i64(Lka, 63);
                    const int64_t Lkb = max(Lenda + Ab, Bb);
                    const int64_t Lpa = wave_shr1_i64(Lka, latest), Lpb = wave_shr1_i64(Lkb, Lenda);
                    const bool aca = aa <= 0 || (rcount > 0 && (ca + Lpa <= ta || ca + Lpa - ta <= rqueue));
                    const bool acb = ab <= 0 || (rcount > 0 && (cb + Lpb <= tb || cb + Lpb - tb <= rqueue));
                    const uint64_t misa = __ballot(oa && aca != spa);
                    // the first wrong prediction of a half: the lanes before it decided, its true decision
                    auto fix = [&](const int m, const bool op, const bool sp, const bool mvv, const int64_t Lk,
                                   const int64_t Lstart, const bool ac, const int av, const int64_t tv,
                                   const int64_t cv, int8_t &d, int64_t &w, uint64_t &r) {
                        if (op && lane < m) {
                            d = sp ? D_PASS : D_BLOCK_FLOW;
                            if (sp && mvv) w = Lk - tv;
                        }
                        latest = m > 0 ? readlane_i64(Lk, m - 1) : Lstart;
                        const int am = __builtin_amdgcn_readlane(av, m);
                        const int64_t tm = readlane_i64(tv, m), cm = readlane_i64(cv, m);
                        const bool pm = (__ballot(ac) >> m) & 1ull;
                        if (lane == m) d = pm ? D_PASS : D_BLOCK_FLOW;
                        if (pm && am > 0) {
                            const int64_t lm = max(latest + cm, tm);
                            if (lane == m) w = lm - tm;
                            latest = lm;
                        }
                        if (am > 0 && cm > 0) pred_c = pm;
                        r &= (m == 63) ? 0ull : (~0ull << (m + 1));
                    };
                    if (misa) {
                        fix(__builtin_ctzll(misa), oa, spa, mva, Lka, latest, aca, aa, ta, ca, da, wa, ra);
                        continue;
                    }
                    if (oa) {  // every open prediction of the first half was right
                        da = spa ? D_PASS : D_BLOCK_FLOW;
                        if (spa && mva) wa = Lka - ta;
                    }
                    ra = 0;
                    const uint64_t misb = __ballot(ob && acb != spb);
                    if (!misb) {
                        if (ob) {
                            db = spb ? D_PASS : D_BLOCK_FLOW;
                            if (spb && mvb) wb = Lkb - tb;
                        }
                        latest = readlane_i64(Lkb, 63);
                        break;
                    }
                    fix(__builtin_ctzll(misb), ob, spb, mvb, Lkb, Lenda, acb, ab, tb, cb, db, wb, rb);
                }
                store_ev(ja, q0, ea, aa, da, wa);
                store_ev(jb, q1, eb, ab, db, wb);
            };
            // Default / WarmUp: once not even the run's smallest acquireCount fits (blocked entries leave
            // the pass count alone), every later entry blocks -- the walk stops there (js) and k_lresults
            // writes the tail's decisions over the whole GPU; the blocked acquire is the run's entry sum
            // less the passes
            uint32_t js = j1;
            // a long RateLimiter run walks k_lwsum's window summaries: a window whose decisions follow from
            // the state it starts at (every costly entry blocks, zero-cost entries pass behind the queue) is
            // skipped, its state left in wstate for k_lresults; the run's first and last windows and any
            // other window are walked as above (RUN_WIN)
            const bool winmode = pace && rcount > 0 && j1 - j0 >= kWinMin;
            if (winmode) {
                const uint32_t wf = j0 / 64, wl = (j1 - 1) / 64;
                const int64_t qp = rqueue > 0 ? rqueue : 0;
                for (uint32_t wb = wf; wb <= wl; wb += 64) {
                    const uint32_t w = wb + (uint32_t)lane;
                    const bool inner = w > wf && w < wl;
                    WinSum s{INT64_MAX, 0, 0, 0, 0, 0};
                    if (inner) s = sc.wsum[w];
                    uint64_t todo = __ballot(w <= wl);
                    while (todo) {
                        const int64_t lo = latest - ts_base, thr = lo - qp;
                        const bool inert = inner && s.kmax < thr &&
                                           (!s.has0 || ((int64_t)s.t0max <= lo && (int64_t)s.t0min >= thr));
                        const uint64_t walk = __ballot(!inert) & todo;
                        const int first = walk ? __builtin_ctzll(walk) : 64;
                        const bool skip = ((todo >> lane) & 1ull) && lane < first;
                        if (skip) {
                            sc.wstate[w] = lo;
                            pa += s.a0;
                            npass += s.n0;
                        }
                        if (__ballot(skip && s.kmax != INT64_MIN)) pred_c = false;  // they blocked
                        if (first == 64) break;
                        const uint32_t g = (wb + (uint32_t)first) * 64;
                        const Payload q = pay[min(max(g + (uint32_t)lane, j0), j1 - 1)];
                        if (lane == first && inner) sc.wstate[w] = kWinWalked;
                        window(g, q);
                        todo &= (first == 63) ? 0ull : (~0ull << (first + 1));
                    }
                }
            }
            for (uint32_t g0 = j0; g0 < j1 && js == j1 && !winmode; g0 += 64 * kWavePf) {
#pragma unroll
                for (int k = 0; k < kWavePf; ++k) {
                    const uint32_t g = g0 + (uint32_t)k * 64;
                    if (pace && pace_pairs) {  // windows k, k + 1 together (kWavePf is even)
                        if (k & 1) continue;
                        const Payload q0 = ring[k], q1 = ring[k + 1];
                        ring[k] = pay[min(g + (uint32_t)(kWavePf * 64 + lane), j1 - 1)];
                        ring[k + 1] = pay[min(g + 64u + (uint32_t)(kWavePf * 64 + lane), j1 - 1)];
                        if (g < j1) pace2(g, q0, q1);  // wave-uniform
                        continue;
                    }
                    const Payload q = ring[k];
                    ring[k] = pay[min(g + (uint32_t)(kWavePf * 64 + lane), j1 - 1)];
                    if (g < j1 && js == j1) {  // wave-uniform
                        if (!pace && !passes(0, 0, amin)) js = g;
                        else window(g, q);
                    }
                }
            }
            pa = wave_sum_i64(pa);
            ba = wave_sum_i64(ba);
            npass = wave_sum_i64(npass);
            if (!pace || winmode) ba = sc.run_asum[r] - pa;
            if (lane == 0) {
                if (pace) rule.latest_passed = latest;
                int64_t *sb = sec_current(node, t0, max_rt);
                int64_t *mb = min_current(node, t0, max_rt);
                const int64_t exc = (int64_t)sc.run_exc[r], exerr = (int64_t)sc.run_exerr[r];
                const int64_t exrt = sc.run_exrt[r], exmin = sc.run_exmin[r];
                int64_t *w2[2] = {sb, mb};
                for (int k = 0; k < 2; ++k) {
                    int64_t *b = w2[k];
                    b[MB_PASS] += pa;
                    b[MB_BLOCK] += ba;
                    b[MB_SUCC] += exc;
                    b[MB_RT] += exrt;
                    b[MB_EXC] += exerr;
                    if (exmin < b[MB_MINRT]) b[MB_MINRT] = exmin;
                }
                node[kNodeThreads] += npass - (int64_t)sc.run_nexit[r];
                sc.run_f[r] = js;  // RUN_POS: entries from js on blocked, not in ev_eidx
                sc.run_mode[r] = winmode ? RUN_WIN : RUN_POS;
            }
            __syncthreads();
        }
        if (prof && lane == 0) {
            const uint64_t dt = wall_clock64() - pt0;
            const uint32_t nev = sc.run_end[r1 - 1] - sc.run_start[r0];
            uint64_t *p = prof + (size_t)(blockIdx.x % 1024) * 8;
            p[0] += 1;
            p[1] += nev;
            p[2] += dt;
            if (dt > p[6]) {
                p[6] = dt;
                p[7] = ((uint64_t)nev << 32) | (uint64_t)(st.res[sc.run_slot[r0]].fast & 0xFFu) |
                       ((uint64_t)(r1 - r0) << 8);
            }
        }
    }
    if (prof && lane == 0) {
        uint64_t *p = prof + (size_t)(blockIdx.x % 1024) * 8;
        p[3] += pr_lrt;
        p[4] += pr_lr;
        p[5] += pr_iter;
    }
}

__global__ __launch_bounds__(64) void k_lheavy(FlowState st, int64_t max_rt, FlowScratch sc,
                                               const Payload *__restrict__ pay, int64_t ts_base,
                                               const int64_t *__restrict__ rt_in,
                                               const uint64_t *__restrict__ param_in, int8_t *decision,
                                               int32_t *wait_ms, uint64_t *prof) {
    // prof (SGA_HEAVY_PROF=1): per workgroup, wall-clock ticks spent in each phase of the chunks
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    __shared__ int64_t lnode[kNodeWords];
    __shared__ FlowRuleDev lrules[kHeavyRules];
    __shared__ CbDev lcbs[kHeavyCbs];
    __shared__ Payload qpay[kHeavyChunk];
    __shared__ int64_t qrt[kHeavyChunk];
    __shared__ uint64_t qpv[kHeavyChunk];
    __shared__ int8_t qd[kHeavyChunk];
    __shared__ int32_t qw[kHeavyChunk];
    // parameter-map entries of the chunk (resources with one token-bucket / throttle parameter rule):
    // resolved by all lanes in parallel, deduplicated into LDS copies, replayed by lane 0 without a
    // global access per event, written back once per chunk
    __shared__ PEntry lent[kHeavySlots];
    __shared__ uint64_t lval[kHeavySlots];  // parameter value of the slot (kLEmpty = free)
    __shared__ uint32_t lgi[kHeavySlots];   // map index of the slot's entry
    __shared__ PEntry tent[kHeavySlots];    // per-value lanes: the value's thread-count entry (ParameterMetric)
    __shared__ uint32_t tgi[kHeavySlots];
    // CacheMap bookkeeping (free mode: the count pass keeps these owners below capacity): the stamp of each
    // slot's last access in the chunk (0: none) and whether its key was present when the chunk began
    __shared__ uint64_t lst[kHeavySlots], tst[kHeavySlots];
    __shared__ uint8_t lp0[kHeavySlots], tp0[kHeavySlots];
    __shared__ int nocache;                 // a parameter event of the chunk got no slot
    __shared__ uint16_t qslot[kHeavyChunk];
    // parameter-only resources: the rule check of each event is decided by the lane that owns the
    // event's value (lane = LDS slot mod 64), every lane walking its values' events in arrival
    // order (the maps of different values are independent); lane 0 then does the statistics
    __shared__ int8_t qpre[kHeavyChunk];
    __shared__ int32_t qpw[kHeavyChunk];
    __shared__ uint16_t qrank[kHeavyChunk], qord[kHeavyChunk];
    __shared__ uint32_t lcnt[64];
    __shared__ int64_t qbq[kHeavyChunk];  // second-window bucket (t / 500) of each event
    __shared__ int64_t qrank_ws[kHeavyChunk];  // breaker-only resources: the breaker's stat window start
    __shared__ int64_t sbad[kHeavyChunk], stot[kHeavyChunk];  // CLOSED-breaker scan: window counts after each exit
    __shared__ int bulk_end;                  // breaker-only resources: where the next bulk part starts
    __shared__ int32_t s_pidx;                // the parameter rule's index in force (applyRealParamIdx)
    __shared__ uint64_t s_tmask;              // the resource's thread-count maps
    const Ctx c{st, max_rt, nullptr, 0, 0, nullptr};
    constexpr uint64_t kLEmpty = ~0ull;  // a value equal to it bypasses the cache (map path)
    constexpr uint32_t kGiNone = 0xFFFFFFFFu, kGiFail = 0xFFFFFFFEu;
    for (int k = threadIdx.x; k < kHeavySlots; k += 64) lval[k] = kLEmpty;
    const uint32_t nheavy = sc.counters[8], nflows = sc.counters[2], nruns = sc.counters[1];
    for (uint32_t h = blockIdx.x; h < nheavy; h += gridDim.x) {
        const uint32_t fl = sc.heavy[h];
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t res = sc.run_slot[r0];
        const ResDev R = st.res[res];
        ResMem g = res_global(c, res, R);
        const bool lr = R.n_rules <= (uint32_t)kHeavyRules, lc = R.n_cbs <= (uint32_t)kHeavyCbs;
        for (int k = threadIdx.x; k < kNodeWords; k += 64) lnode[k] = g.node[k];
        if (lr)
            for (uint32_t k = threadIdx.x; k < R.n_rules; k += 64) lrules[k] = g.rules[k];
        if (lc)
            for (uint32_t k = threadIdx.x; k < R.n_cbs; k += 64) lcbs[k] = g.cbs[k];
        __syncthreads();
        // events in chunks: the 64 lanes stage payloads, RTs and parameters into LDS, lane 0 replays
        // the chunk from LDS, then the lanes store its decisions
        const ResMem m{lnode, lr ? lrules : g.rules, lc ? lcbs : g.cbs};
        // one parameter rule with a map (QPS grade): its entries go through the LDS cache
        const ParamRuleDev *cache_p =
            (R.n_prules == 1 && st.prules[R.prule_off].grade == 1) ? &st.prules[R.prule_off] : nullptr;
        // parameter-only resource: per-value lanes own the rule map entry and the thread-count entry
        const bool par = cache_p && R.n_rules == 0 && R.n_cbs == 0;
        const uint32_t jb = sc.run_start[r0], je = sc.run_end[r1 - 1];
        // ParamFlowSlot.applyRealParamIdx fixes a negative index at the rule's first check: the
        // resource's first entry (events are in arrival order), with args = [param] or [].  The rule
        // is checked by every entry, so its thread-count map exists from then on.
        if (cache_p && threadIdx.x == 0) {
            ParamRuleDev &pr = st.prules[R.prule_off];
            int32_t idx = pr.idx_res;
            uint64_t mask = st.tmapmask[res];
            if (idx == kIdxUnresolved) {
                for (uint32_t j = jb; j < je; ++j) {
                    const Payload q = pay[j];
                    if (q.idx & F_EXIT) continue;
                    idx = param_idx_of(pr, (q.idx & F_PARAM) ? 1u : 0u);
                    break;
                }
            }
            bool any_entry = false;
            for (uint32_t j = jb; j < je && !any_entry; ++j) any_entry = !(pay[j].idx & F_EXIT);
            if (any_entry && idx >= 0 && idx < kMaxParamIdx) {
                mask |= 1ull << idx;
                st.tmapmask[res] = mask;
            }
            s_pidx = idx;
            s_tmask = mask;
        }
        __syncthreads();
        const int32_t pidx = s_pidx;             // kIdxUnresolved: no entry yet (the rule is not checked)
        const bool p_applies = pidx == 0;        // events carry args = [param]: index 0 reads it
        const bool tmap0 = (s_tmask & 1ull) != 0;  // the thread-count map of argument 0 exists
        uint64_t tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint64_t tprev = prof ? wall_clock64() : 0;
        auto tick = [&](int ph) {
            if (prof && threadIdx.x == 0) {
                const uint64_t t = wall_clock64();
                tk[ph] += t - tprev;
                tprev = t;
            }
        };
        for (uint32_t base = jb; base < je; base += kHeavyChunk) {
            const uint32_t cnt = min((uint32_t)kHeavyChunk, je - base);
            for (uint32_t k = threadIdx.x; k < cnt; k += 64) {
                const Payload q = pay[base + k];
                const uint32_t idx = q.idx & F_IDX;
                qpay[k] = q;
                qrt[k] = (q.idx & F_EXIT) ? rt_in[idx] : 0;
                qpv[k] = (q.idx & F_PARAM) ? param_in[idx] : 0;
            }
            __syncthreads();
            tick(0);
            if (threadIdx.x == 0) nocache = 0;
            __syncthreads();
            const bool pt = par && p_applies;  // exits of parameter events go to the value lanes too
            if (cache_p) {
                // 1. the chunk's distinct values into LDS slots (64-bit CAS on the value)
                for (uint32_t k = threadIdx.x; k < cnt; k += 64) {
                    const Payload q = qpay[k];
                    uint16_t sl = 0xFFFF;
                    const bool want = (q.idx & F_PARAM) && (pt || !(q.idx & F_EXIT));
                    if (want && qpv[k] == kLEmpty) nocache = 1;
                    if (want && qpv[k] != kLEmpty) {
                        const uint64_t v = qpv[k];
                        uint32_t h = (uint32_t)splitmix64(v) & (kHeavySlots - 1);
                        for (int probe = 0; probe < kHeavySlots; ++probe) {
                            const uint64_t old = atomicCAS((unsigned long long *)&lval[h], kLEmpty, v);
                            if (old == kLEmpty) {
                                lgi[h] = kGiNone;
                                tgi[h] = kGiNone;
                                lst[h] = 0;
                                tst[h] = 0;
                            }
                            if (old == kLEmpty || old == v) {
                                sl = (uint16_t)h;
                                break;
                            }
                            h = (h + 1) & (kHeavySlots - 1);
                        }
                    }
                    qslot[k] = sl;
                }
                __syncthreads();
                tick(6);
                // 2. find the values' entries (lookups only: nothing is being filled meanwhile).  The
                //    maps stay at most a quarter full, so most values resolve at their home slot: the
                //    home slots of kG of a lane's LDS slots are read together, and only a value whose
                //    home holds another key walks its probe sequence (ptab_get).
                constexpr int kSl = kHeavySlots / 64, kG = 8;
                const uint32_t pown = cache_p->id + 1, town = res + 1;
                uint32_t pfree = 0, tfree = 0;  // bit i: LDS slot lane + 64 i is absent and its home is free
                for (int g0 = 0; g0 < kSl; g0 += kG) {
                    // the whole home entries are loaded together and unconditionally (an empty LDS
                    // slot reads some valid home): a load under a branch would be waited for at the
                    // branch, and an entry found at its home needs no second read
                    uint64_t val[kG];
                    int4 pe0[kG], pe1[kG], te0[kG], te1[kG];
                    uint32_t ph[kG], th[kG];
#pragma unroll
                    for (int u = 0; u < kG; ++u) {
                        val[u] = lval[threadIdx.x + 64 * (g0 + u)];
                        const uint64_t vv = val[u] == kLEmpty ? 0ull : val[u];
                        ph[u] = ptab_home(st.pmask, pown, vv);
                        const int4 *pp = reinterpret_cast<const int4 *>(&st.ptab[ph[u]]);
                        pe0[u] = pp[0];
                        pe1[u] = pp[1];
                        th[u] = ptab_home(st.tmask, town, vv);
                        if (pt) {
                            const int4 *tp = reinterpret_cast<const int4 *>(&st.ttab[th[u]]);
                            te0[u] = tp[0];
                            te1[u] = tp[1];
                        }
                    }
                    auto as_entry = [](const int4 &x, const int4 &y) {
                        PEntry e;
                        e.value = ((uint64_t)(uint32_t)x.y << 32) | (uint32_t)x.x;
                        e.owner = (uint32_t)x.z;
                        e.pad = (uint32_t)x.w;
                        e.a = (int64_t)(((uint64_t)(uint32_t)y.y << 32) | (uint32_t)y.x);
                        e.b = (int64_t)(((uint64_t)(uint32_t)y.w << 32) | (uint32_t)y.z);
                        return e;
                    };
#pragma unroll
                    for (int u = 0; u < kG; ++u) {
                        if (val[u] == kLEmpty) continue;
                        const int h = threadIdx.x + 64 * (g0 + u);
                        const PEntry hp = as_entry(pe0[u], pe1[u]);
                        if (hp.owner == 0) {
                            pfree |= 1u << (g0 + u);
                        } else if (hp.owner == pown && hp.value == val[u]) {
                            lgi[h] = ph[u];
                            lent[h] = hp;
                        } else {
                            PEntry *e = ptab_get(st.ptab, st.pmask, pown, val[u], false, st.overflow);
                            if (e) {
                                lgi[h] = (uint32_t)(e - st.ptab);
                                lent[h] = *e;
                            }
                        }
                        if (pt) {
                            const PEntry ht = as_entry(te0[u], te1[u]);
                            if (ht.owner == 0) {
                                tfree |= 1u << (g0 + u);
                            } else if (ht.owner == town && ht.value == val[u]) {
                                tgi[h] = th[u];
                                tent[h] = ht;
                            } else {
                                PEntry *te = ptab_get(st.ttab, st.tmask, town, val[u], false, st.overflow);
                                if (te) {
                                    tgi[h] = (uint32_t)(te - st.ttab);
                                    tent[h] = *te;
                                }
                            }
                        }
                    }
                }
                __syncthreads();
                tick(7);
                // 3. insert the absent ones (a fresh entry is the reference's "not seen yet"; creating
                //    it for an event that never reaches the rule changes nothing): the claims of the
                //    free home slots go out together, a lost claim walks the probe sequence
                for (int g0 = 0; g0 < kSl; g0 += kG) {
                    uint32_t pc[kG], tc[kG];
#pragma unroll
                    for (int u = 0; u < kG; ++u) {
                        const int h = threadIdx.x + 64 * (g0 + u);
                        pc[u] = tc[u] = 1u;
                        const uint64_t v = lval[h];
                        if (v == kLEmpty) continue;
                        if (lgi[h] == kGiNone && ((pfree >> (g0 + u)) & 1u))
                            pc[u] = atomicCAS(&st.ptab[ptab_home(st.pmask, pown, v)].owner, 0u, pown);
                        if (pt && tgi[h] == kGiNone && ((tfree >> (g0 + u)) & 1u))
                            tc[u] = atomicCAS(&st.ttab[ptab_home(st.tmask, town, v)].owner, 0u, town);
                    }
#pragma unroll
                    for (int u = 0; u < kG; ++u) {
                        const int h = threadIdx.x + 64 * (g0 + u);
                        const uint64_t v = lval[h];
                        if (v == kLEmpty) continue;
                        if (lgi[h] == kGiNone) {
                            PEntry *e;
                            if (pc[u] == 0u) {  // claimed the home slot (the CAS publishes the owner)
                                claim_note(st.ptab, ptab_home(st.pmask, pown, v));
                                e = &st.ptab[ptab_home(st.pmask, pown, v)];
                                e->value = v;
                                e->a = kPAbsent;
                                e->b = kPAbsent;
                            } else {
                                e = ptab_insert_absent(st.ptab, st.pmask, pown, v, st.overflow);
                            }
                            lgi[h] = e ? (uint32_t)(e - st.ptab) : kGiFail;
                            lent[h] = PEntry{v, pown, 0, kPAbsent, kPAbsent};
                        }
                        if (pt && tgi[h] == kGiNone) {
                            PEntry *te;
                            if (tc[u] == 0u) {
                                claim_note(st.ttab, ptab_home(st.tmask, town, v));
                                te = &st.ttab[ptab_home(st.tmask, town, v)];
                                te->value = v;
                                te->a = kPAbsent;
                                te->b = kPAbsent;
                            } else {
                                te = ptab_insert_absent(st.ttab, st.tmask, town, v, st.overflow);
                            }
                            tgi[h] = te ? (uint32_t)(te - st.ttab) : kGiFail;
                            tent[h] = PEntry{v, town, 0, kPAbsent, kPAbsent};
                        }
                    }
                }
            }
            __syncthreads();
            tick(1);
            if (cache_p)  // presence of the chunk's keys before it (found entries as read, inserted ones absent)
                for (int k = threadIdx.x; k < kHeavySlots; k += 64)
                    if (lval[k] != kLEmpty) {
                        lp0[k] = lent[k].a != kPAbsent ? 1 : 0;
                        tp0[k] = (pt && tgi[k] < kGiFail && tent[k].a != kPAbsent) ? 1 : 0;
                    }
            __syncthreads();
            const bool par_ok = pt && !nocache;
            if (par_ok) {
                const int lane = threadIdx.x;
                const uint64_t lt = (1ull << lane) - 1ull;
                lcnt[lane] = 0;
                // stable ranking of the chunk's rule checks by owner lane (ballot-matched owners)
                for (uint32_t r0 = 0; r0 < cnt; r0 += 64) {
                    const uint32_t k = r0 + lane;
                    bool ok = false;
                    uint32_t own = 0;
                    if (k < cnt) {
                        const Payload q = qpay[k];
                        ok = (q.idx & F_PARAM) && qslot[k] != 0xFFFF;  // entries and exits
                        own = qslot[k] & 63u;
                        qpre[k] = 0;
                        qbq[k] = (ts_base + (int64_t)q.ts_off) / kSecW;
                    }
                    uint64_t peers = __ballot(ok);
#pragma unroll
                    for (int b = 0; b < 6; ++b) {
                        const bool bit = (own >> b) & 1u;
                        const uint64_t bb = __ballot(bit);
                        peers &= bit ? bb : ~bb;
                    }
                    uint32_t before = 0;
                    if (ok) before = lcnt[own];
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t my = (uint32_t)__popcll(peers & lt);
                    if (ok && my == 0) lcnt[own] = before + (uint32_t)__popcll(peers);
                    __builtin_amdgcn_wave_barrier();
                    if (k < cnt) qrank[k] = ok ? (uint16_t)(before + my) : (uint16_t)0xFFFF;
                }
                __builtin_amdgcn_wave_barrier();
                const uint32_t mine = lcnt[lane];
                uint32_t x = mine;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(x, o, 64);
                    if (lane >= o) x += y;
                }
                const uint32_t start = x - mine;
                __builtin_amdgcn_wave_barrier();
                lcnt[lane] = start;
                __builtin_amdgcn_wave_barrier();
                for (uint32_t k = lane; k < cnt; k += 64)
                    if (qrank[k] != 0xFFFF) qord[lcnt[qslot[k] & 63u] + qrank[k]] = (uint16_t)k;
                __builtin_amdgcn_wave_barrier();
                Ctx cl = c;
                // the rule in registers: through a generic pointer its fields would be reloaded after
                // every store to the LDS entries (possible aliasing), one global latency per event
                const ParamRuleDev prule = *cache_p;
                for (uint32_t i = start; i < start + mine; ++i) {
                    const uint32_t k = qord[i];
                    const Payload q = qpay[k];
                    PEntry &te = tent[qslot[k]];
                    const bool tmap = tmap0;  // ParameterMetric thread counts exist
                    const uint64_t stamp = lru_stamp(st, q.idx & F_IDX, 0);
                    if (q.idx & F_EXIT) {  // ParameterMetric.decreaseThreadCount (chain_exit)
                        if (tmap) {
                            if (te.a == kPAbsent) te.a = 0;
                            else if (--te.a <= 0) te.a = kPAbsent;
                            tst[qslot[k]] = stamp;
                        }
                        continue;
                    }
                    int64_t w = 0;
                    // a QPS rule does not read the thread count; the entry is read and written back
                    // through LDS directly (a generic pointer would turn every access into a flat op)
                    PEntry pe = lent[qslot[k]];
                    const int aq = (int)(q.acq_prio & 0x7FFFFFFFu);
                    if (param_map_access(cl, prule, qpv[k], aq)) lst[qslot[k]] = stamp;
                    const bool pass = param_pass_qps(cl, prule, pe, qpv[k], aq, ts_base + (int64_t)q.ts_off, &w);
                    lent[qslot[k]] = pe;
                    qpre[k] = pass ? 1 : 2;
                    qpw[k] = (int32_t)w;
                    if (pass && tmap) {  // ParameterMetric.addThreadCount
                        te.a = (te.a == kPAbsent ? 0 : te.a) + 1;
                        tst[qslot[k]] = stamp;
                    }
                }
            }
            __syncthreads();
            tick(2);
            // breaker-only resources: lane 0 runs the breakers event by event (a sequential state
            // machine) and the node statistics in aggregate, as for parameter-only resources
            const bool dgo = R.n_cbs > 0 && R.n_rules == 0 && R.n_prules == 0 && lc;
            const bool agg = par_ok || dgo;
            if (dgo) {  // second-window buckets (and the one breaker's stat window starts) on all lanes:
                        // lane 0 would divide per event
                const int64_t si = R.n_cbs == 1 ? (int64_t)lcbs[0].stat_interval : 1;
                for (uint32_t k = threadIdx.x; k < cnt; k += 64) {
                    const int64_t t = ts_base + (int64_t)qpay[k].ts_off;
                    qbq[k] = t / kSecW;
                    qrank_ws[k] = t - t % si;
                }
                __syncthreads();
            }
            if (agg) {
                // Decisions first (a breaker or a parameter verdict never reads the node statistics),
                // then StatisticSlot in aggregate over all lanes: a parameter-only or breaker-only
                // resource's decisions never read its node, and every event of a 500 ms second-window
                // bucket (nested in one minute bucket) sees the same window rotation, so each run of
                // consecutive same-bucket events is applied once at its first event's time
                // (commutative adds, min RT, thread count).
                const int lane = threadIdx.x;
                if (dgo) {
                    // One breaker: the chunk alternates bulk parts and short replays.  A CLOSED breaker
                    // lets every entry pass and its exits only add to the stat window until one trips
                    // it; an OPEN one blocks every entry before its retry time and its exits only
                    // count.  One segmented scan over the exits (segments = stat windows,
                    // non-decreasing) gives the window counts after every exit; the bulk part ends at
                    // the first exit whose counts trip a CLOSED breaker (cb_trips, the predicate of
                    // cb_on_complete) or at the first entry at or after an OPEN breaker's retry time.
                    // Lane 0 steps the event that ends a bulk part; while the breaker is HALF_OPEN the
                    // entries up to the next exit block in bulk.  Several breakers, or a stat window
                    // that goes back, replay in order on lane 0.
                    uint32_t pos = 0;
                    while (pos < cnt) {
                        const CbDev &b0 = lcbs[0];
                        const int bst = b0.state;
                        uint32_t end = pos;
                        bool seq_rest = R.n_cbs != 1;
                        if (!seq_rest && bst != 2) {
                            int64_t cws = b0.st_start, cbad = b0.st_bad, ctot = b0.st_total;  // running window
                            uint32_t stop = 0xFFFFFFFFu;
                            for (uint32_t r0 = pos; r0 < cnt; r0 += 64) {
                                const uint32_t k = r0 + lane;
                                const bool valid = k < cnt;
                                const bool ex = valid && (qpay[k].idx & F_EXIT);
                                const int64_t ws = ex ? qrank_ws[k] : INT64_MIN;
                                const bool badv = ex && (b0.grade == 0 ? qrt[k] > b0.max_allowed_rt
                                                                       : (qpay[k].idx & F_ERROR) != 0);
                                // previous exit's window: prefix max over the lanes (windows only grow)
                                const int64_t pm = wave_incl_max_i64(ws);
                                int64_t prev = wave_shr1_i64(pm, INT64_MIN);
                                if (prev < cws) prev = cws;  // carry from earlier rounds / the breaker
                                const bool mono = !(ex && prev != kAbsent && ws < prev);
                                if (!__all(mono)) {  // the clock went back: the rest replays in order
                                    stop = r0;
                                    seq_rest = true;
                                    break;
                                }
                                const bool head = ex && (prev == kAbsent || ws != prev);
                                // segmented inclusive scan of (bad, total) over the exits
                                int sb32 = badv ? 1 : 0, st32 = ex ? 1 : 0, hd = head ? 1 : 0;
                                wave_incl_segsum2(sb32, st32, hd);  // counts inside the round (< 64)
                                int64_t sb = sb32, stt = st32;
                                if (!hd) {  // no window start before this lane in the round: continue the carry
                                    sb += (prev == cws) ? cbad : 0;
                                    stt += (prev == cws) ? ctot : 0;
                                }
                                if (ex) {
                                    sbad[k] = sb;
                                    stot[k] = stt;
                                }
                                const uint64_t tb =
                                    bst == 0 ? __ballot(ex && cb_trips(b0, sb, stt))
                                             : __ballot(valid && !ex &&
                                                        ts_base + (int64_t)qpay[k].ts_off >= b0.next_retry);
                                if (tb) {
                                    stop = r0 + (uint32_t)__ffsll((unsigned long long)tb) - 1;
                                    break;
                                }
                                // carry: the round's last exit
                                const uint64_t eb = __ballot(ex);
                                if (eb) {
                                    const int last = 63 - __clzll((unsigned long long)eb);
                                    cws = readlane_i64(ws, last);
                                    cbad = readlane_i64(sb, last);
                                    ctot = readlane_i64(stt, last);
                                }
                            }
                            end = stop == 0xFFFFFFFFu ? cnt : stop;
                        } else if (!seq_rest) {
                            // HALF_OPEN: tryPass blocks every entry (AbstractCircuitBreaker.tryPass) until
                            // the next exit decides the probe (onRequestComplete closes or reopens), so the
                            // bulk part runs up to that exit
                            uint32_t stop = cnt;
                            for (uint32_t r0 = pos; r0 < cnt; r0 += 64) {
                                const uint32_t k = r0 + lane;
                                const uint64_t eb = __ballot(k < cnt && (qpay[k].idx & F_EXIT));
                                if (eb) {
                                    stop = r0 + (uint32_t)__ffsll((unsigned long long)eb) - 1;
                                    break;
                                }
                            }
                            end = stop;
                        }
                        int le = -1;  // last exit inside the bulk part
                        for (uint32_t k = pos + lane; k < end; k += 64) {
                            if (qpay[k].idx & F_EXIT) le = (int)k;
                            else {
                                qd[k] = bst == 0 ? D_PASS : D_BLOCK_DEGRADE;
                                qw[k] = 0;
                            }
                        }
#pragma unroll
                        for (int o = 1; o < 64; o <<= 1) le = max(le, __shfl_xor(le, o, 64));
                        __syncthreads();
                        if (lane == 0) {
                            if (le >= 0) {  // the breaker's window as the scan left it after the bulk part
                                lcbs[0].st_start = qrank_ws[le];
                                lcbs[0].st_bad = sbad[le];
                                lcbs[0].st_total = stot[le];
                            }
                            auto step = [&](uint32_t k) {
                                const Payload q = qpay[k];
                                const int64_t t = ts_base + (int64_t)q.ts_off;
                                if (q.idx & F_EXIT) {
                                    if (R.n_cbs == 1) cb_on_complete_ws(lcbs[0], t, qrank_ws[k], qrt[k], (q.idx & F_ERROR) != 0);
                                    else
                                        for (uint32_t b = 0; b < R.n_cbs; ++b)
                                            cb_on_complete(lcbs[b], t, qrt[k], (q.idx & F_ERROR) != 0);
                                } else {  // DegradeSlot (a block's wait_ms: the breaker's index)
                                    const int kb = degrade_block_index(lcbs, R.n_cbs, t);
                                    qd[k] = kb < 0 ? D_PASS : D_BLOCK_DEGRADE;
                                    qw[k] = kb < 0 ? 0 : kb;
                                }
                            };
                            uint32_t k = end;
                            if (seq_rest) {
                                for (; k < cnt; ++k) step(k);
                            } else if (k < cnt) {  // the event that ended the bulk part (a HALF_OPEN
                                                   // stretch after it is the next bulk part)
                                step(k++);
                            }
                            bulk_end = (int)k;
                        }
                        __syncthreads();
                        pos = (uint32_t)bulk_end;
                    }
                } else {
                    for (uint32_t k = lane; k < cnt; k += 64) {
                        if (qpay[k].idx & F_EXIT) continue;
                        if (qpre[k] == 2) {  // ParamFlowException
                            qd[k] = D_BLOCK_PARAM;
                            qw[k] = 0;
                        } else {  // passed (or the rule does not apply: no argument)
                            qd[k] = D_PASS;
                            qw[k] = qpre[k] == 1 ? qpw[k] : 0;
                        }
                    }
                }
                __syncthreads();
                // s: pass acquire, block acquire, success, rt sum, exceptions, thread delta (uniform
                // over the lanes; lane 0 applies them)
                int64_t cur = INT64_MIN, tf = 0, s[6] = {0, 0, 0, 0, 0, 0}, rt_min = INT64_MAX;
                // per-lane partial sums of the current bucket run, reduced (DPP) only when the run
                // ends or a round crosses a bucket boundary
                int64_t lv[6] = {0, 0, 0, 0, 0, 0}, lmn = INT64_MAX;
                auto fold = [&]() {
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        s[i] += readlane_i64(wave_incl_sum_i64(lv[i]), 63);
                        lv[i] = 0;
                    }
                    const int64_t mn = readlane_i64(wave_incl_min_i64(lmn), 63);
                    if (mn < rt_min) rt_min = mn;
                    lmn = INT64_MAX;
                };
                bool any = false;
                auto flush = [&]() {
                    if (!any || lane != 0) return;
                    int64_t *b = sec_current(lnode, tf, max_rt);
                    int64_t *bm = min_current(lnode, tf, max_rt);
                    int64_t *bs[2] = {b, bm};
                    for (int u = 0; u < 2; ++u) {
                        int64_t *x = bs[u];
                        if (!x) continue;
                        x[MB_PASS] += s[0];
                        x[MB_BLOCK] += s[1];
                        x[MB_SUCC] += s[2];
                        x[MB_RT] += s[3];
                        if (rt_min < x[MB_MINRT]) x[MB_MINRT] = rt_min;
                        x[MB_EXC] += s[4];
                    }
                    lnode[kNodeThreads] += s[5];
                };
                auto open = [&](uint32_t k) {  // a new bucket run starts at event k
                    fold();
                    flush();
                    cur = qbq[k];
                    tf = ts_base + (int64_t)qpay[k].ts_off;
                    for (int i = 0; i < 6; ++i) s[i] = 0;
                    rt_min = INT64_MAX;
                    any = true;
                };
                auto contrib = [&](uint32_t k, int64_t *v, int64_t &mn) {
                    const Payload q = qpay[k];
                    const int64_t a = (int64_t)(int)(q.acq_prio & 0x7FFFFFFFu);
                    if (q.idx & F_EXIT) {  // chain_exit
                        v[2] += a;
                        v[3] += qrt[k];
                        if (qrt[k] < mn) mn = qrt[k];
                        if (q.idx & F_ERROR) v[4] += a;
                        v[5] -= 1;
                    } else if (qd[k] == D_PASS) {
                        v[0] += a;
                        v[5] += 1;
                    } else {
                        v[1] += a;
                    }
                };
                for (uint32_t r0 = 0; r0 < cnt; r0 += 64) {
                    const uint32_t k = r0 + lane;
                    const bool valid = k < cnt;
                    const int64_t b0 = qbq[r0];
                    if (__all(!valid || qbq[k] == b0)) {  // one bucket over the round: a wave reduction
                        if (b0 != cur) open(r0);
                        if (valid) contrib(k, lv, lmn);
                    } else {  // a bucket boundary inside the round: event by event (uniform)
                        fold();
                        const uint32_t e = min(cnt, r0 + 64);
                        for (uint32_t j = r0; j < e; ++j) {
                            if (qbq[j] != cur) open(j);
                            contrib(j, s, rt_min);
                        }
                    }
                }
                fold();
                flush();
            }
            if (!agg && threadIdx.x == 0) {
                Ctx cc = c;
                cc.res = &R;
                for (uint32_t k = 0; k < cnt; ++k) {
                    const Payload q = qpay[k];
                    const int64_t t = ts_base + (int64_t)q.ts_off;
                    const bool hp = (q.idx & F_PARAM) != 0;
                    if (q.idx & F_EXIT) {
                        chain_exit(cc, res, m, t, qrt[k], (int)(q.acq_prio & 0x7FFFFFFFu), (q.idx & F_ERROR) != 0, hp,
                                   qpv[k], PArgs{nullptr, 0}, q.idx & F_IDX);
                    } else {
                        int64_t w = 0;
                        cc.pentry = (cache_p && qslot[k] != 0xFFFF) ? &lent[qslot[k]] : nullptr;
                        cc.pstamp_ref = cc.pentry ? &lst[qslot[k]] : nullptr;
                        cc.pre_param = 0;  // not aggregated: lane 0 decides everything
                        cc.pre_wait = 0;
                        qd[k] = chain_entry(cc, res, m, t, (int)(q.acq_prio & 0x7FFFFFFFu), (q.acq_prio >> 31) != 0,
                                            hp, qpv[k], &w, PArgs{nullptr, 0}, q.idx & F_IDX);
                        qw[k] = (int32_t)w;
                    }
                }
            }
            __syncthreads();
            tick(3);
            if (cache_p) {  // write the chunk's entries back, free the slots
                // (with the keys' stamps and the owners' present counts: free mode, many lanes per owner)
                int pd = 0, td = 0;
                for (int k = threadIdx.x; k < kHeavySlots; k += 64) {
                    if (lval[k] != kLEmpty) {
                        if (lgi[k] < kGiFail) {
                            PEntry *e = st.ptab + lgi[k];
                            e->a = lent[k].a;
                            e->b = lent[k].b;
                            pd += (lent[k].a != kPAbsent ? 1 : 0) - (int)lp0[k];
                            if (lst[k] && st.pstamp) st.pstamp[lgi[k]] = lst[k];
                        }
                        if (par_ok && tgi[k] < kGiFail) {
                            st.ttab[tgi[k]].a = tent[k].a;
                            td += (tent[k].a != kPAbsent ? 1 : 0) - (int)tp0[k];
                            if (tst[k] && st.tstamp) st.tstamp[tgi[k]] = tst[k];
                        }
                        lval[k] = kLEmpty;
                    }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    pd += __shfl_xor(pd, o, 64);
                    td += __shfl_xor(td, o, 64);
                }
                if (threadIdx.x == 0) {
                    if (pd && st.psize) atomicAdd(&st.psize[cache_p->id], (uint32_t)pd);
                    if (td && lru_on_t(st, res)) atomicAdd(&st.tsize[st.tbase[res]], (uint32_t)td);
                }
            }
            for (uint32_t k = threadIdx.x; k < cnt; k += 64) {
                const Payload q = qpay[k];
                if (!(q.idx & F_EXIT)) {
                    decision[q.idx & F_IDX] = qd[k];
                    wait_ms[q.idx & F_IDX] = qw[k];
                }
            }
            __syncthreads();
            tick(4);
        }
        if (prof && threadIdx.x == 0) {
            for (int i = 0; i < 5; ++i) prof[blockIdx.x * 8 + i] += tk[i];
            prof[blockIdx.x * 8 + 6] += tk[6];
            prof[blockIdx.x * 8 + 7] += tk[7];
            prof[blockIdx.x * 8 + 5] += je - jb;
        }
        for (uint32_t r = r0 + threadIdx.x; r < r1; r += 64) sc.run_mode[r] = RUN_DONE;
        __syncthreads();
        for (int k = threadIdx.x; k < kNodeWords; k += 64) g.node[k] = lnode[k];
        if (lr)
            for (uint32_t k = threadIdx.x; k < R.n_rules; k += 64) g.rules[k] = lrules[k];
        if (lc)
            for (uint32_t k = threadIdx.x; k < R.n_cbs; k += 64) g.cbs[k] = lcbs[k];
        __syncthreads();
    }
}

// Resources with a CacheMap in LRU mode (k_lflows lists them): one lane each replays the resource's events
// in arrival order, every map access keeping its owner's recency queue (eviction at capacity).
__global__ __launch_bounds__(64) void k_llru(FlowState st, int64_t max_rt, FlowScratch sc,
                                             const Payload *__restrict__ pay, int64_t ts_base,
                                             const int64_t *__restrict__ rt_in, const uint64_t *__restrict__ param_in,
                                             int8_t *decision, int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const Ctx c{st, max_rt};
    const uint32_t nl = sc.counters[10], nflows = sc.counters[2], nruns = sc.counters[1];
    for (uint32_t i = blockIdx.x * 64 + threadIdx.x; i < nl; i += gridDim.x * 64) {
        const uint32_t fl = sc.lru[i];
        if (fl & 0x80000000u) continue;  // k_llru_ps (parameter-only, chunked)
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t res = sc.run_slot[r0];
        for (uint32_t j = sc.run_start[r0]; j < sc.run_end[r1 - 1]; ++j) {
            const Payload q = pay[j];
            const uint64_t tp = g_lru_prof_on ? wall_clock64() : 0;
            replay_event<true>(c, sc, res, q, ts_base, rt_in, param_in, decision, wait_ms);
            if (tp) atomicAdd(&g_lru_prof[(q.idx & F_EXIT) ? 7 : 6], (unsigned long long)(wall_clock64() - tp));
        }
        for (uint32_t r = r0; r < r1; ++r) sc.run_mode[r] = RUN_DONE;
    }
}

// ---- LRU-mode parameter-only resources, chunked through LDS (k_llru_ps)
// A parameter-only resource (pseg_take's conditions: one QPS-grade ParamFlowRule of argument index 0, no
// FlowRule, no breaker, only the index-0 thread-count map) whose maps are in LRU mode replays its events in
// arrival order with k_llru's results, but a few global round trips per chunk of 64 events instead of ~25
// per event: the lanes load the events, find (or create) each distinct value's entry in the map and the next
// kPsPre records of its LRU queue with their keys' state (registers), the LRU order is replayed on
// wave-uniform bit masks, the token checks run lane-parallel (k_llru_ps below).  Decisions never read the
// node (as for pseg), so the node statistics go in aggregate, run by run.  k_lflows flags these flows in
// sc.lru (kLruPs).
// SGA_LRU_PROF=1 (diagnostics only): k_llru_ps ticks per phase of wave 0, summed over chunks: [0] events [1]
// loads + dedupe [2] leader entries [3] queue records [4] LRU scan [5] rounds [6] write-back [20] queue
// compaction and pushes [7] chunks; [8..15]
// queue pops per map; [16 + wave] the longest resource, [18 + wave] its busiest wave's ticks
__device__ unsigned long long g_lps_prof[22];

__device__ __forceinline__ uint32_t rl32(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}
__device__ __forceinline__ uint64_t rl64(uint64_t x, uint32_t l) {
    return (uint64_t)rl32((uint32_t)x, l) | ((uint64_t)rl32((uint32_t)(x >> 32), l) << 32);
}
// lane l's copy of reg becomes v (v and l wave-uniform)
__device__ __forceinline__ uint32_t wl32(uint32_t reg, uint32_t v, uint32_t l) { return __lane_id() == l ? v : reg; }
__device__ __forceinline__ uint64_t wl64(uint64_t reg, uint64_t v, uint32_t l) { return __lane_id() == l ? v : reg; }
// the entry of (owner, value) if present in the table, its home slot loaded first (the tables stay a quarter
// full, so most keys sit there); kN lookups of one lane issued together
template <int kN>
__device__ __forceinline__ void ptab_find_n(PEntry *tab, uint32_t mask, uint32_t owner, const uint64_t (&v)[kN],
                                            const bool (&want)[kN], PEntry *(&out)[kN], uint32_t *overflow) {
    uint32_t ow[kN];
    uint64_t vv[kN];
#pragma unroll
    for (int i = 0; i < kN; ++i) {
        const uint32_t h = ptab_home(mask, owner, v[i]);
        ow[i] = want[i] ? __hip_atomic_load(&tab[h].owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        vv[i] = want[i] ? tab[h].value : 0ull;
    }
#pragma unroll
    for (int i = 0; i < kN; ++i) {
        if (!want[i] || ow[i] == 0) {
            out[i] = nullptr;
        } else if (ow[i] == owner && vv[i] == v[i]) {
            out[i] = &tab[ptab_home(mask, owner, v[i])];
        } else {
            out[i] = ptab_get(tab, mask, owner, v[i], false, overflow);
        }
    }
}

// ptab_find_n with the entry's `a` and its stamp: the home slot's words are loaded together with its owner and
// value, so a key at its home slot costs one round trip
template <int kN>
__device__ __forceinline__ void ptab_peek_n(PEntry *tab, const uint64_t *tstamp, uint32_t mask, uint32_t owner,
                                            const uint64_t (&v)[kN], const bool (&want)[kN], uint32_t (&slot)[kN],
                                            int64_t (&a)[kN], uint64_t (&ts)[kN], uint32_t *overflow) {
    uint32_t h[kN], ow[kN];
    uint64_t vv[kN];
#pragma unroll
    for (int i = 0; i < kN; ++i) {
        h[i] = ptab_home(mask, owner, v[i]);
        ow[i] = want[i] ? __hip_atomic_load(&tab[h[i]].owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        vv[i] = want[i] ? tab[h[i]].value : 0ull;
        a[i] = want[i] ? ps_ld(&tab[h[i]].a) : kPAbsent;
        ts[i] = want[i] ? ps_ldu(&tstamp[h[i]]) : 0ull;
    }
#pragma unroll
    for (int i = 0; i < kN; ++i) {
        if (!want[i] || ow[i] == 0) {
            slot[i] = 0xFFFFFFFFu;
        } else if (ow[i] == owner && vv[i] == v[i]) {
            slot[i] = h[i];
        } else {
            PEntry *e = ptab_get(tab, mask, owner, v[i], false, overflow);
            slot[i] = e ? (uint32_t)(e - tab) : 0xFFFFFFFFu;
            a[i] = e ? ps_ld(&e->a) : kPAbsent;
            ts[i] = e ? ps_ldu(&tstamp[slot[i]]) : 0ull;
        }
    }
}

// the chunk's leader slots, slot -> leader lane (open addressing in LDS)
constexpr int kPsHash = 256;
__device__ __forceinline__ void ps_hash_put(uint32_t *keys, uint8_t *vals, uint32_t slot, uint32_t lane) {
    uint32_t h = (slot * 2654435761u) >> 24;
    for (;;) {
        const uint32_t prev = atomicCAS(&keys[h], 0xFFFFFFFFu, slot);
        if (prev == 0xFFFFFFFFu || prev == slot) {
            vals[h] = (uint8_t)lane;
            return;
        }
        h = (h + 1) & (kPsHash - 1);
    }
}
__device__ __forceinline__ int ps_hash_get(const uint32_t *keys, const uint8_t *vals, uint32_t slot) {
    uint32_t h = (slot * 2654435761u) >> 24;
    for (;;) {
        const uint32_t k = keys[h];
        if (k == slot) return vals[h];
        if (k == 0xFFFFFFFFu) return -1;
        h = (h + 1) & (kPsHash - 1);
    }
}

// wave-local barrier: the wave's LDS and global writes visible to its other lanes (the workgroup shares
// the CU's L1, so workgroup scope is enough: no other workgroup reads an owner's keys or queue)
__device__ __forceinline__ void ps_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// a wave-uniform value the compiler cannot prove uniform (an atomic load's result): readfirstlane
__device__ __forceinline__ uint32_t ps_uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t ps_uni64(uint64_t x) {
    return (uint64_t)ps_uni32((uint32_t)x) | ((uint64_t)ps_uni32((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ int64_t ps_wave_sum(int64_t x) { return wave_sum_i64(x); }
__device__ __forceinline__ uint32_t ps_wave_max(uint32_t x) { return wave_max_u32(x); }

// Two waves per resource, one chunk apart: wave 0 decides chunk c (the time/token map, the decisions, the node
// statistics) while wave 1 applies chunk c - 1's thread counts (the thread-count map follows the decisions and
// the exits only), each on its own map, queue and LDS; the chunk's events and decisions pass through a double
// buffer.  Per chunk and map:
//  * the leaders' entries (one lane per distinct value) and the next kPsPre queue records with their keys'
//    state go to registers; a record is a candidate for eviction when its key is outside the chunk and live
//    (bit masks `live`), or is a chunk key whose pre-chunk stamp it carries (`link`: live while the key is
//    present and not yet accessed in the chunk);
//  * the LRU scan walks the chunk's accesses in arrival order on wave-uniform bit masks (present, accessed,
//    inserted-absent, evicted): an insert into a full map pops the first candidate (k_llru's lru_evict);
//  * wave 0 then runs the token-bucket / throttle checks lane-parallel in rounds (round r: each value's r-th
//    event, its state in LDS, reset where the scan saw the value absent), wave 1 kept the thread counts in the
//    scan (a count reaching zero removes the key);
//  * the queue's pushes are the accesses in arrival order (one per accessing lane), the copies, the evictions
//    and the last access stamps go back, and the node statistics go in aggregate, run by run.
__global__ __launch_bounds__(128) void k_llru_ps(FlowState st, int64_t max_rt, FlowScratch sc,
                                                 const Payload *__restrict__ pay, int64_t ts_base,
                                                 const uint64_t *__restrict__ param_in, int8_t *decision,
                                                 int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    static_assert(kPsPre == 128, "two loaded queue records per lane");
    __shared__ uint32_t s_hk[2][kPsHash];
    __shared__ uint8_t s_hv[2][kPsHash];
    __shared__ uint8_t s_hasent[64];
    __shared__ uint32_t s_last[2][64];  // per leader lane: 1 + the lane of its value's last access in the chunk
    __shared__ int64_t s_ra[64], s_rb[64];  // wave 0's rounds: each value's (a, b) at its leader's index
    __shared__ int64_t s_tc[64];            // wave 1's rounds: each value's thread count
    __shared__ uint32_t s_first[2][64];     // per leader lane: the lane of its value's first access (64: none)
    __shared__ uint64_t s_dk[128], s_dm[128];  // wave 0's value hash: key, lane mask
    __shared__ uint32_t s_dt[128];             // claim tags
    // chunk handoff (wave 0 -> wave 1): per event flags (bit0 exit, bit1 parameter, bit2 passed), leader,
    // rank among its value's events, request index, value
    __shared__ uint8_t s_bfl[2][64], s_blead[2][64], s_bocc[2][64];
    __shared__ uint32_t s_bidx[2][64];
    __shared__ uint64_t s_bval[2][64];
    // the wave index through readfirstlane: wave-uniform to the compiler, so every branch on the map (and on
    // the masks and counters derived from it) is a scalar branch, not an exec-masked one
    const uint32_t lane = threadIdx.x & 63, wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const Ctx c{st, max_rt};
    const uint32_t nl = sc.counters[10], nflows = sc.counters[2], nruns = sc.counters[1];
    const bool prof = g_lru_prof_on != 0;
    for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
        const uint32_t flx = sc.lru[i];
        if (!(flx & kLruPs)) continue;
        const uint32_t fl = flx & ~kLruPs;
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t res = sc.run_slot[r0];
        const ParamRuleDev p = st.prules[st.res[res].prule_off];
        const uint32_t tj = st.tbase[res];
        const uint32_t jb = sc.run_start[r0], je = sc.run_end[r1 - 1];
        int64_t *node = st.node + (size_t)res * kNodeWords;
        // this wave's map: 0 the rule's time/token map, 1 the index-0 thread-count map
        const int m = (int)wave;
        const uint32_t own = m == 0 ? p.id + 1 : tmap_owner(res, 0);
        PEntry *const tab = m == 0 ? st.ptab : st.ttab;
        const uint32_t tmask = m == 0 ? st.pmask : st.tmask;
        uint64_t *const tstamp = m == 0 ? st.pstamp : st.tstamp;
        const uint64_t qo = m == 0 ? st.pq[p.id] : st.tq[tj];
        LruRec *const area = qo == kNoQueue ? nullptr : st.lpool + qo;
        const uint64_t qcap = 2ull * (m == 0 ? p.cap : (uint32_t)kThreadMapCap) + 2;
        uint64_t head = ps_uni64(area ? ps_ldu(&area[0].value) : 0), tail = ps_uni64(area ? ps_ldu(&area[0].stamp) : 0);
        // the ring positions of head and tail, kept incrementally (no 64-bit division per lane)
        uint32_t hq = area ? (uint32_t)(head % qcap) : 0u, tq = area ? (uint32_t)(tail % qcap) : 0u;
        const uint32_t qc32 = (uint32_t)qcap;
        uint32_t size = ps_uni32(m == 0 ? st.psize[p.id] : st.tsize[tj]);
        const uint32_t cap = m == 0 ? p.cap : (uint32_t)kThreadMapCap;
        uint32_t *const hk = s_hk[m];
        uint8_t *const hv = s_hv[m];
        uint32_t cur_run = 0xFFFFFFFFu;
        int64_t pa = 0, ba = 0, np = 0, thr = 0;
        auto apply_run = [&](uint32_t r) __attribute__((always_inline)) {  // wave 0, lane 0
            const int64_t tf = ts_base + (int64_t)sc.run_t0off[r];
            int64_t *bs[2] = {sec_current(node, tf, max_rt), min_current(node, tf, max_rt)};
            const int64_t exc = (int64_t)sc.run_exc[r], exerr = (int64_t)sc.run_exerr[r];
            const int64_t exrt = sc.run_exrt[r], exmin = sc.run_exmin[r];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                int64_t *b = bs[k];
                if (!b) continue;
                b[MB_PASS] += pa;
                b[MB_BLOCK] += ba;
                b[MB_SUCC] += exc;
                b[MB_RT] += exrt;
                b[MB_EXC] += exerr;
                if (exmin < b[MB_MINRT]) b[MB_MINRT] = exmin;
            }
            thr += np - (int64_t)sc.run_nexit[r];
        };
        uint64_t tp = prof ? wall_clock64() : 0;
        auto mark = [&](int ph) __attribute__((always_inline)) {
            if (!prof) return;
            const uint64_t now = wall_clock64();
            if (lane == 0 && wave == 0) atomicAdd(&g_lps_prof[ph], (unsigned long long)(now - tp));
            tp = now;
        };
        const uint32_t nch = (je - jb + 63) / 64;
        uint64_t n_pop = 0, n_gpop = 0, n_evict = 0, n_acc = 0, busy = 0;  // diagnostics (SGA_LRU_PROF)
        const uint64_t t_res = prof ? wall_clock64() : 0;
        Payload nq{0, 0, 0, 0};  // wave 0: the next chunk's events, loaded during this chunk's LRU scan
        uint32_t nrun = 0;
        for (uint32_t step = 0; step <= nch; ++step) {
            // wave 0: chunk `step`; wave 1: chunk step - 1
            const bool work = wave == 0 ? step < nch : step >= 1;
            const uint32_t ch = wave == 0 ? step : step - 1, bsel = ch & 1;
            if (work) {
                const uint32_t c0 = jb + ch * 64, nk = min(64u, je - c0);
                if (prof && lane == 0 && wave == 0) {
                    atomicAdd(&g_lps_prof[0], (unsigned long long)nk);
                    atomicAdd(&g_lps_prof[7], 1ull);
                }
                tp = prof ? wall_clock64() : 0;
                const uint64_t t_step = tp;
                // 1. the chunk's events (lane k: event k); wave 0 loads them and hands them over
                const bool act = lane < nk;
                uint32_t e_fl, e_lead, e_idx, e_occ = 0;
                uint64_t v;
                uint32_t e_run = 0;
                int64_t e_t = 0;
                int32_t e_acq = 0;
                if (wave == 0) {
                    const uint32_t j = c0 + lane;
                    const Payload q = ch == 0 ? (act ? pay[j] : Payload{0, 0, 0, 0}) : nq;
                    const bool ex = (q.idx & F_EXIT) != 0, hp = act && (q.idx & F_PARAM) != 0;
                    v = hp ? param_in[q.idx & F_IDX] : 0;
                    e_fl = (ex ? 1u : 0u) | (hp ? 2u : 0u);
                    e_idx = q.idx & F_IDX;
                    e_run = ch == 0 ? (act ? sc.ev_run[j] : 0u) : nrun;
                    e_t = ts_base + (int64_t)q.ts_off;
                    e_acq = (int32_t)(q.acq_prio & 0x7FFFFFFFu);
                    // distinct values: the lowest lane of each value leads it; e_occ = the event's rank among
                    // its value's events in the chunk
                    // (an LDS hash of the chunk's values: a claim per slot, then each value's lane mask)
                    s_dt[lane] = 0;
                    s_dt[lane + 64] = 0;
                    s_dm[lane] = 0;
                    s_dm[lane + 64] = 0;
                    ps_wave_sync();
                    uint32_t h = (uint32_t)((v * 0x9E3779B97F4A7C15ull) >> 57);
                    bool done = !hp;
                    while (__ballot(!done)) {
                        if (!done && atomicCAS(&s_dt[h], 0u, lane + 1u) == 0u) s_dk[h] = v;
                        ps_wave_sync();
                        if (!done) {
                            if (s_dk[h] == v) done = true;
                            else h = (h + 1u) & 127u;
                        }
                    }
                    if (hp) atomicOr(&s_dm[h], 1ull << lane);
                    ps_wave_sync();
                    const uint64_t same = hp ? s_dm[h] : 0ull;
                    const uint32_t lead = hp ? (uint32_t)__builtin_ctzll(same) : 64u;
                    e_occ = (uint32_t)__popcll(same & lt_mask);
                    e_lead = lead;
                    s_hasent[lane] = 0;
                    ps_wave_sync();
                    if (hp && !ex) s_hasent[lead] = 1;  // the value's time/token entry is needed only by entries
                    s_bfl[bsel][lane] = (uint8_t)e_fl;
                    s_blead[bsel][lane] = (uint8_t)e_lead;
                    s_bocc[bsel][lane] = (uint8_t)e_occ;
                    s_bidx[bsel][lane] = e_idx;
                    s_bval[bsel][lane] = v;
                } else {
                    e_fl = s_bfl[bsel][lane];
                    e_lead = s_blead[bsel][lane];
                    e_occ = s_bocc[bsel][lane];
                    e_idx = s_bidx[bsel][lane];
                    v = s_bval[bsel][lane];
                }
                for (uint32_t k = lane; k < (uint32_t)kPsHash; k += 64) hk[k] = 0xFFFFFFFFu;
                s_last[m][lane] = 0;
                s_first[m][lane] = 64;
                ps_wave_sync();
                const bool hp = (e_fl & 2u) != 0;
                const bool leader = hp && e_lead == lane;
                const uint64_t my_stamp = lru_stamp(st, e_idx, 0);
                mark(1);
                // 2. the leaders' entries of this wave's map (created, as chain_entry's ptab_get would), kept in
                //    their lanes
                uint32_t c_slot = 0xFFFFFFFFu;
                uint64_t c_st = 0;
                int64_t c_a = kPAbsent, c_b = kPAbsent;
                const bool need = leader && (m == 1 || s_hasent[lane]);
                if (need) {  // the home slot's words together (one round trip for a key at its home slot)
                    const uint32_t h = ptab_home(tmask, own, v);
                    const uint32_t oh = __hip_atomic_load(&tab[h].owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t vh = tab[h].value;
                    const int64_t ah = ps_ld(&tab[h].a), bh = ps_ld(&tab[h].b);
                    const uint64_t sh = ps_ldu(&tstamp[h]);
                    if (oh == own && vh == v) {
                        c_slot = h;
                        c_a = ah;
                        c_b = bh;
                        c_st = sh;
                    } else if (PEntry *e = ptab_get(tab, tmask, own, v, true, st.overflow)) {
                        c_slot = (uint32_t)(e - tab);
                        c_a = ps_ld(&e->a);
                        c_b = ps_ld(&e->b);
                        c_st = ps_ldu(&tstamp[c_slot]);
                    }
                    if (c_slot != 0xFFFFFFFFu) ps_hash_put(hk, hv, c_slot, lane);
                }
                const bool any = __ballot(need) != 0ull;  // this map is touched in the chunk
                // the slot of this event's value (valid only for a parameter event whose entry exists)
                const uint32_t l_slot = (uint32_t)__shfl((int)c_slot, hp ? (int)e_lead : 0, 64);
                const bool slot_ok = hp && l_slot != 0xFFFFFFFFu;
                ps_wave_sync();
                mark(2);
                // 3. the next kPsPre records of the queue (record r * 64 + lane in this lane) with their keys'
                //    state: candidates outside the chunk (live*) and chunk keys' pre-chunk records (link*)
                head = ps_uni64(head);
                tail = ps_uni64(tail);
                size = ps_uni32(size);
                const uint32_t npre = ps_uni32((area && any) ? (uint32_t)min<uint64_t>(kPsPre, tail - head) : 0u);
                uint32_t rslot0 = 0xFFFFFFFFu, rslot1 = 0xFFFFFFFFu, rlink0 = 0, rlink1 = 0;
                uint64_t live0 = 0, live1 = 0, link0 = 0, link1 = 0;
                {
                    uint64_t rv[2], rs[2];
                    bool want[2];
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const uint32_t k = (uint32_t)r * 64 + lane;
                        want[r] = k < npre;
                        const uint32_t ix = hq + k;  // k < npre <= tail - head <= qcap
                        const LruRec *rp = want[r] ? &area[1 + (ix >= qc32 ? ix - qc32 : ix)] : nullptr;
                        rv[r] = want[r] ? ps_ldu(&rp->value) : 0ull;
                        rs[r] = want[r] ? ps_ldu(&rp->stamp) : 0ull;
                    }
                    uint32_t eslot[2];
                    int64_t ea[2];
                    uint64_t ets[2];
                    ptab_peek_n<2>(tab, tstamp, tmask, own, rv, want, eslot, ea, ets, st.overflow);
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const uint32_t slot = eslot[r];
                        const bool gp = slot != 0xFFFFFFFFu && ea[r] != kPAbsent;
                        const uint64_t gs = ets[r];
                        const int link = slot != 0xFFFFFFFFu ? ps_hash_get(hk, hv, slot) : -1;
                        const uint64_t lst = (uint64_t)__shfl((long long)c_st, link >= 0 ? link : 0, 64);
                        const bool lv = want[r] && link < 0 && gp && gs == rs[r];
                        const bool lk = want[r] && link >= 0 && lst == rs[r];
                        if (r == 0) {
                            rslot0 = slot;
                            rlink0 = (uint32_t)max(link, 0);
                            live0 = __ballot(lv);
                            link0 = __ballot(lk);
                        } else {
                            rslot1 = slot;
                            rlink1 = (uint32_t)max(link, 0);
                            live1 = __ballot(lv);
                            link1 = __ballot(lk);
                        }
                    }
                }
                if (wave == 0 && ch + 1 < nch) {  // the next chunk's events (in flight through steps 4-6)
                    const uint32_t jn = c0 + 64 + lane;
                    nq = jn < je ? pay[jn] : Payload{0, 0, 0, 0};
                    nrun = jn < je ? sc.ev_run[jn] : 0u;
                }
                mark(3);
                // 4. the LRU scan: the chunk's accesses in arrival order on wave-uniform masks (bit L: leader L)
                int32_t tdel = 0;  // wave 1: this event's thread-count change
                uint64_t acc;
                const ParamPre e_pre = m == 0 && hp ? param_pre(c, p, v, e_acq) : ParamPre{0, 0};
                if (m == 0) {
                    acc = __ballot(act && !(e_fl & 1u) && slot_ok && param_pre_access(p, e_pre, e_acq));
                } else {
                    tdel = slot_ok ? ((e_fl & 1u) ? -1 : ((e_fl & 4u) ? 1 : 0)) : 0;
                    acc = __ballot(act && tdel != 0);
                }
                uint64_t present = __ballot(c_slot != 0xFFFFFFFFu && c_a != kPAbsent);
                uint64_t touched = 0, reset = 0, evl = 0, evnc0 = 0, evnc1 = 0;
                uint32_t used = 0, nev = 0, ev_slot = 0;
                auto evict = [&]() __attribute__((always_inline)) {
                    n_evict += 1;
                    for (;;) {
                        if (used < npre) {  // the first candidate at or past `used`
                            const uint64_t c0m = used < 64 ? (live0 | link0) & (~0ull << used) : 0ull;
                            const uint64_t c1m = (live1 | link1) & (used < 64 ? ~0ull : (~0ull << (used - 64)));
                            if (!c0m && !c1m) {
                                n_pop += npre - used;
                                used = npre;
                                continue;
                            }
                            const uint32_t idx = c0m ? (uint32_t)__builtin_ctzll(c0m) : 64u + (uint32_t)__builtin_ctzll(c1m);
                            n_pop += idx + 1 - used;
                            used = idx + 1;
                            const uint64_t bit = 1ull << (idx & 63);
                            if (idx < 64 ? (live0 & bit) : (live1 & bit)) {
                                if (idx < 64) evnc0 |= bit;
                                else evnc1 |= bit;
                                size -= 1;
                                return;
                            }
                            const uint32_t L = idx < 64 ? rl32(rlink0, idx) : rl32(rlink1, idx - 64);
                            const uint64_t bL = 1ull << L;
                            if (!(present & bL) || (touched & bL)) continue;
                            present &= ~bL;
                            evl |= bL;
                            if (m == 1) c_a = (int64_t)wl64((uint64_t)c_a, (uint64_t)kPAbsent, L);
                            size -= 1;
                            return;
                        } else if (head + used < tail) {  // past the loaded records: one global pop
                            n_gpop += 1;
                            n_pop += 1;
                            const LruRec *rp = &area[1 + (head + used) % qcap];
                            const uint64_t rv = ps_uni64(ps_ldu(&rp->value)), rs = ps_uni64(ps_ldu(&rp->stamp));
                            PEntry *e = ptab_get(tab, tmask, own, rv, false, st.overflow);
                            const uint32_t slot = ps_uni32(e ? (uint32_t)(e - tab) : 0xFFFFFFFFu);
                            const bool gp = ps_uni32(e && ps_ld(&e->a) != kPAbsent ? 1u : 0u) != 0;
                            const uint64_t gs = ps_uni64(e ? ps_ldu(&tstamp[slot]) : 0ull);
                            const uint64_t hit = __ballot(c_slot == slot && slot != 0xFFFFFFFFu);
                            used += 1;
                            if (hit) {
                                const uint32_t L = (uint32_t)__builtin_ctzll(hit);
                                const uint64_t bL = 1ull << L;
                                if (!(present & bL) || (touched & bL) || rl64(c_st, L) != rs) continue;
                                present &= ~bL;
                                evl |= bL;
                                if (m == 1) c_a = (int64_t)wl64((uint64_t)c_a, (uint64_t)kPAbsent, L);
                                size -= 1;
                                return;
                            }
                            if (slot == 0xFFFFFFFFu || !gp || gs != rs) continue;
                            ev_slot = wl32(ev_slot, slot, nev);
                            nev += 1;
                            size -= 1;
                            return;
                        } else {
                            if (lane == 0) {
                                atomicOr(&st.lru_ctl[1], 2u);  // a full map without a live record: never expected
                                atomicOr(st.overflow, 1u);
                            }
                            return;
                        }
                    }
                };
                // The fast path: in steady state the map is full, each insert evicts the first candidate, and the
                // chunk's keys sit near the queue's tail.  Inserts and removals come from each value's own events
                // (wave 1: its thread counts, lane-parallel in rounds), the number of evictions E from their order;
                // when the first E candidates are all outside the chunk, they are the evictions and no chunk key
                // was evicted, which is the scan's result.  Otherwise the sequential scan below.
                if ((acc >> lane) & 1ull) atomicMin(&s_first[m][e_lead], lane);
                ps_wave_sync();
                const bool first_acc = ((acc >> lane) & 1ull) && s_first[m][e_lead] == lane;
                const uint64_t acc_lead = __ballot(s_first[m][lane] < 64u);  // leaders whose value is accessed
                uint64_t ins;
                uint32_t n_evf = 0, size_f = size;
                int64_t t_cnt = c_a;
                if (m == 0) {
                    ins = __ballot(first_acc && !((present >> e_lead) & 1ull));
                    const uint32_t ni = (uint32_t)__popcll(ins);
                    n_evf = !area ? 0u : (size >= cap ? ni : (ni > cap - size ? ni - (cap - size) : 0u));
                    size_f = size + ni - n_evf;
                } else {
                    if (leader) s_tc[lane] = c_a;
                    const bool ta_me = (acc >> lane) & 1ull;
                    const uint32_t nr = ps_wave_max(ta_me ? e_occ + 1 : 0u);
                    bool my_ins = false, my_rem = false;
                    ps_wave_sync();
                    for (uint32_t r = 0; r < nr; ++r) {
                        if (ta_me && e_occ == r) {
                            int64_t cnt = s_tc[e_lead];
                            if (cnt == kPAbsent) {
                                my_ins = true;
                                cnt = tdel > 0 ? 1 : 0;
                            } else {
                                cnt += tdel;
                                if (tdel < 0 && cnt <= 0) {
                                    my_rem = true;
                                    cnt = kPAbsent;
                                }
                            }
                            s_tc[e_lead] = cnt;
                        }
                        ps_wave_sync();
                    }
                    ins = __ballot(my_ins);
                    const uint64_t rem = __ballot(my_rem);
                    uint32_t sz = size;
                    for (uint64_t am = ins | rem; am; am &= am - 1ull) {
                        if ((ins >> __builtin_ctzll(am)) & 1ull) {
                            sz += 1;
                            if (area && sz > cap) {
                                sz -= 1;
                                n_evf += 1;
                            }
                        } else {
                            sz -= 1;
                        }
                    }
                    size_f = sz;
                    t_cnt = s_tc[lane];
                }
                const uint64_t cand0 = live0 | link0, cand1 = live1 | link1;
                const uint32_t pc0 = (uint32_t)__popcll(cand0), pc1 = (uint32_t)__popcll(cand1);
                const uint64_t sel0 = __ballot(n_evf != 0 && n_evf <= pc0 && ((cand0 >> lane) & 1ull) &&
                                               (uint32_t)__popcll(cand0 & lt_mask) == n_evf - 1);
                const uint64_t sel1 = __ballot(n_evf > pc0 && n_evf - pc0 <= pc1 && ((cand1 >> lane) & 1ull) &&
                                               (uint32_t)__popcll(cand1 & lt_mask) == n_evf - pc0 - 1);
                uint64_t fm0 = 0, fm1 = 0;  // the consumed records: bits up to the n_evf-th candidate
                bool fast = n_evf == 0;
                if (sel0) {
                    const uint32_t pos = (uint32_t)__builtin_ctzll(sel0);
                    fm0 = pos == 63 ? ~0ull : (2ull << pos) - 1ull;
                    fast = true;
                } else if (sel1) {
                    const uint32_t pos = (uint32_t)__builtin_ctzll(sel1);
                    fm0 = ~0ull;
                    fm1 = pos == 63 ? ~0ull : (2ull << pos) - 1ull;
                    fast = true;
                }
                fast = fast && !(link0 & fm0) && !(link1 & fm1);
                if (fast) {
                    evnc0 = live0 & fm0;
                    evnc1 = live1 & fm1;
                    used = (uint32_t)(__popcll(fm0) + __popcll(fm1));
                    size = size_f;
                    touched = acc_lead;
                    reset = ins;
                    if (m == 1 && leader) c_a = t_cnt;
                    n_evict += n_evf;
                    n_pop += used;
                }
                for (uint64_t am = fast ? 0ull : acc; am; am &= am - 1ull) {
                    const uint32_t k = (uint32_t)__builtin_ctzll(am);
                    const uint32_t L = rl32(e_lead, k);
                    const uint64_t bL = 1ull << L;
                    touched |= bL;
                    if (m == 0) {  // time map then token map, one recency order
                        if (!(present & bL)) {
                            present |= bL;
                            reset |= 1ull << k;
                            size += 1;
                            if (area && size > cap) evict();
                        }
                    } else {  // ParameterMetric.add / decreaseThreadCount of index 0 (param_threads)
                        const int64_t td = (int64_t)(int32_t)rl32((uint32_t)tdel, k);
                        const int64_t ta = (int64_t)rl64((uint64_t)c_a, L);
                        int64_t nt;
                        if (ta == kPAbsent) {
                            size += 1;
                            if (area && size > cap) evict();
                            nt = td > 0 ? 1 : 0;
                            present |= bL;
                        } else {
                            nt = ta + td;
                            if (td < 0 && nt <= 0) {
                                nt = kPAbsent;
                                size -= 1;
                                present &= ~bL;
                            }
                        }
                        c_a = (int64_t)wl64((uint64_t)c_a, (uint64_t)nt, L);
                    }
                }
                n_acc += (uint64_t)__popcll(acc);
                if ((acc >> lane) & 1ull) atomicMax(&s_last[m][e_lead], lane + 1);
                ps_wave_sync();
                mark(4);
                // 5. wave 0: the checks, lane-parallel in rounds of each value's events, and the decisions
                const bool ent = act && !(e_fl & 1u);
                int d = D_PASS;
                int64_t w = 0;
                if (m == 0) {
                    if (leader) {
                        s_ra[lane] = c_a;
                        s_rb[lane] = c_b;
                    }
                    const bool tok = ent && slot_ok;
                    if (ent && hp && !slot_ok) d = D_BLOCK_PARAM;  // the map is full: the batch fails (overflow)
                    const uint32_t nr = ps_wave_max(tok ? e_occ + 1 : 0u);
                    const bool rs_me = (reset >> lane) & 1ull;
                    ps_wave_sync();
                    for (uint32_t r = 0; r < nr; ++r) {
                        if (tok && e_occ == r) {
                            struct { int64_t a, b; } e{s_ra[e_lead], s_rb[e_lead]};
                            if (rs_me) e.a = e.b = kPAbsent;
                            if (!param_pass_pre(p, e, e_pre, e_acq, e_t, &w)) {
                                d = D_BLOCK_PARAM;
                                w = 0;  // a block's detail: the rule's index
                            }
                            s_ra[e_lead] = e.a;
                            s_rb[e_lead] = e.b;
                        }
                        ps_wave_sync();
                    }
                    if (ent) {
                        decision[e_idx] = (int8_t)d;
                        wait_ms[e_idx] = (int32_t)w;
                    }
                    s_bfl[bsel][lane] = (uint8_t)(e_fl | (ent && d == D_PASS ? 4u : 0u));
                    // the node statistics, run by run (a chunk's runs are consecutive lanes)
                    for (uint64_t rem = __ballot(act); rem;) {
                        const uint32_t r = rl32(e_run, (uint32_t)__builtin_ctzll(rem));
                        const bool inr = act && e_run == r;
                        rem &= ~__ballot(inr);
                        if (r != cur_run) {
                            if (cur_run != 0xFFFFFFFFu && lane == 0) apply_run(cur_run);
                            cur_run = r;
                            pa = ba = np = 0;
                        }
                        const bool ps_ = inr && ent && d == D_PASS, bk_ = inr && ent && d != D_PASS;
                        pa += ps_wave_sum(ps_ ? (int64_t)e_acq : 0);
                        ba += ps_wave_sum(bk_ ? (int64_t)e_acq : 0);
                        np += (int64_t)__popcll(__ballot(ps_));
                    }
                    if (leader) {
                        c_a = s_ra[lane];
                        c_b = s_rb[lane];
                    }
                }
                mark(5);
                // 6. write back: the copies (an evicted key not accessed since is absent), the evictions, then the
                //    queue's pushes (after a compaction when the ring would overflow: live records kept in order)
                const uint32_t last = s_last[m][lane];
                const uint64_t lst = (uint64_t)__shfl((long long)my_stamp, last ? (int)last - 1 : 0, 64);
                if (c_slot != 0xFFFFFFFFu) {
                    const uint64_t bme = 1ull << lane;
                    if (m == 0) {
                        const bool gone = (evl & bme) && !(touched & bme);
                        tab[c_slot].a = gone ? kPAbsent : c_a;
                        tab[c_slot].b = gone ? kPAbsent : c_b;
                    } else {
                        tab[c_slot].a = c_a;
                        if (evl & bme) tab[c_slot].b = kPAbsent;
                    }
                    tstamp[c_slot] = last ? lst : c_st;
                }
                if ((evnc0 >> lane) & 1ull) {
                    tab[rslot0].a = kPAbsent;
                    tab[rslot0].b = kPAbsent;
                }
                if ((evnc1 >> lane) & 1ull) {
                    tab[rslot1].a = kPAbsent;
                    tab[rslot1].b = kPAbsent;
                }
                if (lane < nev) {
                    tab[ev_slot].a = kPAbsent;
                    tab[ev_slot].b = kPAbsent;
                }
                ps_wave_sync();
                mark(6);
                if (area) {
                    uint64_t h = head + used, t = tail;
                    uint32_t npm = (uint32_t)__popcll(acc);
                    hq = ps_uni32(hq + used >= qc32 ? hq + used - qc32 : hq + used);  // used <= tail - head <= qcap
                    if (t - h + npm > qcap) {  // lru_compact over [h, t), 512 records per round (8 per lane)
                        constexpr int kC = 8;
                        auto ring = [&](uint64_t x) {  // x in [h, h + qcap]: its ring slot
                            const uint32_t r = hq + (uint32_t)(x - h);
                            return 1u + (r >= qc32 ? r - qc32 : r);
                        };
                        uint64_t wpos = h;
                        for (uint64_t b0 = h; b0 < t; b0 += 64 * kC) {
                            uint64_t rv[kC], rs[kC];
                            bool want[kC];
#pragma unroll
                            for (int u = 0; u < kC; ++u) {
                                const uint64_t ix = b0 + (uint64_t)(u * 64) + lane;
                                want[u] = ix < t;
                                const LruRec *rp = want[u] ? &area[ring(ix)] : nullptr;
                                rv[u] = want[u] ? ps_ldu(&rp->value) : 0ull;
                                rs[u] = want[u] ? ps_ldu(&rp->stamp) : 0ull;
                            }
                            uint32_t eslot[kC];
                            int64_t ea[kC];
                            uint64_t ets[kC];
                            ptab_peek_n<kC>(tab, tstamp, tmask, own, rv, want, eslot, ea, ets, st.overflow);
                            bool live[kC];
                            uint64_t bl[kC];
#pragma unroll
                            for (int u = 0; u < kC; ++u) {
                                live[u] = eslot[u] != 0xFFFFFFFFu && ea[u] != kPAbsent && ets[u] == rs[u];
                                bl[u] = __ballot(live[u]);
                            }
                            ps_wave_sync();  // every lane has read its records before any is overwritten
#pragma unroll
                            for (int u = 0; u < kC; ++u) {
                                if (live[u]) area[ring(wpos + (uint64_t)__popcll(bl[u] & lt_mask))] = LruRec{rv[u], rs[u]};
                                wpos += (uint64_t)__popcll(bl[u]);
                            }
                            ps_wave_sync();
                        }
                        t = wpos;
                        tq = ps_uni32(hq + (uint32_t)(t - h) >= qc32 ? hq + (uint32_t)(t - h) - qc32 : hq + (uint32_t)(t - h));
                        if (t - h + npm > qcap) {
                            if (lane == 0) {
                                atomicOr(&st.lru_ctl[1], 2u);
                                atomicOr(st.overflow, 1u);
                            }
                            npm = 0;
                        }
                    }
                    if (npm && ((acc >> lane) & 1ull)) {
                        const uint32_t ix = tq + (uint32_t)__popcll(acc & lt_mask);  // t - h + npm <= qcap
                        area[1 + (ix >= qc32 ? ix - qc32 : ix)] = LruRec{v, my_stamp};
                    }
                    tq = ps_uni32(tq + npm >= qc32 ? tq + npm - qc32 : tq + npm);
                    head = h;
                    tail = t + npm;
                }
                ps_wave_sync();
                mark(20);
                if (prof) busy += wall_clock64() - t_step;
            }
            __syncthreads();  // wave 0's chunk handed over, wave 1's buffer free
        }
        if (prof && lane == 0) {  // per wave: [8 + 4 * wave] pops, global pops, evictions, accesses
            atomicAdd(&g_lps_prof[8 + 4 * wave], (unsigned long long)n_pop);
            atomicAdd(&g_lps_prof[9 + 4 * wave], (unsigned long long)n_gpop);
            atomicAdd(&g_lps_prof[10 + 4 * wave], (unsigned long long)n_evict);
            atomicAdd(&g_lps_prof[11 + 4 * wave], (unsigned long long)n_acc);
            atomicMax(&g_lps_prof[16 + wave], (unsigned long long)(wall_clock64() - t_res));
            atomicMax(&g_lps_prof[18 + wave], (unsigned long long)busy);
        }
        if (lane == 0) {
            if (wave == 0) {
                if (cur_run != 0xFFFFFFFFu) apply_run(cur_run);
                for (uint32_t r = r0; r < r1; ++r) sc.run_mode[r] = RUN_DONE;
                node[kNodeThreads] += thr;
                st.psize[p.id] = size;
            } else {
                st.tsize[tj] = size;
            }
            if (area) {
                area[0].value = head;
                area[0].stamp = tail;
            }
        }
        __syncthreads();
    }
}

// ---- parameter-only resources per (rule, value) segment (pseg_take routes their flows here)
// 1. every parameter event of such a flow names its value's thread-count map entry (owner resource + 1,
//    argument 0; the map exists for the whole batch, pseg_take).  kClaim: make sure the entries exist --
//    the thread-count one for every parameter event, the rule's (time, tokens) one for every entry (two
//    lanes may claim a slot each for one key; the later one in the probe sequence is never found again,
//    its key absent, dropped at the next rehash).  !kClaim: the element (slot << 32 | sorted position),
//    kPsegNone in the slot bits for every other event.
// force_miss (fault injection, SGA_PSEG_FORCE_MISS=1 in the test-only build SGA_TEST_HOOKS): the first parameter event's entry is
// taken as missing, so the device check below fails the batch
template <bool kClaim>
__global__ __launch_bounds__(kT) void k_pseg_key(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                 const uint32_t *__restrict__ keys,
                                                 const uint64_t *__restrict__ param_in, uint32_t m, uint64_t none,
                                                 int force_miss) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const uint32_t nvalid = sc.counters[0];
    const bool any = sc.counters[11] != 0;
    if (kClaim && !any) return;
    for (uint32_t j = blockIdx.x * kT + threadIdx.x; j < m; j += gridDim.x * kT) {
        uint64_t el = none | j;
        if (any && j < nvalid && sc.run_mode[sc.ev_run[j]] == RUN_PSEG) {
            const Payload q = pay[j];
            if (q.idx & F_PARAM) {
                const uint32_t res = keys[j];
                const uint64_t v = param_in[q.idx & F_IDX];
                if (st.tmapmask[res] & 1ull) {  // else an exit-only flow without the map: the exit touches no map
                    PEntry *te = ptab_get(st.ttab, st.tmask, tmap_owner(res, 0), v, kClaim, st.overflow);
                    if (!kClaim && force_miss && j < 64) te = nullptr;
                    if (kClaim && !(q.idx & F_EXIT))
                        ptab_get(st.ptab, st.pmask, st.prules[st.res[res].prule_off].id + 1, v, true, st.overflow);
                    if (!kClaim && te) {
                        el = ((uint64_t)(te - st.ttab) << 32) | j;
                        // the segment's flag word: kPAbsent at rest (k_pseg_solve puts it back), k_pseg_heads ORs
                        // the flags in; only a batch that failed before k_pseg_solve leaves one to reset
                        if (te->b != kPAbsent) te->b = kPAbsent;
                    } else if (!kClaim) {
                        // every parameter event of a RUN_PSEG flow had its thread-count entry claimed (by the
                        // claim launch, or by k_lru_claim in LRU mode); a missing one would leave the event
                        // undecided, so the batch fails: the overflow word's device-error bit (SGA_EIO)
                        atomicOr(st.overflow, kOvfMissingEntry);
                    }
                }
            }
        }
        if (!kClaim) sc.pel[0][j] = el;
    }
}

// SGA_PSEG_DEBUG=1 (diagnostics only): the sorted elements out of order, and pseg elements of resources in
// LRU mode (never expected)
__global__ __launch_bounds__(kT) void k_pseg_check(FlowState st, const uint32_t *__restrict__ keys,
                                                   const uint64_t *__restrict__ el, uint32_t m, uint64_t none,
                                                   uint32_t *out) {
    for (uint32_t e = blockIdx.x * kT + threadIdx.x; e < m; e += gridDim.x * kT) {
        const uint64_t k = el[e] >> 32;
        if (e > 0 && k < (el[e - 1] >> 32)) atomicAdd(&out[0], 1u);
        if (k == none >> 32) continue;
        atomicAdd(&out[1], 1u);
        const uint32_t res = keys[(uint32_t)el[e]];
        if (st.lru_res && st.lru_res[res]) atomicAdd(&out[2], 1u);
        if (st.ttab[k].owner != res + 1) atomicAdd(&out[3], 1u);
    }
}

__device__ __forceinline__ int64_t shfl_up_i64(int64_t v, int o) {
    const int lo = __shfl_up((int)(uint32_t)v, o, 64), hi = __shfl_up((int)(uint32_t)((uint64_t)v >> 32), o, 64);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// 2. segment heads of the sorted elements, the elements' payloads gathered once into sorted order (sc.spay:
//    every later pass streams them)
//    and each segment's flag word (the b word of its thread-count entry, which a thread count never uses: kPAbsent
//    at rest, the flags ORed into its low bits and k_pseg_solve putting kPAbsent back):
//    kSegExit / kSegEntry when it holds exits / entries, kSegIrregular when an entry's acquire count differs
//    from the previous entry's or its time goes back (the closed forms of k_pseg_solve / k_pseg_long need
//    one acquire count and non-decreasing times)
//    Each workgroup takes kHeadsChunk consecutive elements and lists its heads in LDS first: one counter atomic
//    per workgroup (one per wave had all waves of the GPU queue at one address)
constexpr int64_t kSegExit = 1, kSegEntry = 2, kSegIrregular = 4;
constexpr uint32_t kHeadsChunk = 4096;
__global__ __launch_bounds__(kT) void k_pseg_heads(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                   const uint64_t *__restrict__ el, uint32_t m, uint64_t none) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0) || sc.counters[11] == 0) return;
    __shared__ uint32_t hl[kHeadsChunk];
    __shared__ uint32_t hn, hbase;
    if (threadIdx.x == 0) hn = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c0 = blockIdx.x * kHeadsChunk, c1 = min(m, c0 + kHeadsChunk);
    for (uint32_t e0 = c0; e0 < c1; e0 += kT) {  // whole waves in every iteration
        const uint32_t e = e0 + threadIdx.x;
        const uint64_t x = e < m ? el[e] : none;
        const uint64_t k = x >> 32;
        // the previous element and its payload from the lane before (lane 0 loads them): one payload gather
        // per element, stored in sorted order
        uint64_t xp = shfl_up_i64((int64_t)x, 1);
        if (lane == 0) xp = (e > 0 && e - 1 < m) ? el[e - 1] : none;
        const bool head = k != none >> 32 && (e == 0 || (xp >> 32) != k);
        const Payload q = pay[(uint32_t)x];  // every lane (a padding lane reads element 0)
        if (k != none >> 32) sc.spay[e] = q;
        Payload pq;
        pq.idx = (uint32_t)__shfl_up((int)q.idx, 1, 64);
        pq.ts_off = (uint32_t)__shfl_up((int)q.ts_off, 1, 64);
        pq.acq_prio = (uint32_t)__shfl_up((int)q.acq_prio, 1, 64);
        if (lane == 0 && e > 0 && (xp >> 32) != none >> 32) pq = pay[(uint32_t)xp];
        const uint64_t hb = __ballot(head);  // one LDS atomic per wave
        if (hb) {
            const int first = __ffsll((unsigned long long)hb) - 1;
            uint32_t base = 0;
            if ((int)lane == first) base = atomicAdd(&hn, (uint32_t)__popcll(hb));
            base = (uint32_t)__shfl((int)base, first, 64);
            if (head) hl[base + (uint32_t)__popcll(hb & ((1ull << lane) - 1ull))] = e;
        }
        const bool valid = k != none >> 32;
        int64_t f = (q.idx & F_EXIT) ? kSegExit : kSegEntry;
        if (valid && !head && !(q.idx & F_EXIT)) {
            if (!(pq.idx & F_EXIT) && ((pq.acq_prio & 0x7FFFFFFFu) != (q.acq_prio & 0x7FFFFFFFu) || q.ts_off < pq.ts_off))
                f |= kSegIrregular;
        }
        // one flag update per run of equal keys in the wave (the elements are sorted, so a key's lanes are
        // contiguous): its first lane ORs the run's flags in -- a long segment's lanes would otherwise all meet
        // at one address
        const bool lead = valid && (lane == 0 || (xp >> 32) != k);
        const uint64_t ld = __ballot(lead), vm = __ballot(valid);
        const uint64_t mx = __ballot(valid && (f & kSegExit)), me = __ballot(valid && (f & kSegEntry)),
                       mi = __ballot(valid && (f & kSegIrregular));
        if (!lead) continue;
        const uint64_t after = lane == 63 ? 0ull : (ld & (~0ull << (lane + 1)));
        const int rend = after ? __builtin_ctzll(after) : 64;  // the run: lanes [lane, rend)
        const uint64_t run = (rend == 64 ? ~0ull : ((1ull << rend) - 1ull)) & (~0ull << lane) & vm;
        const int64_t fr = ((mx & run) ? kSegExit : 0) | ((me & run) ? kSegEntry : 0) | ((mi & run) ? kSegIrregular : 0);
        int64_t *w = &st.ttab[k].b;
        if ((*w & fr) != fr) atomicOr((unsigned long long *)w, (unsigned long long)fr);  // a read first: hot segments
    }
    __syncthreads();
    const uint32_t n = hn;
    if (threadIdx.x == 0 && n) hbase = atomicAdd(&sc.counters[12], n);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n; t += kT) sc.seg[hbase + t] = hl[t];
}

// 3. one lane per segment: the value's events in arrival order against its entries held in registers
//    (ParamFlowChecker.passDefaultLocalCheck / passThrottleLocalCheck via param_pass_qps, ParameterMetric
//    add/decreaseThreadCount as param_threads), the entries, their access stamps and the owners' present
//    counts written back once (free mode: the count pass keeps these owners below capacity)
constexpr int kPsegG = 8;       // elements loaded ahead
#ifndef SGA_PSEG_LONG
#define SGA_PSEG_LONG 64
#endif
constexpr int kPsegLong = SGA_PSEG_LONG;  // regular entry segments this long go to k_pseg_long (C4: 6.17 / 6.04 / 6.21 / 6.45
                                          // ms per step at 512 / 128 / 64 / 32 with the scattered block fill;
                                          // without it, round-6 end: 3.82 / 3.86 / 4.00 ms at 64 / 128 / 256)
__global__ __launch_bounds__(kT) void k_pseg_solve(FlowState st, int64_t max_rt, FlowScratch sc,
                                                   const Payload *__restrict__ pay, const uint32_t *__restrict__ keys,
                                                   const uint64_t *__restrict__ el, uint32_t m, int64_t ts_base,
                                                   const uint64_t *__restrict__ param_in, int8_t *decision,
                                                   int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const Ctx c{st, max_rt};
    const uint32_t nseg = sc.counters[12];
    for (uint32_t s = blockIdx.x * kT + threadIdx.x; s < nseg; s += gridDim.x * kT) {
        const uint32_t e0 = sc.seg[s];
        const uint64_t key = el[e0] >> 32;
        const uint32_t j0 = (uint32_t)el[e0];
        const uint32_t res = keys[j0];
        const ParamRuleDev prule = st.prules[st.res[res].prule_off];
        const uint64_t v = param_in[sc.spay[e0].idx & F_IDX];
        PEntry *const tp = st.ttab + key;
        int64_t ta = tp->a;
        const bool t0 = ta != kPAbsent;
        PEntry *pp = nullptr;
        PEntry pe{};
        bool p0 = false;
        uint64_t pst = 0, tst = 0;  // the last access stamps
        bool more = true;
        const int64_t flags = tp->b & (kSegExit | kSegEntry | kSegIrregular);
        tp->b = kPAbsent;  // the flag word back to the thread-count entry's unused value (a present-key count
                           // and a rehash test a != absent || b != absent)
        if (flags == kSegExit || flags == kSegEntry) {
            // the segment's end: galloping search on the keys
            uint32_t lo = e0 + 1, step = 1, hi = e0 + 1;
            while (hi < m && (el[hi] >> 32) == key) {
                lo = hi + 1;
                hi = min(m, hi + step);
                step <<= 1;
            }
            while (lo < hi) {  // first index in [lo, hi) with another key (hi: one, or m)
                const uint32_t mid = (lo + hi) >> 1;
                if ((el[mid] >> 32) == key) lo = mid + 1;
                else hi = mid;
            }
            const uint32_t e1 = lo;
            if (flags == kSegEntry && e1 - e0 >= (uint32_t)kPsegLong) {  // one wave decides it (k_pseg_long)
                const uint32_t li = atomicAdd(&sc.counters[14], 1u);
                sc.plong[2 * li] = e0;
                sc.plong[2 * li + 1] = e1 - e0;
                continue;
            }
            if (flags == kSegExit) {
                // exits only: decreaseThreadCount n times (absent -> 0, 0 or 1 -> absent, c -> c - 1)
                const int64_t n = e1 - e0;
                int64_t st0 = ta;
                int64_t rem = n;
                if (ta != kPAbsent && ta >= 1) {
                    if (n < ta) {
                        st0 = ta - n;
                        rem = 0;
                    } else {
                        st0 = kPAbsent;
                        rem = n - ta;
                    }
                }
                if (rem) st0 = ((rem & 1) ? (st0 == kPAbsent ? 0 : kPAbsent) : st0);
                ta = st0;
                tst = lru_stamp(st, sc.spay[e1 - 1].idx & F_IDX, 0);
                more = false;
            }
        }
        for (uint32_t g = e0; more; g += kPsegG) {
            uint64_t x[kPsegG];
            Payload q[kPsegG];
#pragma unroll
            for (int u = 0; u < kPsegG; ++u) x[u] = el[min(g + u, m - 1)];
#pragma unroll
            for (int u = 0; u < kPsegG; ++u) q[u] = sc.spay[min(g + u, m - 1)];
#pragma unroll
            for (int u = 0; u < kPsegG; ++u) {
                if (!more || g + u >= m || (x[u] >> 32) != key) {
                    more = false;
                    continue;
                }
                const uint32_t idx = q[u].idx & F_IDX;
                const uint64_t stamp = lru_stamp(st, idx, 0);
                if (q[u].idx & F_EXIT) {  // decreaseThreadCount: an absent count is put as 0, a count reaching 0 removed
                    ta = ta == kPAbsent ? 0 : (ta - 1 <= 0 ? kPAbsent : ta - 1);
                    tst = stamp;
                    continue;
                }
                if (!pp) {
                    pp = ptab_get(st.ptab, st.pmask, prule.id + 1, v, false, st.overflow);
                    if (!pp) {  // overflow: the batch fails (-ENOMEM)
                        more = false;
                        continue;
                    }
                    pe = *pp;
                    p0 = pe.a != kPAbsent;
                }
                const int aq = (int)(q[u].acq_prio & 0x7FFFFFFFu);
                if (param_map_access(c, prule, v, aq)) pst = stamp;
                int64_t w = 0;
                const bool pass = param_pass_qps(c, prule, pe, v, aq, ts_base + (int64_t)q[u].ts_off, &w);
                decision[idx] = pass ? D_PASS : D_BLOCK_PARAM;
                wait_ms[idx] = pass ? (int32_t)w : 0;  // a block's detail: the rule's index (0)
                if (pass) {  // addThreadCount
                    ta = (ta == kPAbsent ? 0 : ta) + 1;
                    tst = stamp;
                }
            }
        }
        if (pp) {
            pp->a = pe.a;
            pp->b = pe.b;
            if (pst && st.pstamp) st.pstamp[pp - st.ptab] = pst;
            const int d = (pe.a != kPAbsent ? 1 : 0) - (p0 ? 1 : 0);
            if (d && st.psize) atomicAdd(&st.psize[prule.id], (uint32_t)d);
        }
        tp->a = ta;
        if (tst && st.tstamp) st.tstamp[key] = tst;
        const int d = (ta != kPAbsent ? 1 : 0) - (t0 ? 1 : 0);
        if (d && lru_on_t(st, res)) atomicAdd(&st.tsize[st.tbase[res]], (uint32_t)d);
    }
}

// Breaker-only flows (cb_take): one wave each, the breaker in registers (uniform over the lanes).
//   entries only: HALF_OPEN blocks every entry; OPEN blocks every entry but the first at or after the retry
//     time, which passes and moves the breaker to HALF_OPEN (DegradeSlot.entry, AbstractCircuitBreaker.tryPass);
//   exits only (onRequestComplete, cb_on_complete_ws): the stat window (LeapArray(1, statIntervalMs)) counts
//     as a segmented scan over the exits in rounds of 64 x kCbI (segments = windows, non-decreasing); a CLOSED
//     breaker opens at the first exit whose window counts trip it, and exits after that only count; a
//     HALF_OPEN one is decided by its first exit, stepped alone; a window that goes back in time (a detached
//     bucket) sends the rest of the flow to the step-by-step replay.
constexpr int kCbI = 16;
constexpr int64_t kCbNone = INT64_MIN + 1;
__device__ __forceinline__ CbAgg cb_combine(const CbAgg &p, const CbAgg &x) {
    if (x.ws == kCbNone) return p;
    if (x.ws == p.ws) return CbAgg{x.ws, p.bad + x.bad, p.tot + x.tot};
    return x;
}
constexpr int kCbW = 8;  // waves per flow: a round covers kCbW x 64 x kCbI exits
constexpr uint32_t kCbRound = 64u * kCbW * kCbI;
constexpr uint32_t kCbTiled = 1u << 31;        // a cbf word's flow taken by the tile kernels (k_cbt_*)
constexpr uint32_t kCbTileMin = 2 * kCbRound;  // exits of the shortest flow they take
// a wave's 64 x kCbI exits of a round, loaded coalesced and read back per lane (kCbI consecutive each; one pad
// slot per kCbI items keeps those strided reads off one bank)
constexpr int kCbStage = 64 * kCbI + 64;
template <int kW>
struct CbLds {
    int64_t w[kW][5];  // per wave: total {ws, bad, tot}, first and last window
    uint32_t min, bad;
    uint32_t ts[kW][kCbStage], fx[kW][kCbStage];
    int64_t rt[kW][kCbStage];
};
struct CbRound {
    CbAgg total;    // carry combined with the round's exits
    uint32_t trip;  // the first exit whose counts trip a CLOSED breaker (je: none, or !want_trip)
    bool bad;       // a window went back (inside the round or against the carry): the round is not taken
    int64_t first, last;  // the round's first and last windows (INT64_MAX / INT64_MIN: no exit)
};
// One round of a flow's exits (kW waves x 64 lanes x kCbI consecutive exits from base, clipped at je) against
// the carry: the stat window's counts as a segmented scan (segments = windows, non-decreasing) and, when
// want_trip, the first exit whose window counts trip the breaker (cb_trips).  Every thread of the workgroup
// calls it with the same arguments.
template <int kW>
__device__ CbRound cb_round(CbLds<kW> &L, const CbDev &b, const CbAgg &carry, uint32_t base, uint32_t je, bool want_trip,
                            const Payload *__restrict__ pay, const int64_t *__restrict__ rt_sorted, int64_t ts_base) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr uint32_t kWaveItems = 64u * kCbI;
    const int64_t si = b.stat_interval;
    int64_t wsv[kCbI];
    uint32_t badm = 0, valm = 0;
    const uint32_t wb = base + (uint32_t)wave * kWaveItems;
    const uint32_t j0 = wb + (uint32_t)lane * kCbI;
    // the wave's items through LDS: coalesced loads at clamped indices, then each lane's run
    {
#pragma unroll
        for (int i = 0; i < kCbI; ++i) {
            const uint32_t k = (uint32_t)i * 64 + (uint32_t)lane;
            const uint32_t j = min(wb + k, je - 1);
            const Payload q = pay[j];
            L.ts[wave][k + k / kCbI] = q.ts_off;
            L.fx[wave][k + k / kCbI] = q.idx;
            if (b.grade == 0) L.rt[wave][k + k / kCbI] = rt_sorted[j];  // sorted order (k_lexits)
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    uint32_t tso[kCbI], fx[kCbI];
#pragma unroll
    for (int i = 0; i < kCbI; ++i) {
        const uint32_t k = (uint32_t)lane * kCbI + (uint32_t)i;
        tso[i] = L.ts[wave][k + k / kCbI];
        fx[i] = L.fx[wave][k + k / kCbI];
    }
    if (b.grade == 0) {
#pragma unroll
        for (int i = 0; i < kCbI; ++i) {
            const uint32_t k = (uint32_t)lane * kCbI + (uint32_t)i;
            badm |= (L.rt[wave][k + k / kCbI] > b.max_allowed_rt ? 1u : 0u) << i;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kCbI; ++i) badm |= ((fx[i] & F_ERROR) ? 1u : 0u) << i;
    }
    int64_t cw = kCbNone;  // the window of the previous item: most items share it (no division)
#pragma unroll
    for (int i = 0; i < kCbI; ++i) {
        const int64_t t = ts_base + (int64_t)tso[i];
        if (cw == kCbNone || t < cw || t - cw >= si) cw = t - t % si;
        wsv[i] = j0 + i < je ? cw : kCbNone;
        valm |= (j0 + i < je ? 1u : 0u) << i;
    }
    badm &= valm;
    bool mono = true;  // inside the lane
    int64_t first = kCbNone, last = kCbNone;
#pragma unroll
    for (int i = 0; i < kCbI; ++i) {
        if (!((valm >> i) & 1u)) continue;
        if (first == kCbNone) first = wsv[i];
        else if (wsv[i] < last) mono = false;
        last = wsv[i];
    }
    CbAgg agg{kCbNone, 0, 0};
#pragma unroll
    for (int i = 0; i < kCbI; ++i)
        if ((valm >> i) & 1u) agg = cb_combine(agg, CbAgg{wsv[i], (int64_t)((badm >> i) & 1u), 1});
    // the lanes' tail-window counts as one DPP segmented scan: a lane starts a segment when its
    // tail window starts inside it or differs from the windows before it (windows only grow, so
    // the window of everything up to a lane is the prefix maximum)
    const int64_t prev_last = wave_incl_max_i64(last == kCbNone ? INT64_MIN : last);
    const int64_t before = wave_shr1_i64(prev_last, INT64_MIN);  // windows of the lanes before
    const bool has = agg.ws != kCbNone;
    int hd = (has && (first != agg.ws || (before != INT64_MIN && before != agg.ws))) ? 1 : 0;
    int sb = (int)agg.bad, stt = (int)agg.tot;
    wave_incl_segsum2(sb, stt, hd);
    const int64_t iws = prev_last == INT64_MIN ? kCbNone : prev_last;  // window of lanes <= this one
    // the waves' totals, first and last windows: each wave's carry is the round's carry and the
    // totals of the waves before it
    {
        const int64_t fmin = wave_incl_min_i64(first == kCbNone ? INT64_MAX : first);
        if (lane == 63) {
            L.w[wave][0] = iws;
            L.w[wave][1] = sb;
            L.w[wave][2] = stt;
            L.w[wave][3] = fmin;  // first window of the wave (INT64_MAX: none)
            L.w[wave][4] = prev_last;
        }
        if (threadIdx.x == 0) L.bad = 0;
    }
    __syncthreads();
    CbAgg cwv = carry;
    int64_t wlim = carry.ws == kCbNone ? INT64_MIN : carry.ws;
    for (int w = 0; w < wave; ++w) {
        cwv = cb_combine(cwv, CbAgg{L.w[w][0], L.w[w][1], L.w[w][2]});
        wlim = max(wlim, L.w[w][4]);
    }
    // windows must not go back: across lanes, across waves and against the carry
    const int64_t lim = max(before, wlim);
    if (first != kCbNone && first < lim) mono = false;
    if (!mono) L.bad = 1;
    CbRound out{carry, je, false, INT64_MAX, INT64_MIN};
    for (int w = 0; w < kW; ++w) {
        out.total = cb_combine(out.total, CbAgg{L.w[w][0], L.w[w][1], L.w[w][2]});
        out.first = min(out.first, L.w[w][3]);
        out.last = max(out.last, L.w[w][4]);
    }
    __syncthreads();
    if (L.bad) {
        out.bad = true;
        __syncthreads();
        return out;
    }
    CbAgg inc{iws, sb, stt};
    if (!hd && iws != kCbNone && iws == cwv.ws) {
        inc.bad += cwv.bad;
        inc.tot += cwv.tot;
    }
    if (iws == kCbNone) inc = cwv;  // nothing up to this lane: the carry alone
    CbAgg run{wave_shr1_i64(inc.ws, cwv.ws), wave_shr1_i64(inc.bad, cwv.bad), wave_shr1_i64(inc.tot, cwv.tot)};
    if (threadIdx.x == 0) L.min = je;
    __syncthreads();
    if (want_trip) {
        uint32_t trip = je;
#pragma unroll
        for (int i = 0; i < kCbI; ++i) {
            if (!((valm >> i) & 1u)) continue;
            run = cb_combine(run, CbAgg{wsv[i], (int64_t)((badm >> i) & 1u), 1});
            if (trip == je && cb_trips(b, run.bad, run.tot)) trip = j0 + i;
        }
        if (trip < je) atomicMin(&L.min, trip);
    }
    __syncthreads();
    out.trip = L.min;
    __syncthreads();
    return out;
}

// kW waves per flow: k_cb_flows<kCbW> takes the flows of at least kCbShort events, k_cb_flows<1> the others (many
// one-wave workgroups per CU: most flows are short)
constexpr uint32_t kCbShort = 4096;
template <int kW>
__global__ __launch_bounds__(64 * kW) void k_cb_flows(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                      int64_t ts_base, const int64_t *__restrict__ rt_in,
                                                      int8_t *decision, int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    __shared__ CbLds<kW> L;
    constexpr uint32_t kRound = 64u * kW * kCbI;
    const uint32_t ncb = sc.counters[13], nflows = sc.counters[2], nruns = sc.counters[1];
    for (uint32_t h = blockIdx.x; h < ncb; h += gridDim.x) {
        const uint32_t fl = sc.cbf[h];
        if (fl & kCbTiled) continue;  // decided by the tile kernels (k_cbt_*)
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t res = sc.run_slot[r0];
        const uint32_t jb = sc.run_start[r0], je = sc.run_end[r1 - 1];
        if ((je - jb >= kCbShort) != (kW == kCbW)) continue;  // the other launch's
        CbDev *gb = st.cbs + st.res[res].cb_off;
        CbDev b = *gb;  // every thread holds the same copy and takes the same steps
        if (!(pay[jb].idx & F_EXIT)) {  // entries only (the breaker is not CLOSED)
            uint32_t probe = je;
            if (b.state == 1) {
                for (uint32_t base = jb; base < je && probe == je; base += kRound) {
                    if (threadIdx.x == 0) L.min = je;
                    __syncthreads();
                    for (int i = 0; i < kCbI; ++i) {  // coalesced; a thread's later items are later entries
                        const uint32_t j = base + (uint32_t)i * (64u * kW) + threadIdx.x;
                        if (j < je && ts_base + (int64_t)pay[j].ts_off >= b.next_retry) {
                            atomicMin(&L.min, j);
                            break;
                        }
                    }
                    __syncthreads();
                    probe = L.min;
                    __syncthreads();
                }
                if (probe < je) {  // fromOpenToHalfOpen: the probe passes
                    b.state = 2;
                    b.probe_t = ts_base + (int64_t)pay[probe].ts_off;
                }
            }
            for (uint32_t j = jb + threadIdx.x; j < je; j += 64 * kW) {
                const uint32_t idx = pay[j].idx & F_IDX;
                decision[idx] = j == probe ? D_PASS : D_BLOCK_DEGRADE;
                wait_ms[idx] = 0;  // a block's detail: the breaker's index
            }
        } else {  // exits only
            const int64_t si = b.stat_interval;
            CbAgg carry{b.st_start == kAbsent ? kCbNone : b.st_start, b.st_bad, b.st_total};
            bool seq = false;
            uint32_t base = jb;
            while (base < je && !seq) {
                if (b.state == 2) {  // the probe's completion decides HALF_OPEN alone
                    const Payload q = pay[base];
                    const int64_t t = ts_base + (int64_t)q.ts_off;
                    b.st_start = carry.ws == kCbNone ? kAbsent : carry.ws;
                    b.st_bad = carry.bad;
                    b.st_total = carry.tot;
                    cb_on_complete_ws(b, t, t - t % si, rt_in[q.idx & F_IDX], (q.idx & F_ERROR) != 0);
                    carry = CbAgg{b.st_start == kAbsent ? kCbNone : b.st_start, b.st_bad, b.st_total};
                    ++base;
                    continue;
                }
                const CbRound o = cb_round(L, b, carry, base, je, b.state == 0, pay, sc.rt_sorted, ts_base);
                if (o.bad) {
                    seq = true;
                    break;
                }
                if (o.trip < je) cb_to_open(b, ts_base + (int64_t)pay[o.trip].ts_off);  // the first exit that trips it
                carry = o.total;
                base += kRound;
            }
            b.st_start = carry.ws == kCbNone ? kAbsent : carry.ws;
            b.st_bad = carry.bad;
            b.st_total = carry.tot;
            if (seq)  // step by step (every thread the same steps)
                for (uint32_t j = base; j < je; ++j) {
                    const Payload q = pay[j];
                    const int64_t t = ts_base + (int64_t)q.ts_off;
                    cb_on_complete_ws(b, t, t - t % si, rt_in[q.idx & F_IDX], (q.idx & F_ERROR) != 0);
                }
        }
        __syncthreads();
        if (threadIdx.x == 0) *gb = b;
        __syncthreads();
    }
}

// Long breaker-only flows over the whole GPU: the flow in tiles of one round (kCbRound), one workgroup per tile.
// Exit flows of a CLOSED or OPEN breaker: the stat window's counts combine associatively (cb_combine), so
//   k_cbt_plan         lists the flows with at least kCbTileMin events and numbers their tiles;
//   k_cbt_tiles<0>     each tile's counts from an empty carry, and its first and last windows;
//   k_cbt_scan         per flow, each tile's carry in tile order -- a window that goes back anywhere (inside a
//                      tile, between tiles, against the breaker's window) hands the whole flow back to k_cb_flows;
//   k_cbt_tiles<1>     a CLOSED breaker's first tripping exit: each tile's against its carry, the flow's first by
//                      atomicMin (nothing after the trip can change the breaker: OPEN exits only count, and only
//                      an entry moves OPEN on);
//   k_cbt_fin          the breaker's window = the flow's total, cb_to_open at the first trip.
// Entry flows (OPEN or HALF_OPEN): k_cbt_tiles<0> finds an OPEN breaker's probe (the first entry at or after the
// retry time, atomicMin over the tiles), k_cbt_tiles<1> writes every entry's decision, k_cbt_fin moves the
// breaker to HALF_OPEN at the probe.
// k_cb_flows skips the flows k_cbt_scan took (kCbTiled in their cbf word).
__global__ __launch_bounds__(kT) void k_cbt_plan(FlowState st, FlowScratch sc, const Payload *__restrict__ pay) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const uint32_t ncb = sc.counters[13], nflows = sc.counters[2], nruns = sc.counters[1];
    for (uint32_t h = blockIdx.x * kT + threadIdx.x; h < ncb; h += gridDim.x * kT) {
        const uint32_t fl = sc.cbf[h];
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        const uint32_t jb = sc.run_start[r0], je = sc.run_end[r1 - 1];
        if (je - jb < kCbTileMin) continue;
        // exits: CLOSED or OPEN at the start (HALF_OPEN: the first exit alone decides); entries: any
        const CbDev &b = st.cbs[st.res[sc.run_slot[r0]].cb_off];
        if ((pay[jb].idx & F_EXIT) && b.state == 2) continue;
        const uint32_t ntile = (je - jb + kCbRound - 1) / kCbRound;
        // the flows' and tiles' numbering is arbitrary (a tile names its flow)
        const uint32_t k = atomicAdd(&sc.cbt_ctl[0], 1u), t0 = atomicAdd(&sc.cbt_ctl[1], ntile);
        sc.cbt_flow[k] = h;
        sc.cbt_off[k] = t0;
        sc.cbt_trip[k] = 0xFFFFFFFFu;
        sc.cbt_state[k] = 0;
        for (uint32_t i = 0; i < ntile; ++i) sc.cbt_tile[t0 + i] = k;
    }
}

// a tiled flow's exit range [jb, je) and breaker
__device__ __forceinline__ void cbt_flow(const FlowState &st, const FlowScratch &sc, uint32_t k, uint32_t &h,
                                         uint32_t &jb, uint32_t &je, CbDev *&gb) {
    const uint32_t nflows = sc.counters[2], nruns = sc.counters[1];
    h = sc.cbt_flow[k];
    const uint32_t fl = sc.cbf[h] & ~kCbTiled;
    const uint32_t r0 = sc.flow_first_run[fl];
    const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
    jb = sc.run_start[r0];
    je = sc.run_end[r1 - 1];
    gb = st.cbs + st.res[sc.run_slot[r0]].cb_off;
}

template <bool kTrip>
__global__ __launch_bounds__(64 * kCbW) void k_cbt_tiles(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                         int64_t ts_base, int8_t *decision, int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    __shared__ CbLds<kCbW> L;
    const uint32_t ntiles = sc.cbt_ctl[1];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t k = sc.cbt_tile[t];
        uint32_t h, jb, je;
        CbDev *gb;
        cbt_flow(st, sc, k, h, jb, je, gb);
        const uint32_t base = jb + (t - sc.cbt_off[k]) * kCbRound, end = min(base + kCbRound, je);
        const CbDev b = *gb;
        if (!(pay[jb].idx & F_EXIT)) {  // entries: an OPEN breaker's probe, then every entry's decision
            if (!kTrip) {
                if (b.state != 1) continue;
                if (threadIdx.x == 0) L.min = je;
                __syncthreads();
                for (uint32_t j = base + threadIdx.x; j < end; j += 64 * kCbW)
                    if (ts_base + (int64_t)pay[j].ts_off >= b.next_retry) {  // a thread's later items are later
                        atomicMin(&L.min, j);
                        break;
                    }
                __syncthreads();
                if (threadIdx.x == 0 && L.min < je) atomicMin(&sc.cbt_trip[k], L.min);
                __syncthreads();
            } else {
                const uint32_t probe = b.state == 1 ? sc.cbt_trip[k] : 0xFFFFFFFFu;
                for (uint32_t j = base + threadIdx.x; j < end; j += 64 * kCbW) {
                    const uint32_t idx = pay[j].idx & F_IDX;
                    decision[idx] = j == probe ? D_PASS : D_BLOCK_DEGRADE;
                    wait_ms[idx] = 0;  // a block's detail: the breaker's index
                }
            }
        } else if (!kTrip) {
            const CbRound o = cb_round(L, b, CbAgg{kCbNone, 0, 0}, base, je, false, pay, sc.rt_sorted, ts_base);
            if (threadIdx.x == 0) {
                CbTile &T = sc.cbt[t];
                T.agg = o.total;
                T.first = o.first;
                T.last = o.last;
                T.bad = o.bad ? 1 : 0;
            }
        } else {
            if (sc.cbt_state[k] != 1 || b.state != 0) continue;  // taken, CLOSED
            const CbRound o = cb_round(L, b, sc.cbt[t].carry, base, je, true, pay, sc.rt_sorted, ts_base);
            if (threadIdx.x == 0 && o.trip < je) atomicMin(&sc.cbt_trip[k], o.trip);
        }
    }
}

// one lane per tiled flow: the tiles' carries in order, the windows checked; cbt_state 1 = taken, 2 = back
// to k_cb_flows
__global__ __launch_bounds__(kT) void k_cbt_scan(FlowState st, FlowScratch sc, const Payload *__restrict__ pay) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const uint32_t nf = sc.cbt_ctl[0];
    for (uint32_t k = blockIdx.x * kT + threadIdx.x; k < nf; k += gridDim.x * kT) {
        uint32_t h, jb, je;
        CbDev *gb;
        cbt_flow(st, sc, k, h, jb, je, gb);
        const CbDev b = *gb;
        if (!(pay[jb].idx & F_EXIT)) {  // entries: always taken
            sc.cbt_state[k] = 1;
            sc.cbf[h] |= kCbTiled;
            continue;
        }
        CbAgg carry{b.st_start == kAbsent ? kCbNone : b.st_start, b.st_bad, b.st_total};
        int64_t lim = carry.ws == kCbNone ? INT64_MIN : carry.ws;
        const uint32_t t0 = sc.cbt_off[k], t1 = t0 + (je - jb + kCbRound - 1) / kCbRound;
        bool ok = true;
        for (uint32_t t = t0; t < t1 && ok; ++t) {
            const CbTile T = sc.cbt[t];
            if (T.bad || (T.first != INT64_MAX && T.first < lim)) ok = false;
            sc.cbt[t].carry = carry;
            carry = cb_combine(carry, T.agg);
            lim = max(lim, T.last);
        }
        sc.cbt_state[k] = ok ? 1u : 2u;
        if (ok) {
            sc.cbt_total[k] = carry;
            sc.cbf[h] |= kCbTiled;
        }
    }
}

__global__ __launch_bounds__(kT) void k_cbt_fin(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                int64_t ts_base) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const uint32_t nf = sc.cbt_ctl[0];
    for (uint32_t k = blockIdx.x * kT + threadIdx.x; k < nf; k += gridDim.x * kT) {
        if (sc.cbt_state[k] != 1) continue;
        uint32_t h, jb, je;
        CbDev *gb;
        cbt_flow(st, sc, k, h, jb, je, gb);
        CbDev b = *gb;
        const uint32_t trip = sc.cbt_trip[k];
        if (!(pay[jb].idx & F_EXIT)) {  // entries: an OPEN breaker's probe passes (fromOpenToHalfOpen)
            if (b.state == 1 && trip < je) {
                b.state = 2;
                b.probe_t = ts_base + (int64_t)pay[trip].ts_off;
                *gb = b;
            }
            continue;
        }
        if (b.state == 0 && trip < je) cb_to_open(b, ts_base + (int64_t)pay[trip].ts_off);
        const CbAgg c = sc.cbt_total[k];
        b.st_start = c.ws == kCbNone ? kAbsent : c.ws;
        b.st_bad = c.bad;
        b.st_total = c.tot;
        *gb = b;
    }
}

// 3b. a long segment of entries with one acquire count and non-decreasing times: one wave, by stretches
//    instead of events.  Token bucket (passDefaultLocalCheck): between two refills (pass_time > duration)
//    the first floor(tokens / acquire) entries pass and the rest block, so a stretch is one search for the
//    next refill time and two fills; the refill itself is one exact step.  Throttle (passThrottleLocalCheck):
//    an entry passes iff expected - t < maxQueueingTimeMs or expected <= t, so the next pass is one search
//    for the first t >= expected - max(maxQueueingTimeMs - 1, 0).  Searches are 64-ary (a probe per lane),
//    fills write the decisions on all lanes.
__device__ __forceinline__ int64_t pseg_time(const Payload *__restrict__ spay, int64_t ts_base, uint32_t e) {
    return ts_base + (int64_t)spay[e].ts_off;
}
// first e in [lo, hi) with time > x (hi if none); times non-decreasing over [lo, hi)
__device__ uint32_t pseg_upper(const Payload *__restrict__ sp, int64_t ts_base, uint32_t lo, uint32_t hi, int64_t x) {
    const int lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t p = lo + (uint32_t)lane * step;
        const bool gt = p < hi && pseg_time(sp, ts_base, p) > x;
        const uint64_t b = __ballot(gt);
        if (!b) {  // every probe <= x: the answer is past the last probe inside [lo, hi)
            lo = lo + ((hi - lo - 1) / step) * step + 1;
            continue;
        }
        const int f = __ffsll((unsigned long long)b) - 1;
        if (f == 0) return lo;
        hi = lo + (uint32_t)f * step;  // satisfies
        lo = lo + (uint32_t)(f - 1) * step + 1;
    }
    const uint32_t p = lo + (uint32_t)lane;
    const uint64_t b = __ballot(p < hi && pseg_time(sp, ts_base, p) > x);
    return b ? lo + (uint32_t)(__ffsll((unsigned long long)b) - 1) : hi;
}
__global__ __launch_bounds__(64) void k_pseg_long(FlowState st, int64_t max_rt, FlowScratch sc,
                                                  const Payload *__restrict__ pay, const uint32_t *__restrict__ keys,
                                                  const uint64_t *__restrict__ el, int64_t ts_base,
                                                  const uint64_t *__restrict__ param_in, int8_t *decision,
                                                  int32_t *wait_ms) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const Ctx c{st, max_rt};
    const int lane = threadIdx.x;
    const uint32_t nl = sc.counters[14];
    for (uint32_t h = blockIdx.x; h < nl; h += gridDim.x) {
        const uint32_t e0 = sc.plong[2 * h], e1 = e0 + sc.plong[2 * h + 1];
        const uint64_t key = el[e0] >> 32;
        const Payload *__restrict__ sp = sc.spay;
        const Payload q0 = sp[e0];
        const uint32_t res = keys[(uint32_t)el[e0]];
        const ParamRuleDev prule = st.prules[st.res[res].prule_off];
        const uint64_t v = param_in[q0.idx & F_IDX];
        const int a = (int)(q0.acq_prio & 0x7FFFFFFFu);
        PEntry *const tp = st.ttab + key;
        PEntry *const pp = ptab_get(st.ptab, st.pmask, prule.id + 1, v, false, st.overflow);
        if (!pp) continue;  // overflow: the batch fails
        PEntry pe = *pp;
        const bool p0 = pe.a != kPAbsent;
        int64_t npass = 0;
        uint32_t last_pass = e1;
        // decisions of [lo, hi) on all lanes (blocks: the default k_lclassify wrote)
        auto fill = [&](uint32_t lo, uint32_t hi, bool pass) {
            if (!pass) return;
            const int8_t d = D_PASS;
            for (uint32_t e = lo + lane; e < hi; e += 4 * 64) {
                uint32_t ix[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) ix[u] = sp[min(e + 64 * u, hi - 1)].idx & F_IDX;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (e + 64 * u < hi) {
                        decision[ix[u]] = d;
                        wait_ms[ix[u]] = 0;
                    }
            }
            if (pass && hi > lo) {
                npass += hi - lo;
                last_pass = hi - 1;
            }
        };
        auto one = [&](uint32_t e, bool pass, int64_t w) {
            if (lane == 0) {
                const uint32_t ix = sp[e].idx & F_IDX;
                decision[ix] = pass ? D_PASS : D_BLOCK_PARAM;
                wait_ms[ix] = pass ? (int32_t)w : 0;
            }
            if (pass) {
                ++npass;
                last_pass = e;
            }
        };
        const bool access = param_map_access(c, prule, v, a);
        if (!access) {
            fill(e0, e1, false);  // a zero threshold, or acquire > maxCount: every entry blocks, no map access
        } else {
            int64_t token_count = j_d2l(prule.count), hot;
            if (hot_lookup(c, prule, v, &hot)) token_count = hot;
            uint32_t e = e0;
            if (prule.behavior == 2) {
                const int64_t cost =
                    j_round(1.0 * 1000 * (double)a * (double)prule.duration / (double)token_count);
                const int64_t slack = prule.max_queue > 0 ? prule.max_queue - 1 : 0;
                while (e < e1) {
                    if (pe.a == kPAbsent) {
                        pe.a = pseg_time(sp, ts_base, e);
                        one(e++, true, 0);
                        continue;
                    }
                    if (cost == 0 && pseg_time(sp, ts_base, e) >= pe.a) {
                        // a zero cost (token count above 2000 x acquire x duration): with times
                        // non-decreasing every entry from here passes without a wait, the last one's time kept
                        fill(e, e1, true);
                        pe.a = pseg_time(sp, ts_base, e1 - 1);
                        break;
                    }
                    const int64_t expected = pe.a + cost;
                    const uint32_t r = pseg_upper(sp, ts_base, e, e1, expected - slack - 1);
                    fill(e, r, false);
                    if (r >= e1) break;
                    const int64_t tr = pseg_time(sp, ts_base, r);
                    const int64_t w = expected - tr;
                    pe.a = w > 0 ? expected : tr;
                    one(r, true, w > 0 ? w : 0);
                    e = r + 1;
                }
            } else {
                const int64_t max_count = lwrap_add(token_count, prule.burst);
                const int64_t dur_ms = lwrap_mul(prule.duration, 1000);
                while (e < e1) {
                    if (pe.a == kPAbsent) {
                        pe.a = pseg_time(sp, ts_base, e);
                        if (pe.b == kPAbsent) pe.b = max_count - a;
                        one(e++, true, 0);
                        continue;
                    }
                    const uint32_t r = pseg_upper(sp, ts_base, e, e1, pe.a + dur_ms);  // the next refill
                    int64_t k = 0;
                    if (pe.b != kPAbsent && pe.b >= 0) k = a > 0 ? min((int64_t)(r - e), pe.b / a) : (int64_t)(r - e);
                    fill(e, e + (uint32_t)k, true);
                    fill(e + (uint32_t)k, r, false);
                    if (pe.b != kPAbsent) pe.b -= k * a;
                    e = r;
                    if (e >= e1) break;
                    int64_t w = 0;  // the refill: one exact step
                    const bool ok = param_pass_qps(c, prule, pe, v, a, pseg_time(sp, ts_base, e), &w);
                    one(e++, ok, w);
                }
            }
        }
        if (lane == 0) {
            pp->a = pe.a;
            pp->b = pe.b;
            if (access && st.pstamp) st.pstamp[pp - st.ptab] = lru_stamp(st, sp[e1 - 1].idx & F_IDX, 0);
            const int d = (pe.a != kPAbsent ? 1 : 0) - (p0 ? 1 : 0);
            if (d && st.psize) atomicAdd(&st.psize[prule.id], (uint32_t)d);
            if (npass) {  // addThreadCount per pass
                const int64_t ta0 = tp->a;
                tp->a = (ta0 == kPAbsent ? 0 : ta0) + npass;
                if (st.tstamp) st.tstamp[key] = lru_stamp(st, sp[last_pass].idx & F_IDX, 0);
                if (ta0 == kPAbsent && lru_on_t(st, res)) atomicAdd(&st.tsize[st.tbase[res]], 1u);
            }
        }
    }
}

// 4. each run's pass / block acquire sums and passes (the decisions are in), pre-reduced over a thread's
//    consecutive events
__global__ __launch_bounds__(kT) void k_pseg_runs(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                  const int8_t *__restrict__ decision) {
    __shared__ uint32_t srun[kStagePad];
    __shared__ uint64_t sia[kStagePad];  // idx | acq_prio << 32 (stage_idx_acq)
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0) || sc.counters[11] == 0) return;
    const uint32_t nvalid = sc.counters[0];
    const uint32_t base = blockIdx.x * kTileElems;
    if (base >= nvalid) return;  // the whole block
    stage_tile(srun, sc.ev_run, base, nvalid, 0u);
    stage_idx_acq(sia, pay, base, nvalid);
    __syncthreads();
    const uint32_t e0 = (blockIdx.x * kT + threadIdx.x) * kItems;
    uint32_t cur = 0xFFFFFFFFu, np = 0;
    int64_t pa = 0, ba = 0;
    auto flush = [&]() {
        if (cur == 0xFFFFFFFFu) return;
        if (pa) atomicAdd((unsigned long long *)&sc.run_pa[cur], (unsigned long long)pa);
        if (ba) atomicAdd((unsigned long long *)&sc.run_ba[cur], (unsigned long long)ba);
        if (np) atomicAdd(&sc.run_np[cur], np);
    };
    for (int i = 0; i < kItems && e0 + i < nvalid; ++i) {
        const uint32_t e = e0 + i;
        const uint32_t r = srun[sslot(base, e)];
        if (sc.run_mode[r] != RUN_PSEG) continue;
        const uint64_t qv = sia[sslot(base, e)];
        const uint32_t qf = (uint32_t)qv;
        if ((qf & F_EXIT) && !(qf & F_SPECIAL)) continue;
        if (r != cur) {
            flush();
            cur = r;
            pa = ba = 0;
            np = 0;
        }
        const int64_t a = (int64_t)((uint32_t)(qv >> 32) & 0x7FFFFFFFu);
        if (qf & F_SPECIAL) {  // a revoke takes its pass back and counts a block; a block outside the engine counts
            if (qf & F_EXIT) pa -= a;
            ba += a;
            continue;
        }
        const int8_t d = decision[qf & F_IDX];
        if (d == D_PASS || d == D_PASS_WAIT) {
            pa += a;
            ++np;
        } else {
            ba += a;
        }
    }
    // a long run covers whole waves: one atomic per wave instead of one per lane
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur);
    if (__all(cur == c0) && c0 != 0xFFFFFFFFu) {
        pa = readlane_i64(wave_incl_sum_i64(pa), 63);
        ba = readlane_i64(wave_incl_sum_i64(ba), 63);
        np = (uint32_t)readlane_i64(wave_incl_sum_i64((int64_t)np), 63);
        if ((threadIdx.x & 63) != 0) cur = 0xFFFFFFFFu;
    }
    flush();
}

// 5. one lane per flow: StatisticSlot in aggregate, run by run in order -- every event of a run (one 500 ms
//    bucket, nested in one minute bucket) sees the same window rotation, applied at the run's first event
//    (a detached bucket takes none of the run's adds, as it would take none of its events')
__global__ __launch_bounds__(kT) void k_pseg_apply(FlowState st, int64_t max_rt, FlowScratch sc, int64_t ts_base) {
    if (!gate_is(st.gate, kGateSeq | kGateBad, 0)) return;
    const uint32_t nf = sc.counters[11], nflows = sc.counters[2], nruns = sc.counters[1];
    for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < nf; i += gridDim.x * kT) {
        const uint32_t fl = sc.pseg[i];
        const uint32_t r0 = sc.flow_first_run[fl];
        const uint32_t r1 = fl + 1 < nflows ? sc.flow_first_run[fl + 1] : nruns;
        int64_t *node = st.node + (size_t)sc.run_slot[r0] * kNodeWords;
        int64_t thr = 0;
        for (uint32_t r = r0; r < r1; ++r) {
            const int64_t tf = ts_base + (int64_t)sc.run_t0off[r];
            int64_t *bs[2] = {sec_current(node, tf, max_rt), min_current(node, tf, max_rt)};
            const int64_t pa = sc.run_pa[r], ba = sc.run_ba[r];
            const int64_t exc = (int64_t)sc.run_exc[r], exerr = (int64_t)sc.run_exerr[r];
            const int64_t exrt = sc.run_exrt[r], exmin = sc.run_exmin[r];
            for (int k = 0; k < 2; ++k) {
                int64_t *b = bs[k];
                if (!b) continue;
                b[MB_PASS] += pa;
                b[MB_BLOCK] += ba;
                b[MB_SUCC] += exc;
                b[MB_RT] += exrt;
                b[MB_EXC] += exerr;
                if (exmin < b[MB_MINRT]) b[MB_MINRT] = exmin;
            }
            thr += (int64_t)sc.run_np[r] - (int64_t)sc.run_nexit[r];
            sc.run_mode[r] = RUN_DONE;
        }
        node[kNodeThreads] += thr;
    }
}

// ---- CacheMap capacity: before each batch (flow.hpp LruRec)
// 1. count pass: per owner in free mode, the distinct keys absent at the batch start that its events name
//    (the keys it could insert).  Two launches: the first claims every such key's slot (lanes of one owner
//    run together here, so two lanes may claim a slot each for the same key: the later one in the probe
//    sequence is never found again), marks each slot it gets back without a value (claimed now, or absent
//    since an earlier claim) with the batch's stamp mark and lists the events that marked one first; the
//    second walks only those, looks each of their keys up -- its first slot in the probe sequence -- and the
//    first to meet an absent one marks it counted and counts it.  Every absent key's first slot was marked
//    by its claimant or by an event that found it, so one listed event names it: the counts are those of a
//    walk over every event, and the second launch's work is the batch's distinct absent keys, not its events.
constexpr uint64_t kStampCounted = 1ull << 62;
template <bool kCount>
__device__ __forceinline__ bool lru_count_key(PEntry *tab, uint64_t *stamp, uint32_t mask, uint32_t owner, uint64_t v,
                                              uint32_t *ctr, uint64_t mark, uint32_t *overflow) {
    PEntry *e = ptab_get(tab, mask, owner, v, !kCount, overflow);
    if (!e || e->a != kPAbsent) return false;  // a claimant always reads its own kPAbsent
    uint64_t *sp = &stamp[e - tab];
    const uint64_t m = kCount ? mark | kStampCounted : mark;
    if (__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == m) return false;
    const bool first = atomicExch((unsigned long long *)sp, (unsigned long long)m) != m;
    if (kCount && first) atomicAdd(ctr, 1u);
    return first;
}

template <bool kCount>
__device__ __forceinline__ bool lru_count_event(const FlowState &st, uint32_t i, const uint8_t *__restrict__ kind,
                                                const uint32_t *__restrict__ resource, const uint8_t *__restrict__ flags,
                                                const uint64_t *__restrict__ param_in,
                                                const uint64_t *__restrict__ pvals, uint64_t mark) {
    const uint32_t r = resource[i];
    if (r >= st.nres || kind[i] == SGA_KIND_BLOCKED) return false;  // a revoke touches the maps as an exit does
    const ResDev R = st.res[r];
    if (!R.n_prules) return false;
    bool need = false;
    const uint8_t fl = flags ? flags[i] : 0;
    const bool hp = (fl & SGA_EV_HAS_PARAM) != 0;
    const uint64_t pv = param_in ? param_in[i] : 0;
    PArgs pa{nullptr, 0};
    if ((fl & SGA_EV_ARGS) && pvals) {
        pa.args = pvals + (pv >> 32);
        pa.pvals = pvals;
        pa.nargs = (uint32_t)pv;
    } else if (hp && (fl & SGA_EV_PARAM_LIST) && pvals) {
        pa = PArgs{pvals + (pv >> 32), (uint32_t)pv};
    }
    const uint32_t nargs = ev_nargs(pa, hp);
    uint64_t kmask = st.tmapmask ? st.tmapmask[r] : 0ull;  // thread-count maps the event may reach
    for (uint32_t k = 0; k < R.n_prules; ++k) {
        const ParamRuleDev &p = st.prules[R.prule_off + k];
        int32_t idx = p.idx_res;
        if (idx == kIdxUnresolved) {  // as applyRealParamIdx would resolve it for this event
            idx = p.param_idx;
            if (idx < 0) idx = (-idx <= (int32_t)nargs) ? (int32_t)nargs + idx : -idx;
        }
        if (idx >= 0 && idx < kMaxParamIdx) kmask |= 1ull << idx;
        if (!kCount && p.cluster && p.grade == 1 && st.cluster_on && st.cpst.ctl && kind[i] == 0 &&
            (int64_t)nargs > (int64_t)idx) {
            // the embedded server's keys of this call (their count decides the CacheMap switch)
            const uint32_t slot = prule_lookup(st.cpst, p.cflow);
            const uint64_t *vals;
            uint32_t nv;
            if (slot != 0xFFFFFFFFu && st.cpst.param[slot].active && ev_arg(pa, (uint32_t)idx, pv, &vals, &nv) != ARG_NULL)
                for (uint32_t q = 0; q < nv; ++q) {
                    const uint32_t vid = vid_of(st.cpst, (int64_t)vals[q], true);
                    if (vid != 0xFFFFFFFFu) key_of(st.cpst, slot, vid, (int64_t)vals[q], true);
                }
        }
        if (kind[i] != 0 || p.grade != 1 || st.pq[p.id] != kNoQueue || (int64_t)nargs <= (int64_t)idx) continue;
        const uint64_t *vals;
        uint32_t nv;
        if (ev_arg(pa, (uint32_t)idx, pv, &vals, &nv) == ARG_NULL) continue;
        for (uint32_t q = 0; q < nv; ++q)
            need |= lru_count_key<kCount>(st.ptab, st.pstamp, st.pmask, p.id + 1, vals[q], &st.pnew[p.id], mark,
                                          st.overflow);
    }
    if (st.tbase[r] == kNoTBase) return need;
    for (uint32_t k = 0; k < nargs && k < (uint32_t)kMaxParamIdx; ++k) {
        if (!((kmask >> k) & 1ull)) continue;
        const uint32_t j = st.tbase[r] + k;
        if (st.tq[j] != kNoQueue) continue;
        const uint64_t *vals;
        uint32_t nv;
        if (ev_arg(pa, k, pv, &vals, &nv) == ARG_NULL) continue;
        for (uint32_t q = 0; q < nv; ++q)
            need |= lru_count_key<kCount>(st.ttab, st.tstamp, st.tmask, tmap_owner(r, k), vals[q], &st.tnew[j], mark,
                                          st.overflow);
    }
    return need;
}

// the claim launch (every event; those that marked a slot first into st.lneed).  Each workgroup takes kLruChunk
// consecutive events and lists its own in LDS first: one list atomic per workgroup (one per wave queued the
// waves of the whole GPU at one address)
constexpr uint32_t kLruChunk = 4096;
__global__ __launch_bounds__(kT) void k_lru_claim(FlowState st, const uint8_t *__restrict__ kind,
                                                  const uint32_t *__restrict__ resource,
                                                  const uint8_t *__restrict__ flags,
                                                  const uint64_t *__restrict__ param_in,
                                                  const uint64_t *__restrict__ pvals, uint32_t n) {
    __shared__ uint32_t ll[kLruChunk];
    __shared__ uint32_t ln, lbase;
    if (threadIdx.x == 0) ln = 0;
    __syncthreads();
    const uint64_t mark = kStampMark | st.seq_base;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c0 = blockIdx.x * kLruChunk, c1 = min(n, c0 + kLruChunk);
    for (uint32_t i0 = c0; i0 < c1; i0 += kT) {  // whole waves go round the loop together (the ballot below)
        const uint32_t i = i0 + threadIdx.x;
        const bool need = i < c1 && lru_count_event<false>(st, i, kind, resource, flags, param_in, pvals, mark);
        const uint64_t bal = __ballot(need);
        if (!bal) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&ln, (uint32_t)__popcll(bal));
        base = __shfl(base, 0);
        if (need) ll[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = i;
    }
    __syncthreads();
    const uint32_t cnt = ln;
    if (threadIdx.x == 0 && cnt) lbase = atomicAdd(&st.lru_ctl[2], cnt);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < cnt; t += kT) st.lneed[lbase + t] = ll[t];
}

// the count launch over the listed events
__global__ __launch_bounds__(kT) void k_lru_count(FlowState st, const uint8_t *__restrict__ kind,
                                                  const uint32_t *__restrict__ resource,
                                                  const uint8_t *__restrict__ flags,
                                                  const uint64_t *__restrict__ param_in,
                                                  const uint64_t *__restrict__ pvals) {
    const uint64_t mark = kStampMark | st.seq_base;
    const uint32_t m = st.lru_ctl[2];
    for (uint32_t t = blockIdx.x * kT + threadIdx.x; t < m; t += gridDim.x * kT)
        (void)lru_count_event<true>(st, st.lneed[t], kind, resource, flags, param_in, pvals, mark);
}

// 2. owners that could pass their capacity switch to LRU mode: a queue area from the pool, marked
//    for the collect pass (head = kLruBuilding), their resource replayed in arrival order from now on
constexpr uint64_t kLruBuilding = ~0ull;
__global__ __launch_bounds__(kT) void k_lru_decide(FlowState st) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i == 0) st.lru_ctl[2] = 0;  // the count launch (ahead of this one) is done with the list
    if (i >= st.nprid + st.ntslot) return;
    const bool th = i >= st.nprid;
    const uint32_t j = th ? i - st.nprid : i;
    uint32_t *ctr = th ? &st.tnew[j] : &st.pnew[j];
    const uint32_t c = *ctr;
    if (!c) return;
    *ctr = 0;
    uint64_t *q = th ? &st.tq[j] : &st.pq[j];
    const uint32_t cap = th ? kThreadMapCap : st.pcap[j];
    const uint32_t size = th ? st.tsize[j] : st.psize[j];
    if (*q != kNoQueue || (uint64_t)size + c <= (uint64_t)cap) return;
    const uint64_t need = 2ull * cap + 3;  // meta + 2 cap + 2 records
    const unsigned long long off = atomicAdd(st.lcursor, (unsigned long long)need);
    if (off + need > st.lpool_cap) {
        atomicOr(&st.lru_ctl[1], 1u);
        atomicOr(st.overflow, 1u);
        return;
    }
    st.lpool[off] = LruRec{kLruBuilding, 0};
    *q = off;
    st.lru_list[atomicAdd(&st.lru_ctl[0], 1u)] = th ? (kLruThread | j) : j;
    const uint32_t res = th ? st.tres[j / kMaxParamIdx] : st.pres[j];
    if (res < st.nres) st.lru_res[res] = 1;
}

// 3. the switched owners' present keys into their queues (every map slot once)
__global__ __launch_bounds__(kT) void k_lru_collect(FlowState st) {
    if (st.lru_ctl[0] == 0) return;
    const uint32_t np = st.pmask + 1, nt = st.tmask + 1;
    for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < np + nt; i += gridDim.x * kT) {
        const bool th = i >= np;
        const uint32_t s = th ? i - np : i;
        const PEntry e = th ? st.ttab[s] : st.ptab[s];
        if (e.owner == 0 || e.a == kPAbsent) continue;
        uint64_t qo;
        if (!th) {
            if (e.owner - 1 >= st.nprid) continue;
            qo = st.pq[e.owner - 1];
        } else {
            const uint32_t r = (e.owner & 0xFFFFFFu) - 1u, k = e.owner >> 24;
            if (r >= st.nres || st.tbase[r] == kNoTBase) continue;
            qo = st.tq[st.tbase[r] + k];
        }
        if (qo == kNoQueue || st.lpool[qo].value != kLruBuilding) continue;
        const unsigned long long pos = atomicAdd((unsigned long long *)&st.lpool[qo].stamp, 1ull);
        st.lpool[qo + 1 + pos] = LruRec{e.value, th ? st.tstamp[s] : st.pstamp[s]};
    }
}

// 4. each switched owner's records ordered by stamp (oldest first): one workgroup per owner, bitonic
//    (in LDS up to kLruLds records, else in the queue area itself, which holds 2 cap + 2 >= the padding)
constexpr int kLruSortThreads = 256, kLruLds = 4096;
__global__ __launch_bounds__(kLruSortThreads) void k_lru_sort(FlowState st) {
    __shared__ uint64_t ks[kLruLds], vs[kLruLds];
    const uint32_t nsw = st.lru_ctl[0];
    for (uint32_t w = blockIdx.x; w < nsw; w += gridDim.x) {
        const uint32_t id = st.lru_list[w];
        const bool th = (id & kLruThread) != 0;
        const uint32_t j = id & ~kLruThread;
        const uint64_t qo = th ? st.tq[j] : st.pq[j];
        const uint32_t cap = th ? kThreadMapCap : st.pcap[j];
        const uint32_t size = th ? st.tsize[j] : st.psize[j];
        LruRec *rec = st.lpool + qo + 1;
        const uint32_t n = (uint32_t)st.lpool[qo].stamp;
        uint32_t np2 = 1;
        while (np2 < n) np2 <<= 1;
        if (threadIdx.x == 0 && (n != size || n > cap)) {  // the present counts were kept exactly
            atomicOr(&st.lru_ctl[1], 4u);
            atomicOr(st.overflow, 1u);
        }
        if (np2 <= (uint32_t)kLruLds) {
            for (uint32_t k = threadIdx.x; k < np2; k += kLruSortThreads) {
                ks[k] = k < n ? rec[k].stamp : ~0ull;
                vs[k] = k < n ? rec[k].value : 0ull;
            }
            __syncthreads();
            for (uint32_t kk = 2; kk <= np2; kk <<= 1)
                for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                    for (uint32_t a = threadIdx.x; a < np2; a += kLruSortThreads) {
                        const uint32_t b = a ^ jj;
                        if (b > a) {
                            const bool up = (a & kk) == 0;
                            if ((ks[a] > ks[b]) == up) {
                                const uint64_t tk = ks[a], tv = vs[a];
                                ks[a] = ks[b];
                                vs[a] = vs[b];
                                ks[b] = tk;
                                vs[b] = tv;
                            }
                        }
                    }
                    __syncthreads();
                }
            for (uint32_t k = threadIdx.x; k < n; k += kLruSortThreads) rec[k] = LruRec{vs[k], ks[k]};
        } else {
            for (uint32_t k = n + threadIdx.x; k < np2; k += kLruSortThreads) rec[k] = LruRec{0, ~0ull};
            __syncthreads();
            for (uint32_t kk = 2; kk <= np2; kk <<= 1)
                for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                    for (uint32_t a = threadIdx.x; a < np2; a += kLruSortThreads) {
                        const uint32_t b = a ^ jj;
                        if (b > a) {
                            const bool up = (a & kk) == 0;
                            const LruRec x = rec[a], y = rec[b];
                            if ((x.stamp > y.stamp) == up) {
                                rec[a] = y;
                                rec[b] = x;
                            }
                        }
                    }
                    __syncthreads();
                }
        }
        __syncthreads();
        if (threadIdx.x == 0) st.lpool[qo] = LruRec{0, n};  // head 0, tail n
        __syncthreads();
    }
}

// after a parameter-rule load: a resource keeps arrival-order replay while one of its current owners
// is in LRU mode
__global__ __launch_bounds__(kT) void k_lru_res_refresh(FlowState st) {
    const uint32_t r = blockIdx.x * kT + threadIdx.x;
    if (r >= st.nres) return;
    const ResDev R = st.res[r];
    bool any = false;
    for (uint32_t k = 0; k < R.n_prules; ++k) any |= st.pq[st.prules[R.prule_off + k].id] != kNoQueue;
    if (st.tbase[r] != kNoTBase)
        for (uint32_t k = 0; k < (uint32_t)kMaxParamIdx; ++k) any |= st.tq[st.tbase[r] + k] != kNoQueue;
    st.lru_res[r] = any ? 1 : 0;
}

__global__ __launch_bounds__(kT) void k_lresults(FlowState st, FlowScratch sc, const Payload *__restrict__ pay,
                                                 int8_t *decision, int32_t *wait_ms) {
    if (!gate_is(sc.gate, kGateSeq | kGateBad, 0)) return;
    const uint32_t nvalid = sc.counters[0];
    const uint32_t j = blockIdx.x * kT + threadIdx.x;
    if (j >= nvalid) return;
    const uint32_t r = sc.ev_run[j];
    const uint8_t mode = sc.run_mode[r];
    if (mode == RUN_DONE) return;
    const Payload q = pay[j];
    if (q.idx & F_EXIT) return;
    if (mode == RUN_FAST) {
        decision[q.idx & F_IDX] = sc.ev_eidx[j] < sc.run_f[r] ? D_PASS : D_BLOCK_FLOW;
    } else {
        if (mode == RUN_POS && j >= sc.run_f[r]) {  // k_lwave's saturated tail
            decision[q.idx & F_IDX] = D_BLOCK_FLOW;
            if (wait_ms) wait_ms[q.idx & F_IDX] = 0;
            return;
        }
        if (mode == RUN_WIN) {  // an interior window k_lwave skipped: RateLimiterController.java:46-89 at its state
            const uint32_t w = j / 64;
            const int64_t lo = (w != sc.run_start[r] / 64 && w != (sc.run_end[r] - 1) / 64) ? sc.wstate[w] : kWinWalked;
            if (lo != kWinWalked) {
                const int aq = (int)(q.acq_prio & 0x7FFFFFFFu);
                const double rcount = st.rules[st.res[sc.run_slot[r]].rule_off].count;
                const int64_t cost = aq > 0 ? j_round(1.0 * aq / rcount * 1000) : 0;
                decision[q.idx & F_IDX] = cost > 0 ? D_BLOCK_FLOW : D_PASS;
                if (wait_ms) wait_ms[q.idx & F_IDX] = (cost == 0 && aq > 0) ? (int32_t)(lo - (int64_t)q.ts_off) : 0;
                return;
            }
        }
        const uint32_t v = sc.ev_eidx[j];
        if (v == ~0u) return;
        decision[q.idx & F_IDX] = (v & 1u) ? D_BLOCK_FLOW : D_PASS;
        if (wait_ms) wait_ms[q.idx & F_IDX] = (int32_t)(v >> 1);
    }
}

__global__ void k_node_view(FlowState st, int64_t max_rt, uint32_t r, int64_t now, double *dv, int64_t *iv) {
    if (threadIdx.x || blockIdx.x) return;
    const Ctx c{st, max_rt};
    int64_t *node = st.node + (size_t)r * kNodeWords;
    // StatisticNode getters (each rotates the current window first)
    dv[0] = node_pass_qps(c, node, now);
    sec_current(node, now, max_rt);
    dv[1] = (double)sec_sum(node, now, MB_BLOCK) / 1.0;
    dv[2] = (double)sec_sum(node, now, MB_SUCC) / 1.0;
    dv[3] = (double)sec_sum(node, now, MB_EXC) / 1.0;
    dv[4] = (double)sec_sum(node, now, MB_OPASS) / 1.0;
    const int64_t succ = sec_sum(node, now, MB_SUCC);
    dv[5] = succ == 0 ? 0.0 : (double)sec_sum(node, now, MB_RT) * 1.0 / (double)succ;
    int64_t mr = max_rt;
    for (int j = 0; j < 2; ++j) {
        const int64_t *b = node + kNodeSec + kMB * j;
        if (b[0] != kAbsent && !(now - b[0] > kSecInterval) && b[MB_MINRT] < mr) mr = b[MB_MINRT];
    }
    dv[6] = (double)(mr < 1 ? 1 : mr);
    dv[7] = node_prev_pass_qps(c, node, now);
    {  // maxSuccessQps: ArrayMetric.maxSuccess() (currentWindow, max over values(), at least 1) x 2 / 1.0
        sec_current(node, now, max_rt);
        int64_t ms = 0;
        for (int j = 0; j < 2; ++j) {
            const int64_t *b = node + kNodeSec + kMB * j;
            if (b[0] != kAbsent && !(now - b[0] > kSecInterval) && b[MB_SUCC] > ms) ms = b[MB_SUCC];
        }
        dv[8] = (double)(ms < 1 ? 1 : ms) * 2.0 / 1.0;
    }
    dv[9] = node_prev_qps(c, node, now, MB_BLOCK);
    min_current(node, now, max_rt);
    iv[0] = min_sum(node, now, MB_PASS);
    iv[1] = min_sum(node, now, MB_BLOCK);
    iv[2] = min_sum(node, now, MB_SUCC);
    iv[3] = min_sum(node, now, MB_EXC);
    iv[4] = node[kNodeThreads];
    iv[5] = node_waiting(node, now);
}

__global__ void k_init_nodes(int64_t *node, uint32_t n, int64_t max_rt) {
    const uint32_t r = blockIdx.x * kT + threadIdx.x;
    if (r >= n) return;
    int64_t *p = node + (size_t)r * kNodeWords;
    for (int j = 0; j < 2; ++j) {
        p[kNodeSec + kMB * j] = kAbsent;
        mb_zero(p + kNodeSec + kMB * j, max_rt);
        p[kNodeBor + 2 * j] = kAbsent;
        p[kNodeBor + 2 * j + 1] = 0;
    }
    for (int j = 0; j < 60; ++j) {
        p[kNodeMin + kMB * j] = kAbsent;
        mb_zero(p + kNodeMin + kMB * j, max_rt);
    }
    p[kNodeThreads] = 0;
    p[kNodeLastFetch] = -1;
}

// StatisticNode.metrics() (CORE/node/StatisticNode.java:120-157) over ArrayMetric.details()
// (ArrayMetric.java:166-218): rotate the minute window at now, then every listed bucket
// (LeapArray.list(now): not deprecated) becomes a MetricNode; those newer than lastFetchTime,
// older than the current second and with a non-zero field are emitted.
__global__ __launch_bounds__(kT) void k_metrics(FlowState st, int64_t max_rt, int64_t now, sga_metric_node *out,
                                                uint32_t cap, uint32_t *count) {
    const uint32_t r = blockIdx.x * kT + threadIdx.x;
    if (r > st.nres) return;  // node nres = ENTRY_NODE
    int64_t *node = st.node + (size_t)r * kNodeWords;
    const int64_t cur = now - now % 1000;
    min_current(node, now, max_rt);
    const int64_t last = node[kNodeLastFetch];
    int64_t nlast = last;
    for (int j = 0; j < 60; ++j) {
        const int64_t *b = node + kNodeMin + kMB * j;
        if (b[0] == kAbsent || now - b[0] > kMinInterval) continue;
        sga_metric_node m;
        m.timestamp = b[0];
        m.pass_qps = b[MB_PASS];
        m.block_qps = b[MB_BLOCK];
        m.success_qps = b[MB_SUCC];
        m.exception_qps = b[MB_EXC];
        m.rt = m.success_qps != 0 ? b[MB_RT] / m.success_qps : b[MB_RT];
        m.occupied_pass_qps = b[MB_OPASS];
        m.resource = r == st.nres ? SGA_ENTRY_NODE : r;
        m.concurrency = 0;
        const bool in_time = m.timestamp > last && m.timestamp < cur;
        const bool valid = m.pass_qps > 0 || m.block_qps > 0 || m.success_qps > 0 || m.exception_qps > 0 ||
                           m.rt > 0 || m.occupied_pass_qps > 0;
        if (in_time && valid) {
            const uint32_t k = atomicAdd(count, 1u);
            if (k < cap) out[k] = m;
            nlast = m.timestamp > nlast ? m.timestamp : nlast;
        }
    }
    node[kNodeLastFetch] = nlast;
}

__global__ void k_clear_ptab(PEntry *t, uint32_t n) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i < n) t[i] = PEntry{0, 0, 0, kPAbsent, kPAbsent};
}

// slots claimed by a map and keys present in it (one atomic pair per workgroup).  A rule map's entry is
// {time, tokens}; a thread-count entry (tt) keeps its count in a, and b is the per-segment flag word
// k_pseg_heads ORs into it, which may be left off kPAbsent when a batch stops at a gate check, so only a
// counts there.
__device__ __forceinline__ bool pentry_present(const PEntry &e, bool tt) {
    return e.a != kPAbsent || (!tt && e.b != kPAbsent);
}
__global__ void k_count_keys(const PEntry *__restrict__ t, uint32_t n, uint32_t *__restrict__ out, int tt) {
    __shared__ uint32_t ws[2][kT / 64];
    uint32_t c = 0, p = 0;
    for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
        const PEntry e = t[i];
        c += e.owner != 0 ? 1u : 0u;
        p += (e.owner != 0 && pentry_present(e, tt)) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c += (uint32_t)__shfl_down((int)c, o, 64);
        p += (uint32_t)__shfl_down((int)p, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        ws[0][threadIdx.x >> 6] = c;
        ws[1][threadIdx.x >> 6] = p;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t2 = 0, p2 = 0;
        for (int w = 0; w < kT / 64; ++w) {
            t2 += ws[0][w];
            p2 += ws[1][w];
        }
        if (t2) atomicAdd(out, t2);
        if (p2) atomicAdd(out + 1, p2);
    }
}

// every present key of `old` (with its stamp) into the empty table `nt` (same hash as ptab_get; entries
// keep their counters); claimed slots of absent keys are dropped
__global__ void k_rehash(const PEntry *__restrict__ old, const uint64_t *__restrict__ ostamp, uint32_t oldn,
                         PEntry *__restrict__ nt, uint64_t *__restrict__ nstamp, uint32_t nmask, uint32_t *overflow,
                         int tt) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i >= oldn) return;
    const PEntry e = old[i];
    if (e.owner == 0 || !pentry_present(e, tt)) return;
    uint32_t h = (uint32_t)splitmix64(e.value ^ ((uint64_t)e.owner << 40) ^ 0xA5A5ULL) & nmask;
    for (uint32_t probe = 0; probe <= nmask; ++probe) {
        if (atomicCAS(&nt[h].owner, 0u, e.owner) == 0u) {
            claim_note(nt, h);
            nt[h].value = e.value;
            nt[h].a = e.a;
            nt[h].b = tt ? kPAbsent : e.b;
            if (nstamp) nstamp[h] = ostamp ? ostamp[i] : 0;
            return;
        }
        h = (h + 1) & nmask;
    }
    atomicOr(overflow, 1u);
}

}  // namespace

// ======================================================================== host side
// a parameter map's slots start after its claim counters
static PEntry *tab_data(const DevBuf<PEntry> &d) { return d.p ? d.p + kClaimHdr : nullptr; }
static size_t tab_slots(const DevBuf<PEntry> &d) { return d.n > kClaimHdr ? d.n - kClaimHdr : 0; }

FlowState FlowEngine::state() const {
    FlowState s{};
    s.node = d_node.p;
    s.rules = d_rules.p;
    s.prules = d_prules.p;
    s.hot_v = d_hot_v.p;
    s.hot_t = d_hot_t.p;
    s.cbs = d_cbs.p;
    s.res = d_res.p;
    s.ptab = tab_data(d_ptab);
    s.ttab = tab_data(d_ttab);
    s.pmask = tab_slots(d_ptab) ? (uint32_t)(tab_slots(d_ptab) - 1) : 0;
    s.tmask = tab_slots(d_ttab) ? (uint32_t)(tab_slots(d_ttab) - 1) : 0;
    s.nres = nres;
    s.overflow = d_overflow.p;
    s.cst = cluster_st;
    s.cluster_on = cluster_on;
    s.gate = nullptr;
    s.tmapmask = d_tmapmask.p;
    s.cpst = cparam_st;
    s.cpst.seq = seq;  // access stamps of the embedded server's parameter maps: this batch's events
    // CacheMap capacity (null until parameter rules are loaded)
    const bool lru = d_psize.p != nullptr;
    s.pstamp = lru ? d_pstamp.p : nullptr;
    s.tstamp = lru ? d_tstamp.p : nullptr;
    s.psize = d_psize.p;
    s.pq = d_pq.p;
    s.pcap = d_pcap.p;
    s.pres = d_pres.p;
    s.tbase = lru ? d_tbase.p : nullptr;
    s.tres = d_tres.p;
    s.tsize = d_tsize.p;
    s.tq = d_tq.p;
    s.lpool = d_lpool.p;
    s.lpool_cap = d_lpool.n;
    s.lcursor = d_lcursor.p;
    s.pnew = d_pnew.p;
    s.tnew = d_tnew.p;
    s.lru_res = lru ? d_lru_res.p : nullptr;
    static const bool lru_ps = !(getenv("SGA_LRU_PS") && atoi(getenv("SGA_LRU_PS")) == 0);
    s.lru_ps = lru_ps ? 1 : 0;
    s.lru_ctl = d_lru_ctl.p;
    s.lru_list = d_lru_list.p;
    s.lneed = d_lneed.p;
    s.nprid = lru ? (uint32_t)d_psize.n : 0;
    s.ntslot = lru ? ntbase * (uint32_t)kMaxParamIdx : 0;
    s.seq_base = seq;
    return s;
}

// Per-id and per-slot CacheMap arrays after a parameter-rule load: new rule ids start empty in free mode,
// resources with rules get thread-map owner slots (kept for good), the queue pool covers every current
// owner switching once.
__global__ void k_fill_u32(uint32_t *p, uint32_t v, size_t n) {
    const size_t i = (size_t)blockIdx.x * kT + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_fill_u64(uint64_t *p, uint64_t v, size_t n) {
    const size_t i = (size_t)blockIdx.x * kT + threadIdx.x;
    if (i < n) p[i] = v;
}
template <class T>
static void grow_fill(DevBuf<T> &b, size_t n, T v, hipStream_t s) {
    const size_t old = b.p ? b.n : 0;
    if (n <= old) return;
    b.grow(n, s);
    const size_t m = n - old;
    if (sizeof(T) == 8)
        hipLaunchKernelGGL(k_fill_u64, dim3((unsigned)((m + kT - 1) / kT)), dim3(kT), 0, s, (uint64_t *)(b.p + old),
                           (uint64_t)v, m);
    else
        hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)((m + kT - 1) / kT)), dim3(kT), 0, s, (uint32_t *)(b.p + old),
                           (uint32_t)v, m);
}

void FlowEngine::lru_sync_rules() {
    const size_t nid = std::max<size_t>(next_prule_id, 1);
    grow_fill<uint32_t>(d_psize, nid, 0u, stream);
    grow_fill<uint32_t>(d_pnew, nid, 0u, stream);
    grow_fill<uint64_t>(d_pq, nid, kNoQueue, stream);
    std::vector<uint32_t> pcap(nid, 0), pres(nid, 0xFFFFFFFFu);
    if (d_pcap.p && d_pcap.n) {  // ids of earlier rules keep their values
        std::vector<uint32_t> o(d_pcap.n), r(d_pres.n);
        SGA_HIP_CHECK(hipMemcpyAsync(o.data(), d_pcap.p, o.size() * 4, hipMemcpyDeviceToHost, stream));
        SGA_HIP_CHECK(hipMemcpyAsync(r.data(), d_pres.p, r.size() * 4, hipMemcpyDeviceToHost, stream));
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        std::copy(o.begin(), o.end(), pcap.begin());
        std::copy(r.begin(), r.end(), pres.begin());
    }
    uint64_t pool = 0;
    for (size_t k = 0; k < h_prules.size(); ++k) {
        const ParamRuleDev &d = h_prules[k];
        pcap[d.id] = d.cap;
        pres[d.id] = h_prule_src[k].resource;
        pool += 2 * (2ull * d.cap + 3);  // its time/token map and one thread-count map
    }
    for (uint32_t r = 0; r < nres; ++r)
        if (h_res[r].n_prules && h_tbase[r] == kNoTBase) h_tbase[r] = (ntbase++) * (uint32_t)kMaxParamIdx;
    std::vector<uint32_t> tres(std::max<uint32_t>(ntbase, 1), 0xFFFFFFFFu);
    for (uint32_t r = 0; r < nres; ++r)
        if (h_tbase[r] != kNoTBase) tres[h_tbase[r] / kMaxParamIdx] = r;
    d_pcap.alloc(nid);
    d_pres.alloc(nid);
    SGA_HIP_CHECK(hipMemcpyAsync(d_pcap.p, pcap.data(), nid * 4, hipMemcpyHostToDevice, stream));
    SGA_HIP_CHECK(hipMemcpyAsync(d_pres.p, pres.data(), nid * 4, hipMemcpyHostToDevice, stream));
    const size_t nts = std::max<size_t>((size_t)ntbase * kMaxParamIdx, 1);
    grow_fill<uint32_t>(d_tsize, nts, 0u, stream);
    grow_fill<uint32_t>(d_tnew, nts, 0u, stream);
    grow_fill<uint64_t>(d_tq, nts, kNoQueue, stream);
    d_tres.alloc(tres.size());
    SGA_HIP_CHECK(hipMemcpyAsync(d_tres.p, tres.data(), tres.size() * 4, hipMemcpyHostToDevice, stream));
    if (d_tbase.n < std::max<size_t>(nres, 1)) d_tbase.alloc(std::max<size_t>(nres, 1));
    SGA_HIP_CHECK(hipMemcpyAsync(d_tbase.p, h_tbase.data(), (size_t)nres * 4, hipMemcpyHostToDevice, stream));
    if (d_lru_list.n < nid + nts) d_lru_list.alloc(nid + nts);
    if (!d_lru_ctl.p) {
        d_lru_ctl.alloc(4);
        SGA_HIP_CHECK(hipMemsetAsync(d_lru_ctl.p, 0, 16, stream));
        d_lcursor.alloc(1);
        SGA_HIP_CHECK(hipMemsetAsync(d_lcursor.p, 0, 8, stream));
    }
    if (!d_lru_res.p) {
        d_lru_res.alloc(std::max<size_t>(nres, 1));
        SGA_HIP_CHECK(hipMemsetAsync(d_lru_res.p, 0, std::max<size_t>(nres, 1), stream));
    }
    if (!d_pstamp.p) {
        d_pstamp.alloc(tab_slots(d_ptab));
        d_tstamp.alloc(tab_slots(d_ttab));
        SGA_HIP_CHECK(hipMemsetAsync(d_pstamp.p, 0, tab_slots(d_ptab) * 8, stream));
        SGA_HIP_CHECK(hipMemsetAsync(d_tstamp.p, 0, tab_slots(d_ttab) * 8, stream));
    }
    // the pool: what is in use plus every current owner switching once (queue areas are not reused)
    unsigned long long used = 0;
    SGA_HIP_CHECK(hipMemcpyAsync(&used, d_lcursor.p, 8, hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    if (d_lpool.n < used + pool) d_lpool.grow(used + pool + 1024, stream);
    upload_res();
    const FlowState st = state();
    hipLaunchKernelGGL(k_lru_res_refresh, dim3((nres + kT - 1) / kT), dim3(kT), 0, stream, st);
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
}

void FlowEngine::lru_prepare(const uint8_t *kind, const uint32_t *resource, const uint8_t *flags, const uint64_t *param,
                             const uint64_t *pvals, uint32_t n, hipStream_t s) {
    if (!d_psize.p || h_prules.empty()) return;
    if (d_lneed.n < n) d_lneed.grow(n, s);
    const FlowState st = state();
    const uint32_t nb = std::min<uint32_t>((n + kT - 1) / kT, 2048);
    hipLaunchKernelGGL(k_lru_claim, dim3(std::max<uint32_t>((n + kLruChunk - 1) / kLruChunk, 1)), dim3(kT), 0, s, st,
                       kind, resource, flags, param, pvals, n);
    hipLaunchKernelGGL(k_lru_count, dim3(std::max<uint32_t>(nb, 1)), dim3(kT), 0, s, st, kind, resource, flags,
                       param, pvals);
    const uint32_t no = st.nprid + st.ntslot;
    hipLaunchKernelGGL(k_lru_decide, dim3((no + kT - 1) / kT), dim3(kT), 0, s, st);
    hipLaunchKernelGGL(k_lru_collect, dim3(2048), dim3(kT), 0, s, st);
    hipLaunchKernelGGL(k_lru_sort, dim3(64), dim3(kLruSortThreads), 0, s, st);
    if (cparam_hook && has_cluster_prules && cluster_on && cparam_st.ctl) cparam_hook(s);
    static const int prof = getenv("SGA_LRU_PROF") ? atoi(getenv("SGA_LRU_PROF")) : 0;  // diagnostics only
    if (prof) {
        static bool on = false;
        unsigned long long v[22];
        if (on) {  // the previous batch's counters
            SGA_HIP_CHECK(hipMemcpyFromSymbolAsync(v, HIP_SYMBOL(g_lru_prof), 8 * sizeof(v[0]), 0, hipMemcpyDeviceToHost, s));
            SGA_HIP_CHECK(hipStreamSynchronize(s));
            fprintf(stderr, "lru_prof pushes %llu compactions %llu scanned %llu compact_ticks %llu evictions %llu popped %llu "
                    "entry_ticks %llu exit_ticks %llu\n", v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
            SGA_HIP_CHECK(hipMemcpyFromSymbolAsync(v, HIP_SYMBOL(g_lps_prof), sizeof(v), 0, hipMemcpyDeviceToHost, s));
            SGA_HIP_CHECK(hipStreamSynchronize(s));
            fprintf(stderr, "lps_prof events %llu chunks %llu ticks: loads %llu leaders %llu records %llu scan %llu rounds "
                    "%llu write-back %llu queue %llu; longest resource: wave 0 %llu wave 1 %llu, busy %llu / %llu; time map: pops "
                    "%llu global %llu evictions %llu accesses %llu; thread map: pops %llu global %llu evictions %llu "
                    "accesses %llu\n", v[0], v[7], v[1], v[2], v[3], v[4], v[5], v[6], v[20], v[16], v[17], v[18], v[19], v[8], v[9],
                    v[10], v[11], v[12], v[13], v[14], v[15]);
        }
        std::memset(v, 0, sizeof(v));
        SGA_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lps_prof), v, sizeof(v), 0, hipMemcpyHostToDevice, s));
        const int one = 1;
        SGA_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lru_prof), v, 8 * sizeof(v[0]), 0, hipMemcpyHostToDevice, s));
        SGA_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lru_prof_on), &one, sizeof(one), 0, hipMemcpyHostToDevice, s));
        on = true;
    }
    static const int dbg = getenv("SGA_LRU_DEBUG") ? atoi(getenv("SGA_LRU_DEBUG")) : 0;  // diagnostics only
    if (dbg) {
        uint32_t ctl[4];
        SGA_HIP_CHECK(hipMemcpyAsync(ctl, d_lru_ctl.p, 16, hipMemcpyDeviceToHost, s));
        SGA_HIP_CHECK(hipStreamSynchronize(s));
        std::vector<uint32_t> lst(std::min<uint32_t>(ctl[0], 8));
        if (!lst.empty())
            SGA_HIP_CHECK(hipMemcpy(lst.data(), d_lru_list.p, lst.size() * 4, hipMemcpyDeviceToHost));
        fprintf(stderr, "lru_prepare seq=%llu n=%u switched=%u err=%u", (unsigned long long)seq, n, ctl[0], ctl[1]);
        for (uint32_t x : lst) {
            const bool th = x & kLruThread;
            const uint32_t j = x & ~kLruThread;
            uint32_t sz = 0;
            SGA_HIP_CHECK(hipMemcpy(&sz, (th ? d_tsize.p : d_psize.p) + j, 4, hipMemcpyDeviceToHost));
            fprintf(stderr, " %s%u(size %u)", th ? "t" : "p", j, sz);
        }
        fprintf(stderr, "\n");
    }
    SGA_HIP_CHECK(hipMemsetAsync(d_lru_ctl.p, 0, 4, s));  // switches of this batch done
}

__global__ void k_set_cslot(FlowRuleDev *rules, const uint32_t *idx, const int32_t *slot, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rules[idx[i]].cslot = slot[i];
}

// The token server's slot of every cluster-mode rule's flowId (-1: no active cluster rule), written
// into the device rules without touching their controller state.  A flowId shared by the cluster
// rules of two resources would be decided by two lanes at once: refused.
int FlowEngine::resolve_cluster(const std::function<int32_t(int64_t)> &slot_of_flow, uint64_t gen) {
    if (!has_cluster_rules || gen == cluster_resolved_gen) return 0;
    std::vector<uint32_t> idx;
    std::vector<int32_t> slot;
    std::vector<std::pair<int64_t, uint32_t>> owner;
    for (uint32_t r = 0; r < nres; ++r)
        for (uint32_t k = 0; k < h_res[r].n_rules; ++k) {
            FlowRuleDev &d = h_rules[h_res[r].rule_off + k];
            if (!d.cluster) continue;
            const int32_t sl = slot_of_flow(d.cflow);
            if (sl == -2) return SGA_ENOSYS;  // the flowId's namespace has a GlobalRequestLimiter
            d.cslot = sl;
            idx.push_back(h_res[r].rule_off + k);
            slot.push_back(sl);
            owner.emplace_back(d.cflow, r);
        }
    std::sort(owner.begin(), owner.end());
    for (size_t i = 1; i < owner.size(); ++i)
        if (owner[i].first == owner[i - 1].first && owner[i].second != owner[i - 1].second) return SGA_ENOSYS;
    if (!idx.empty()) {
        DevBuf<uint32_t> di;
        DevBuf<int32_t> ds;
        di.alloc(idx.size());
        ds.alloc(slot.size());
        SGA_HIP_CHECK(hipMemcpyAsync(di.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipMemcpyAsync(ds.p, slot.data(), slot.size() * 4, hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(k_set_cslot, dim3((unsigned)((idx.size() + kT - 1) / kT)), dim3(kT), 0, stream, d_rules.p,
                           di.p, ds.p, (uint32_t)idx.size());
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }
    cluster_resolved_gen = gen;
    return 0;
}

int FlowEngine::set_resources(uint32_t n) {
    if (n == nres) return 0;
    if (nres != 0) return SGA_EINVAL;  // resource table is fixed once set
    if (n >= (1u << 24)) return SGA_EINVAL;  // thread-count map owners: resource + 1 in 24 bits
    nres = n;
    d_tmapmask.alloc((size_t)n + 1);
    SGA_HIP_CHECK(hipMemsetAsync(d_tmapmask.p, 0, ((size_t)n + 1) * 8, stream));
    d_node.alloc(((size_t)n + 1) * kNodeWords);  // + Constants.ENTRY_NODE at index n
    hipLaunchKernelGGL(k_init_nodes, dim3((n + 1 + kT - 1) / kT), dim3(kT), 0, stream, d_node.p, n + 1,
                       (int64_t)cfg.statistic_max_rt);
    h_res.assign(n, ResDev{});
    h_tbase.assign(n, kNoTBase);
    d_overflow.alloc(1);
    SGA_HIP_CHECK(hipMemsetAsync(d_overflow.p, 0, 4, stream));
    // parameter tables: power of two, sized for the batch capacity
    size_t pc = 1;
    while (pc < (size_t)cfg.max_batch * 2) pc <<= 1;
    pc = std::max<size_t>(pc, 1 << 16);
    d_ptab.alloc(pc + kClaimHdr);
    d_ttab.alloc(pc + kClaimHdr);
    for (DevBuf<PEntry> *t : {&d_ptab, &d_ttab}) {
        SGA_HIP_CHECK(hipMemsetAsync(t->p, 0, kClaimHdr * sizeof(PEntry), stream));  // claim counters
        hipLaunchKernelGGL(k_clear_ptab, dim3((unsigned)((pc + kT - 1) / kT)), dim3(kT), 0, stream, tab_data(*t),
                           (uint32_t)pc);
    }
    upload_res();
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    return 0;
}

void FlowEngine::upload_res() {
    for (uint32_t r = 0; r < nres; ++r) {
        ResDev &R = h_res[r];
        R.fast &= 2u;  // bit1 (a thread-count map exists) is sticky
        if (R.n_rules == 1 && R.n_prules == 0 && R.n_cbs == 0 && !(R.fast & 2u)) {
            const FlowRuleDev &fr = h_rules[R.rule_off];
            if (fr.cluster) {
                // cluster-mode rule: every entry asks the token server (per-event replay)
            } else if (fr.grade == 1 && (fr.behavior == 0 || fr.behavior == 1)) R.fast = 1;
            else if (fr.grade == 1 && fr.behavior == 2) R.fast = 4;  // pacing only: k_lflows register loop
        }
    }
    if (d_res.n < std::max<size_t>(nres, 1)) d_res.alloc(std::max<size_t>(nres, 1));
    if (nres) SGA_HIP_CHECK(hipMemcpyAsync(d_res.p, h_res.data(), nres * sizeof(ResDev), hipMemcpyHostToDevice, stream));
}

// FlowRuleManager.loadRules -> FlowRuleUtil.buildFlowRuleMap/generateRater: raters regenerated
// (controller state reset), node statistics kept.  FlowRuleUtil.java:84-195
int FlowEngine::load_flow_rules(const sga_flow_rule *rules, size_t n) {
    if (!nres) return SGA_EINVAL;
    std::vector<std::vector<FlowRuleDev>> per(nres);
    int valid = 0;
    for (size_t i = 0; i < n; ++i) {
        const sga_flow_rule &r = rules[i];
        if (r.resource >= nres) continue;
        bool ok = r.count >= 0 && r.grade >= 0 && r.strategy >= 0 && r.control_behavior >= 0 && r.strategy == 0;
        if (ok && r.cluster_mode) {  // FlowRuleUtil.checkClusterField / checkClusterConcurrentField (:197-240)
            ok = r.cluster_flow_id > 0 && r.cluster_sample_count > 0 && r.cluster_window_ms > 0 &&
                 r.cluster_window_ms % r.cluster_sample_count == 0 && (r.grade != 1 || r.cluster_strategy == 0);
        }
        if (ok && r.grade == 1) {
            switch (r.control_behavior) {
            case 1: ok = r.warm_up_period_sec > 0; break;
            case 2: ok = r.max_queueing_time_ms > 0; break;
            case 3: ok = r.warm_up_period_sec > 0 && r.max_queueing_time_ms > 0; break;
            default: break;
            }
        } else if (ok && r.grade != 0) {
            ok = false;
        }
        if (!ok) continue;
        FlowRuleDev d{};
        d.behavior = r.grade == 1 ? r.control_behavior : 0;
        if (d.behavior < 0 || d.behavior > 3) d.behavior = 0;
        d.grade = r.grade;
        d.count = r.count;
        d.max_queue = r.max_queueing_time_ms;
        d.cold_factor = cfg.cold_factor;
        d.latest_passed = -1;
        d.cluster = r.cluster_mode ? 1 : 0;
        d.cfallback = r.cluster_fallback ? 1 : 0;
        d.cflow = r.cluster_flow_id;
        d.cslot = -1;
        if (d.behavior == 1 || d.behavior == 3) {  // WarmUpController.construct, :83-106
            d.warning_token = j_d2i((double)r.warm_up_period_sec * r.count) / (cfg.cold_factor - 1);
            d.max_token = d.warning_token + j_d2i(2 * r.warm_up_period_sec * r.count / (1.0 + cfg.cold_factor));
            d.slope = (cfg.cold_factor - 1.0) / r.count / (double)(d.max_token - d.warning_token);
        }
        per[r.resource].push_back(d);
        valid++;
    }
    h_rules.clear();
    has_cluster_rules = false;
    cluster_resolved_gen = ~0ull;
    for (uint32_t r = 0; r < nres; ++r) {
        for (const FlowRuleDev &d : per[r]) has_cluster_rules |= d.cluster != 0;
        h_res[r].rule_off = (uint32_t)h_rules.size();
        h_res[r].n_rules = (uint32_t)per[r].size();
        h_rules.insert(h_rules.end(), per[r].begin(), per[r].end());
    }
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    d_rules.alloc(std::max<size_t>(h_rules.size(), 1));
    if (!h_rules.empty())
        SGA_HIP_CHECK(hipMemcpyAsync(d_rules.p, h_rules.data(), h_rules.size() * sizeof(FlowRuleDev),
                                     hipMemcpyHostToDevice, stream));
    upload_res();
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    return valid;
}

// ParamFlowRule.equals (ParamFlowRule.java:192-210) of a loaded rule -- whose paramIdx the slot may have
// rewritten (applyRealParamIdx mutates the rule object): aidx is the index in force -- and a new rule
static bool prule_equal(const sga_param_rule &a, int32_t aidx, const std::vector<uint64_t> &av,
                        const std::vector<int32_t> &at, const sga_param_rule &b) {
    if (a.resource != b.resource || a.grade != b.grade || a.count != b.count || a.control_behavior != b.control_behavior ||
        a.max_queueing_time_ms != b.max_queueing_time_ms || a.burst_count != b.burst_count ||
        aidx != b.param_idx || a.duration_in_sec != b.duration_in_sec || a.n_hot != b.n_hot ||
        a.cluster_mode != b.cluster_mode)
        return false;
    if (a.cluster_mode && (a.cluster_fallback != b.cluster_fallback || a.cluster_flow_id != b.cluster_flow_id ||
                           a.cluster_sample_count != b.cluster_sample_count || a.cluster_window_ms != b.cluster_window_ms))
        return false;
    for (uint32_t i = 0; i < b.n_hot; ++i)
        if (av[i] != b.hot_values[i] || at[i] != b.hot_thresholds[i]) return false;
    return true;
}

// ParamFlowRuleUtil.isValidRule + checkCluster (ParamFlowRuleUtil.java:46-69)
static bool prule_valid(const sga_param_rule &r) {
    if (!(r.count >= 0 && r.grade >= 0 && r.duration_in_sec > 0 && r.burst_count >= 0 && r.control_behavior >= 0 &&
          r.max_queueing_time_ms >= 0))
        return false;
    if (r.param_idx < -kMaxParamIdx || r.param_idx >= kMaxParamIdx) return false;  // engine limit (header)
    if (!r.cluster_mode) return true;
    if (!(r.cluster_sample_count > 0 && r.cluster_window_ms > 0 && r.cluster_window_ms % r.cluster_sample_count == 0))
        return false;
    return r.cluster_flow_id > 0;
}

// ParameterMetric.clearForRule / ParameterMetricStorage.clearParamMetricForResource: the thread-count
// entries of the cleared (resource, index) maps read as absent, and the maps no longer exist
__global__ void k_tmap_clear(PEntry *ttab, uint32_t n, const uint64_t *clear, uint32_t nres, uint64_t *tmapmask,
                             const uint32_t *tbase, uint32_t *tsize, uint64_t *tq) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nres) {
        tmapmask[i] &= ~clear[i];
        if (tbase && tbase[i] != kNoTBase)  // a new map: empty, free mode
            for (int k = 0; k < kMaxParamIdx; ++k)
                if ((clear[i] >> k) & 1ull) {
                    tsize[tbase[i] + k] = 0;
                    tq[tbase[i] + k] = kNoQueue;
                }
    }
    if (i >= n) return;
    const uint32_t o = ttab[i].owner;
    if (!o) return;
    const uint32_t r = (o & 0xFFFFFFu) - 1u, k = o >> 24;
    if (r < nres && ((clear[r] >> k) & 1ull)) ttab[i].a = kPAbsent;
}

// ParamFlowRuleManager.loadRules (ParamFlowRuleManager.java:101-150): rules grouped by resource in list
// order; ParameterMetric maps are keyed by the rule, so an equal rule keeps its maps (ids), a new one
// starts empty.  aggregateAndPrepareParamRules: no rules at all clears every metric; a resource left
// without rules loses its metric; each removed rule clears its maps and the thread-count map of its index.
int FlowEngine::load_param_rules(const sga_param_rule *rules, size_t n) {
    if (!nres) return SGA_EINVAL;
    // the indices the slot resolved on the device (applyRealParamIdx) take part in the equality
    std::vector<ParamRuleDev> cur(h_prules.size());
    if (!cur.empty())
        SGA_HIP_CHECK(hipMemcpyAsync(cur.data(), d_prules.p, cur.size() * sizeof(ParamRuleDev), hipMemcpyDeviceToHost,
                                     stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    std::vector<std::vector<size_t>> per(nres);
    for (size_t i = 0; i < n; ++i) {
        const sga_param_rule &r = rules[i];
        if (r.resource >= nres) continue;
        if (!prule_valid(r)) continue;
        if (r.n_hot && (!r.hot_values || !r.hot_thresholds)) continue;
        per[r.resource].push_back(i);
    }
    std::vector<ParamRuleDev> nr;
    std::vector<sga_param_rule> nsrc;
    std::vector<std::vector<uint64_t>> nhv;
    std::vector<std::vector<int32_t>> nht;
    std::vector<uint64_t> hv;
    std::vector<int32_t> ht;
    std::vector<bool> used(h_prule_src.size(), false);
    auto idx_in_force = [&](size_t k) {
        return (k < cur.size() && cur[k].idx_res != kIdxUnresolved) ? cur[k].idx_res : h_prule_src[k].param_idx;
    };
    int valid = 0;
    for (uint32_t res = 0; res < nres; ++res) {
        h_res[res].prule_off = (uint32_t)nr.size();
        h_res[res].n_prules = (uint32_t)per[res].size();
        for (size_t i : per[res]) {
            const sga_param_rule &r = rules[i];
            uint32_t id = 0xFFFFFFFFu;
            int32_t idx_res = kIdxUnresolved;
            for (size_t k = 0; k < h_prule_src.size(); ++k)
                if (!used[k] && prule_equal(h_prule_src[k], idx_in_force(k), h_prule_hot_v[k], h_prule_hot_t[k], r)) {
                    used[k] = true;
                    id = h_prules[k].id;
                    if (k < cur.size()) idx_res = cur[k].idx_res;
                    break;
                }
            if (id == 0xFFFFFFFFu) id = next_prule_id++;
            ParamRuleDev d{};
            d.grade = r.grade;
            d.behavior = r.control_behavior;
            d.count = r.count;
            d.max_queue = r.max_queueing_time_ms;
            d.burst = r.burst_count;
            d.param_idx = r.param_idx;
            d.duration = r.duration_in_sec;
            d.n_hot = (int32_t)r.n_hot;
            d.hot_off = (uint32_t)hv.size();
            d.id = id;
            d.idx_res = idx_res;
            d.cluster = r.cluster_mode ? 1 : 0;
            d.cfallback = r.cluster_fallback ? 1 : 0;
            d.cflow = r.cluster_flow_id;
            // ParameterMetric.initialize: Math.min(BASE_PARAM_MAX_CAPACITY * durationInSec, TOTAL_MAX_CAPACITY)
            d.cap = (uint32_t)std::min<int64_t>((int64_t)4000 * (int64_t)r.duration_in_sec, 200000);
            for (uint32_t h = 0; h < r.n_hot; ++h) {
                hv.push_back(r.hot_values[h]);
                ht.push_back(r.hot_thresholds[h]);
            }
            nr.push_back(d);
            sga_param_rule src = r;
            src.hot_values = nullptr;
            src.hot_thresholds = nullptr;
            nsrc.push_back(src);
            nhv.emplace_back(r.hot_values, r.hot_values + r.n_hot);
            nht.emplace_back(r.hot_thresholds, r.hot_thresholds + r.n_hot);
            valid++;
        }
    }
    // thread-count maps cleared by the reload
    std::vector<uint64_t> clear(nres, 0);
    bool any_clear = false;
    for (size_t k = 0; k < h_prule_src.size(); ++k) {
        const uint32_t res = h_prule_src[k].resource;
        if (res >= nres) continue;
        if (valid == 0 || per[res].empty()) {
            clear[res] = ~0ull;  // clearParamMetricForResource / every metric cleared
            any_clear = true;
        } else if (!used[k]) {
            const int32_t idx = idx_in_force(k);  // clearForRule: threadCountMap.remove(rule.getParamIdx())
            if (idx >= 0 && idx < kMaxParamIdx) {
                clear[res] |= 1ull << idx;
                any_clear = true;
            }
        }
    }
    has_cluster_prules = false;
    for (uint32_t res = 0; res < nres; ++res) {
        if (h_res[res].n_prules) h_res[res].fast |= 2u;  // the resource has parameter rules
        else h_res[res].fast &= ~2u;
    }
    for (const ParamRuleDev &d : nr) has_cluster_prules |= d.cluster != 0;
    h_prules = nr;
    h_prule_src = nsrc;
    h_prule_hot_v = nhv;
    h_prule_hot_t = nht;
    d_prules.alloc(std::max<size_t>(nr.size(), 1));
    d_hot_v.alloc(std::max<size_t>(hv.size(), 1));
    d_hot_t.alloc(std::max<size_t>(ht.size(), 1));
    if (!nr.empty())
        SGA_HIP_CHECK(hipMemcpyAsync(d_prules.p, nr.data(), nr.size() * sizeof(ParamRuleDev), hipMemcpyHostToDevice, stream));
    if (!hv.empty()) {
        SGA_HIP_CHECK(hipMemcpyAsync(d_hot_v.p, hv.data(), hv.size() * 8, hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipMemcpyAsync(d_hot_t.p, ht.data(), ht.size() * 4, hipMemcpyHostToDevice, stream));
    }
    if (any_clear) {
        DevBuf<uint64_t> dc;
        dc.alloc(nres);
        SGA_HIP_CHECK(hipMemcpyAsync(dc.p, clear.data(), (size_t)nres * 8, hipMemcpyHostToDevice, stream));
        const uint32_t tn = (uint32_t)tab_slots(d_ttab);
        const uint32_t m = std::max(tn, nres);
        hipLaunchKernelGGL(k_tmap_clear, dim3((m + kT - 1) / kT), dim3(kT), 0, stream, tab_data(d_ttab), tn, dc.p, nres,
                           d_tmapmask.p, d_tbase.p, d_tsize.p, d_tq.p);
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }
    lru_sync_rules();  // uploads the resources too
    return valid;
}

// DegradeRuleManager.loadRules: an unchanged rule keeps its breaker (state and statistics).
int FlowEngine::load_degrade_rules(const sga_degrade_rule *rules, size_t n) {
    if (!nres) return SGA_EINVAL;
    // current breaker states come back from the device first
    if (!h_cbs.empty()) {
        SGA_HIP_CHECK(hipMemcpyAsync(h_cbs.data(), d_cbs.p, h_cbs.size() * sizeof(CbDev), hipMemcpyDeviceToHost, stream));
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }
    std::vector<CbDev> nc;
    std::vector<sga_degrade_rule> nsrc;
    std::vector<bool> used(h_cb_src.size(), false);
    int valid = 0;
    for (uint32_t res = 0; res < nres; ++res) {
        h_res[res].cb_off = (uint32_t)nc.size();
        uint32_t cnt = 0;
        for (size_t i = 0; i < n; ++i) {
            const sga_degrade_rule &r = rules[i];
            if (r.resource != res) continue;
            bool ok = r.count >= 0 && r.time_window > 0 && r.min_request_amount > 0 && r.stat_interval_ms > 0;
            if (ok) {
                switch (r.grade) {
                case 0: ok = r.slow_ratio_threshold >= 0 && r.slow_ratio_threshold <= 1; break;
                case 1: ok = r.count <= 1; break;
                case 2: break;
                default: ok = false;
                }
            }
            if (!ok) continue;
            int keep = -1;
            for (size_t k = 0; k < h_cb_src.size(); ++k) {
                const sga_degrade_rule &o = h_cb_src[k];
                if (!used[k] && o.resource == r.resource && o.grade == r.grade && o.count == r.count &&
                    o.time_window == r.time_window && o.min_request_amount == r.min_request_amount &&
                    o.slow_ratio_threshold == r.slow_ratio_threshold && o.stat_interval_ms == r.stat_interval_ms) {
                    used[k] = true;
                    keep = (int)k;
                    break;
                }
            }
            CbDev d{};
            if (keep >= 0) {
                d = h_cbs[keep];
            } else {
                d.grade = r.grade;
                d.min_req = r.min_request_amount;
                d.count = r.count;
                d.slow_ratio = r.slow_ratio_threshold;
                d.stat_interval = r.stat_interval_ms;
                d.state = 0;
                d.recovery_ms = (int64_t)r.time_window * 1000;
                d.max_allowed_rt = j_round(r.count);
                d.next_retry = 0;
                d.st_start = kAbsent;
            }
            nc.push_back(d);
            nsrc.push_back(r);
            cnt++;
            valid++;
        }
        h_res[res].n_cbs = cnt;
    }
    h_cbs = nc;
    h_cb_src = nsrc;
    d_cbs.alloc(std::max<size_t>(nc.size(), 1));
    if (!nc.empty())
        SGA_HIP_CHECK(hipMemcpyAsync(d_cbs.p, nc.data(), nc.size() * sizeof(CbDev), hipMemcpyHostToDevice, stream));
    upload_res();
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    return valid;
}

static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }


void FlowEngine::grow_map(DevBuf<PEntry> &tab, DevBuf<uint64_t> &stamp, size_t &ub, size_t add) {
    const bool tt = &tab == &d_ttab;  // the thread-count table
    const size_t n = tab_slots(tab);
    if (ub + add <= n / 4) {
        ub += add;
        return;
    }
    // the exact count of claimed slots: the table's claim counters (a 2 KB read, not a table scan)
    PEntry hdr[kClaimHdr];
    SGA_HIP_CHECK(hipMemcpyAsync(hdr, tab.p, sizeof(hdr), hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    uint64_t claimed = 0;
    for (const PEntry &h : hdr) claimed += (uint64_t)h.a;
    ub = claimed;
    if (ub + add > n / 4) {
        // rehash the present keys (claimed slots of absent keys -- evicted or removed ones -- are dropped)
        // into a table that stays at most a quarter full for two batches like this one (so the next batch
        // needs no counter read either)
        if (!d_keycount.p || d_keycount.n < 2) d_keycount.alloc(2);
        SGA_HIP_CHECK(hipMemsetAsync(d_keycount.p, 0, 8, stream));
        hipLaunchKernelGGL(k_count_keys, dim3((unsigned)std::min<size_t>((n + kT - 1) / kT, 2048)), dim3(kT), 0,
                           stream, tab_data(tab), (uint32_t)n, d_keycount.p, tt ? 1 : 0);
        uint32_t keys[2] = {0, 0};  // claimed slots, present keys
        SGA_HIP_CHECK(hipMemcpyAsync(keys, d_keycount.p, 8, hipMemcpyDeviceToHost, stream));
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        size_t nn = n;
        const size_t room = (keys[1] + 2 * add) * 4 <= ((size_t)1 << 31) ? 2 * add : add;  // 32-bit slot indices
        while (keys[1] + room > nn / 4) nn <<= 1;
        DevBuf<PEntry> nt;
        nt.alloc(nn + kClaimHdr);
        DevBuf<uint64_t> ns;
        if (stamp.p) ns.alloc(nn);
        SGA_HIP_CHECK(hipMemsetAsync(nt.p, 0, kClaimHdr * sizeof(PEntry), stream));
        hipLaunchKernelGGL(k_clear_ptab, dim3((unsigned)((nn + kT - 1) / kT)), dim3(kT), 0, stream, tab_data(nt),
                           (uint32_t)nn);
        hipLaunchKernelGGL(k_rehash, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, stream, tab_data(tab), stamp.p,
                           (uint32_t)n, tab_data(nt), ns.p, (uint32_t)(nn - 1), d_overflow.p, tt ? 1 : 0);
        ub = keys[1];
        uint32_t ovf = 0;
        SGA_HIP_CHECK(hipMemcpyAsync(&ovf, d_overflow.p, 4, hipMemcpyDeviceToHost, stream));
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        if (ovf) {  // a key found no slot in the new table: keep the old one, report -ENOMEM
            SGA_HIP_CHECK(hipMemsetAsync(d_overflow.p, 0, 4, stream));
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
            throw std::bad_alloc();
        }
        std::swap(tab.p, nt.p);
        std::swap(tab.n, nt.n);
        if (stamp.p) {
            std::swap(stamp.p, ns.p);
            std::swap(stamp.n, ns.n);
        }
    }
    ub += add;
}

// Before a batch of m events the maps get room for every key the batch could add: m per parameter rule of
// a resource for the rule maps, and m per argument index with a rule for the thread counts (one event claims
// a thread-count entry for each of its resource's rule indices, tmap_owner(r, k); the rule count bounds the
// distinct indices).  CacheMap capacity bounds the present keys, and a rehash drops the claimed slots of
// evicted / removed ones.
int FlowEngine::ensure_maps(size_t m) {
    // an event claims at most one (rule, value) entry per parameter rule of its resource, and one thread-count
    // entry per distinct argument index those rules name (ParameterMetric's threadCountMap per index)
    uint32_t mpr = 0, midx = 0;
    for (const ResDev &r : h_res) {
        mpr = std::max<uint32_t>(mpr, r.n_prules);
        uint64_t seen = 0;  // argument indices 0..63 (kMaxParamIdx); a negative index (resolved on the device
        uint32_t other = 0;  // against each call's argument count) or a larger one counts once per rule
        for (uint32_t k = 0; k < r.n_prules; ++k) {
            const int32_t ix = h_prules[r.prule_off + k].param_idx;
            if (ix >= 0 && ix < kMaxParamIdx) seen |= 1ull << ix;
            else ++other;
        }
        midx = std::max<uint32_t>(midx, (uint32_t)__builtin_popcountll(seen) + other);
    }
    if (!mpr) return 0;
    const size_t limit = (size_t)1 << 31;  // 32-bit map indices
    if ((pkeys_ub + m * mpr) * 4 > limit || (tkeys_ub + m * midx) * 4 > limit) return SGA_ENOMEM;
    grow_map(d_ptab, d_pstamp, pkeys_ub, m * mpr);
    grow_map(d_ttab, d_tstamp, tkeys_ub, m * midx);
    return 0;
}

// SGA_NO_PSEG=1 (A/B knob): parameter-only resources keep the event-by-event replay
static bool pseg_on() {
    static const bool off = getenv("SGA_NO_PSEG") && atoi(getenv("SGA_NO_PSEG")) == 1;
    return !off;
}

void FlowEngine::launch_pseg(const FlowState &st, const FlowScratch &g, const Payload *pay, const uint32_t *keys,
                             int64_t ts_base, const int64_t *rt, const uint64_t *param, int8_t *decision,
                             int32_t *wait_ms, uint32_t m, hipStream_t s) {
    if (!g.pseg || m == 0) return;
    FlowScratch gs = g;
    const uint64_t none = ((uint64_t)st.tmask + 1) << 32;  // after every map slot
    int sbits = 1;
    while ((1ull << sbits) <= (uint64_t)st.tmask + 1) ++sbits;
    const uint32_t nb = std::min<uint32_t>((m + kT - 1) / kT, 2048);
    if (!h_prules.empty()) {
        // the count pass (lru_prepare, whenever parameter rules are loaded) has claimed every key these events
        // name in free-mode maps already; the claim launch is for an engine without it
#ifdef SGA_TEST_HOOKS  // the test-only build (libsentinel_amd_testhooks.so): fault injection
        static const int force_miss = getenv("SGA_PSEG_FORCE_MISS") ? atoi(getenv("SGA_PSEG_FORCE_MISS")) : 0;
#else
        constexpr int force_miss = 0;
#endif
        if (!d_psize.p)
            hipLaunchKernelGGL(k_pseg_key<true>, dim3(nb), dim3(kT), 0, s, st, gs, pay, keys, param, m, none, 0);
        hipLaunchKernelGGL(k_pseg_key<false>, dim3(nb), dim3(kT), 0, s, st, gs, pay, keys, param, m, none, force_miss);
        // the slot bits sorted in pieces of at most 24 bits (3 radix passes each), least significant first
        uint64_t *el = gs.pel[0], *alt = gs.pel[1];
        const int pieces = (sbits + 23) / 24, pb = (sbits + pieces - 1) / pieces;
        int np = 0;
        for (int lo = 0; lo < sbits; lo += pb) {
            np = radix_sort_u64(el, alt, m, 32 + lo, std::min(pb, sbits - lo), gs.radix, s, false);
            if (np < 0) {  // never expected (at most 24 bits per call)
                fprintf(stderr, "sentinel_amd: parameter segment sort of %d bits refused\n", sbits);
                abort();
            }
            if (np & 1) std::swap(el, alt);
        }
        hipLaunchKernelGGL(k_pseg_heads, dim3((m + kHeadsChunk - 1) / kHeadsChunk), dim3(kT), 0, s, st, gs, pay, el, m,
                           none);
        static const bool dbg = getenv("SGA_PSEG_DEBUG") && atoi(getenv("SGA_PSEG_DEBUG")) == 1;
        if (dbg) {
            uint32_t h[4] = {0, 0, 0, 0}, *dd = gs.radix.err;  // the radix error words are free here
            SGA_HIP_CHECK(hipMemsetAsync(dd, 0, 16, s));
            hipLaunchKernelGGL(k_pseg_check, dim3(nb), dim3(kT), 0, s, st, keys, el, m, none, dd);
            SGA_HIP_CHECK(hipMemcpyAsync(h, dd, 16, hipMemcpyDeviceToHost, s));
            uint32_t c[16];
            SGA_HIP_CHECK(hipMemcpyAsync(c, gs.counters, 64, hipMemcpyDeviceToHost, s));
            SGA_HIP_CHECK(hipStreamSynchronize(s));
            fprintf(stderr, "pseg m=%u flows=%u segs=%u elements=%u unsorted=%u lru=%u wrong_owner=%u sbits=%d np=%d\n", m,
                    c[11], c[12], h[1], h[0], h[2], h[3], sbits, np);
        }
        hipLaunchKernelGGL(k_pseg_solve, dim3(std::min<uint32_t>((m + kT - 1) / kT, 4096)), dim3(kT), 0, s, st,
                           (int64_t)cfg.statistic_max_rt, gs, pay, keys, el, m, ts_base, param, decision, wait_ms);
        hipLaunchKernelGGL(k_pseg_long, dim3(std::min<uint32_t>(m / kPsegLong + 1, 2048)), dim3(64), 0, s, st,
                           (int64_t)cfg.statistic_max_rt, gs, pay, keys, el, ts_base, param, decision, wait_ms);
    }
    if (!h_cbs.empty() && m >= kCbTileMin) {  // long exit-only flows over the whole GPU
        const uint32_t tg = std::min<uint32_t>(2 * (m / kCbRound) + 16, 4096);
        SGA_HIP_CHECK(hipMemsetAsync(gs.cbt_ctl, 0, 8, s));
        hipLaunchKernelGGL(k_cbt_plan, dim3(std::min<uint32_t>(m / kT + 1, 256)), dim3(kT), 0, s, st, gs, pay);
        hipLaunchKernelGGL(k_cbt_tiles<false>, dim3(tg), dim3(64 * kCbW), 0, s, st, gs, pay, ts_base, decision, wait_ms);
        hipLaunchKernelGGL(k_cbt_scan, dim3(m / kCbTileMin / kT + 1), dim3(kT), 0, s, st, gs, pay);
        hipLaunchKernelGGL(k_cbt_tiles<true>, dim3(tg), dim3(64 * kCbW), 0, s, st, gs, pay, ts_base, decision, wait_ms);
        hipLaunchKernelGGL(k_cbt_fin, dim3(m / kCbTileMin / kT + 1), dim3(kT), 0, s, st, gs, pay, ts_base);
    }
    if (!h_cbs.empty()) {
        if (m >= kCbShort)
            hipLaunchKernelGGL(k_cb_flows<kCbW>, dim3(std::min<uint32_t>(m / kCbShort, 1024)), dim3(64 * kCbW), 0, s, st,
                               gs, pay, ts_base, rt, decision, wait_ms);
        hipLaunchKernelGGL(k_cb_flows<1>, dim3(std::min<uint32_t>(std::max<uint32_t>(1, m / 64), 4096)), dim3(64), 0, s, st,
                           gs, pay, ts_base, rt, decision, wait_ms);
    }
    hipLaunchKernelGGL(k_pseg_runs, dim3((m + kTileElems - 1) / kTileElems), dim3(kT), 0, s, st, gs, pay, decision);
    const uint32_t fthreads = std::min<uint32_t>(m, nres);
    hipLaunchKernelGGL(k_pseg_apply, dim3((fthreads + kT - 1) / kT), dim3(kT), 0, s, st, (int64_t)cfg.statistic_max_rt,
                       gs, ts_base);
}

// SGA_HEAVY_PROF=1: k_lheavy phase timers (1024 workgroups x 8 counters), printed by
// FlowEngine::print_heavy_prof at engine release.  Diagnostics only.
static uint64_t *g_heavy_prof = nullptr;
static uint64_t *heavy_prof() {
    static const bool on = getenv("SGA_HEAVY_PROF") && atoi(getenv("SGA_HEAVY_PROF")) == 1;
    if (on && !g_heavy_prof) {
        SGA_HIP_CHECK(hipMalloc((void **)&g_heavy_prof, 1024 * 8 * sizeof(uint64_t)));
        SGA_HIP_CHECK(hipMemset(g_heavy_prof, 0, 1024 * 8 * sizeof(uint64_t)));
    }
    return on ? g_heavy_prof : nullptr;
}

// SGA_LWAVE_PROF=1: k_lwave per-workgroup counters, printed after every launch (diagnostics only)
static uint64_t *g_lwave_prof = nullptr;
static uint64_t *lwave_prof() {
    static const bool on = getenv("SGA_LWAVE_PROF") && atoi(getenv("SGA_LWAVE_PROF")) == 1;
    if (on && !g_lwave_prof) SGA_HIP_CHECK(hipMalloc((void **)&g_lwave_prof, 1024 * 8 * sizeof(uint64_t)));
    if (on) SGA_HIP_CHECK(hipMemset(g_lwave_prof, 0, 1024 * 8 * sizeof(uint64_t)));
    return on ? g_lwave_prof : nullptr;
}
static void print_lwave_prof(hipStream_t s) {
    if (!g_lwave_prof) return;
    std::vector<uint64_t> h(1024 * 8);
    SGA_HIP_CHECK(hipStreamSynchronize(s));
    SGA_HIP_CHECK(hipMemcpy(h.data(), g_lwave_prof, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<int> o(1024);
    for (int b = 0; b < 1024; ++b) o[b] = b;
    std::sort(o.begin(), o.end(), [&](int a, int b) { return h[a * 8 + 2] > h[b * 8 + 2]; });
    for (int k = 0; k < 4; ++k) {
        const uint64_t *p = &h[o[k] * 8];
        fprintf(stderr, "k_lwave wg %d: resources %llu events %llu ms %.2f lane_run %llu (%.2f ms) iters %llu; "
                "longest resource %.2f ms, %llu events, %llu runs, fast %llu\n", o[k], (unsigned long long)p[0],
                (unsigned long long)p[1], p[2] / 1e5, (unsigned long long)p[4], p[3] / 1e5,
                (unsigned long long)p[5], p[6] / 1e5, (unsigned long long)(p[7] >> 32),
                (unsigned long long)((p[7] >> 8) & 0xFFFFFFu), (unsigned long long)(p[7] & 0xFFu));
    }
}

void print_heavy_prof() {
    if (!g_heavy_prof) return;
    std::vector<uint64_t> h(1024 * 8);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h.data(), g_heavy_prof, h.size() * 8, hipMemcpyDeviceToHost);
    int best = 0;
    for (int b = 0; b < 1024; ++b)
        if (h[b * 8 + 5] > h[best * 8 + 5]) best = b;
    fprintf(stderr, "k_lheavy busiest workgroup %d: %llu events; ms stage %.2f insert %.2f "
            "lanes %.2f replay %.2f writeback+stores %.2f dedupe %.2f find %.2f (100 MHz wall clock)\n", best,
            (unsigned long long)h[best * 8 + 5], h[best * 8] / 1e5, h[best * 8 + 1] / 1e5, h[best * 8 + 2] / 1e5,
            h[best * 8 + 3] / 1e5, h[best * 8 + 4] / 1e5, h[best * 8 + 6] / 1e5, h[best * 8 + 7] / 1e5);
    (void)hipMemset(g_heavy_prof, 0, 1024 * 8 * sizeof(uint64_t));
}

int FlowEngine::ensure_scratch() {
    const size_t cap = cfg.max_batch;
    if (cap > F_IDX) return SGA_ERANGE;
    if (scratch_cap < cap) {
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        size_t hist = 0;
        for (int b = 1; b <= 32; ++b) hist = std::max(hist, radix_hist_entries(cap, b));
        const size_t ntiles = (cap + kTileElems - 1) / kTileElems + 1;
        size_t bytes = 2 * al(cap * 4) + 2 * al(cap * sizeof(Payload)) + 2 * al(cap * 4) + 11 * al(cap * 4) +
                       4 * al(cap * 8) + al(cap) + 3 * al(cap * 4) + 2 * al(ntiles * sizeof(LAgg)) + al(ntiles * 4) +
                       al(64) + 2 * al(hist * 4) + al(scan_partials_needed(hist) * 4 + 64) + al(cap * 4) +
                       2 * al(cap * 8) + al(cap * 4) + 2 * al(cap * 8) + al(cap * 4) + al(kRadixGhistWords * 4) + al(64) + al(cap * 4) + al((cap / 256 + 16) * 8) + al(cap * 8) +
                       al(cap * 8) +  // run_asum
                       al((cap / 64 + 2) * sizeof(WinSum)) + al((cap / 64 + 2) * 8) +  // wsum, wstate
                       al(cap * 8) +  // ev_param
                       al(cap * sizeof(Payload)) +  // spay
                       4 * al((cap / kCbTileMin + 2) * 4) + al((cap / kCbTileMin + 2) * sizeof(CbAgg)) +  // cbt_*
                       al((2 * (cap / kCbRound) + 16) * 4) + al((2 * (cap / kCbRound) + 16) * sizeof(CbTile)) + al(64);
        d_scratch.alloc(bytes);
        char *p = (char *)d_scratch.p;
        auto take = [&](size_t b) {
            void *r = p;
            p += al(b);
            return r;
        };
        sc.keys[0] = (uint32_t *)take(cap * 4);
        sc.keys[1] = (uint32_t *)take(cap * 4);
        sc.pay[0] = (Payload *)take(cap * sizeof(Payload));
        sc.pay[1] = (Payload *)take(cap * sizeof(Payload));
        sc.ev_run = (uint32_t *)take(cap * 4);
        sc.ev_eidx = (uint32_t *)take(cap * 4);
        sc.run_start = (uint32_t *)take(cap * 4);
        sc.run_end = (uint32_t *)take(cap * 4);
        sc.run_slot = (uint32_t *)take(cap * 4);
        sc.run_t0off = (uint32_t *)take(cap * 4);
        sc.run_nent = (uint32_t *)take(cap * 4);
        sc.run_cp = (uint32_t *)take(cap * 4);
        sc.run_amin = (int32_t *)take(cap * 4);
        sc.run_amax = (int32_t *)take(cap * 4);
        sc.run_asum = (int64_t *)take(cap * 8);
        sc.run_nexit = (uint32_t *)take(cap * 4);
        sc.run_f = (uint32_t *)take(cap * 4);
        sc.run_exc = (uint64_t *)take(cap * 8);
        sc.run_exerr = (uint64_t *)take(cap * 8);
        sc.run_exrt = (int64_t *)take(cap * 8);
        sc.run_exmin = (int64_t *)take(cap * 8);
        sc.run_mode = (uint8_t *)take(cap);
        sc.flow_first_run = (uint32_t *)take(cap * 4);
        sc.heavy = (uint32_t *)take(cap * 4);
        sc.pace = (uint32_t *)take(cap * 4);
        sc.lru = (uint32_t *)take(cap * 4);
        sc.tile_agg = take(ntiles * sizeof(LAgg));
        sc.tile_carry = take(ntiles * sizeof(LAgg));
        sc.tile_valid = (uint32_t *)take(ntiles * 4);
        sc.counters = (uint32_t *)take(64);
        sc.radix.hist = (uint32_t *)take(hist * 4);
        sc.radix.hist_scan = (uint32_t *)take(hist * 4);
        sc.radix.partial = (uint32_t *)take(scan_partials_needed(hist) * 4 + 64);
        sc.pseg = (uint32_t *)take(cap * 4);
        sc.cbf = (uint32_t *)take(cap * 4);
        sc.plong = (uint32_t *)take((cap / 256 + 16) * 8);
        sc.rt_sorted = (int64_t *)take(cap * 8);
        sc.pel[0] = (uint64_t *)take(cap * 8);
        sc.pel[1] = (uint64_t *)take(cap * 8);
        sc.seg = (uint32_t *)take(cap * 4);
        sc.run_pa = (int64_t *)take(cap * 8);
        sc.run_ba = (int64_t *)take(cap * 8);
        sc.run_np = (uint32_t *)take(cap * 4);
        sc.radix.ghist = (uint32_t *)take(kRadixGhistWords * 4);
        sc.radix.err = (uint32_t *)take(64);
        sc.wsum = (WinSum *)take((cap / 64 + 2) * sizeof(WinSum));
        sc.wstate = (int64_t *)take((cap / 64 + 2) * 8);
        sc.ev_param = (uint64_t *)take(cap * 8);
        sc.spay = (Payload *)take(cap * sizeof(Payload));
        {
            const size_t nf = cap / kCbTileMin + 2, nt = 2 * (cap / kCbRound) + 16;
            sc.cbt_flow = (uint32_t *)take(nf * 4);
            sc.cbt_off = (uint32_t *)take(nf * 4);
            sc.cbt_trip = (uint32_t *)take(nf * 4);
            sc.cbt_state = (uint32_t *)take(nf * 4);
            sc.cbt_total = (CbAgg *)take(nf * sizeof(CbAgg));
            sc.cbt_tile = (uint32_t *)take(nt * 4);
            sc.cbt = (CbTile *)take(nt * sizeof(CbTile));
            sc.cbt_ctl = (uint32_t *)take(64);
        }
        sc.cap = cap;
        scratch_cap = cap;
        d_kind.alloc(cap);
        d_flags.alloc(cap);
        d_resid.alloc(cap);
        d_ts.alloc(cap);
        d_acq.alloc(cap);
        d_rt.alloc(cap);
        d_param.alloc(cap);
        d_dec.alloc(cap);
        d_wait.alloc(cap);
    }
    return 0;
}

// One small chunk (FlowEngine::kSmallEvents): the events and their argument words packed into page-locked memory,
// one copy to the device, the CacheMap bookkeeping (lru_prepare), k_lsmall, one copy back of the decisions,
// waits and the overflow word.
int FlowEngine::submit_small(const uint8_t *kind, const uint32_t *resource, const int32_t *acquire,
                             const uint8_t *flags, const int64_t *rt, const uint64_t *param, const uint32_t *ts_off,
                             int64_t lo, uint32_t m, int8_t *decision, int32_t *wait_ms, const uint64_t *pvals,
                             size_t npvals) {
    auto a8 = [](size_t x) { return (x + 7) & ~(size_t)7; };
    const size_t o_kind = 0, o_flags = a8(o_kind + kSmallEvents), o_res = a8(o_flags + kSmallEvents),
                 o_ts = o_res + 4 * kSmallEvents, o_acq = o_ts + 4 * kSmallEvents, o_rt = o_acq + 4 * kSmallEvents,
                 o_param = o_rt + 8 * kSmallEvents, o_vals = o_param + 8 * kSmallEvents,
                 in_bytes = o_vals + 8 * (size_t)kSmallWords;
    const size_t o_dec = in_bytes, o_wait = a8(o_dec + kSmallEvents), o_ovf = o_wait + 4 * kSmallEvents,
                 all_bytes = o_ovf + 8;
    if (!h_small.p) h_small.alloc(all_bytes);
    if (!d_small.p) d_small.alloc(all_bytes);
    uint8_t *h = h_small.p, *d = d_small.p;
    std::memcpy(h + o_kind, kind, m);
    if (flags) std::memcpy(h + o_flags, flags, m);
    else std::memset(h + o_flags, 0, m);
    std::memcpy(h + o_res, resource, 4 * (size_t)m);
    std::memcpy(h + o_ts, ts_off, 4 * (size_t)m);
    std::memcpy(h + o_acq, acquire, 4 * (size_t)m);
    if (rt) std::memcpy(h + o_rt, rt, 8 * (size_t)m);
    else std::memset(h + o_rt, 0, 8 * (size_t)m);
    if (param) std::memcpy(h + o_param, param, 8 * (size_t)m);
    else std::memset(h + o_param, 0, 8 * (size_t)m);
    if (npvals) std::memcpy(h + o_vals, pvals, 8 * npvals);
    // The kernels read the page-locked buffer in place and write the results into it (it is mapped into the
    // device's address space, coherent): no copy operation either way, one launch (plus the CacheMap
    // bookkeeping when parameter rules exist).  SGA_SMALL_COPY=1 (A/B knob) copies to HBM first.
    static const bool copy = getenv("SGA_SMALL_COPY") && atoi(getenv("SGA_SMALL_COPY")) == 1;
    if (copy) {
        const size_t up = npvals ? o_vals + 8 * npvals : o_vals;  // the argument words end the input region
        SGA_HIP_CHECK(hipMemcpyAsync(d, h, up, hipMemcpyHostToDevice, stream));
    } else {
        d = h;
    }
    const bool maps = d_psize.p && !h_prules.empty();  // lru_prepare runs (and may flag the overflow word)
    if (maps) SGA_HIP_CHECK(hipMemsetAsync(d_overflow.p, 0, 4, stream));
    const uint8_t *dk = d + o_kind, *dfl = d + o_flags;
    const uint32_t *dres = (const uint32_t *)(d + o_res), *dts = (const uint32_t *)(d + o_ts);
    const int32_t *dacq = (const int32_t *)(d + o_acq);
    const int64_t *drt = (const int64_t *)(d + o_rt);
    const uint64_t *dpar = (const uint64_t *)(d + o_param), *dvals = npvals ? (const uint64_t *)(d + o_vals) : nullptr;
    lru_prepare(dk, dres, dfl, dpar, dvals, m, stream);  // CacheMap capacity
    FlowScratch fs = sc;
    fs.in_kind = dk;
    fs.in_flags = dfl;
    fs.in_param = dpar;
    fs.pvals = dvals;
    hipLaunchKernelGGL(k_lsmall, dim3(1), dim3(kLSmall), 0, stream, state(), (int64_t)cfg.statistic_max_rt, fs, dres,
                       dts, lo, dacq, drt, m, (int8_t *)(d + o_dec), (int32_t *)(d + o_wait), (uint32_t *)(d + o_ovf),
                       maps ? 0 : 1);
    SGA_HIP_CHECK(hipGetLastError());
    if (copy) SGA_HIP_CHECK(hipMemcpyAsync(h + o_dec, d + o_dec, all_bytes - o_dec, hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    std::memcpy(decision, h + o_dec, m);
    if (wait_ms) std::memcpy(wait_ms, h + o_wait, 4 * (size_t)m);
    uint32_t ovf;
    std::memcpy(&ovf, h + o_ovf, 4);
    if (ovf & kOvfMissingEntry) throw HipError(kMissingEntryText, __FILE__, __LINE__);  // SGA_EIO
    if (ovf) return SGA_ENOMEM;  // parameter maps full
    return 0;
}

// The chunk's view of the scratch for F_SPECIAL events: a new epoch marks their resources (res_special), the
// original kind / flags / parameters / value lists are what the per-resource replay reads for them.
FlowScratch FlowEngine::special_scratch(const FlowScratch &base, const uint8_t *d_kind_in, const uint8_t *d_flags_in,
                                        const uint64_t *d_param_in, const uint64_t *d_pvals) {
    if (d_res_special.n < (size_t)nres + 1) {
        d_res_special.alloc((size_t)nres + 1);
        SGA_HIP_CHECK(hipMemset(d_res_special.p, 0, d_res_special.bytes()));
        epoch = 0;
    }
    if (++epoch >= (1u << 30)) {  // wrapped (res_special holds epoch << 2 | level): no resource may hold the new one
        SGA_HIP_CHECK(hipMemsetAsync(d_res_special.p, 0, d_res_special.bytes(), stream));
        epoch = 1;
    }
    FlowScratch f = base;
    f.res_special = d_res_special.p;
    f.epoch = epoch;
    f.in_kind = d_kind_in;
    f.in_flags = d_flags_in;
    f.in_param = d_param_in;
    f.pvals = d_pvals;
    return f;
}

int FlowEngine::submit(const uint8_t *kind, const uint32_t *resource, const int64_t *ts, const int32_t *acquire,
                       const uint8_t *flags, const int64_t *rt, const uint64_t *param, size_t n, int8_t *decision,
                       int32_t *wait_ms, const uint64_t *pvals, size_t npvals) {
    if (!nres) return SGA_EINVAL;
    if (n == 0) return 0;
    // Collection / array arguments (SGA_EV_PARAM_LIST): the value array goes to the device once;
    // chunks holding such events are replayed in arrival order by one lane (k_lseq)
    // and whole argument vectors (SGA_EV_ARGS: word pairs, lists inside param_values)
    auto is_list = [&](size_t i) {
        return (flags[i] & SGA_EV_ARGS) ||
               (flags[i] & (SGA_EV_PARAM_LIST | SGA_EV_HAS_PARAM)) == (SGA_EV_PARAM_LIST | SGA_EV_HAS_PARAM);
    };
    auto list_ok = [&](size_t i) {
        const uint64_t off = param[i] >> 32, na = param[i] & 0xFFFFFFFFu;
        if (!(flags[i] & SGA_EV_ARGS)) return off + na <= npvals;
        if (off + 2 * na > npvals) return false;
        for (uint64_t k = 0; k < na; ++k) {
            const uint64_t h = pvals[off + 2 * k], w = pvals[off + 2 * k + 1];
            if ((h >> 62) > 2 || ((h >> 62) == SGA_ARG_LIST && w + (h & 0xFFFFFFFFu) > npvals)) return false;
        }
        return true;
    };
    bool any_list = false;
    for (size_t i = 0; flags && param && i < n; ++i) {
        if (!is_list(i)) continue;
        if ((npvals && !pvals) || !list_ok(i)) return SGA_EINVAL;  // an empty args vector needs no values
        any_list = true;
    }
    if (any_list) {
        if (d_pvals.n < std::max<size_t>(npvals, 1)) d_pvals.alloc(std::max<size_t>(npvals, 1));
        if (npvals) SGA_HIP_CHECK(hipMemcpyAsync(d_pvals.p, pvals, npvals * 8, hipMemcpyHostToDevice, stream));
    }
    const size_t cap = cfg.max_batch;
    if (const int rc = ensure_scratch()) return rc;
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)nres + 1) ++bits;
    std::vector<uint32_t> off;
    std::vector<int64_t> zero_rt;
    for (size_t b = 0; b < n;) {
        size_t m = std::min(cap, n - b);
        int64_t lo = ts[b], hi = ts[b];
        for (size_t i = 0; i < m; ++i) {
            const int64_t t = ts[b + i];
            if (t < 0 || acquire[b + i] < 0) return SGA_EINVAL;
            const int64_t nlo = std::min(lo, t), nhi = std::max(hi, t);
            if (nhi - nlo > (int64_t)0xFFFFFFFFLL) {
                m = i;
                break;
            }
            lo = nlo;
            hi = nhi;
        }
        off.resize(m);
        for (size_t i = 0; i < m; ++i) off[i] = (uint32_t)(ts[b + i] - lo);
        if (const int rc = ensure_maps(m + (any_list ? npvals : 0))) return rc;
        bool has_in = false, has_list = false;
        for (size_t i = 0; flags && i < m && !has_in; ++i) has_in = (flags[b + i] & SGA_EV_INBOUND) && resource[b + i] < nres;
        for (size_t i = 0; any_list && i < m && !has_list; ++i) has_list = is_list(b + i);
        for (size_t i = 0; i < m; ++i)
            if (kind[b + i] > SGA_KIND_REVOKE) return SGA_EINVAL;
        if (m <= small_max && !(has_in && sys.check) && (!has_list || npvals <= kSmallWords)) {
            if (const int rc = submit_small(kind + b, resource + b, acquire + b, flags ? flags + b : nullptr,
                                            rt ? rt + b : nullptr, param ? param + b : nullptr, off.data(), lo,
                                            (uint32_t)m, decision + b, wait_ms ? wait_ms + b : nullptr,
                                            has_list ? pvals : nullptr, has_list ? npvals : 0))
                return rc;
            b += m;
            seq += m;
            continue;
        }
        SGA_HIP_CHECK(hipMemcpyAsync(d_kind.p, kind + b, m, hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipMemcpyAsync(d_resid.p, resource + b, m * 4, hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipMemcpyAsync(d_ts.p, off.data(), m * 4, hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipMemcpyAsync(d_acq.p, acquire + b, m * 4, hipMemcpyHostToDevice, stream));
        if (flags) SGA_HIP_CHECK(hipMemcpyAsync(d_flags.p, flags + b, m, hipMemcpyHostToDevice, stream));
        else SGA_HIP_CHECK(hipMemsetAsync(d_flags.p, 0, m, stream));
        if (rt) SGA_HIP_CHECK(hipMemcpyAsync(d_rt.p, rt + b, m * 8, hipMemcpyHostToDevice, stream));
        else SGA_HIP_CHECK(hipMemsetAsync(d_rt.p, 0, m * 8, stream));
        if (param) SGA_HIP_CHECK(hipMemcpyAsync(d_param.p, param + b, m * 8, hipMemcpyHostToDevice, stream));
        else SGA_HIP_CHECK(hipMemsetAsync(d_param.p, 0, m * 8, stream));
        SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, 64, stream));
        // per chunk: a probe sequence that overflowed in an earlier (failed) batch must not fail
        // every later one.  A failed batch has been partly applied (its node and breaker updates
        // stay); the call reports -ENOMEM.
        SGA_HIP_CHECK(hipMemsetAsync(d_overflow.p, 0, 4, stream));
        // CacheMap capacity: owners that could pass theirs switch to LRU mode (both paths below)
        lru_prepare(d_kind.p, d_resid.p, flags ? d_flags.p : nullptr, param ? d_param.p : nullptr,
                    any_list ? d_pvals.p : nullptr, (uint32_t)m, stream);
        const FlowState st = state();
        const uint32_t nb = (uint32_t)((m + kT - 1) / kT);
        // kind 2 / 3 events and argument lists stay on the parallel pipeline (their resources replay per resource,
        // F_SPECIAL); SystemRules read ENTRY_NODE across resources: one lane in arrival order
        if (has_in && sys.check) {
            hipLaunchKernelGGL(k_lseq, dim3(1), dim3(64), 0, stream, st, (int64_t)cfg.statistic_max_rt, sys, d_kind.p,
                               d_resid.p, d_ts.p, lo, d_acq.p, d_flags.p, d_rt.p, d_param.p, (uint32_t)m, d_dec.p,
                               d_wait.p, has_list ? d_pvals.p : nullptr);
            SGA_HIP_CHECK(hipGetLastError());
            SGA_HIP_CHECK(hipMemcpyAsync(decision + b, d_dec.p, m, hipMemcpyDeviceToHost, stream));
            if (wait_ms) SGA_HIP_CHECK(hipMemcpyAsync(wait_ms + b, d_wait.p, m * 4, hipMemcpyDeviceToHost, stream));
            uint32_t ovf = 0;
            SGA_HIP_CHECK(hipMemcpyAsync(&ovf, d_overflow.p, 4, hipMemcpyDeviceToHost, stream));
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
            if (ovf & kOvfMissingEntry) throw HipError(kMissingEntryText, __FILE__, __LINE__);  // SGA_EIO
            if (ovf) return SGA_ENOMEM;
            b += m;
            seq += m;
            continue;
        }
        FlowScratch fsc = special_scratch(sc, d_kind.p, flags ? d_flags.p : nullptr, param ? d_param.p : nullptr,
                                          has_list ? d_pvals.p : nullptr);
        const uint64_t *evp = fsc.ev_param;
        hipLaunchKernelGGL(k_lclassify, dim3(nb), dim3(kT), 0, stream, st, fsc, d_kind.p, d_resid.p, d_ts.p, lo, d_acq.p,
                           d_flags.p, param ? d_param.p : nullptr, (uint32_t)m, sc.keys[0], sc.pay[0], d_dec.p, d_wait.p);
        const int np = radix_sort_pairs(sc.keys[0], sc.pay[0], sc.keys[1], sc.pay[1], m, bits, sc.radix, stream);
        const uint32_t *keys = sc.keys[np & 1];
        const Payload *pay = sc.pay[np & 1];
        const uint32_t ntiles = (uint32_t)((m + kTileElems - 1) / kTileElems);
        hipLaunchKernelGGL(k_lruns_up, dim3(ntiles), dim3(kT), 0, stream, keys, pay, (uint32_t)m, nres,
                           (LAgg *)sc.tile_agg, sc.tile_valid);
        hipLaunchKernelGGL(k_lruns_tiles, dim3(1), dim3(kT), 0, stream, (const LAgg *)sc.tile_agg, sc.tile_valid, ntiles,
                           (LAgg *)sc.tile_carry, sc.counters);
        hipLaunchKernelGGL(k_lruns_down, dim3(ntiles), dim3(kT), 0, stream, keys, pay, d_rt.p, nres,
                           (const LAgg *)sc.tile_carry, sc);
        hipLaunchKernelGGL(k_lexits, dim3(ntiles), dim3(kT), 0, stream, pay, d_rt.p, sc);
        const uint32_t fthreads = (uint32_t)std::min<size_t>(m, nres);
        FlowScratch fsc_p = fsc;  // the flows and the per-value segments (pseg off: null)
        if ((h_prules.empty() && h_cbs.empty()) || !pseg_on()) fsc_p.pseg = nullptr;
        hipLaunchKernelGGL(k_lflows, dim3((fthreads + kT - 1) / kT), dim3(kT), 0, stream, st,
                           (int64_t)cfg.statistic_max_rt, fsc_p, pay, keys, lo, d_rt.p, evp, d_dec.p, d_wait.p);
        launch_pseg(st, fsc_p, pay, keys, lo, d_rt.p, evp, d_dec.p, d_wait.p, (uint32_t)m, stream);
        if (st.lru_res) {
            hipLaunchKernelGGL(k_llru, dim3(64), dim3(64), 0, stream, st, (int64_t)cfg.statistic_max_rt, fsc, pay, lo,
                               d_rt.p, evp, d_dec.p, d_wait.p);
            hipLaunchKernelGGL(k_llru_ps, dim3(256), dim3(128), 0, stream, st, (int64_t)cfg.statistic_max_rt, fsc, pay, lo,
                               evp, d_dec.p, d_wait.p);
        }
        hipLaunchKernelGGL(k_lwsum, dim3((unsigned)((m / 64 + 3) / 4 + 1)), dim3(256), 0, stream, st, fsc, pay);
        for (int rl = 0; rl < 2; ++rl)
            hipLaunchKernelGGL(rl ? k_lwave<1> : k_lwave<0>,
                               dim3(std::max<uint32_t>(1, std::min<uint32_t>(4096, (uint32_t)(m / 4096)))),
                               dim3(64), 0, stream, st, (int64_t)cfg.statistic_max_rt, fsc, pay, lo, d_rt.p, evp,
                               d_dec.p, d_wait.p, lwave_prof());
        print_lwave_prof(stream);
        hipLaunchKernelGGL(k_lheavy, dim3(std::max<uint32_t>(1, std::min<uint32_t>(1024, (uint32_t)(m / kHeavyEvents)))),
                           dim3(64), 0, stream, st, (int64_t)cfg.statistic_max_rt, fsc, pay, lo, d_rt.p, evp,
                           d_dec.p, d_wait.p, heavy_prof());
        if (heavy_prof()) print_heavy_prof();
        hipLaunchKernelGGL(k_lresults, dim3(nb), dim3(kT), 0, stream, st, fsc, pay, d_dec.p, d_wait.p);
        if (has_in)  // ENTRY_NODE statistics of the inbound events
            hipLaunchKernelGGL(k_entry_stats, dim3(1), dim3(kEnTile), 0, stream, st, (int64_t)cfg.statistic_max_rt,
                               d_kind.p, d_resid.p, d_ts.p, lo, d_acq.p, d_flags.p, d_rt.p, d_dec.p, (uint32_t)m);
        SGA_HIP_CHECK(hipGetLastError());
        SGA_HIP_CHECK(hipMemcpyAsync(decision + b, d_dec.p, m, hipMemcpyDeviceToHost, stream));
        if (wait_ms) SGA_HIP_CHECK(hipMemcpyAsync(wait_ms + b, d_wait.p, m * 4, hipMemcpyDeviceToHost, stream));
        uint32_t ovf = 0;
        SGA_HIP_CHECK(hipMemcpyAsync(&ovf, d_overflow.p, 4, hipMemcpyDeviceToHost, stream));
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        if (ovf & kOvfMissingEntry) throw HipError(kMissingEntryText, __FILE__, __LINE__);  // SGA_EIO
        if (ovf) return SGA_ENOMEM;  // parameter maps full
        debug_size_check();
        b += m;
        seq += m;
    }
    return 0;
}

// SGA_SIZE_CHECK=1 (diagnostics only): after each host batch, every free-mode owner's kept present count
// against a count of its present map keys
void FlowEngine::debug_size_check() {
    static const bool on = getenv("SGA_SIZE_CHECK") && atoi(getenv("SGA_SIZE_CHECK")) == 1;
    if (!on || !d_psize.p) return;
    const FlowState st = state();
    std::vector<PEntry> pt(st.pmask + 1), tt(st.tmask + 1);
    SGA_HIP_CHECK(hipMemcpy(pt.data(), tab_data(d_ptab), pt.size() * sizeof(PEntry), hipMemcpyDeviceToHost));
    SGA_HIP_CHECK(hipMemcpy(tt.data(), tab_data(d_ttab), tt.size() * sizeof(PEntry), hipMemcpyDeviceToHost));
    std::vector<uint32_t> ps(st.nprid), ts(st.ntslot);
    std::vector<uint64_t> pq(st.nprid), tq(st.ntslot);
    SGA_HIP_CHECK(hipMemcpy(ps.data(), d_psize.p, ps.size() * 4, hipMemcpyDeviceToHost));
    SGA_HIP_CHECK(hipMemcpy(ts.data(), d_tsize.p, ts.size() * 4, hipMemcpyDeviceToHost));
    SGA_HIP_CHECK(hipMemcpy(pq.data(), d_pq.p, pq.size() * 8, hipMemcpyDeviceToHost));
    SGA_HIP_CHECK(hipMemcpy(tq.data(), d_tq.p, tq.size() * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> pc(st.nprid), tc(st.ntslot);
    for (const PEntry &e : pt)
        if (e.owner && e.a != kPAbsent && e.owner - 1 < st.nprid) ++pc[e.owner - 1];
    for (const PEntry &e : tt) {
        if (!e.owner || e.a == kPAbsent) continue;
        const uint32_t r = (e.owner & 0xFFFFFFu) - 1u, k = e.owner >> 24;
        if (r < h_tbase.size() && h_tbase[r] != kNoTBase) ++tc[h_tbase[r] + k];
    }
    int shown = 0;
    for (uint32_t i = 0; i < st.nprid && shown < 12; ++i)
        if (pq[i] == kNoQueue && pc[i] != ps[i] && ++shown)
            fprintf(stderr, "size check seq=%llu: rule id %u size %u present %u\n", (unsigned long long)seq, i, ps[i], pc[i]);
    for (uint32_t j = 0; j < st.ntslot && shown < 24; ++j)
        if (tq[j] == kNoQueue && tc[j] != ts[j] && ++shown)
            fprintf(stderr, "size check seq=%llu: thread slot %u size %u present %u\n", (unsigned long long)seq, j, ts[j], tc[j]);
    if (!shown) fprintf(stderr, "size check seq=%llu: ok\n", (unsigned long long)seq);
}

// Device entry: one chunk of events already in HBM, launched on s without a host wait.  What the host
// entry decides by scanning the events (arrival-order replay, inbound statistics, validation) is
// decided by k_lgate on the device: both the parallel pipeline and k_lseq are launched and the gate
// word lets exactly one of them act.  Errors surface through device_status.
int FlowEngine::submit_device(const uint8_t *d_kind_in, const uint32_t *d_resource, int64_t ts_base,
                              const uint32_t *d_ts_off, const int32_t *d_acquire, const uint8_t *d_flags_in,
                              const int64_t *d_rt_in, const uint64_t *d_param_in, size_t n,
                              const uint64_t *d_param_values, size_t n_values, int8_t *d_decision, int32_t *d_wait,
                              hipStream_t s) {
    if (!nres) return SGA_EINVAL;
    if (n == 0) return 0;
    if (n > cfg.max_batch) return SGA_ERANGE;
    if (const int rc = ensure_scratch()) return rc;
    if (const int rc = ensure_maps(n + n_values)) return rc;
    if (!d_gate.p) {
        d_gate.alloc(2);
        SGA_HIP_CHECK(hipMemsetAsync(d_gate.p, 0, 8, s));
    }
    const uint32_t m = (uint32_t)n;
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)nres + 1) ++bits;
    // absent optional columns read as zeros
    if (!d_rt_in) SGA_HIP_CHECK(hipMemsetAsync(d_rt.p, 0, n * 8, s));
    if (!d_param_in) SGA_HIP_CHECK(hipMemsetAsync(d_param.p, 0, n * 8, s));
    if (!d_flags_in) SGA_HIP_CHECK(hipMemsetAsync(d_flags.p, 0, n, s));
    const int64_t *rt_p = d_rt_in ? d_rt_in : d_rt.p;
    const uint64_t *param_p = d_param_in ? d_param_in : d_param.p;
    const uint8_t *flags_p = d_flags_in ? d_flags_in : d_flags.p;
    int32_t *wait_p = d_wait ? d_wait : this->d_wait.p;
    SGA_HIP_CHECK(hipMemsetAsync(sc.counters, 0, 64, s));
    SGA_HIP_CHECK(hipMemsetAsync(d_overflow.p, 0, 4, s));
    SGA_HIP_CHECK(hipMemsetAsync(d_gate.p, 0, 4, s));
    const uint32_t nb = (m + kT - 1) / kT;
    const uint32_t gb = std::min<uint32_t>(nb, 1024);
    hipLaunchKernelGGL(k_lgate, dim3(gb), dim3(kT), 0, s, d_kind_in, d_resource, d_acquire, flags_p, param_p, m, nres,
                       (int)sys.check, (uint64_t)(d_param_values ? n_values : 0), d_gate.p, d_param_values);
    lru_prepare(d_kind_in, d_resource, flags_p, param_p, d_param_values, m, s);  // CacheMap capacity
    FlowState st = state();
    st.gate = d_gate.p;
    FlowScratch gsc = special_scratch(sc, d_kind_in, flags_p, param_p, d_param_values);
    gsc.gate = d_gate.p;
    hipLaunchKernelGGL(k_lclassify, dim3(nb), dim3(kT), 0, s, st, gsc, d_kind_in, d_resource, d_ts_off, ts_base, d_acquire,
                       flags_p, param_p, m, gsc.keys[0], gsc.pay[0], d_decision, wait_p);
    const uint64_t *evp = gsc.ev_param;  // what the parallel kernels read as the event's parameter
    const int np = radix_sort_pairs(gsc.keys[0], gsc.pay[0], gsc.keys[1], gsc.pay[1], m, bits, gsc.radix, s);
    const uint32_t *keys = gsc.keys[np & 1];
    const Payload *pay = gsc.pay[np & 1];
    const uint32_t ntiles = (m + kTileElems - 1) / kTileElems;
    hipLaunchKernelGGL(k_lruns_up, dim3(ntiles), dim3(kT), 0, s, keys, pay, m, nres, (LAgg *)gsc.tile_agg,
                       gsc.tile_valid);
    hipLaunchKernelGGL(k_lruns_tiles, dim3(1), dim3(kT), 0, s, (const LAgg *)gsc.tile_agg, gsc.tile_valid, ntiles,
                       (LAgg *)gsc.tile_carry, gsc.counters);
    hipLaunchKernelGGL(k_lruns_down, dim3(ntiles), dim3(kT), 0, s, keys, pay, rt_p, nres, (const LAgg *)gsc.tile_carry,
                       gsc);
    hipLaunchKernelGGL(k_lexits, dim3(ntiles), dim3(kT), 0, s, pay, rt_p, gsc);
    const uint32_t fthreads = std::min<uint32_t>(m, nres);
    if ((h_prules.empty() && h_cbs.empty()) || !pseg_on()) gsc.pseg = nullptr;
    hipLaunchKernelGGL(k_lflows, dim3((fthreads + kT - 1) / kT), dim3(kT), 0, s, st, (int64_t)cfg.statistic_max_rt, gsc,
                       pay, keys, ts_base, rt_p, evp, d_decision, wait_p);
    launch_pseg(st, gsc, pay, keys, ts_base, rt_p, evp, d_decision, wait_p, m, s);
    if (st.lru_res) {
        hipLaunchKernelGGL(k_llru, dim3(64), dim3(64), 0, s, st, (int64_t)cfg.statistic_max_rt, gsc, pay, ts_base, rt_p,
                           evp, d_decision, wait_p);
        hipLaunchKernelGGL(k_llru_ps, dim3(256), dim3(128), 0, s, st, (int64_t)cfg.statistic_max_rt, gsc, pay, ts_base,
                           evp, d_decision, wait_p);
    }
    hipLaunchKernelGGL(k_lwsum, dim3((m / 64 + 3) / 4 + 1), dim3(256), 0, s, st, gsc, pay);
    for (int rl = 0; rl < 2; ++rl)
        hipLaunchKernelGGL(rl ? k_lwave<1> : k_lwave<0>, dim3(std::max<uint32_t>(1, std::min<uint32_t>(4096, m / 4096))),
                           dim3(64), 0, s, st, (int64_t)cfg.statistic_max_rt, gsc, pay, ts_base, rt_p, evp, d_decision,
                           wait_p, lwave_prof());
    print_lwave_prof(s);
    hipLaunchKernelGGL(k_lheavy, dim3(std::max<uint32_t>(1, std::min<uint32_t>(1024, m / kHeavyEvents))), dim3(64), 0, s,
                       st, (int64_t)cfg.statistic_max_rt, gsc, pay, ts_base, rt_p, evp, d_decision, wait_p,
                       heavy_prof());
        if (heavy_prof()) print_heavy_prof();
    hipLaunchKernelGGL(k_lresults, dim3(nb), dim3(kT), 0, s, st, gsc, pay, d_decision, wait_p);
    hipLaunchKernelGGL(k_entry_stats, dim3(1), dim3(kEnTile), 0, s, st, (int64_t)cfg.statistic_max_rt, d_kind_in,
                       d_resource, d_ts_off, ts_base, d_acquire, flags_p, rt_p, d_decision, m);
    // arrival-order chunks (inbound events under system rules): k_lseq acts only when the gate says so
    hipLaunchKernelGGL(k_lseq, dim3(1), dim3(64), 0, s, st, (int64_t)cfg.statistic_max_rt, sys, d_kind_in,
                       d_resource, d_ts_off, ts_base, d_acquire, flags_p, rt_p, param_p, m, d_decision, wait_p,
                       d_param_values);
    hipLaunchKernelGGL(k_lfail, dim3(gb), dim3(kT), 0, s, d_gate.p, d_overflow.p, d_gate.p + 1, m, d_decision, wait_p);
    SGA_HIP_CHECK(hipGetLastError());
    seq += n;
    return 0;
}

int FlowEngine::device_status() {
    if (!d_gate.p) return 0;
    uint32_t e = 0;
    SGA_HIP_CHECK(hipMemcpyAsync(&e, d_gate.p + 1, 4, hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipMemsetAsync(d_gate.p + 1, 0, 4, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    if (e & 1u) return SGA_EINVAL;
    if (e & 4u) throw HipError(kMissingEntryText, __FILE__, __LINE__);  // SGA_EIO
    if (e & 2u) return SGA_ENOMEM;
    return 0;
}

int FlowEngine::query(uint32_t r, int64_t now, sga_node_view *out) {
    if (r == SGA_ENTRY_NODE && nres) r = nres;
    else if (r >= nres) return SGA_EINVAL;
    if (now < 0 || !out) return SGA_EINVAL;
    if (!d_view.p || d_view.n < 24) d_view.alloc(24);
    hipLaunchKernelGGL(k_node_view, dim3(1), dim3(64), 0, stream, state(), (int64_t)cfg.statistic_max_rt, r, now,
                       (double *)d_view.p, d_view.p + 16);
    double dv[16];
    int64_t iv[8];
    SGA_HIP_CHECK(hipMemcpyAsync(dv, d_view.p, 128, hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipMemcpyAsync(iv, d_view.p + 16, 64, hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    out->pass_qps = dv[0];
    out->block_qps = dv[1];
    out->success_qps = dv[2];
    out->exception_qps = dv[3];
    out->occupied_pass_qps = dv[4];
    out->avg_rt = dv[5];
    out->min_rt = dv[6];
    out->previous_pass_qps = dv[7];
    out->total_pass = iv[0];
    out->total_block = iv[1];
    out->total_success = iv[2];
    out->total_exception = iv[3];
    out->cur_thread_num = iv[4];
    out->waiting = iv[5];
    out->max_success_qps = dv[8];
    out->previous_block_qps = dv[9];
    return 0;
}

int FlowEngine::metrics(int64_t now, sga_metric_node *out, size_t cap, size_t *n) {
    if (now < 0 || !n || (cap && !out)) return SGA_EINVAL;
    *n = 0;
    if (nres == 0) return 0;
    const size_t dcap = std::max<size_t>(cap, 1);
    if (d_metrics.n < dcap) d_metrics.alloc(dcap);
    if (!d_mcount.p) d_mcount.alloc(1);
    SGA_HIP_CHECK(hipMemsetAsync(d_mcount.p, 0, 4, stream));
    hipLaunchKernelGGL(k_metrics, dim3((nres + 1 + kT - 1) / kT), dim3(kT), 0, stream, state(),
                       (int64_t)cfg.statistic_max_rt, now, d_metrics.p, (uint32_t)cap, d_mcount.p);
    uint32_t cnt = 0;
    SGA_HIP_CHECK(hipMemcpyAsync(&cnt, d_mcount.p, 4, hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    const size_t w = std::min<size_t>(cnt, cap);
    if (w) SGA_HIP_CHECK(hipMemcpy(out, d_metrics.p, w * sizeof(sga_metric_node), hipMemcpyDeviceToHost));
    *n = w;
    return cnt > cap ? SGA_ERANGE : 0;
}

// SystemPropertyListener.configUpdate + loadSystemConf, SystemRuleManager.java:191-300
int FlowEngine::load_system_rules(const sga_system_rule *r, size_t n) {
    const double dmax = 1.7976931348623157e308;
    sys.check = 0;
    sys.load = dmax;
    sys.cpu = dmax;
    sys.qps = dmax;
    sys.max_rt = INT64_MAX;
    sys.max_thread = INT64_MAX;
    sys.load_set = 0;
    sys.cpu_set = 0;
    int applied = 0;
    for (size_t i = 0; i < n; ++i) {
        int st = 0;
        if (r[i].highest_system_load >= 0) {
            sys.load = std::min(sys.load, r[i].highest_system_load);
            sys.load_set = 1;
            st = 1;
        }
        if (r[i].highest_cpu_usage >= 0 && r[i].highest_cpu_usage <= 1) {  // > 1: "Ignoring invalid SystemRule"
            sys.cpu = std::min(sys.cpu, r[i].highest_cpu_usage);
            sys.cpu_set = 1;
            st = 1;
        }
        if (r[i].avg_rt >= 0) {
            sys.max_rt = std::min(sys.max_rt, r[i].avg_rt);
            st = 1;
        }
        if (r[i].max_thread >= 0) {
            sys.max_thread = std::min(sys.max_thread, r[i].max_thread);
            st = 1;
        }
        if (r[i].qps >= 0) {
            sys.qps = std::min(sys.qps, r[i].qps);
            st = 1;
        }
        sys.check = st;  // checkSystemStatus.set(checkStatus) per rule: the last rule decides
        applied += st;
    }
    return applied;
}

int FlowEngine::cb_state(uint32_t r, uint32_t k) {
    if (r >= nres || k >= h_res[r].n_cbs) return -1;
    CbDev d;
    SGA_HIP_CHECK(hipMemcpyAsync(&d, d_cbs.p + h_res[r].cb_off + k, sizeof(CbDev), hipMemcpyDeviceToHost, stream));
    SGA_HIP_CHECK(hipStreamSynchronize(stream));
    return d.state;
}

}  // namespace sga
