// Device restatement of one cluster parameter token request (DefaultTokenService.requestParamToken,
// CS/flow/DefaultTokenService.java:52-64 -> ClusterParamFlowChecker.acquireClusterToken,
// CS/flow/ClusterParamFlowChecker.java:37-120, over ClusterParamMetric / ClusterParameterLeapArray):
// the key store and window helpers the cluster parameter kernels (cluster.hip) use, and the exact
// single-request form the local path's ParamFlowSlot calls for cluster-mode parameter rules decided by
// the embedded token server (ParamFlowChecker.passClusterCheck, ParamFlowChecker.java:305-333).
#pragma once
#include <hip/hip_runtime.h>

#include "cluster.hpp"
#include "cluster_exact.hpp"

namespace sga {

constexpr uint32_t kErrKeys = 1, kErrPool = 2;

__device__ __forceinline__ uint32_t prule_lookup(const CParamState &st, int64_t fid) {
    uint32_t h = (uint32_t)hash_flow_id(fid) & st.hmask;
    for (uint32_t probe = 0; probe <= st.hmask; ++probe) {
        const HashEntry e = st.htab[h];
        if (e.key == fid) return e.slot;
        if (e.key == 0) break;
        h = (h + 1) & st.hmask;
    }
    return 0xFFFFFFFFu;
}

// ParamFlowRule.retrieveExclusiveItemCount + calcGlobalThreshold (ClusterParamFlowChecker.java:101-120)
__device__ __forceinline__ double prule_threshold(const CParamState &st, const PRuleParam &P, int64_t value) {
    double count = P.count;
    uint32_t lo = 0, hi = P.n_hot;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (st.hot_v[P.hot_off + m] < value) lo = m + 1;
        else hi = m;
    }
    if (lo < P.n_hot && st.hot_v[P.hot_off + lo] == value) count = (double)st.hot_c[P.hot_off + lo];
    if (P.threshold_type == 1) return count;  // FLOW_THRESHOLD_GLOBAL
    return count * (double)(P.ns >= 0 ? st.ns_connected[P.ns] : 0);
}

// value -> vid (insert-only open addressing on the 64-bit value)
__device__ __forceinline__ uint32_t vid_of(const CParamState &st, int64_t v, bool insert) {
    if (v == kAbsent) return st.vmask + 1;
    uint32_t h = (uint32_t)hash_flow_id(v) & st.vmask;
    for (uint32_t probe = 0; probe <= st.vmask; ++probe) {
        int64_t cur = st.vtab[h];
        if (cur == v) return h;
        if (cur == kAbsent) {
            if (!insert) return 0xFFFFFFFFu;
            const unsigned long long prev = atomicCAS((unsigned long long *)&st.vtab[h], (unsigned long long)kAbsent,
                                                      (unsigned long long)v);
            if ((int64_t)prev == kAbsent || (int64_t)prev == v) return h;
        }
        h = (h + 1) & st.vmask;
    }
    return 0xFFFFFFFFu;
}

// (slot, vid) -> kidx; the inserting lane allocates and initialises the key's record
// [stamp x S][count x S][access x S] and counts the key for its rule (nkeys: the CacheMap capacity trigger)
__device__ __forceinline__ uint32_t key_of(const CParamState &st, uint32_t slot, uint32_t vid, int64_t value,
                                           bool insert) {
    const uint64_t key = ((uint64_t)(slot + 1) << 32) | vid;
    uint32_t h = (uint32_t)splitmix64(key) & st.kmask;
    for (uint32_t probe = 0; probe <= st.kmask; ++probe) {
        const uint64_t cur = st.ktab[h];
        if (cur == key) return h;
        if (cur == 0) {
            if (!insert) return 0xFFFFFFFFu;
            const unsigned long long prev = atomicCAS((unsigned long long *)&st.ktab[h], 0ull, key);
            if (prev == 0) {
                const int S = st.param[slot].S;
                const uint32_t off = atomicAdd(&st.ctl[0], (uint32_t)(3 * S));
                if ((uint64_t)off + 3 * S > st.krec_cap) {
                    atomicOr(&st.ctl[1], kErrPool);
                    st.koff[h] = 0;
                } else {
                    st.koff[h] = off;
                    for (int j = 0; j < S; ++j) {
                        st.krec[off + j] = kAbsent;
                        st.krec[off + S + j] = 0;
                        st.krec[off + 2 * S + j] = 0;
                    }
                }
                st.kslot[h] = slot;
                st.kval[h] = value;
                atomicAdd(&st.nkeys[slot], 1u);
                return h;
            }
            if (prev == key) return h;
        }
        h = (h + 1) & st.kmask;
    }
    atomicOr(&st.ctl[1], kErrKeys);
    return 0xFFFFFFFFu;
}

// ---- CacheMap capacity (strict LRU).  Each bucket's map is a ConcurrentLinkedHashMapWrapper of the
// metric's maxCapacity (ClusterParamMetric.java:37-49, ClusterParameterLeapArray.java:40-47; CLHM 1.4.2
// is not vendored: restated as strict LRU, oracle/oracle_cparam.c).  An access is getSum's get of a
// present key (every valid bucket, :57-62) or addValue's putIfAbsent of a present one; a new key into a
// full map evicts the least recently accessed key (:79-88); a bucket reset empties the map.
// Every path keeps the key's last access stamp per bucket (record word 2S + j, stamp order = arrival
// order: ((seq + request) << 16) | (getSum: value index, add: 0x8000 | value index)).  A rule whose
// key count passes its capacity switches to LRU mode (k_plru_decide / collect / sort, once): per bucket
// a queue area [meta {head, tail}][2 cap + 2 records] of (key, stamp) pushes in access order, a record
// live while its key is in the map with that stamp; from then on the rule takes the sequential path and
// an insert past the capacity pops records from the head until a live one, whose key leaves the map.
__device__ __forceinline__ uint64_t pstamp(const CParamState &st, uint32_t req, uint32_t low) {
    return ((st.seq + req) << 16) | low;
}
constexpr uint32_t kPAddLow = 0x8000u;
__device__ __forceinline__ bool plru_on(const CParamState &st, const PRuleParam &P) {
    return st.pq != nullptr && st.pq[P.boff] != kPNoQueue;
}
__device__ __forceinline__ uint64_t plru_qcap(const PRuleParam &P) { return 2ull * P.cap + 2; }
__device__ __forceinline__ bool plru_live(const CParamState &st, const PRuleParam &P, int j, const PLruRec &r) {
    const int64_t *rec = st.krec + st.koff[r.kidx];
    return rec[j] == st.rstart[P.boff + j] && (uint64_t)rec[2 * P.S + j] == r.stamp;
}
__device__ void plru_push(const CParamState &st, const PRuleParam &P, int j, uint32_t kidx, uint64_t stamp) {
    PLruRec *a = st.lpool + st.pq[P.boff + j];
    const uint64_t qcap = plru_qcap(P);
    if (a[0].stamp - a[0].kidx >= qcap) {  // full: keep the live records (<= cap + 1 of them)
        uint64_t w = a[0].kidx;
        for (uint64_t i = a[0].kidx; i < a[0].stamp; ++i) {
            const PLruRec r = a[1 + i % qcap];
            if (plru_live(st, P, j, r)) a[1 + (w++) % qcap] = r;
        }
        a[0].stamp = w;
        if (w - a[0].kidx >= qcap) {
            atomicOr(&st.ctl[1], 4u);
            return;
        }
    }
    a[1 + a[0].stamp % qcap] = PLruRec{kidx, stamp};
    a[0].stamp += 1;
}
__device__ void plru_evict(const CParamState &st, const PRuleParam &P, int j) {
    PLruRec *a = st.lpool + st.pq[P.boff + j];
    const uint64_t qcap = plru_qcap(P);
    while (a[0].kidx < a[0].stamp) {
        const PLruRec r = a[1 + a[0].kidx % qcap];
        a[0].kidx += 1;
        if (plru_live(st, P, j, r)) {
            st.krec[st.koff[r.kidx] + j] = kAbsent;
            st.psize[P.boff + j] -= 1;
            return;
        }
    }
    atomicOr(&st.ctl[1], 4u);  // a full map without a live record: never expected
}

// ClusterParamMetric over the rule-level starts for one call at t (exact, any time order):
// currentWindow(t) (LeapArray.java:121-222) then the key's sum over valid buckets.
__device__ __forceinline__ int pm_window(const CParamState &st, const PRuleParam &P, int64_t t) {
    const int idx = (int)((t / P.W) % P.S);
    const int64_t ws = t - t % P.W;
    int64_t &rs = st.rstart[P.boff + idx];
    if (rs == kAbsent || ws > rs) {  // newEmptyBucket / resetWindowTo: the bucket's map is empty
        rs = ws;
        if (plru_on(st, P)) {
            st.lpool[st.pq[P.boff + idx]] = PLruRec{0, 0};
            st.psize[P.boff + idx] = 0;
        }
        return idx;
    }
    return ws == rs ? idx : -1;  // -1: detached bucket (clock went backwards), adds lost
}

// sum without accesses (getTopValues keeps the maps' order: it reads every key oldest first)
__device__ __forceinline__ int64_t pm_key_sum(const CParamState &st, const PRuleParam &P, const int64_t *rec,
                                              int64_t t) {
    int64_t s = 0;
    for (int j = 0; j < P.S; ++j) {
        const int64_t rs = st.rstart[P.boff + j];
        if (rs == kAbsent || t - rs > (int64_t)P.interval) continue;
        if (rec[j] == rs) s += rec[P.S + j];
    }
    return s;
}

// getSum(value): every valid bucket holding the key is accessed
__device__ __forceinline__ int64_t pm_key_sum_access(const CParamState &st, const PRuleParam &P, uint32_t kidx,
                                                     int64_t t, uint64_t stamp) {
    int64_t *rec = st.krec + st.koff[kidx];
    const bool lru = plru_on(st, P);
    int64_t s = 0;
    for (int j = 0; j < P.S; ++j) {
        const int64_t rs = st.rstart[P.boff + j];
        if (rs == kAbsent || t - rs > (int64_t)P.interval) continue;
        if (rec[j] != rs) continue;
        s += rec[P.S + j];
        rec[2 * P.S + j] = (int64_t)stamp;
        if (lru) plru_push(st, P, j, kidx, stamp);
    }
    return s;
}

// addValue into bucket idx (pm_window's index, its start current): putIfAbsent + add
__device__ __forceinline__ void pm_key_add(const CParamState &st, const PRuleParam &P, uint32_t kidx, int idx, int32_t a,
                                           uint64_t stamp) {
    int64_t *rec = st.krec + st.koff[kidx];
    const int64_t rs = st.rstart[P.boff + idx];
    const bool lru = plru_on(st, P);
    rec[2 * P.S + idx] = (int64_t)stamp;
    if (rec[idx] != rs) {  // a new key in the map
        rec[idx] = rs;
        rec[P.S + idx] = a;
        if (lru) {
            st.psize[P.boff + idx] += 1;
            plru_push(st, P, idx, kidx, stamp);
            if (st.psize[P.boff + idx] > P.cap) plru_evict(st, P, idx);
        }
        return;
    }
    rec[P.S + idx] += a;
    if (lru) plru_push(st, P, idx, kidx, stamp);
}

// One requestParamToken(flowId, acquireCount, values) at time t, in arrival order with every other
// request of the rule (the local path's sequential lanes): validation, rule lookup, then for each value
// rem = threshold(value) - sum(value) / intervalInSec - acquire; any rem < 0 -> BLOCKED with no adds;
// all pass -> every value added, OK with remaining (int) rem of the last value (-1 for several).
// The namespace limiter is not applied (the host refuses namespaces that have one).
__device__ inline uint64_t cparam_request_exact(const CParamState &st, int64_t flow_id, int32_t a,
                                                const uint64_t *values, uint32_t nv, int64_t t, uint32_t req) {
    if (flow_id <= 0 || a <= 0 || nv == 0) return pack_result(TRS_BAD_REQUEST, 0, 0);
    if (!st.ctl) return pack_result(TRS_NO_RULE_EXISTS, 0, 0);
    const uint32_t slot = prule_lookup(st, flow_id);
    if (slot == 0xFFFFFFFFu || !st.param[slot].active) return pack_result(TRS_NO_RULE_EXISTS, 0, 0);
    const PRuleParam P = st.param[slot];
    double remaining = -1;
    bool passed = true;
    for (uint32_t v = 0; v < nv; ++v) {
        const int64_t x = (int64_t)values[v];
        pm_window(st, P, t);
        const uint32_t vid = vid_of(st, x, false);
        const uint32_t kidx = vid == 0xFFFFFFFFu ? 0xFFFFFFFFu : key_of(st, slot, vid, x, false);
        const int64_t sum = kidx == 0xFFFFFFFFu ? 0 : pm_key_sum_access(st, P, kidx, t, pstamp(st, req, min(v, 0x7FFFu)));
        const double next = prule_threshold(st, P, x) - (double)sum / P.isec - (double)a;
        remaining = next;
        if (next < 0) {
            passed = false;
            break;
        }
    }
    if (passed) {
        for (uint32_t v = 0; v < nv; ++v) {
            const int64_t x = (int64_t)values[v];
            const int idx = pm_window(st, P, t);
            const uint32_t vid = vid_of(st, x, true);
            const uint32_t kidx = vid == 0xFFFFFFFFu ? 0xFFFFFFFFu : key_of(st, slot, vid, x, true);
            if (vid == 0xFFFFFFFFu) atomicOr(&st.ctl[1], kErrKeys);
            if (idx < 0 || kidx == 0xFFFFFFFFu) continue;
            pm_key_add(st, P, kidx, idx, a, pstamp(st, req, kPAddLow | min(v, 0x7FFFu)));
        }
    }
    if (nv > 1) remaining = -1;
    st.tmax[slot] = t > st.tmax[slot] ? t : st.tmax[slot];
    return passed ? pack_result(TRS_OK, j_d2i(remaining), 0) : pack_result(TRS_BLOCKED, 0, 0);
}

}  // namespace sga
