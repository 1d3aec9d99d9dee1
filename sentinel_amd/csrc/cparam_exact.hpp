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
                const uint32_t off = atomicAdd(&st.ctl[0], (uint32_t)(2 * S));
                if ((uint64_t)off + 2 * S > st.krec_cap) {
                    atomicOr(&st.ctl[1], kErrPool);
                    st.koff[h] = 0;
                } else {
                    st.koff[h] = off;
                    for (int j = 0; j < S; ++j) {
                        st.krec[off + j] = kAbsent;
                        st.krec[off + S + j] = 0;
                    }
                }
                st.kslot[h] = slot;
                st.kval[h] = value;
                return h;
            }
            if (prev == key) return h;
        }
        h = (h + 1) & st.kmask;
    }
    atomicOr(&st.ctl[1], kErrKeys);
    return 0xFFFFFFFFu;
}

// ClusterParamMetric over the rule-level starts for one call at t (exact, any time order):
// currentWindow(t) (LeapArray.java:121-222) then the key's sum over valid buckets.
__device__ __forceinline__ int pm_window(const CParamState &st, const PRuleParam &P, int64_t t) {
    const int idx = (int)((t / P.W) % P.S);
    const int64_t ws = t - t % P.W;
    int64_t &rs = st.rstart[P.boff + idx];
    if (rs == kAbsent || ws > rs) {  // newEmptyBucket / resetWindowTo: the bucket's map is empty
        rs = ws;
        return idx;
    }
    return ws == rs ? idx : -1;  // -1: detached bucket (clock went backwards), adds lost
}

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

// One requestParamToken(flowId, acquireCount, values) at time t, in arrival order with every other
// request of the rule (the local path's sequential lanes): validation, rule lookup, then for each value
// rem = threshold(value) - sum(value) / intervalInSec - acquire; any rem < 0 -> BLOCKED with no adds;
// all pass -> every value added, OK with remaining (int) rem of the last value (-1 for several).
// The namespace limiter is not applied (the host refuses namespaces that have one).
__device__ inline uint64_t cparam_request_exact(const CParamState &st, int64_t flow_id, int32_t a,
                                                const uint64_t *values, uint32_t nv, int64_t t) {
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
        const int64_t sum = kidx == 0xFFFFFFFFu ? 0 : pm_key_sum(st, P, st.krec + st.koff[kidx], t);
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
            int64_t *rec = st.krec + st.koff[kidx];
            const int64_t rs = st.rstart[P.boff + idx];
            if (rec[idx] != rs) {
                rec[idx] = rs;
                rec[P.S + idx] = 0;
            }
            rec[P.S + idx] += a;
        }
    }
    if (nv > 1) remaining = -1;
    st.tmax[slot] = t > st.tmax[slot] ? t : st.tmax[slot];
    return passed ? pack_result(TRS_OK, j_d2i(remaining), 0) : pack_result(TRS_BLOCKED, 0, 0);
}

}  // namespace sga
