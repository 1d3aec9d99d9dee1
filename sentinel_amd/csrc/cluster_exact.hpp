// Device restatement of one cluster token request against a rule's window record: the exact
// per-request replay of ClusterFlowChecker.acquireClusterToken / SimpleClusterFlowChecker (used by
// the cluster kernels for runs the closed form does not cover, and by the local path's FlowSlot for
// cluster-mode rules decided by the embedded token server, FlowRuleChecker.passClusterCheck).
#pragma once
#include <hip/hip_runtime.h>

#include "cluster.hpp"

namespace sga {

enum : int8_t { TRS_BAD_REQUEST = -4, TRS_TOO_MANY_REQUEST = -2, TRS_FAIL = -1, TRS_OK = 0, TRS_BLOCKED = 1,
                TRS_SHOULD_WAIT = 2, TRS_NO_RULE_EXISTS = 3 };

// TokenResult packed as sga_token_result: remaining | waitInMs << 32 | status << 48
__device__ __forceinline__ uint64_t pack_result(int8_t status, int32_t remaining, int32_t wait) {
    return (uint64_t)(uint32_t)remaining | ((uint64_t)(uint16_t)(int16_t)wait << 32) |
           ((uint64_t)(uint8_t)status << 48);
}

// ---------------------------------------------------------------- exact per-request replay (device)
// Window state of a rule lives in one contiguous record of 8 x S + 12 int64, padded to an even number
// of 64-byte units (rec_units: 12 units = 768 bytes for S = 10, so every record starts on a 128-byte line):
//   header  [per bucket j: start, PASS] [occupy state: occupyCounter PASS, PASS_REQUEST, hasOccupied]
//           [cache: the six other counters of one bucket] [cache tag: that bucket's start] [threshold]
//   array   [per bucket j: WAITING, BLOCK, PASS_REQUEST, BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK]
// The window sums read the dense vector of 16-byte pairs; for S = 10 the header is exactly two
// 128-byte lines, so a cold rule's closed form (k_cold_fused) reads two lines: the pairs, the occupy
// state, the current bucket's counters (the cache, valid while its tag equals that bucket's start) and
// the rule's threshold (a copy of SlotParam::thr, written at every rule load by k_rec_thr).  The array
// is authoritative and always written; the cache is only read by the closed forms, and a writer that
// changes a bucket's array counters without refreshing the cache clears the tag (metric_add).
constexpr int kOccWords = 4;  // SlotOcc inside the record
static_assert(sizeof(SlotOcc) <= kOccWords * 8, "occupy state fits its words");
constexpr int kCacheWords = 6;  // the cached counter group (array order)
__host__ __device__ constexpr int rec_hdr_words(int S) { return 2 * S + kOccWords + kCacheWords + 2; }
__host__ __device__ constexpr uint32_t rec_units(int S) {
    return ((uint32_t)(8 * S + 12 + 7) / 8 + 1u) & ~1u;  // 64-byte units, even (128-byte aligned records)
}
static_assert(rec_hdr_words(10) == 32 && rec_units(10) == 12, "S = 10: a two-line header, 768-byte record");
struct Rec {
    int64_t *r;
    int S;
    __device__ __forceinline__ int64_t &start(int j) const { return r[2 * j]; }
    __device__ __forceinline__ SlotOcc &occ() const { return *reinterpret_cast<SlotOcc *>(r + 2 * S); }
    __device__ __forceinline__ int64_t *cache() const { return r + 2 * S + kOccWords; }
    __device__ __forceinline__ int64_t &tag() const { return r[2 * S + kOccWords + kCacheWords]; }
    __device__ __forceinline__ double &thr() const {
        return *reinterpret_cast<double *>(r + 2 * S + kOccWords + kCacheWords + 1);
    }
    __device__ __forceinline__ int64_t *group(int j) const { return r + rec_hdr_words(S) + 6 * j; }
    __device__ __forceinline__ int64_t &cnt(int ev, int j) const {
        if (ev == CEV_PASS) return r[2 * j + 1];
        if (ev == CEV_WAITING) return group(j)[0];
        return group(j)[ev];  // BLOCK..OCCUPIED_BLOCK = ordinals 1..5
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
__device__ inline WinRef cur_window(const ClusterState &st, const SlotParam &P, uint32_t s, int64_t t) {
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
        SlotOcc &o = R.occ();
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

__device__ inline int64_t values_sum(const ClusterState &st, const SlotParam &P, int64_t t, int ev) {
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
    if (w.detached) return;
    const Rec R = rec_of(st, P);
    R.cnt(ev, w.j) += n;
    if (ev != CEV_PASS && R.tag() == R.start(w.j)) R.tag() = kAbsent;  // the cached group is stale now
}

// ClusterMetricLeapArray.getFirstCountOfWindow(PASS) = getValidHead(now).value().get(PASS)
__device__ __forceinline__ int64_t head_pass(const ClusterState &st, const SlotParam &P, int64_t t) {
    const Rec R = rec_of(st, P);
    const int j = (int)(((t + P.W) / P.W) % P.S);
    const int64_t w = R.start(j);
    return (w != kAbsent && !(t - w > (int64_t)P.interval)) ? R.cnt(CEV_PASS, j) : 0;
}

// ClusterFlowChecker.acquireClusterToken / SimpleClusterFlowChecker.acquireClusterToken for one request
__device__ inline uint64_t request_exact(const ClusterState &st, uint32_t s, int64_t t, int32_t a, bool p, int simple) {
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
            SlotOcc &o = rec_of(st, P).occ();
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


}  // namespace sga
