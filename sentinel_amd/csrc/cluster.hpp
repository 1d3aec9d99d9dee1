// Device-side state and launch interface of the cluster token server path
// (ClusterFlowChecker + ClusterMetric over ClusterMetricLeapArray).
#pragma once
#include "common.hpp"
#include "radix_sort.hpp"

namespace sga {

// Per rule slot, read-only during a batch (48 bytes).
struct SlotParam {
    double thr;         // calcGlobalThreshold(rule) * exceedCount   ClusterFlowChecker.java:38-48,68
    double thr_simple;  // rule.count * exceedCount                  SimpleClusterFlowChecker.java:43
    double isec;        // LeapArray.intervalInSecond = intervalInMs / 1000.0  LeapArray.java:68
    uint32_t boff;      // bucket offset of this slot's ClusterMetricLeapArray (record at rec[8*boff])
    int32_t S;          // sampleCount of the metric (fixed at metric creation)
    int32_t W;          // windowLengthInMs = interval / sampleCount
    int32_t interval;   // intervalInMs
    int32_t active;     // rule present (FLOW_RULES contains the flowId)
    int32_t ns;         // namespace index
};

// Per slot mutable occupy state: ClusterMetricLeapArray.occupyCounter/hasOccupied
struct SlotOcc {
    int64_t occ_pass;   // occupyCounter[PASS]
    int64_t occ_preq;   // occupyCounter[PASS_REQUEST]
    int32_t has_occ;    // hasOccupied
    int32_t pad;
};

// Bucket field ordinals = ClusterFlowEvent ordinals.
enum : int { CEV_PASS = 0, CEV_BLOCK, CEV_PASS_REQUEST, CEV_BLOCK_REQUEST, CEV_OCCUPIED_PASS, CEV_OCCUPIED_BLOCK,
             CEV_WAITING, CEV_N };

// flowId -> slot hash entry (16 B, one load per probe); key 0 = empty (flowIds are > 0)
struct alignas(16) HashEntry {
    int64_t key;
    uint32_t slot;
    uint32_t W;  // windowLengthInMs of the slot's metric
};

struct ClusterState {
    const SlotParam *param;
    SlotOcc *occ;
    int64_t *rec;            // per slot: 8 fields x S buckets at rec[8*boff]; field 0 = window start
                             // (kAbsent = null), fields 1..7 = LongAdder sums per ClusterFlowEvent
    const HashEntry *htab;   // open-addressing flowId -> (slot, windowLengthInMs)
    const uint32_t *dense;   // when flowIds are dense: dense[flowId - 1] = slot | wcode << 24 (~0u: none)
    const uint32_t *wtab;    // wcode -> windowLengthInMs
    uint32_t dense_n;        // dense table length (0: hash lookup)
    uint32_t hmask;
    uint32_t nslots;
    double max_occupy_ratio;
};

// GlobalRequestLimiter / RequestLimiter of one namespace over UnaryLeapArray(10, 1000)
// (CS/flow/statistic/limit/RequestLimiter.java:29-87, GlobalRequestLimiter.java:32-55).
struct NsLimiterDev {
    int64_t start[10];  // window start (kAbsent = null)
    int64_t cnt[10];    // LongAdder
};

struct LimiterPass {
    int32_t ns;           // namespace index
    double qps_allowed;   // RequestLimiter.qpsAllowed
    NsLimiterDev *state;  // device
};

// Per-run decision record written by k_flows, read by k_results (40 B).
struct RunOut {
    int64_t s0;     // window PASS sum before the run (closed form)
    double thr;     // threshold used
    double isec;    // intervalInSecond
    uint32_t f;     // passing prefix length
    uint32_t cpf;   // prioritized requests inside the prefix
    uint32_t cw;    // occupied (SHOULD_WAIT) requests among the prioritized after the prefix
    uint16_t wait;  // waitInMs = 1000 / sampleCount
    uint8_t mode;   // 0 closed form, 1 replayed (results already written)
    uint8_t pad;
};

// Results-side scan value (a projection of the run scan): run heads so far, run head seen,
// prioritized requests since the last run head.
struct RAgg {
    uint32_t nh, flag, cnt;
};

// Per-batch scratch (device), sized for max_batch events.
struct BatchScratch {
    uint64_t *el[2];          // packed sort elements (double buffer)
    // run records (index = run id, runs in sorted order)
    uint32_t *run_start, *run_slot, *run_idx0, *run_cp, *run_p0;
    int32_t *run_acq;         // common acquire count, 0 = mixed / escaped (replay)
    uint32_t *flow_first_run; // per rule touched in the batch: its first run
    uint32_t *plist;          // sorted positions of prioritized requests (ascending)
    uint32_t *deferred;       // (flow, run) pairs handed from k_flows to k_flows_slow
    RunOut *run_out;
    RAgg *wave_carry;         // per 512-request wave slice: scan carry for k_results
    void *tile_agg;
    void *tile_carry;
    uint32_t *tile_valid;
    uint32_t *counters;  // [0]=nvalid [1]=nruns [2]=nflows [4]=limited [5]=limiter runs [6]=deferred flows
    uint32_t *lim_partial;  // scan partials over max_batch elements (namespace limiter pre-pass)
    RadixScratch radix;
    size_t cap = 0;
};

// Requests per batch are indexed with 26 bits inside the packed sort element; rule slots with 24.
constexpr size_t kMaxBatch = (size_t)1 << 26;
constexpr uint32_t kMaxSlots = (1u << 24) - 2;

size_t batch_scratch_bytes(size_t cap, uint32_t nslots_cap);
void batch_scratch_carve(BatchScratch &b, void *base, size_t cap, uint32_t nslots_cap);

// Runs the whole decision pipeline for one batch on `stream` (asynchronous).
// simple != 0 selects SimpleClusterFlowChecker semantics (Envoy RLS).
void cluster_decide_batch(const ClusterState &st, BatchScratch &sc, const int64_t *flow_id, const int32_t *acquire,
                          const uint8_t *prio, int64_t ts_base, const uint32_t *ts_off, uint32_t n, int simple,
                          void *out /* sga_token_result */, hipStream_t stream, const LimiterPass *lims = nullptr,
                          int nlims = 0);

// Fresh limiter state (every bucket absent).
void cluster_init_limiter(NsLimiterDev *d, hipStream_t stream);

// ClusterMetric.getSum for all 7 events at `now` (rotates the current window as the reference does).
void cluster_metric_sums(const ClusterState &st, uint32_t slot, int64_t now, int64_t *d_out7, hipStream_t stream);

// Fresh metrics: every bucket of each listed slot absent, occupy counters zero.
void cluster_init_slots(const ClusterState &st, const uint32_t *d_slots, uint32_t n, hipStream_t stream);

}  // namespace sga
