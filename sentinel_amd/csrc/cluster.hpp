// Device-side state and launch interface of the cluster token server path
// (ClusterFlowChecker + ClusterMetric over ClusterMetricLeapArray).
#pragma once
#include "../../include/sentinel_amd.h"
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

// Per slot mutable occupy state: ClusterMetricLeapArray.occupyCounter/hasOccupied (kept inside the
// slot's window record, after the (start, PASS) pairs)
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
    int64_t *rec;            // per slot: 8 fields x S buckets at rec[8*boff]; field 0 = window start
                             // (kAbsent = null), fields 1..7 = LongAdder sums per ClusterFlowEvent
    const HashEntry *htab;   // open-addressing flowId -> (slot, windowLengthInMs)
    const uint32_t *dense;   // when flowIds are dense, per flowId - 1: slot | wcode << 24 (all ones: no rule)
    uint32_t *dkey;          // the hot path's copy of `dense` (one per scratch set): a hot rule's entry is
                             // kDkHot | hot id instead, so the key pass's one 4-byte gather answers both
                             // (written when the hot set changes); no rule = kDkNone; wcode < 127 here
    const uint32_t *wtab;    // wcode -> windowLengthInMs
    const int64_t *slot_fid; // flowId per slot
    uint32_t dense_n;        // dense table length (0: hash lookup)
    uint32_t hmask;
    uint32_t nslots;
    double max_occupy_ratio;
    // Uniform geometry (every allocated slot has sampleCount uni_S, windowLength uni_W, interval uni_iv and
    // its record at slot * rec_units(uni_S) 64-byte units, the layout of one load of equal rules): a slot's record
    // address needs no parameter load, so the record loads do not wait for one.  uni_S = 0: not uniform.
    int32_t uni_S, uni_W, uni_iv, uni_pad;
};

constexpr uint32_t kDkHot = 0x80000000u, kDkNone = 0x7FFFFFFFu;

// A batch's requests as the device entries receive them: four arrays (int64 flowId, int32
// acquireCount, u8 prioritized or none, u32 time offset), or the packed 12-byte records of
// sga_token_request (3 words: flowId, time offset, acquireCount | flags << 16).
struct ReqIn {
    const int64_t *flow = nullptr;
    const int32_t *acq = nullptr;
    const uint8_t *prio = nullptr;
    const uint32_t *ts = nullptr;
    const uint32_t *pk = nullptr;
    __device__ __forceinline__ uint32_t ts_at(uint32_t i) const { return pk ? pk[3 * (size_t)i + 1] : ts[i]; }
    __device__ __forceinline__ int32_t acq_at(uint32_t i) const {
        return pk ? (int32_t)(pk[3 * (size_t)i + 2] & 0xFFFFu) : acq[i];
    }
    __device__ __forceinline__ bool prio_at(uint32_t i) const {
        return pk ? ((pk[3 * (size_t)i + 2] >> 16) & 1u) != 0 : (prio && prio[i]);
    }
    __device__ __forceinline__ int64_t flow_at(uint32_t i) const { return pk ? (int64_t)pk[3 * (size_t)i] : flow[i]; }
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
struct alignas(16) RunOut {  // 48 B: three 16-byte stores / loads
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

// Per-run record of a hot rule (k_hot_flows), read per request by k_hot_final / k_prio_results.
// The first 32 bytes are all that a non-prioritized request needs.
struct HotRun {
    int64_t s0;       // window PASS sum before the run
    double thr;       // threshold used
    double isec;      // intervalInSecond
    uint32_t f;       // passing prefix length
    uint32_t start;   // rank of the run's first request among the rule's requests of the batch
    uint32_t n;       // requests in the run (0: the rule has no request in this bucket)
    uint32_t p0;      // index of the run's first prioritized request in the prioritized region
    uint32_t cpf;     // prioritized requests inside the prefix
    uint32_t cw;      // occupied (SHOULD_WAIT) requests among the prioritized after the prefix
    uint16_t wait;    // waitInMs = 1000 / sampleCount
    uint8_t ok;       // closed form applied (0: never expected, counted in the error flags)
    uint8_t pad;
    uint32_t pad2[3];
};
static_assert(sizeof(HotRun) == 64, "hot run record");

// Hot path geometry.
constexpr int kHot = 4096;          // hot ids (12 bits in the request code)
constexpr uint16_t kColdId = 0xFFFF;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;  // hot_next: id not taken
constexpr int kHotCtlWords = 128;        // hot_ctl: [0..8) state, [8..40) count bins, [64..96) bin cursors
constexpr int kHotSeg = 8192;       // requests per wave segment of k_hot_classify (one count row)
constexpr int kSubSeg = 1024;       // cold compaction segment = sort input segment (4 per sort tile)
constexpr int kHotBuckets = 64;     // window buckets a batch may span on the hot path (6 bits)
constexpr int kHotGroupRows = 16;   // count rows per group of the column scan
constexpr int kHotCand = 1 << 16;   // next-hot-set candidates gathered per batch
constexpr int kSegStat = 4;         // seg_stat words per rank segment
// Cold partition (hot path): the cold elements are scattered once into kPartBins bins of consecutive
// rule slots (slot >> part_lb), and k_cold_fused orders each bin in its workgroup (SURVEY hard part 4)
constexpr int kPartBits = 11;
constexpr int kPartBins = 1 << kPartBits;
constexpr int kPartGroup = 64;      // key segments per group of the column scan
constexpr int kPartMaxLow = 10;     // slot bits below the bin (the in-workgroup digit) at most

// Per-batch control words (BatchScratch::counters, zeroed per batch).
enum : int {
    CTL_NVALID = 0, CTL_NRUNS = 1, CTL_NFLOWS = 2, CTL_LIMITED = 4, CTL_LIMRUNS = 5, CTL_DEFERRED = 6,
    CTL_FLAGS = 16,      // hot-path fallback reasons (kFlag*)
    CTL_NPRIO = 19,      // prioritized hot requests (pass 0; sorted on their own)
    CTL_NSORT = 20,      // elements to sort (the cold ones)
    CTL_NCOLD = 21,      // cold elements (the sorted elements the run kernels read)
    CTL_NPRE = 22,       // hot buckets starting inside a rank segment (k_hot_pre rows)
    CTL_BDLO = 23,       // hot bucket delta of the batch's first request
    CTL_BDHI = 24,       // largest hot bucket delta
    CTL_MODE = 25,       // 1: the batch runs the hot path
    CTL_HOTERR = 26,     // hot runs that needed a replay (never expected)
    CTL_WORDS = 64
};
enum : uint32_t {
    kFlagUnsorted = 1,   // timestamps decrease somewhere: no bucket order to rank by
    kFlagMixed = 2,      // a hot request with acquireCount != 1
    kFlagBucket = 4,     // the batch spans more than kHotBuckets hot buckets
    kFlagHotKey = 8,     // a key-table entry names a hot id outside the hot set (never expected)
    kFlagRerun = 15,     // any of the above: pass 1 re-classifies every request as cold
    kFlagState = 16      // a hot rule's window holds a bucket newer than the batch (precheck)
};

// Per batch and window-length code: windowLengthInMs, ts_base mod W, 1 / W (bucket deltas without
// int64 division).
struct WConst {
    uint32_t W, r0;
    double inv;
};

// Per-batch scratch (device), sized for max_batch events.
struct BatchScratch {
    uint64_t *el[2];          // packed sort elements (double buffer)
    // run records (index = run id, runs in sorted order)
    uint32_t *run_start, *run_slot, *run_idx0, *run_cp, *run_p0;
    int32_t *run_acq;         // common acquire count, 0 = mixed / escaped (replay)
    uint8_t *run_bd;          // bucket delta of the run
    uint32_t *flow_first_run; // per rule touched in the batch: its first run
    uint32_t *plist;          // sorted positions of prioritized requests (ascending)
    uint32_t *deferred;       // (flow, run) pairs handed from k_flows to k_flows_slow
    RunOut *run_out;
    RAgg *wave_carry;         // per 512-request wave slice: scan carry for k_results
    void *tile_agg;
    void *tile_carry;
    uint32_t *tile_valid;
    uint32_t *counters;       // CTL_* words
    uint32_t *counters_last;  // the last hot-path batch's CTL_* words (k_hot_fin saves them, then clears
                              // the live ones for the next batch: no clearing launch per batch)
    int counters_clean = 0;   // host: the live words are zero once the queued work has run
    uint32_t *lim_partial;    // scan partials over max_batch elements (namespace limiter pre-pass)
    RadixScratch radix;
    size_t cap = 0;
    // ---- hot path.  The hot set persists across batches (chosen from the previous batch's
    // per-rule request counts); it only decides how a request reaches its decision, never what
    // is decided.
    uint16_t *hot_of;         // per rule slot: hot id, kColdId = cold
    uint32_t *hot_slot;       // per hot id: rule slot
    uint32_t *hot_next;       // next batch's hot set while it is picked
    uint32_t *hot_ctl;        // [0] hot ids in use [1] picks [2] hot window length [3] next window length
                              // [4..5] best (count << 32 | slot) [6] candidates [7] last pick threshold
                              // [8..40) log2 count bins
    uint64_t *el_tile;        // classify output per 1024-request segment: cold elements, arrival order
    uint32_t *tile_nc;        // per 1024-request segment: elements
    uint64_t *pel_tile;       // per rank segment (kHotSeg requests): the prioritized hot requests (key = hot id),
                              // compacted in arrival order; seg_stat holds their count
    uint32_t *prow;           // [kPsGroups][kHot]: the prioritized requests per group of segments and hot id
    uint32_t *ppre;           // [kPsGroups][kHot]: the earlier groups' (k_psort_cols)
    uint32_t *ptot;           // [kHot]: per hot id
    uint64_t *pel[2];         // the prioritized hot requests sorted by hot id (double buffer of their own sort)
    uint32_t *hcode;          // per request: hot id | in-segment rank << 12 | bucket << 25 | prioritized << 31
                              // (~0: not a hot request)
    uint16_t *hcnt;           // [segment][kHot] hot requests per hot id
    uint32_t *hbase;          // [segment][kHot] rank of the segment's first request of the hot id
    uint32_t *hgsum;          // [group][kHot] group sums, then exclusive prefixes over groups
    uint16_t *hpre;           // [kHotBuckets][kHot] the segment's hot requests before the bucket's first
    uint32_t *hbnd;           // [kHotBuckets] the bucket's first request
    HotRun *hrun;             // [kHotBuckets][kHot]
    uint4 *hfin;              // [kHotBuckets][kHot]: (s0, f, start) of each hot run, what k_hot_final caches
    uint2 *hfs;               // [kHotBuckets][kHot]: (f, start) of each hot run, what k_hot_final_p stages
    double2 *hthr;            // [kHot] threshold and intervalInSecond of each hot rule (k_hot_flows)
    uint32_t *prank;          // per prioritized hot request (order of pel): its rank among its rule's requests
    uint32_t *plo, *phi;      // per hot id: its range in the prioritized region
    uint32_t *hot_tot;        // per hot id: requests in the batch
    WConst *wconst;           // [256] per window-length code
    uint32_t *seg_stat;       // per rank segment (kSegStat words): prioritized hot requests, largest hot bucket
                              // delta, latest request time (offset)
    unsigned long long *tmax_all;  // latest request time of every hot-path batch classified so far (precheck of
                                   // pipelined batches; shared by an engine's scratch sets)
    const uint64_t *el_sorted = nullptr, *pel_sorted = nullptr;  // stage 1's sorted cold / prioritized elements
    bool hot_early = false;   // host: the batch's hot runs and results were queued in stage 1 (beside the cold sort)
    bool sched2 = false;      // host: stream schedule 2 (cluster.hip hot_sched): the cold partition on `side`, the
                              // hot results on `side2`; the cold stage waits for ev_fork
    uint32_t *hot_cand;       // [kHotCand] (slot, count) of cold rules with >= hot_min requests (hot_ctl[6])
    // cold partition: [segment][bin] counts (then in-group exclusive prefixes), [group][bin] group sums
    // (then prefixes), [bin] bin starts (+ the total); part_lb: slot bits below the bin (host, 0 = LSD sort)
    uint32_t *phist, *pgrp, *pstart;
    int part_lb = 0;
    int hot_enabled = 1;      // host policy (sga_set_hot_rules)
    uint32_t small_max = 4096; // batches of at most this many requests take the one-workgroup path (sga_set_small_batch)
    int hot_lane_order = 0;   // lds_lane_order_ok() held on this device (set when the scratch is made)
    uint32_t hot_min = 64;    // smallest per-batch request count that makes a rule hot
    // hot/cold overlap: after the sort the hot side (ranks, hot runs, hot results) runs on `side`
    // beside the cold stage on the batch's stream (fork and join by events; made on first use)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_fork0 = nullptr, ev_mid = nullptr;
    // the prioritized hot requests' sort on a stream of its own (beside the hot count scans on `side`)
    hipStream_t side2 = nullptr;
    hipEvent_t ev_prio = nullptr;
};

// The hot path's in-order ranks come from LDS atomics whose same-word lanes are served in lane
// order; this probes that on the current device (once per engine scratch).
bool lds_lane_order_ok(hipStream_t stream);

// Forget the hot set (rule slots changed or scratch re-carved).
void hot_reset(const ClusterState &st, BatchScratch &b, uint32_t nslots_cap, hipStream_t stream);
// Releases the side stream and events of a scratch (engine teardown).
void batch_scratch_release(BatchScratch &b);

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
// The same over packed requests (sga_token_request): the hot path reads them directly; the other paths
// unpack them into the hot path's scratch (pel, prank) first.
void cluster_decide_batch_packed(const ClusterState &st, BatchScratch &sc, const uint32_t *pk, int64_t ts_base,
                                 uint32_t n, void *out, hipStream_t stream, const LimiterPass *lims = nullptr,
                                 int nlims = 0);

// Whether a batch takes the hot path (the small path and the limiter / RLS / look-back sort paths do not).
bool cluster_hot_eligible(const ClusterState &st, const BatchScratch &sc, uint32_t n, int simple, int nlims);
// The hot path in two stages for pipelined batches (sga_request_tokens_device_pipelined): stage 1 reads only the
// batch's inputs, the dense flowId table and the hot rules' window starts (the precheck refuses a batch that
// starts before an earlier batch's latest time); stage 2 decides.  A batch's stage 2 must follow its stage 1 and
// every earlier batch's stage 2; the next batch on the same scratch may start stage 1 once this stage 2 is done.
void cluster_classify_hot(const ClusterState &st, BatchScratch &sc, const int64_t *flow_id, const int32_t *acquire,
                          const uint8_t *prio, int64_t ts_base, const uint32_t *ts_off, uint32_t n, void *out,
                          hipStream_t stream);
void cluster_decide_hot(const ClusterState &st, BatchScratch &sc, const int32_t *acquire, const uint8_t *prio,
                        int64_t ts_base, const uint32_t *ts_off, uint32_t n, void *out, hipStream_t stream);

// ---------------------------------------------------------------------------------------------
// Cluster parameter flow (ClusterParamFlowChecker + ClusterParamMetric, CS/flow/ClusterParamFlowChecker.java:37-120,
// CS/flow/statistic/metric/ClusterParamMetric.java:41-88).  Per rule slot the rule-level LeapArray
// starts; per (rule, value) key a record [stamp x S][count x S][access x S] where stamp = start of the
// rule bucket the count belongs to (a count is live -- the key is in that bucket's map -- while its
// stamp equals the rule's start: resetWindowTo clearing a bucket's map = the rule start moving past the
// stamp) and access = the key's last access in that bucket's map (LRU order, see cparam_exact.hpp).
struct PRuleParam {
    double count;        // ParamFlowRule.count
    double isec;         // intervalInMs / 1000.0
    uint32_t boff;       // rule-level starts at rstart[boff .. boff + S)
    int32_t S, W, interval;
    int32_t active, ns, threshold_type;
    uint32_t hot_off, n_hot;  // hot items (ascending value) at hot_v/hot_c[hot_off ..)
    uint32_t cap;        // each bucket map's capacity (ClusterParamMetric maxCapacity, default 4000)
};

// LRU-mode queue record (cparam_exact.hpp): the key and the access stamp it was pushed with
struct PLruRec {
    uint64_t kidx;
    uint64_t stamp;
};
constexpr uint64_t kPNoQueue = ~0ull;
constexpr uint64_t kPLruBuilding = ~0ull;  // meta.kidx of an area the switch is filling

struct CParamState {
    const PRuleParam *param;
    int64_t *rstart;          // rule-level window starts (kAbsent = null)
    int64_t *tmax;            // per rule slot: latest call time seen
    uint8_t *coupled;         // per rule slot, per batch: needs the sequential path
    const HashEntry *htab;    // flowId -> slot (open addressing)
    uint32_t hmask, nslots;
    const int64_t *hot_v;
    const int32_t *hot_c;
    const int32_t *ns_connected;
    int64_t *vtab;            // value table: value -> vid = index (kAbsent = empty; kAbsent itself -> vid vcap)
    uint32_t vmask;
    uint64_t *ktab;           // key table: ((slot + 1) << 32 | vid) -> kidx = index (0 = empty)
    uint32_t kmask;
    uint32_t *koff;           // per kidx: record offset (int64 units) in krec
    uint32_t *kslot;          // per kidx: rule slot
    int64_t *kval;            // per kidx: value
    int64_t *krec;
    uint64_t krec_cap;        // int64 units
    uint32_t *ctl;            // [0] krec cursor  [1] error flags (1 key table full, 2 record pool full,
                              //     4 LRU queue check)  [2] slow requests  [3] global slow (timestamps
                              //     not ascending)  [4] rules switching to LRU mode (k_plru_decide)
    // CacheMap capacity (strict LRU, cparam_exact.hpp)
    uint32_t *nkeys;          // per rule slot: keys ever created (a bucket map can only overflow past cap keys)
    uint64_t *pq;             // per rule bucket (boff + j): LRU queue area in lpool (kPNoQueue: free mode)
    uint32_t *psize;          // per rule bucket, LRU mode: keys in the bucket's map
    PLruRec *lpool;
    uint32_t *sw_list;        // rules switching this batch
    uint64_t seq;             // access stamp base of this batch / call
};

struct CParamScratch {
    uint64_t *els[2];         // sequential-path elements (slot << 40 | request index)
    uint32_t *vkey;           // per value of the batch: kidx
};

// off[i] = ts[i] - lo, ts int32 deltas from the batch's first time (host-buffer batches ship those)
void cluster_ts_offsets(const int32_t *ts, int64_t lo, uint32_t *off, uint32_t n, hipStream_t s);
// registered host buffers: int64 times on the device; minmax[0..1] = their min / max; off = ts - lo
void cluster_ts_minmax(const int64_t *ts, uint32_t n, int64_t *minmax, hipStream_t s);
void cluster_ts_offsets64(const int64_t *ts, int64_t lo, uint32_t *off, uint32_t n, hipStream_t s);

size_t cparam_scratch_bytes(size_t cap);
void cparam_scratch_carve(CParamScratch &ps, void *base, size_t cap);

// Batched DefaultTokenService.requestParamToken over DEVICE buffers (host API drives it and reads
// st.ctl between the stages).  Stage 1: validation, rule lookup, namespace limiter, value/key
// insertion, path choice.  Stage 2: key-parallel closed form + sequential per-rule replay.
void cparam_stage1(const CParamState &st, BatchScratch &sc, CParamScratch &ps, const int64_t *flow_id,
                   const int32_t *acquire, const uint32_t *voff, const int64_t *values, int64_t ts_base,
                   const uint32_t *ts_off, uint32_t n, void *out, hipStream_t stream, const LimiterPass *lims,
                   int nlims);
void cparam_stage2(const CParamState &st, BatchScratch &sc, CParamScratch &ps, const int32_t *acquire,
                   const uint32_t *voff, const int64_t *values, int64_t ts_base, const uint32_t *ts_off, uint32_t n,
                   uint32_t nslow, void *out, hipStream_t stream);
// ClusterParamMetric.getSum(value) at now (rotation side effect included); *d_out = -1 if no key
void cparam_sum(const CParamState &st, uint32_t slot, int64_t value, int64_t now, int64_t *d_out, hipStream_t s);
void cparam_init_rule(const CParamState &st, uint32_t slot, hipStream_t s);
// CacheMap capacity: rules whose key count passed their capacity switch to LRU mode (the sequential
// path from then on).  decide lists them (count in ctl[4]); the host assigns each an area of S x
// (2 cap + 3) records (qoff, one per listed rule; max_s = their largest S) and calls switch, which
// fills the areas from the access stamps.
void cparam_lru_decide(const CParamState &st, hipStream_t s);
void cparam_lru_switch(const CParamState &st, const uint64_t *d_qoff, uint32_t nsw, uint32_t max_s, hipStream_t s);
// ClusterParamMetric.getTopValues(number) of one rule at now: d_list holds 2 x (kmask + 1) int64.
void cparam_top_values(const CParamState &st, uint32_t slot, int64_t now, uint32_t number, int64_t *d_list,
                       uint32_t *d_count, int64_t *d_val, double *d_qps, uint32_t *d_n, hipStream_t s);

// ClusterMetricNodeGenerator.flowToMetricNode for every active slot (out: sga_cluster_metric_node,
// count: device u32; slot_fid: flowId per slot).
void cluster_metric_nodes(const ClusterState &st, const int64_t *slot_fid, int64_t now, void *out, uint32_t cap,
                          uint32_t *count, hipStream_t stream);

// Fresh limiter state (every bucket absent).
void cluster_init_limiter(NsLimiterDev *d, hipStream_t stream);
// Envoy RLS over device buffers: descriptors -> token requests, token results -> codes
void rls_expand(const uint32_t *off, uint32_t nreq, const int64_t *dfid, const int32_t *hits, const uint32_t *ts_off,
                int64_t *fid_out, int32_t *acq_out, uint32_t *ts_out, hipStream_t s);
void rls_finish(const uint32_t *off, uint32_t nreq, const int32_t *hits, const uint64_t *res, int8_t *desc_status,
                int32_t *desc_rem, int32_t *code, hipStream_t s);

// ClusterMetric.getSum for all 7 events at `now` (rotates the current window as the reference does).
void cluster_metric_sums(const ClusterState &st, uint32_t slot, int64_t now, int64_t *d_out7, hipStream_t stream);

// Fresh metrics: every bucket of each listed slot absent, occupy counters zero.
void cluster_init_slots(const ClusterState &st, const uint32_t *d_slots, uint32_t n, hipStream_t stream);
// copy SlotParam::thr into the header of every allocated slot < n (Rec::thr, cluster_exact.hpp)
void cluster_sync_rec_thr(const ClusterState &st, uint32_t n, hipStream_t stream);

}  // namespace sga
