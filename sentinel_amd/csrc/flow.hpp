// Local path (StatisticSlot + ParamFlowSlot + FlowSlot + DegradeSlot) -- device engine.
#pragma once
#include <functional>

#include "cluster.hpp"
#include "../../include/sentinel_amd.h"
#include "common.hpp"
#include "radix_sort.hpp"

#include <vector>

namespace sga {

// FlowState::overflow bits: any other bit = a parameter map filled (SGA_ENOMEM); kOvfMissingEntry = a
// parameter event of a per-value segment flow found no thread-count entry, which every such event had
// claimed before (never expected: the batch fails with SGA_EIO instead of leaving the event undecided)
constexpr uint32_t kOvfMissingEntry = 0x80000000u;
constexpr const char *kMissingEntryText =
    "parameter event without its thread-count map entry (k_pseg_key device check); the batch failed";


// ---- node record (one ClusterNode per resource), int64 words -------------------
// second window: OccupiableBucketLeapArray(2, 1000)  (StatisticNode.java:99-100)
// borrow window: FutureBucketLeapArray(2, 1000)      (OccupiableBucketLeapArray.java:33-37)
// minute window: BucketLeapArray(60, 60000)          (StatisticNode.java:106)
// MetricBucket fields: start, PASS, BLOCK, EXCEPTION, SUCCESS, RT, OCCUPIED_PASS, minRt
constexpr int kMB = 8;
enum : int { MB_START = 0, MB_PASS, MB_BLOCK, MB_EXC, MB_SUCC, MB_RT, MB_OPASS, MB_MINRT };
constexpr int kNodeSec = 0;                       // 2 x 8
constexpr int kNodeBor = kNodeSec + 2 * kMB;      // 2 x 2 (start, PASS)
constexpr int kNodeMin = kNodeBor + 4;            // 60 x 8
constexpr int kNodeThreads = kNodeMin + 60 * kMB; // curThreadNum
constexpr int kNodeLastFetch = kNodeThreads + 1;  // StatisticNode.lastFetchTime (-1 initially)
constexpr int kNodeWords = kNodeThreads + 4;      // 504 words = 4032 B (64-B aligned)

struct FlowRuleDev {    // one rater (TrafficShapingController) + its FlowRule fields
    int32_t behavior, grade;
    double count;
    int32_t max_queue, cold_factor;
    int32_t warning_token, max_token;
    double slope;
    int64_t latest_passed;   // RateLimiterController / WarmUpRateLimiterController latestPassedTime
    int64_t stored_tokens;   // WarmUpController.storedTokens
    int64_t last_filled;     // WarmUpController.lastFilledTime
    // FlowRule.clusterMode (FlowRuleChecker.passClusterCheck): the token server's rule slot for the
    // rule's flowId (-1: no such cluster rule -> NO_RULE_EXISTS), resolved on the host before a batch
    int32_t cluster, cfallback;
    int64_t cflow;
    int32_t cslot, cpad;
};

struct ParamRuleDev {
    int32_t grade, behavior;
    double count;
    int32_t max_queue, burst;
    int32_t param_idx, n_hot;
    int64_t duration;
    uint32_t hot_off, id;   // id: global param-rule id (hash-table key part)
    // ParamFlowSlot.applyRealParamIdx (ParamFlowSlot.java:56-66) rewrites a negative index on the rule at
    // its first check: the index in force (kIdxUnresolved until then), kept by equal rules on reload
    int32_t idx_res;
    // ParamFlowRule.clusterMode (QPS grade): decided by the embedded server's parameter path
    int32_t cluster, cfallback;
    int32_t cpad;
    int64_t cflow;
    uint32_t cap;   // ParameterMetric: the rule's time / token CacheMap capacity, min(4000 * durationInSec, 200000)
    uint32_t pad2;
};
constexpr int32_t kIdxUnresolved = INT32_MIN;
constexpr int kMaxParamIdx = 64;  // thread-count maps exist for argument indices 0..63

struct CbDev {
    int32_t grade, min_req;
    double count, slow_ratio;
    int32_t stat_interval, state;   // state: 0 CLOSED, 1 OPEN, 2 HALF_OPEN
    int64_t recovery_ms, max_allowed_rt, next_retry;
    int64_t st_start, st_bad, st_total;  // LeapArray(1, statIntervalMs) bucket
    int64_t probe_t;  // time of the entry that moved it OPEN -> HALF_OPEN (its revoke moves it back)
};

struct ResDev {
    uint32_t rule_off, n_rules;
    uint32_t prule_off, n_prules;
    uint32_t cb_off, n_cbs;
    uint32_t fast;   // bit0: single QPS Default/WarmUp rule, no param rules, no breakers;
                     // bit1: the resource has a parameter thread-count map (sticky)
    uint32_t pad;
};

// (rule, value) -> {time, tokens} for ParameterMetric rule maps; (resource, value) -> thread count
struct alignas(32) PEntry {
    uint64_t value;
    uint32_t owner;   // rule id + 1 (param maps) or resource + 1 (thread counts); 0 = empty
    uint32_t pad;
    int64_t a;        // time counter / thread count
    int64_t b;        // token counter
};
constexpr int64_t kPAbsent = INT64_MIN;

// ParameterMetric's CacheMaps (ConcurrentLinkedHashMapWrapper, strict LRU; ParameterMetric.java:37-39,95-121).
// Every key access stamps the key's map slot with ((event sequence) << 16 | element index): within an
// owner (a rule's time/token map, or a resource's thread-count map of one argument index) stamps grow
// with the access order.  An owner whose keys cannot exceed its capacity in a batch (count pass) stays in
// free mode (any kernel, sizes kept exactly); one that could is switched to LRU mode for good: its
// present keys go into a recency queue (records {value, stamp}, oldest first), its resource is decided
// in arrival order by one lane, every access appends a record, and an insert into a full map evicts the
// oldest record whose stamp still matches its key.
struct LruRec {
    uint64_t value;
    uint64_t stamp;  // the queue area's first record holds {head, tail}
};
constexpr uint64_t kNoQueue = ~0ull;        // free mode
constexpr uint32_t kNoTBase = 0xFFFFFFFFu;  // a resource without thread-count map owner slots
constexpr uint32_t kThreadMapCap = 4000;    // ParameterMetric.THREAD_COUNT_MAX_CAPACITY
constexpr uint64_t kStampMark = 1ull << 63;  // count pass: an absent key first met in this batch

// SystemRuleManager thresholds (SystemRuleManager.java:62-74) + SystemStatusListener readings
struct SysDev {
    int32_t check, load_set, cpu_set, pad;
    double load, cpu, qps;
    int64_t max_rt, max_thread;
    double cur_load, cur_cpu;
};

struct FlowState {
    int64_t *node;
    FlowRuleDev *rules;
    ParamRuleDev *prules;
    const uint64_t *hot_v;
    const int32_t *hot_t;
    CbDev *cbs;
    const ResDev *res;
    PEntry *ptab;      // param time/token maps
    PEntry *ttab;      // thread-count maps
    uint32_t pmask, tmask;
    uint32_t nres;
    uint32_t *overflow;  // set when a param table is full (bit kOvfMissingEntry: a device check failed)
    // embedded cluster token server for cluster-mode FlowRules (sga_set_cluster_server 1)
    ClusterState cst;
    int32_t cluster_on;
    int32_t lru_ps;              // k_llru_ps takes LRU-mode parameter-only resources (SGA_LRU_PS=0: k_llru)
    // device entry (sga_submit_events_device): the chunk's gate word, written by k_lgate; nullptr on
    // the host entry, which chooses the kernels itself
    const uint32_t *gate;
    // per resource: bit k set once a parameter rule with (resolved) index k was checked -- the
    // ParameterMetric thread-count map of argument k exists (ParameterMetric.initialize, :113-121)
    uint64_t *tmapmask;
    // embedded cluster server's parameter path for cluster-mode parameter rules (ctl null: no rules)
    CParamState cpst;
    // CacheMap capacity (LruRec above)
    uint64_t *pstamp, *tstamp;   // per map slot: stamp of the key's last access
    uint32_t *psize;             // per parameter-rule id: keys present in its time/token map
    uint64_t *pq;                // per parameter-rule id: LRU queue area in lpool (kNoQueue: free mode)
    const uint32_t *pcap, *pres; // per parameter-rule id: capacity, resource
    const uint32_t *tbase;       // per resource: first of its kMaxParamIdx thread-map owner slots
    const uint32_t *tres;        // per thread-slot base (tbase / kMaxParamIdx): its resource
    uint32_t *tsize;             // per thread-map owner slot: keys present
    uint64_t *tq;                // per thread-map owner slot: LRU queue area (kNoQueue: free mode)
    LruRec *lpool;
    uint64_t lpool_cap;
    unsigned long long *lcursor; // next free record of lpool
    uint32_t *pnew, *tnew;       // count pass: distinct absent keys the batch may insert, per owner
    uint8_t *lru_res;            // per resource: an owner in LRU mode (its events replay in arrival order)
    uint32_t *lru_ctl;           // [0] owners switched this batch [1] error bits (1 queue pool full, 2 queue check)
                                 // [2] events in lneed
    uint32_t *lru_list;          // owners switched this batch: param id, or kLruThread | thread slot
    uint32_t *lneed;             // count pass input: the batch's events with a key absent at its start ([2] of lru_ctl)
    uint32_t nprid, ntslot;      // parameter-rule ids, thread-map owner slots
    uint64_t seq_base;           // event sequence of the batch's first event
};
constexpr uint32_t kLruThread = 1u << 31;

// A RateLimiter window's state-independent summary (flow.hip k_lwsum): its entries with a nonzero
// cost block while latestPassedTime L is past kmax + maxQueueingTime (kmax: the largest ts_off - cost),
// and its zero-cost entries pass with L unchanged while L - maxQueueingTime <= t0min and t0max <= L;
// n0 / a0: the entries that then pass (zero cost or acquireCount 0), their count and acquire sum; has0: any
// zero-cost entry with a positive acquireCount (t0min / t0max hold)
struct WinSum {
    int64_t kmax;
    int64_t a0;
    uint32_t t0min, t0max, n0, has0;
};

struct CbAgg {
    int64_t ws, bad, tot;  // a breaker stat window's counts: the last window's start (kCbNone: no exit), bad, total
};
struct CbTile {  // one tile of a long exit-only breaker flow (k_cbt_*)
    CbAgg agg, carry;
    int64_t first, last;  // windows
    uint32_t bad;         // a window went back inside the tile
};

struct FlowScratch {
    uint32_t *keys[2];
    Payload *pay[2];
    uint32_t *ev_run, *ev_eidx;
    uint32_t *run_start, *run_end, *run_slot, *run_t0off, *run_nent, *run_cp;
    int32_t *run_amin, *run_amax;
    int64_t *run_asum;            // entries' acquire counts per run (k_lwave's saturated tail: blocks = sum - passes)
    uint64_t *run_exc, *run_exerr;
    int64_t *run_exrt, *run_exmin;
    uint32_t *run_nexit;
    uint32_t *run_f;
    uint8_t *run_mode;
    uint32_t *flow_first_run;
    uint32_t *heavy;  // flows replayed by k_lheavy (count in counters[8])
    uint32_t *pace;   // long single-rule fast-path flows decided by k_lwave (count in counters[9])
    uint32_t *lru;    // flows of resources with a map in LRU mode, replayed by k_llru (count in counters[10])
    // parameter-only resources decided per (rule, value) segment (flow.hip k_pseg_*): their flows (count in
    // counters[11]), the events as (thread-count map slot << 32 | sorted position), sorted by slot, the
    // segments' first elements (count in counters[12]), and each run's pass / block acquire sums and passes
    uint32_t *pseg;
    uint32_t *plong;  // long regular entry segments (first element, length; count in counters[14], k_pseg_long)
    uint32_t *cbf;       // the breaker-only flows that move their breaker (count in counters[13], k_cb_flows)
    int64_t *rt_sorted;  // each exit's response time at its sorted position (k_lexits; k_cb_flows reads it in order)
    // long exit-only breaker flows over the whole GPU (k_cbt_*): per taken flow its cbf index, first tile, first
    // tripping exit, state and total; per tile its flow, counts and carry; [0] flows [1] tiles
    uint32_t *cbt_flow, *cbt_off, *cbt_trip, *cbt_state, *cbt_tile, *cbt_ctl;
    CbTile *cbt;
    CbAgg *cbt_total;
    uint64_t *pel[2];
    Payload *spay;  // the per-value segments' payloads in sorted order (k_pseg_gather): one gather, then streams
    uint32_t *seg;
    int64_t *run_pa, *run_ba;
    uint32_t *run_np;
    WinSum *wsum;     // per 64-event window (j / 64) of a RateLimiter k_lwave run (k_lwsum)
    int64_t *wstate;  // per window: the state k_lwave skipped it at, or kWinWalked (flow.hip RUN_WIN)
    void *tile_agg, *tile_carry;
    uint32_t *tile_valid;
    uint32_t *counters;
    RadixScratch radix;
    size_t cap = 0;
    const uint32_t *gate = nullptr;  // as FlowState::gate
    // Events the slot chain replays with their original arguments (F_SPECIAL: kind 2 / 3 events, argument
    // vectors and Collection arguments k_lclassify could not restate as one value): their resources are
    // marked res_special[r] == epoch for this chunk and go to the per-resource replay.  ev_param: every
    // event's parameter after that restatement (what the parallel kernels read as param_in).
    uint64_t *ev_param = nullptr;
    uint32_t *res_special = nullptr;
    uint32_t epoch = 0;
    const uint8_t *in_kind = nullptr, *in_flags = nullptr;
    const uint64_t *in_param = nullptr, *pvals = nullptr;
};

void print_heavy_prof();  // SGA_HEAVY_PROF=1 diagnostics (flow.hip)

struct FlowEngine {
    sga_config cfg{};
    hipStream_t stream = nullptr;
    uint32_t nres = 0;
    DevBuf<int64_t> d_node;
    DevBuf<FlowRuleDev> d_rules;
    DevBuf<ParamRuleDev> d_prules;
    DevBuf<uint64_t> d_hot_v;
    DevBuf<int32_t> d_hot_t;
    DevBuf<CbDev> d_cbs;
    DevBuf<ResDev> d_res;
    DevBuf<PEntry> d_ptab, d_ttab;
    DevBuf<uint32_t> d_overflow;
    DevBuf<uint32_t> d_keycount;
    DevBuf<uint64_t> d_tmapmask;  // FlowState::tmapmask
    DevBuf<uint32_t> d_res_special;  // FlowScratch::res_special (per resource, the chunk epoch that marked it)
    uint32_t epoch = 0;
    // CacheMap capacity (FlowState: pstamp .. seq_base)
    DevBuf<uint64_t> d_pstamp, d_tstamp, d_pq, d_tq;
    DevBuf<uint32_t> d_psize, d_pcap, d_pres, d_pnew, d_tbase, d_tres, d_tsize, d_tnew, d_lru_ctl, d_lru_list, d_lneed;
    DevBuf<uint8_t> d_lru_res;
    DevBuf<LruRec> d_lpool;
    DevBuf<unsigned long long> d_lcursor;
    std::vector<uint32_t> h_tbase;  // per resource (kNoTBase until it gets parameter rules)
    uint32_t ntbase = 0;            // resources given thread-map owner slots
    uint64_t seq = 0;               // events submitted so far (stamps)
    void lru_sync_rules();          // per-id / per-slot arrays after a parameter-rule load
    // parameter-only resources per (rule, value) segment, after k_lflows took their flows (flow.hip k_pseg_*)
    void launch_pseg(const FlowState &st, const FlowScratch &g, const Payload *pay, const uint32_t *keys,
                     int64_t ts_base, const int64_t *rt, const uint64_t *param, int8_t *decision, int32_t *wait_ms,
                     uint32_t m, hipStream_t s);
    void debug_size_check();  // SGA_SIZE_CHECK=1 diagnostics
    void lru_prepare(const uint8_t *kind, const uint32_t *resource, const uint8_t *flags, const uint64_t *param,
                     const uint64_t *pvals, uint32_t n, hipStream_t s);  // count pass + switches, before a batch
    int lru_error(hipStream_t s);   // sticky queue errors (host wait)
    CParamState cparam_st{};      // set before each batch (the engine's cluster parameter state)
    bool has_cluster_prules = false;
    // after the count pass (which creates the cluster-mode rules' keys): the engine switches cluster
    // parameter rules past their CacheMap capacity to LRU mode and refreshes cparam_st (host wait)
    std::function<void(hipStream_t)> cparam_hook;
    // upper bounds of the keys held by the parameter / thread-count maps (exact after a count);
    // the maps are rehashed into more room before a batch could fill them past a quarter
    size_t pkeys_ub = 0, tkeys_ub = 0;
    int ensure_maps(size_t m);
    void grow_map(DevBuf<PEntry> &tab, DevBuf<uint64_t> &stamp, size_t &ub, size_t add);
    DevBuf<uint8_t> d_scratch;
    FlowScratch sc;
    size_t scratch_cap = 0;
    // host mirrors for rule reloads
    std::vector<FlowRuleDev> h_rules;
    std::vector<sga_flow_rule> h_flow_src;
    std::vector<ParamRuleDev> h_prules;
    std::vector<sga_param_rule> h_prule_src;
    std::vector<std::vector<uint64_t>> h_prule_hot_v;
    std::vector<std::vector<int32_t>> h_prule_hot_t;
    std::vector<CbDev> h_cbs;
    std::vector<sga_degrade_rule> h_cb_src;
    std::vector<ResDev> h_res;
    uint32_t next_prule_id = 0;
    // staging for host API
    DevBuf<uint8_t> d_kind, d_flags;
    DevBuf<uint32_t> d_resid, d_ts;
    DevBuf<int32_t> d_acq;
    DevBuf<int64_t> d_rt;
    DevBuf<uint64_t> d_param;
    DevBuf<int8_t> d_dec;
    DevBuf<int32_t> d_wait;
    DevBuf<int64_t> d_view;

    void init(const sga_config &c, hipStream_t s) {
        cfg = c;
        stream = s;
    }
    void release() { print_heavy_prof(); }
    FlowState state() const;
    // cluster-mode FlowRules: the engine's cluster state and ClusterStateManager mode, set before
    // each batch (sga_set_cluster_server); resolve_cluster fills every cluster rule's slot
    ClusterState cluster_st{};
    int32_t cluster_on = 0;
    bool has_cluster_rules = false;
    uint64_t cluster_resolved_gen = ~0ull;
    int resolve_cluster(const std::function<int32_t(int64_t)> &slot_of_flow, uint64_t gen);
    int set_resources(uint32_t n);
    int load_flow_rules(const sga_flow_rule *r, size_t n);
    int load_param_rules(const sga_param_rule *r, size_t n);
    int load_degrade_rules(const sga_degrade_rule *r, size_t n);
    void upload_res();
    int submit(const uint8_t *kind, const uint32_t *resource, const int64_t *ts, const int32_t *acquire,
               const uint8_t *flags, const int64_t *rt, const uint64_t *param, size_t n, int8_t *decision,
               int32_t *wait_ms, const uint64_t *pvals = nullptr, size_t npvals = 0);
    FlowScratch special_scratch(const FlowScratch &base, const uint8_t *d_kind_in, const uint8_t *d_flags_in,
                                const uint64_t *d_param_in, const uint64_t *d_pvals);
    DevBuf<uint64_t> d_pvals;  // values of Collection / array arguments (SGA_EV_PARAM_LIST)
    // the same over device buffers, asynchronous on s: one chunk of n <= max_batch events
    // small host batches (<= kSmallEvents events, <= kSmallWords argument words, no SystemRule check): one
    // packed page-locked copy each way and one replay kernel (k_lsmall) instead of the pipeline
    static constexpr uint32_t kSmallEvents = 1024, kSmallWords = 16384;
    uint32_t small_max = kSmallEvents;  // sga_set_small_batch (0: off)
    PinnedBuf h_small;
    DevBuf<uint8_t> d_small;
    int submit_small(const uint8_t *kind, const uint32_t *resource, const int32_t *acquire, const uint8_t *flags,
                     const int64_t *rt, const uint64_t *param, const uint32_t *ts_off, int64_t lo, uint32_t m,
                     int8_t *decision, int32_t *wait_ms, const uint64_t *pvals, size_t npvals);
    int submit_device(const uint8_t *d_kind, const uint32_t *d_resource, int64_t ts_base, const uint32_t *d_ts_off,
                      const int32_t *d_acquire, const uint8_t *d_flags, const int64_t *d_rt_in,
                      const uint64_t *d_param_in, size_t n, const uint64_t *d_param_values, size_t n_values,
                      int8_t *d_decision, int32_t *d_wait, hipStream_t s);
    int device_status();  // sticky error of the device entry since the last call (host wait)
    int ensure_scratch();
    DevBuf<uint32_t> d_gate;  // [0] gate word of the running chunk, [1] sticky error bits
    int query(uint32_t resource, int64_t now, sga_node_view *out);
    int cb_state(uint32_t resource, uint32_t k);
    int metrics(int64_t now, sga_metric_node *out, size_t cap, size_t *n);
    int load_system_rules(const sga_system_rule *r, size_t n);
    SysDev sys{0, 0, 0, 0, 1.7976931348623157e308, 1.7976931348623157e308, 1.7976931348623157e308, INT64_MAX,
               INT64_MAX, -1.0, -1.0};
    DevBuf<sga_metric_node> d_metrics;
    DevBuf<uint32_t> d_mcount;
};

}  // namespace sga
