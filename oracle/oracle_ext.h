/*
 * ORACLE / TEST INFRASTRUCTURE ONLY (see sentinel_oracle.h).
 * Hot-parameter flow control (PF module) and DegradeSlot circuit breakers,
 * plugged into the local flow engine (orc_flow) in the reference's slot order:
 *   StatisticSlot -> ParamFlowSlot(-3000) -> FlowSlot(-2000) -> DegradeSlot(-1000)
 * (CORE/Constants.java:76-83, PF/slots/block/flow/param/ParamFlowSlot.java:34-93).
 *
 * Engine-level restriction: an entry carries at most one parameter value
 * (args[0], a 64-bit key); rules with paramIdx 0 (or -1) see it, other indexes see
 * "args.length <= paramIdx" and pass (ParamFlowChecker.java:55-58).
 * Parameter maps never evict: identical to the reference while each rule's
 * ConcurrentLinkedHashMap stays below min(4000*durationInSec, 200000) keys
 * (ParameterMetric.java:37-39,99,108); above that the reference's eviction order
 * is unspecified (parity unpinned).
 */
#ifndef SENTINEL_ORACLE_EXT_H
#define SENTINEL_ORACLE_EXT_H
#include "sentinel_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_param_rule {
    uint32_t resource;
    int32_t grade;              /* FLOW_GRADE_QPS (1) / THREAD (0) */
    double count;
    int32_t control_behavior;   /* 0 default token bucket, 2 RATE_LIMITER (throttle) */
    int32_t max_queueing_time_ms;
    int32_t burst_count;
    int32_t param_idx;
    int64_t duration_in_sec;
    uint32_t n_hot;             /* parsed hot items (ParamFlowRuleUtil.parseHotItems) */
    const uint64_t *hot_values;
    const int32_t *hot_thresholds;
    /* ParamFlowRule.clusterMode + ParamFlowClusterConfig (ParamFlowClusterConfig.java:32-44) */
    int32_t cluster_mode;
    int32_t cluster_fallback;   /* fallbackToLocalWhenFail, default false */
    int64_t cluster_flow_id;
    int32_t cluster_sample_count;
    int32_t cluster_window_ms;
} orc_param_rule;

typedef struct orc_degrade_rule {
    uint32_t resource;
    int32_t grade;              /* DEGRADE_GRADE_RT 0, EXCEPTION_RATIO 1, EXCEPTION_COUNT 2 */
    double count;
    int32_t time_window;        /* seconds */
    int32_t min_request_amount; /* default 5 */
    double slow_ratio_threshold;/* default 1.0 */
    int32_t stat_interval_ms;   /* default 1000 */
} orc_degrade_rule;

/* ParamFlowRuleManager.loadRules / DegradeRuleManager.loadRules on the engine. */
int orc_flow_load_param_rules(orc_flow *f, const orc_param_rule *rules, size_t n);
int orc_flow_load_degrade_rules(orc_flow *f, const orc_degrade_rule *rules, size_t n);

/* SphU.entry(resource, IN/OUT, acquire, args...) with an optional single
 * parameter.  Returns ORC_PASS / ORC_BLOCK_PARAM / ORC_BLOCK_FLOW /
 * ORC_BLOCK_DEGRADE / ORC_PASS_WAIT. */
int orc_flow_entry_p(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int has_param,
                     uint64_t param, int64_t *wait_ms);
/* Entry.exit of a passed entry: stats, param thread counts, circuit breakers. */
void orc_flow_exit_p(orc_flow *f, uint32_t resource, int64_t now, int64_t rt, int count, int error, int has_param,
                     uint64_t param);
/* Argument vectors (SGA_EV_ARGS): events flagged 32 carry args[0 .. nargs) as word pairs in pvals:
 * param = offset << 32 | nargs; pair k = pvals[offset + 2k] (kind << 62 | list length: kind 0 scalar,
 * 1 null, 2 Collection / array) and pvals[offset + 2k + 1] (the scalar's key, or the offset of the
 * list's elements in pvals).  Flags bit 4 (PARAM_LIST) keeps its round-2 meaning for args[0]. */
void orc_flow_replay_args(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                          const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                          const uint64_t *pvals, int8_t *decision, int32_t *wait_ms);
/* the resolved parameter index of resource r's k-th parameter rule (ParamFlowSlot.applyRealParamIdx sets it
 * on the rule at its first check), or INT32_MIN while unresolved */
int32_t orc_flow_param_idx(const orc_flow *f, uint32_t r, int k);
/* circuit breaker state of the k-th breaker of a resource: 0 CLOSED, 1 OPEN, 2 HALF_OPEN */
int orc_flow_cb_state(orc_flow *f, uint32_t resource, int k);

/* Batch replay with parameters: kind 0 entry / 1 exit; flags bit0 prioritized,
 * bit1 error (exit), bit2 has_param. */
/* SystemRule fields (CORE/slots/system/SystemRule.java:43-50); negative = not set */
typedef struct orc_system_rule {
    double highest_system_load;
    double highest_cpu_usage;
    double qps;
    int64_t avg_rt;
    int64_t max_thread;
} orc_system_rule;
int orc_flow_load_system_rules(orc_flow *f, const orc_system_rule *rules, size_t n);
void orc_flow_set_system_status(orc_flow *f, double avg_load, double cpu_usage);
int orc_flow_entry_x(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int has_param,
                     uint64_t param, int inbound, int64_t *wait_ms);
void orc_flow_exit_x(orc_flow *f, uint32_t resource, int64_t now, int64_t rt, int count, int error, int has_param,
                     uint64_t param, int inbound);
orc_node *orc_flow_entry_node(orc_flow *f);

void orc_flow_replay_p(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                       const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                       int8_t *decision, int32_t *wait_ms);
/* flags bit 4: args[0] is a Collection / array (pvals[param >> 32 ..], param & 0xffffffff values) */
void orc_flow_replay_pl(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                        const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                        const uint64_t *pvals, int8_t *decision, int32_t *wait_ms);

/* Standalone ParamFlowChecker.passSingleValueCheck on one rule (KATs): the rule's
 * maps persist in the handle. */
typedef struct orc_prule orc_prule;
orc_prule *orc_prule_new(const orc_param_rule *r);
void orc_prule_free(orc_prule *p);
/* LRU CacheMap introspection (tests): which 0 = time map, 1 = token map, 2 = the resource's thread map */
size_t orc_prule_map_size(const orc_prule *p, int which);
uint64_t orc_prule_map_evictions(const orc_prule *p, int which);
size_t orc_prule_map_keys(const orc_prule *p, int which, uint64_t *keys, int64_t *vals, size_t cap);
size_t orc_flow_param_map_size(const orc_flow *f, uint32_t r, int k, int which);
int orc_prule_pass_single(orc_prule *p, uint64_t value, int acquire, int64_t now, int64_t thread_count,
                          int64_t *wait_ms);

#ifdef __cplusplus
}
#endif
#endif
