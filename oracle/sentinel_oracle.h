/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- "parity oracle" for the MI355X
 * admission engine.  A single-threaded C restatement of the reference's
 * statistics-and-decision hot path (Alibaba Sentinel 1.8.4-SNAPSHOT, the
 * Gepeng18/Sentinel fork) under a mocked TimeUtil clock: every call takes the
 * virtual time `now` (ms) that TimeUtil.currentTimeMillis() would return.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker.  The product (sentinel_amd/)
 * never links or calls it.
 *
 * Path aliases (relative to the reference root):
 *   CORE = sentinel-core/src/main/java/com/alibaba/csp/sentinel
 *   PF   = sentinel-extension/sentinel-parameter-flow-control/src/main/java/com/alibaba/csp/sentinel
 *   CS   = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster
 *   RLS  = sentinel-cluster/sentinel-cluster-server-envoy-rls/src/main/java/com/alibaba/csp/sentinel/cluster/server/envoy/rls
 *
 * Parity pinning: the restatement is checked against the known-answer tests
 * transcribed from the reference's JUnit suites (the JSON fixtures under tests/golden/, see
 * tests/golden/README.md); Java could not be run in this container (no JDK).
 */
#ifndef SENTINEL_ORACLE_H
#define SENTINEL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- leap arrays (CORE/slots/statistic/base/LeapArray.java) ---------------- */
enum orc_leap_kind {
    ORC_LEAP_BUCKET = 0,     /* BucketLeapArray            CORE/slots/statistic/metric/BucketLeapArray.java */
    ORC_LEAP_OCCUPIABLE = 1, /* OccupiableBucketLeapArray  CORE/slots/statistic/metric/occupy/OccupiableBucketLeapArray.java */
    ORC_LEAP_FUTURE = 2,     /* FutureBucketLeapArray      CORE/slots/statistic/metric/occupy/FutureBucketLeapArray.java */
    ORC_LEAP_CLUSTER = 3,    /* ClusterMetricLeapArray     CS/flow/statistic/metric/ClusterMetricLeapArray.java */
    ORC_LEAP_UNARY = 4       /* UnaryLeapArray (LongAdder) CORE/slots/statistic/base/UnaryLeapArray.java */
};

/* MetricEvent ordinals (CORE/slots/statistic/MetricEvent.java:21-39) */
enum { ORC_EV_PASS = 0, ORC_EV_BLOCK, ORC_EV_EXCEPTION, ORC_EV_SUCCESS, ORC_EV_RT, ORC_EV_OCCUPIED_PASS };
/* ClusterFlowEvent ordinals (CS/flow/statistic/data/ClusterFlowEvent.java:22-52) */
enum { ORC_CEV_PASS = 0, ORC_CEV_BLOCK, ORC_CEV_PASS_REQUEST, ORC_CEV_BLOCK_REQUEST, ORC_CEV_OCCUPIED_PASS,
       ORC_CEV_OCCUPIED_BLOCK, ORC_CEV_WAITING };

typedef struct orc_leap orc_leap;

orc_leap *orc_leap_new(int kind, int sample_count, int interval_ms);
void orc_leap_free(orc_leap *l);
/* currentWindow(t): returns window start or INT64_MIN when t < 0 (null). */
int64_t orc_leap_current_window(orc_leap *l, int64_t t);
/* currentWindow(t).value().add(ev, n) */
void orc_leap_add(orc_leap *l, int64_t t, int ev, int64_t n);
void orc_leap_add_rt(orc_leap *l, int64_t t, int64_t rt);
/* counter of the bucket that currentWindow(t) returns */
int64_t orc_leap_current_get(orc_leap *l, int64_t t, int ev);
/* values(t): sum of ev over valid buckets; *count receives the list size */
int64_t orc_leap_values_sum(orc_leap *l, int64_t t, int ev, int *count);
/* getPreviousWindow(t) evaluated at mocked clock `now`; returns 1 if non-null */
int orc_leap_previous_window(orc_leap *l, int64_t t, int64_t now, int64_t *start, int64_t *pass);
/* getValidHead(now); returns 1 if non-null */
int orc_leap_valid_head(orc_leap *l, int64_t now, int64_t *start, int64_t *pass);
/* occupiable only */
void orc_leap_add_waiting(orc_leap *l, int64_t t, int n);
int64_t orc_leap_current_waiting(orc_leap *l, int64_t now);
/* getWindowValue(t).pass() or -1 when null */
int64_t orc_leap_window_value_pass(orc_leap *l, int64_t t);

/* ---- StatisticNode (CORE/node/StatisticNode.java) --------------------------- */
typedef struct orc_node orc_node;
orc_node *orc_node_new(void);
void orc_node_free(orc_node *n);
double orc_node_pass_qps(orc_node *n, int64_t now);
double orc_node_block_qps(orc_node *n, int64_t now);
double orc_node_success_qps(orc_node *n, int64_t now);
double orc_node_exception_qps(orc_node *n, int64_t now);
double orc_node_previous_pass_qps(orc_node *n, int64_t now);
double orc_node_avg_rt(orc_node *n, int64_t now);
double orc_node_min_rt(orc_node *n, int64_t now);
double orc_node_occupied_pass_qps(orc_node *n, int64_t now);
int64_t orc_node_total_pass(orc_node *n, int64_t now);
int64_t orc_node_total_block(orc_node *n, int64_t now);
int64_t orc_node_total_success(orc_node *n, int64_t now);
int64_t orc_node_total_exception(orc_node *n, int64_t now);
int32_t orc_node_cur_thread_num(orc_node *n);
int64_t orc_node_waiting(orc_node *n, int64_t now);
void orc_node_add_pass_request(orc_node *n, int64_t now, int count);
void orc_node_add_rt_and_success(orc_node *n, int64_t now, int64_t rt, int count);
void orc_node_increase_block_qps(orc_node *n, int64_t now, int count);
void orc_node_increase_exception_qps(orc_node *n, int64_t now, int count);
void orc_node_increase_thread_num(orc_node *n);
void orc_node_decrease_thread_num(orc_node *n);
int64_t orc_node_try_occupy_next(orc_node *n, int64_t now, int acquire, double threshold);
void orc_node_add_waiting_request(orc_node *n, int64_t future_time, int acquire);
void orc_node_add_occupied_pass(orc_node *n, int64_t now, int acquire);
/* Mock node: passQps/previousPassQps/curThreadNum stubbed (Mockito in the JUnit tests). */
orc_node *orc_node_new_mock(double pass_qps, double previous_pass_qps, int32_t threads);
void orc_node_set_mock(orc_node *n, double pass_qps, double previous_pass_qps, int32_t threads);

/* ---- traffic shaping controllers (CORE/slots/block/flow/controller) ------ */
enum { ORC_CTRL_DEFAULT = 0, ORC_CTRL_WARM_UP = 1, ORC_CTRL_RATE_LIMITER = 2, ORC_CTRL_WARM_UP_RATE_LIMITER = 3 };
enum { ORC_GRADE_THREAD = 0, ORC_GRADE_QPS = 1 };
/* decision codes shared with include/sentinel_amd.h */
enum { ORC_PASS = 0, ORC_BLOCK_FLOW = 1, ORC_BLOCK_PARAM = 2, ORC_BLOCK_DEGRADE = 3, ORC_PASS_WAIT = 4,
       ORC_BLOCK_SYSTEM = 5 };

typedef struct orc_ctrl orc_ctrl;
orc_ctrl *orc_ctrl_new(int behavior, int grade, double count, int warm_up_period_sec, int max_queueing_time_ms,
                       int cold_factor);
void orc_ctrl_free(orc_ctrl *c);
/* rater.canPass(node, acquire, prioritized) at mocked time `now`.  Returns an
 * ORC_* decision; *wait_ms receives the sleep the reference would perform. */
int orc_ctrl_can_pass(orc_ctrl *c, orc_node *node, int64_t now, int acquire, int prioritized, int64_t *wait_ms);
/* state peeks for parity tests */
int64_t orc_ctrl_latest_passed_time(const orc_ctrl *c);
int64_t orc_ctrl_stored_tokens(const orc_ctrl *c);
int64_t orc_ctrl_last_filled_time(const orc_ctrl *c);
int32_t orc_ctrl_warning_token(const orc_ctrl *c);
int32_t orc_ctrl_max_token(const orc_ctrl *c);
double orc_ctrl_slope(const orc_ctrl *c);

/* ---- local flow engine: StatisticSlot + FlowSlot replay (one default ctx) -- */
typedef struct orc_flow_rule {
    uint32_t resource;     /* dense resource id (the engine's name table is host side) */
    int32_t grade;         /* RuleConstant.FLOW_GRADE_* */
    double count;
    int32_t control_behavior;
    int32_t warm_up_period_sec;
    int32_t max_queueing_time_ms;
    int32_t strategy;      /* only DIRECT(0) is supported by the engine */
    /* FlowRule.clusterMode + ClusterFlowConfig (FlowRuleChecker.passClusterCheck, :168-230) */
    int32_t cluster_mode;
    int32_t cluster_fallback;      /* fallbackToLocalWhenFail */
    int64_t cluster_flow_id;
    int32_t cluster_sample_count;  /* validity only (FlowRuleUtil.checkClusterField) */
    int32_t cluster_window_ms;
    int32_t cluster_strategy;
    int32_t reserved;
} orc_flow_rule;

typedef struct orc_flow orc_flow;
orc_flow *orc_flow_new(uint32_t n_resources, int cold_factor);
void orc_flow_free(orc_flow *f);
/* FlowRuleManager.loadRules: validity filter, rater regenerated (controller
 * state reset), node statistics kept.  Returns #valid rules. */
int orc_flow_load_rules(orc_flow *f, const orc_flow_rule *rules, size_t n);
/* ClusterStateManager for cluster-mode rules (FlowRuleChecker.pickClusterService): mode 0 = neither
 * client nor server (fallbackToLocalOrPass), 1 = embedded token server `server` (its
 * DefaultTokenService decides the rule's flowId). */
typedef struct orc_cluster orc_cluster;
void orc_flow_set_cluster(orc_flow *f, orc_cluster *server, int mode);
/* SphU.entry(resource, type, acquire) -> decision (ORC_*), wait ms */
int orc_flow_entry(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int64_t *wait_ms);
/* Entry.exit for a PASSED entry: rt = now - createTimestamp supplied by caller */
void orc_flow_exit(orc_flow *f, uint32_t resource, int64_t now, int64_t rt, int count, int error);
orc_node *orc_flow_node(orc_flow *f, uint32_t resource);
/* batch replay: events in order; kind 0 = entry, 1 = exit */
void orc_flow_replay(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                     const int32_t *acquire, const uint8_t *flags, const int64_t *rt, int8_t *decision,
                     int32_t *wait_ms);

/* MetricNode (CORE/node/metric/MetricNode.java:28-51), same layout as sga_metric_node */
typedef struct orc_metric_node {
    int64_t timestamp;
    int64_t pass_qps, block_qps, success_qps, exception_qps, rt, occupied_pass_qps;
    uint32_t resource;
    int32_t concurrency;
} orc_metric_node;
/* StatisticNode.metrics(): returns the number of due nodes (writes up to cap) */
size_t orc_node_metrics(orc_node *n, int64_t now, uint32_t resource, orc_metric_node *out, size_t cap);
size_t orc_flow_metrics(orc_flow *f, int64_t now, orc_metric_node *out, size_t cap);
#define ORC_ENTRY_NODE 0xFFFFFFFFu /* resource id of Constants.ENTRY_NODE in metric rows and node queries */
double orc_node_max_success_qps(orc_node *n, int64_t now);
double orc_node_previous_block_qps(orc_node *n, int64_t now);

/* ---- cluster token server (CS/flow) ---------------------------------------- */
typedef struct orc_cluster_rule {
    int64_t flow_id;
    double count;
    int32_t threshold_type; /* ClusterRuleConstant.FLOW_THRESHOLD_AVG_LOCAL=0 / GLOBAL=1 */
    int32_t sample_count;   /* ClusterFlowConfig.sampleCount (default 10) */
    int32_t window_interval_ms;
    int32_t grade;          /* must be QPS for token requests */
    int32_t strategy;       /* ClusterFlowConfig.strategy (NORMAL=0) */
    int32_t reserved;
    int64_t resource_timeout_ms;    /* ClusterFlowConfig.resourceTimeout (2000) */
    int64_t client_offline_time_ms; /* ClusterFlowConfig.clientOfflineTime (2000) */
} orc_cluster_rule;

typedef struct orc_token_result {
    int32_t status;     /* TokenResultStatus */
    int32_t remaining;
    int32_t wait_in_ms;
} orc_token_result;

typedef struct orc_cluster orc_cluster;
orc_cluster *orc_cluster_new(double exceed_count, double max_occupy_ratio);
void orc_cluster_free(orc_cluster *c);
/* ClusterFlowRuleManager.loadRules(namespace, rules); returns #applied */
int orc_cluster_load_rules(orc_cluster *c, const char *ns, const orc_cluster_rule *rules, size_t n);
/* ClusterServerConfigManager namespace QPS limiter (GlobalRequestLimiter.initIfAbsent) */
void orc_cluster_set_namespace_limit(orc_cluster *c, const char *ns, double max_allowed_qps);
void orc_cluster_set_connected_count(orc_cluster *c, const char *ns, int32_t n);
/* DefaultTokenService.requestToken(flowId, acquire, prioritized) at `now` */
orc_token_result orc_cluster_request_token(orc_cluster *c, int64_t flow_id, int32_t acquire, int prioritized,
                                           int64_t now);
/* SimpleClusterFlowChecker (Envoy RLS) on the same metric store */
orc_token_result orc_cluster_request_token_simple(orc_cluster *c, int64_t flow_id, int32_t acquire, int64_t now);
void orc_cluster_replay(orc_cluster *c, size_t n, const int64_t *flow_id, const int32_t *acquire,
                        const uint8_t *prio, const int64_t *ts, orc_token_result *out);
/* SimpleClusterFlowChecker per descriptor, in order (Envoy RLS front end). */
void orc_cluster_replay_simple(orc_cluster *c, size_t n, const int64_t *flow_id, const int32_t *acquire,
                               const int64_t *ts, orc_token_result *out);
/* sum of a ClusterFlowEvent over valid buckets of flow's metric at now (ClusterMetric.getSum) */
int64_t orc_cluster_metric_sum(orc_cluster *c, int64_t flow_id, int ev, int64_t now);
/* standalone ClusterMetric (CS/flow/statistic/metric/ClusterMetric.java) for KATs */
typedef struct orc_cmetric orc_cmetric;
orc_cmetric *orc_cmetric_new(int sample_count, int interval_ms);
void orc_cmetric_free(orc_cmetric *m);
void orc_cmetric_add(orc_cmetric *m, int64_t now, int ev, int64_t n);
int64_t orc_cmetric_sum(orc_cmetric *m, int64_t now, int ev);
double orc_cmetric_avg(orc_cmetric *m, int64_t now, int ev);
int32_t orc_cmetric_try_occupy_next(orc_cmetric *m, int64_t now, int ev, int32_t acquire, double threshold);
/* RequestLimiter (CS/flow/statistic/limit/RequestLimiter.java) */
typedef struct orc_limiter orc_limiter;
orc_limiter *orc_limiter_new(double qps_allowed);
void orc_limiter_free(orc_limiter *l);
void orc_limiter_add(orc_limiter *l, int64_t now, int x);
int64_t orc_limiter_sum(orc_limiter *l, int64_t now);
double orc_limiter_qps(orc_limiter *l, int64_t now);
int orc_limiter_can_pass(orc_limiter *l, int64_t now);
int orc_limiter_try_pass(orc_limiter *l, int64_t now);

/* ---- cluster parameter flow (CS/flow/ClusterParamFlowChecker) ---------------- */
typedef struct orc_cparam_rule {
    int64_t flow_id;            /* ParamFlowClusterConfig.flowId */
    double count;
    int32_t threshold_type;     /* AVG_LOCAL = 0 (default), GLOBAL = 1 */
    int32_t sample_count;       /* default 10 */
    int32_t window_interval_ms; /* default 1000 */
    int32_t grade;              /* ParamFlowRuleUtil.isValidRule fields */
    int32_t burst_count;
    int32_t control_behavior;
    int32_t max_queueing_time_ms;
    int32_t param_idx_set;      /* paramIdx != null */
    int64_t duration_in_sec;
    int32_t n_hot;              /* parsed hot items value -> count */
    int32_t reserved;
    const int64_t *hot_values;
    const int32_t *hot_counts;
} orc_cparam_rule;

/* ClusterParamFlowRuleManager.loadRules(namespace, rules); returns #applied */
int orc_cluster_load_param_rules(orc_cluster *c, const char *ns, const orc_cparam_rule *rules, size_t n);
/* per-bucket CacheMap capacity of the ClusterParamMetrics created afterwards (default 4000; tests) */
void orc_cluster_set_param_capacity(size_t cap);
/* DefaultTokenService.requestParamToken(flowId, acquire, values) at `now` */
orc_token_result orc_cluster_request_param_token(orc_cluster *c, int64_t flow_id, int32_t acquire,
                                                 const int64_t *values, size_t nvalues, int64_t now);
void orc_cluster_param_replay(orc_cluster *c, size_t n, const int64_t *flow_id, const int32_t *acquire,
                              const uint32_t *value_offsets, const int64_t *values, const int64_t *ts,
                              orc_token_result *out);
/* standalone ClusterParamMetric (CS/flow/statistic/metric/ClusterParamMetric.java:41-88) for KATs */
typedef struct orc_pmetric orc_pmetric;
orc_pmetric *orc_pmetric_new(int sample_count, int interval_ms);
void orc_pmetric_free(orc_pmetric *m);
void orc_pmetric_add(orc_pmetric *m, int64_t now, int64_t value, int32_t count);
int64_t orc_pmetric_sum(orc_pmetric *m, int64_t now, int64_t value);
double orc_pmetric_avg(orc_pmetric *m, int64_t now, int64_t value);
/* ClusterParamMetric.getSum(value) at now; -1 when the flow has no metric */
int64_t orc_cluster_param_sum(orc_cluster *c, int64_t flow_id, int64_t value, int64_t now);

/* ClusterParamMetric.getTopValues(number) at now; returns the values written */
size_t orc_cluster_param_top_values(orc_cluster *c, int64_t flow_id, int64_t now, size_t number, int64_t *vals,
                                    double *qps);

/* ---- cluster concurrency tokens (oracle_conc.c) ----------------------------- */
#define ORC_CLIENT_NONE 0xFFFFFFFFu
typedef struct orc_conc_result {
    int32_t status;   /* TokenResultStatus */
    int32_t reserved;
    int64_t token_id; /* TokenResult.tokenId when OK */
} orc_conc_result;
orc_conc_result orc_cluster_concurrent_acquire(orc_cluster *c, uint32_t client, int64_t flow_id, int32_t acquire,
                                               int64_t now, int64_t token_id);
int32_t orc_cluster_concurrent_release(orc_cluster *c, int64_t token_id);
uint64_t orc_cluster_concurrent_expire(orc_cluster *c, int64_t now, const uint32_t *online_bits, uint32_t nclients);
int orc_cluster_concurrent_now_calls(orc_cluster *c, int64_t flow_id, int32_t *out);
size_t orc_cluster_concurrent_tokens(orc_cluster *c);
int orc_cluster_concurrent_get(orc_cluster *c, int64_t token_id, int64_t *flow_id, int64_t *client_deadline,
                               int64_t *resource_deadline, int32_t *acquire);

/* ---- Java numerics exposed for tests ---------------------------------------- */
int64_t orc_java_round(double d);
double orc_java_next_up(double d);
int32_t orc_java_d2i(double d);
int64_t orc_java_d2l(double d);
int32_t orc_java_string_hash(const char *utf8);

#ifdef __cplusplus
}
#endif
#endif
