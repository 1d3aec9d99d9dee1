/*
 * sentinel_amd.h -- C-ABI of the MI355X-native admission engine for Sentinel's
 * statistics-and-decision hot path.  Drop-in boundary: these are the calls a
 * JNI shim (GpuTokenService / GpuStatisticSlot / rule-manager hooks, see
 * INTEGRATION.md) binds.  Plain pointers and sizes only; every function
 * returns 0 or a negative errno-style code; no exception crosses the ABI.
 *
 * Reference interfaces replaced (paths relative to the reference root; aliases
 * CORE / CS / RLS as in SURVEY.md):
 *   sga_request_tokens*       <- TokenService.requestToken(Long, int, boolean)
 *                                CORE/cluster/TokenService.java:36 ;
 *                                DefaultTokenService.requestToken CS/flow/DefaultTokenService.java:39-50
 *   sga_load_cluster_flow_rules <- ClusterFlowRuleManager.loadRules(String, List<FlowRule>)
 *                                CS/flow/rule/ClusterFlowRuleManager.java:254-260 (apply :310-364)
 *   sga_set_namespace_limit   <- GlobalRequestLimiter.initIfAbsent / applyMaxQpsChange
 *                                CS/flow/statistic/limit/GlobalRequestLimiter.java:32-80
 *   sga_set_connected_count   <- ConnectionManager.getConnectedCount (AVG_LOCAL thresholds)
 *                                CS/flow/rule/ClusterFlowRuleManager.java:333-343
 *   sga_cluster_metric_sums   <- ClusterMetric.getSum(ClusterFlowEvent)  CS/flow/statistic/metric/ClusterMetric.java:53-62
 *   sga_rls_check_descriptors <- SentinelEnvoyRlsServiceImpl.checkToken -> SimpleClusterFlowChecker
 *                                RLS/SentinelEnvoyRlsServiceImpl.java:116-125, RLS/flow/SimpleClusterFlowChecker.java:33-65
 */
#ifndef SENTINEL_AMD_H
#define SENTINEL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGA_ABI_VERSION 1

/* error codes (negated errno values) */
#define SGA_OK 0
#define SGA_EINVAL (-22)
#define SGA_ENOMEM (-12)
#define SGA_EIO (-5)      /* HIP/device error; sga_last_error() has the text */
#define SGA_ENODEV (-19)  /* no usable gfx950 device */
#define SGA_ERANGE (-34)  /* batch larger than the configured capacity */
#define SGA_ENOSYS (-38)  /* feature not available on this build */

/* TokenResultStatus codes, CORE/cluster/TokenResultStatus.java:27-60 */
#define SGA_TOKEN_BAD_REQUEST (-4)
#define SGA_TOKEN_TOO_MANY_REQUEST (-2)
#define SGA_TOKEN_FAIL (-1)
#define SGA_TOKEN_OK 0
#define SGA_TOKEN_BLOCKED 1
#define SGA_TOKEN_SHOULD_WAIT 2
#define SGA_TOKEN_NO_RULE_EXISTS 3

/* ClusterFlowEvent ordinals, CS/flow/statistic/data/ClusterFlowEvent.java:22-52 */
#define SGA_CEV_PASS 0
#define SGA_CEV_BLOCK 1
#define SGA_CEV_PASS_REQUEST 2
#define SGA_CEV_BLOCK_REQUEST 3
#define SGA_CEV_OCCUPIED_PASS 4
#define SGA_CEV_OCCUPIED_BLOCK 5
#define SGA_CEV_WAITING 6

typedef struct sga_engine sga_engine;

typedef struct sga_config {
    int32_t device;            /* HIP device ordinal */
    uint32_t max_batch;        /* events per submit (device scratch is sized for it) */
    uint32_t max_rules;        /* initial rule-slot capacity (grows on load) */
    int32_t cold_factor;       /* csp.sentinel.flow.cold.factor, SentinelConfig.java:68 (3) */
    int32_t statistic_max_rt;  /* csp.sentinel.statistic.max.rt, SentinelConfig.java:69 (5000) */
    int32_t reserved0;
    double exceed_count;       /* ServerFlowConfig.DEFAULT_EXCEED_COUNT (1.0), ServerFlowConfig.java:26 */
    double max_occupy_ratio;   /* ServerFlowConfig.DEFAULT_MAX_OCCUPY_RATIO (1.0), ServerFlowConfig.java:27 */
} sga_config;

/* Cluster flow rule = FlowRule{count, grade, strategy, clusterMode=true} +
 * ClusterFlowConfig{flowId, thresholdType, sampleCount, windowIntervalMs}
 * (CORE/slots/block/flow/FlowRule.java:52-95, CORE/slots/block/flow/ClusterFlowConfig.java:34-74). */
typedef struct sga_cluster_flow_rule {
    int64_t flow_id;
    double count;
    int32_t threshold_type;     /* ClusterRuleConstant: AVG_LOCAL = 0, GLOBAL = 1 */
    int32_t sample_count;       /* default 10 (ClusterRuleConstant.DEFAULT_CLUSTER_SAMPLE_COUNT) */
    int32_t window_interval_ms; /* default 1000 */
    int32_t grade;              /* RuleConstant.FLOW_GRADE_QPS = 1 */
    int32_t strategy;           /* ClusterFlowConfig.strategy, NORMAL = 0 */
    int32_t reserved;
} sga_cluster_flow_rule;

/* TokenResult as the engine writes it: 8 bytes per decision.
 * (CORE/cluster/TokenResult.java: status, remaining, waitInMs) */
typedef struct sga_token_result {
    int32_t remaining;
    int16_t wait_in_ms;
    int8_t status;
    int8_t reserved;
} sga_token_result;

void sga_config_default(sga_config *cfg);
int sga_create(const sga_config *cfg, sga_engine **out);
int sga_destroy(sga_engine *e);
const char *sga_last_error(const sga_engine *e);
int sga_abi_version(void);

/* ClusterFlowRuleManager.loadRules(namespace, rules): invalid rules dropped
 * (FlowRuleUtil.isValidRule), metrics of flowIds that stay are kept, metrics of
 * dropped flowIds removed, new flowIds get a fresh ClusterMetric. Returns the
 * number of rules applied (>= 0) or an error. */
int sga_load_cluster_flow_rules(sga_engine *e, const char *ns, const sga_cluster_flow_rule *rules, size_t n);
int sga_set_namespace_limit(sga_engine *e, const char *ns, double max_allowed_qps);
int sga_set_connected_count(sga_engine *e, const char *ns, int32_t connected);

/* Batched DefaultTokenService.requestToken over host buffers; synchronous.
 * Requests are decided in array order as if issued one by one under a mocked
 * TimeUtil returning ts[i] (epoch ms).  Host-pinned or pageable buffers. */
int sga_request_tokens(sga_engine *e, const int64_t *flow_id, const int32_t *acquire, const uint8_t *prioritized,
                       const int64_t *ts, size_t n, sga_token_result *out);

/* Same over DEVICE buffers, asynchronous on `hip_stream` (NULL = engine stream).
 * Timestamps are ts_base + ts_off[i].  Inputs must stay valid until the stream
 * reaches the end of the call's work. */
int sga_request_tokens_device(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                              const uint8_t *d_prioritized, int64_t ts_base, const uint32_t *d_ts_off, size_t n,
                              sga_token_result *d_out, void *hip_stream);

/* ClusterMetric.getSum(event) for every ClusterFlowEvent at virtual time `now`
 * (rotation side effects included, as in the reference). out[7]. */
int sga_cluster_metric_sums(sga_engine *e, int64_t flow_id, int64_t now, int64_t *out7);

/* Number of flow slots and device bytes of window state (for roofline tools). */
int sga_cluster_stats(sga_engine *e, uint64_t *n_active_rules, uint64_t *state_bytes);

/* Envoy RLS: SentinelEnvoyRlsServiceImpl.shouldRateLimit over a batch of
 * requests.  Each request has desc_count descriptors; descriptor d has flowId
 * d_flow_id (= Integer.MAX_VALUE + key.hashCode(), EnvoySentinelRuleConverter.java:67-72)
 * and hitsAddend.  Every descriptor consumes (no short-circuit).  code[r]:
 * 1 = OK, 2 = OVER_LIMIT (envoy RateLimitResponse.Code); per-descriptor status
 * in desc_status (TokenResultStatus). */
int sga_rls_should_rate_limit(sga_engine *e, const uint32_t *desc_offsets, size_t n_requests,
                              const int64_t *desc_flow_id, const int32_t *hits_addend, const int64_t *ts,
                              int8_t *desc_status, int32_t *code);

/* Optional helper for tools: HIP stream of the engine (hipStream_t as void*). */
void *sga_engine_stream(sga_engine *e);

#ifdef __cplusplus
}
#endif
#endif
