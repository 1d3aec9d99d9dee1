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
 *   sga_load_cluster_param_rules <- ClusterParamFlowRuleManager.loadRules(String, List<ParamFlowRule>)
 *                                CS/flow/rule/ClusterParamFlowRuleManager.java:270-276 (apply :318-368)
 *   sga_request_param_tokens  <- TokenService.requestParamToken(Long, int, Collection<Object>)
 *                                CORE/cluster/TokenService.java:46 ; DefaultTokenService.requestParamToken
 *                                CS/flow/DefaultTokenService.java:52-64
 *   sga_rls_should_rate_limit <- SentinelEnvoyRlsServiceImpl.shouldRateLimit -> SimpleClusterFlowChecker
 *                                RLS/SentinelEnvoyRlsServiceImpl.java:51-134, RLS/flow/SimpleClusterFlowChecker.java:33-65
 *   sga_submit_events         <- SphU.entry(String, EntryType, int, Object...) / Entry.exit(int, Object...)
 *                                CORE/SphU.java:84-208, CORE/Entry.java:86-111 through the slot chain
 *                                StatisticSlot (CORE/slots/statistic/StatisticSlot.java:64-187) ->
 *                                ParamFlowSlot (PF/slots/block/flow/param/ParamFlowSlot.java:34-93) ->
 *                                FlowSlot (CORE/slots/block/flow/FlowSlot.java:161-189) ->
 *                                DegradeSlot (CORE/slots/block/degrade/DegradeSlot.java:41-89)
 *   sga_load_flow_rules       <- FlowRuleManager.loadRules(List<FlowRule>)  CORE/slots/block/flow/FlowRuleManager.java:125-127
 *   sga_load_param_rules      <- ParamFlowRuleManager.loadRules(List<ParamFlowRule>)  PF/slots/block/flow/param/ParamFlowRuleManager.java:52
 *   sga_load_degrade_rules    <- DegradeRuleManager.loadRules(List<DegradeRule>)  CORE/slots/block/degrade/DegradeRuleManager.java:108
 *   sga_query_node            <- Node views (ClusterNode) CORE/node/Node.java:40-203, StatisticNode.java:185-250
 *   sga_metrics_snapshot      <- StatisticNode.metrics() as polled by MetricTimerListener.run
 *                                CORE/node/StatisticNode.java:120-157, CORE/node/metric/MetricTimerListener.java:44-65
 *   sga_cluster_metric_nodes* <- ClusterMetricNodeGenerator.flowToMetricNode
 *                                CS/flow/statistic/ClusterMetricNodeGenerator.java:75-91
 */
#ifndef SENTINEL_AMD_H
#define SENTINEL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGA_ABI_VERSION 3

/* error codes (negated errno values) */
#define SGA_OK 0
#define SGA_EINVAL (-22)
#define SGA_ENOMEM (-12)
#define SGA_EIO (-5)      /* HIP/device error; sga_last_error() has the text */
#define SGA_ENODEV (-19)  /* no usable gfx950 device */
#define SGA_ERANGE (-34)  /* batch larger than the configured capacity */
#define SGA_ENOSYS (-38)  /* feature not available on this build */
#define SGA_EAGAIN (-11)  /* sga_poll: the request is not decided yet */

/* TokenResultStatus codes, CORE/cluster/TokenResultStatus.java:27-60 */
#define SGA_TOKEN_BAD_REQUEST (-4)
#define SGA_TOKEN_TOO_MANY_REQUEST (-2)
#define SGA_TOKEN_FAIL (-1)
#define SGA_TOKEN_OK 0
#define SGA_TOKEN_BLOCKED 1
#define SGA_TOKEN_SHOULD_WAIT 2
#define SGA_TOKEN_NO_RULE_EXISTS 3
#define SGA_TOKEN_RELEASE_OK 6
#define SGA_TOKEN_ALREADY_RELEASE 7

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
    uint32_t max_param_keys;   /* cluster parameter flow: (rule, value) keys kept on the device
                                  (0 = 1M; at most 4M) */
    double exceed_count;       /* ServerFlowConfig.DEFAULT_EXCEED_COUNT (1.0), ServerFlowConfig.java:26 */
    double max_occupy_ratio;   /* ServerFlowConfig.DEFAULT_MAX_OCCUPY_RATIO (1.0), ServerFlowConfig.java:27 */
} sga_config;

/* Cluster flow rule = FlowRule{count, grade, strategy, clusterMode=true} +
 * ClusterFlowConfig{flowId, thresholdType, sampleCount, windowIntervalMs, resourceTimeout,
 * clientOfflineTime} (CORE/slots/block/flow/FlowRule.java:52-95,
 * CORE/slots/block/flow/ClusterFlowConfig.java:34-105). */
typedef struct sga_cluster_flow_rule {
    int64_t flow_id;
    double count;
    int32_t threshold_type;     /* ClusterRuleConstant: AVG_LOCAL = 0, GLOBAL = 1 */
    int32_t sample_count;       /* default 10 (ClusterRuleConstant.DEFAULT_CLUSTER_SAMPLE_COUNT) */
    int32_t window_interval_ms; /* default 1000 */
    int32_t grade;              /* RuleConstant.FLOW_GRADE_QPS = 1 (THREAD = 0: concurrency tokens) */
    int32_t strategy;           /* ClusterFlowConfig.strategy, NORMAL = 0 */
    int32_t reserved;
    int64_t resource_timeout_ms;     /* ClusterFlowConfig.resourceTimeout (default 2000) */
    int64_t client_offline_time_ms;  /* ClusterFlowConfig.clientOfflineTime (default 2000) */
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

/* Engine tuning, no reference counterpart (decisions never depend on it): the cluster token
 * path decides the requests of its hottest rules (at most 4096, each with at least `min_requests`
 * requests in the previous batch, one window length) in input order without sorting them: each
 * request's rank among its rule's requests comes from a per-segment count and a column prefix
 * (DESIGN.md section 3).  enabled = 0 sends every request through the radix sort.  Default:
 * enabled, min_requests 64. */
int sga_set_hot_rules(sga_engine *e, int32_t enabled, uint32_t min_requests);
/* Engine tuning (no reference counterpart): token batches of at most max_requests requests (capped
 * at 4096, 0 = off; default 4096) are classified and ordered by one workgroup instead of the
 * multi-launch sort pipeline -- the latency path of a single requestToken.  Decisions are the same
 * either way.  The same setting (capped at 1024) sends host chunks of local events (sga_submit_events,
 * the sga_event_* queue) of at most that many events, without inbound events under SystemRules, to one
 * replay kernel instead of the local pipeline. */
int sga_set_small_batch(sga_engine *e, uint32_t max_requests);

/* Batched DefaultTokenService.requestToken over host buffers; synchronous.
 * Requests are decided in array order as if issued one by one under a mocked
 * TimeUtil returning ts[i] (epoch ms).  Host-pinned or pageable buffers. */
int sga_request_tokens(sga_engine *e, const int64_t *flow_id, const int32_t *acquire, const uint8_t *prioritized,
                       const int64_t *ts, size_t n, sga_token_result *out);

/* Engine tuning (no reference counterpart): page-lock a long-lived host buffer of the caller (a front
 * end's request / result pool) for this engine's DMA.  sga_request_tokens batches of at least 2^20
 * requests whose arrays all lie in registered buffers are copied straight from / to them; other large
 * batches are staged through the engine's own page-locked slots by host threads.  Decisions are the
 * same either way.  Unregister before freeing the memory. */
int sga_host_register(sga_engine *e, void *ptr, size_t bytes);
int sga_host_unregister(sga_engine *e, void *ptr);

/* Coalescing queue for single requests.  TokenService.requestToken is called once per request from
 * many threads (FlowRequestProcessor.java:43 -> DefaultTokenService.requestToken,
 * CS/flow/DefaultTokenService.java:39-54); calling sga_request_tokens with n = 1 from each would
 * launch one pipeline per request.  sga_token_submit enqueues one request (lock-free, any thread)
 * and returns a ticket; sga_poll returns SGA_OK with its TokenResult once decided, SGA_EAGAIN before
 * (a poller that finds no batch running decides every queued request as one batch, so concurrent
 * callers share a launch); each ticket is polled to SGA_OK exactly once.  sga_request_token_one =
 * submit + poll until decided (the drop-in for a synchronous requestToken).  Decisions equal one
 * sga_request_tokens batch per request in ticket order.  A batch that fails answers
 * TokenResultStatus.FAIL (-1). */
int sga_token_submit(sga_engine *e, int64_t flow_id, int32_t acquire, uint8_t prioritized, int64_t ts,
                     uint64_t *ticket);
int sga_poll(sga_engine *e, uint64_t ticket, sga_token_result *out);
int sga_request_token_one(sga_engine *e, int64_t flow_id, int32_t acquire, uint8_t prioritized, int64_t ts,
                          sga_token_result *out);

/* Same over DEVICE buffers, asynchronous on `hip_stream` (NULL = engine stream).
 * Timestamps are ts_base + ts_off[i].  Inputs must stay valid until the stream
 * reaches the end of the call's work.  A caller stream first waits for all earlier engine work
 * and the engine stream then waits for the batch, so later engine calls (rule loads, other
 * batches on any stream) never overlap it. */
int sga_request_tokens_device(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                              const uint8_t *d_prioritized, int64_t ts_base, const uint32_t *d_ts_off, size_t n,
                              sga_token_result *d_out, void *hip_stream);

/* One token request in the packed 12-byte form (SURVEY.md 8(d) E_in: flowId u32, ts offset u32,
 * acquireCount u16, flags u16): what a front end that decodes Netty frames (FlowRequestData:
 * flowId, count, priority -- CS/server/codec/data/FlowRequestDataDecoder.java:35-48) into a device
 * batch writes, for engines whose flowIds fit 32 bits.  flow_id = 0 and acquire = 0 answer
 * BAD_REQUEST as flowId <= 0 / acquireCount <= 0 do (DefaultTokenService.notValidRequest, :87-89);
 * flags bit 0 = prioritized, the other bits are reserved: a request with any of them set answers
 * BAD_REQUEST. */
typedef struct sga_token_request {
    uint32_t flow_id;
    uint32_t ts_off;   /* time = ts_base + ts_off (ms) */
    uint16_t acquire;
    uint16_t flags;
} sga_token_request;
#define SGA_REQ_PRIORITIZED 1u

/* sga_request_tokens_device over packed requests (12 B each, 4-byte aligned): same decisions as the
 * unpacked entry on the same requests (DefaultTokenService.requestToken in arrival order,
 * CS/flow/DefaultTokenService.java:39-50); the hot path reads the records directly, every other path
 * unpacks them on the device first. */
int sga_request_tokens_packed_device(sga_engine *e, const sga_token_request *d_req, int64_t ts_base, size_t n,
                                     sga_token_result *d_out, void *hip_stream);

/* Round-1 name of sga_request_tokens_device (kept for its callers): the device entry already
 * returns once the batch is queued on the engine stream, and batches run in submission order. */
int sga_request_tokens_device_async(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                                    const uint8_t *d_prio, int64_t ts_base, const uint32_t *d_ts_off, size_t n,
                                    sga_token_result *d_out, void *hip_stream);
/* Pipelined form of sga_request_tokens_device for a stream of hot-path batches: the batch's classification
 * (key pass, count scans, sorts) starts once the inputs are ready on hip_stream, beside the previous batch's
 * decisions; decisions still run in submission order after every earlier engine call.  The outputs are
 * ready on hip_stream only after sga_stream_wait(e, hip_stream) (or sga_sync).  A batch the hot path does
 * not take runs as sga_request_tokens_device.  Same decisions as one sga_request_tokens_device per batch
 * (DefaultTokenService.requestToken in arrival order, CS/flow/DefaultTokenService.java:39-50). */
int sga_request_tokens_device_pipelined(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                                        const uint8_t *d_prioritized, int64_t ts_base, const uint32_t *d_ts_off,
                                        size_t n, sga_token_result *d_out, void *hip_stream);
/* Make `hip_stream` wait for every queued engine batch (no host wait). */
int sga_stream_wait(sga_engine *e, void *hip_stream);
/* Host wait for every queued batch. */
int sga_sync(sga_engine *e);

/* ClusterMetric.getSum(event) for every ClusterFlowEvent at virtual time `now`
 * (rotation side effects included, as in the reference). out[7]. */
int sga_cluster_metric_sums(sga_engine *e, int64_t flow_id, int64_t now, int64_t *out7);

/* Cluster parameter flow rule = ParamFlowRule{count, grade, paramIdx, burstCount, controlBehavior,
 * durationInSec, maxQueueingTimeMs, parsed hot items, clusterMode=true} + ParamFlowClusterConfig
 * {flowId, thresholdType, sampleCount, windowIntervalMs}
 * (PF/slots/block/flow/param/ParamFlowRule.java:45-83, ParamFlowClusterConfig.java:32-44).
 * Fields other than flow_id / count / threshold_type / window geometry / hot items only take part
 * in ParamFlowRuleUtil.isValidRule (PF/.../ParamFlowRuleUtil.java:46-70). */
typedef struct sga_cluster_param_rule {
    int64_t flow_id;
    double count;
    int32_t threshold_type;       /* AVG_LOCAL = 0 (ParamFlowClusterConfig default), GLOBAL = 1 */
    int32_t sample_count;         /* default 10 */
    int32_t window_interval_ms;   /* default 1000 */
    int32_t grade;                /* QPS = 1 */
    int32_t burst_count;          /* default 0 */
    int32_t control_behavior;     /* default 0 */
    int32_t max_queueing_time_ms; /* default 0 */
    int32_t param_idx_set;        /* paramIdx != null */
    int64_t duration_in_sec;      /* default 1 */
    int32_t n_hot;                /* parsed hot items (value -> count), later entries win */
    int32_t reserved;
    const int64_t *hot_values;
    const int32_t *hot_counts;
} sga_cluster_param_rule;

/* ClusterParamFlowRuleManager.loadRules(namespace, rules)  CS/flow/rule/ClusterParamFlowRuleManager.java:270-368:
 * invalid rules dropped, metrics of flowIds that stay are kept (geometry fixed at creation), metrics
 * of dropped flowIds removed.  Returns the number of rules applied or an error. */
int sga_load_cluster_param_rules(sga_engine *e, const char *ns, const sga_cluster_param_rule *rules, size_t n);

/* Batched DefaultTokenService.requestParamToken(flowId, acquireCount, params)
 * (CS/flow/DefaultTokenService.java:52-64 -> ClusterParamFlowChecker.acquireClusterToken):
 * request i carries the parameter values values[value_offsets[i] .. value_offsets[i+1]) (Java
 * Objects as 64-bit values: the caller maps each parameter to a stable int64, e.g. the long value
 * or a 64-bit hash of a String).  Decided in array order under a mocked clock ts[i].  Host buffers,
 * synchronous.  -ENOMEM when the device key store (sga_config.max_param_keys) is exhausted. */
int sga_request_param_tokens(sga_engine *e, const int64_t *flow_id, const int32_t *acquire,
                             const uint32_t *value_offsets, const int64_t *values, const int64_t *ts, size_t n,
                             sga_token_result *out);

/* Each bucket map's capacity of the ClusterParamMetrics created from now on (the maxCapacity argument of
 * ClusterParamMetric(sampleCount, intervalInMs, maxCapacity), ClusterParamMetric.java:44-49; 0 restores
 * DEFAULT_CLUSTER_MAX_CAPACITY = 4000).  Existing metrics keep theirs.  A map at capacity evicts its least
 * recently accessed value (getSum's get and addValue's putIfAbsent are accesses). */
int sga_cluster_set_param_capacity(sga_engine *e, uint32_t capacity);

/* ClusterParamMetric.getSum(value) of a flow at `now` (rotation side effect included; the gets are
 * accesses in LRU order). */
int sga_cluster_param_sum(sga_engine *e, int64_t flow_id, int64_t value, int64_t now, int64_t *out);

/* ClusterParamMetric.getTopValues(number) of a param flow at `now` (rotation side effect included):
 * up to `number` (1..1024) values with the largest sums over the valid buckets, as value keys and
 * qps = sum / intervalInSecond, largest first (equal sums: smaller value key first; the reference's
 * order among equal sums is its HashMap's).  *n_out = 0 when the flow has no metric. */
int sga_cluster_param_top_values(sga_engine *e, int64_t flow_id, int64_t now, uint32_t number, int64_t *values,
                                 double *qps, uint32_t *n_out);

/* Number of flow slots and device bytes of window state (for roofline tools). */
int sga_cluster_stats(sga_engine *e, uint64_t *n_active_rules, uint64_t *state_bytes);
/* Host-side event routing for a node of G engines (no reference
 * counterpart -- the reference runs one token server): order[] receives the request indices of a
 * global batch grouped by shard = splitmix64(flowId) mod G, arrival order kept inside a shard (a
 * stable counting sort); shard g's requests are order[shard_off[g] .. shard_off[g + 1]).
 * n_threads host threads (slices counted in parallel, one offset scan).  n < 2^32. */
int sga_route_shards(const int64_t *flow_id, size_t n, uint32_t n_shards, uint32_t n_threads, uint32_t *order,
                     uint64_t *shard_off);

/* Diagnostics of the last token batch (no reference counterpart): out[0] 1 when it ran the hot
 * path, [1] fallback flags, [2] sorted elements, [3] cold elements, [4] prioritized hot requests,
 * [5] hot rules for the next batch, [6..7] first / last hot bucket delta, [8] hot runs that
 * needed a replay (always 0), [9] in-segment bucket boundaries, [10] 1 when the device passed the
 * LDS lane-order probe the hot path's ranking relies on (else the hot path stays off).
 * Synchronous. */
int sga_cluster_batch_info(sga_engine *e, uint32_t *out, size_t n);

/* ---------------------------------------------------------------------------
 * Cluster concurrency tokens: TokenService.requestConcurrentToken / releaseConcurrentToken
 * (CORE/cluster/TokenService.java:58-73) -> DefaultTokenService.java:67-86 ->
 * ConcurrentClusterFlowChecker.java:37-104, TokenCacheNodeManager, CurrentConcurrencyManager,
 * RegularExpireStrategy.java:78-134 (CS = sentinel-cluster-server-default/.../cluster).
 * Client addresses are dense ids of a host table (SGA_CLIENT_NONE = null or "").
 * ------------------------------------------------------------------------- */
#define SGA_CONCURRENT_ACQUIRE 0
#define SGA_CONCURRENT_RELEASE 1
#define SGA_CLIENT_NONE 0xFFFFFFFFu

typedef struct sga_concurrent_result {
    int64_t token_id;  /* TokenResult.tokenId (acquire OK; 0 otherwise) */
    int32_t status;    /* TokenResultStatus: OK, BLOCKED, NO_RULE_EXISTS, BAD_REQUEST, RELEASE_OK,
                          ALREADY_RELEASE */
    int32_t reserved;
} sga_concurrent_result;

/* TokenCacheNode (TokenCacheNode.java:25-60); the timeouts are absolute, as the setters store them. */
typedef struct sga_token_cache_node {
    int64_t token_id;
    int64_t flow_id;
    int64_t client_timeout;    /* clientOfflineTime + creation time */
    int64_t resource_timeout;  /* resourceTimeout + creation time */
    int32_t acquire_count;
    uint32_t client;
} sga_token_cache_node;

/* A batch of acquire / release operations decided in arrival order.  op[i] = SGA_CONCURRENT_*;
 * acquire: id = flowId (ruleId), client[i], acquire[i], ts[i] = TimeUtil/System time of the call;
 * release: id = tokenId (client / acquire ignored).  Token ids are 64-bit values unique per engine
 * (the reference draws UUID.randomUUID().getMostSignificantBits()). */
int sga_concurrent_ops(sga_engine *e, const uint8_t *op, const uint32_t *client, const int64_t *id,
                       const int32_t *acquire, const int64_t *ts, size_t n, sga_concurrent_result *out);

/* One RegularExpireStrategy pass at `now` over every cached token.  online_bits: bit c set when
 * client c is connected (ConnectionManager.isClientOnline).  *n_removed = tokens removed. */
int sga_concurrent_expire(sga_engine *e, int64_t now, const uint32_t *online_bits, uint32_t n_clients,
                          uint64_t *n_removed);

/* CurrentConcurrencyManager.get(flowId): returns 1 and *now_calls when present, 0 when absent. */
int sga_concurrent_now_calls(sga_engine *e, int64_t flow_id, int32_t *now_calls);

/* TokenCacheNodeManager.getSize() */
int sga_concurrent_token_count(sga_engine *e, uint64_t *n);

/* TokenCacheNodeManager.getTokenCacheNode(tokenId): 1 and *out when cached, 0 when absent. */
int sga_concurrent_get_token(sga_engine *e, int64_t token_id, sga_token_cache_node *out);

/* Envoy RLS: SentinelEnvoyRlsServiceImpl.shouldRateLimit over a batch of
 * requests.  Each request has desc_count descriptors; descriptor d has flowId
 * d_flow_id (= Integer.MAX_VALUE + key.hashCode(), EnvoySentinelRuleConverter.java:67-72)
 * and hitsAddend.  Every descriptor consumes (no short-circuit).  code[r]:
 * 1 = OK, 2 = OVER_LIMIT (envoy RateLimitResponse.Code), -1 = hitsAddend < 0 (onError).
 * Optional per-descriptor outputs: desc_status = the TokenResult status of
 * SimpleClusterFlowChecker.acquireClusterToken (NO_RULE_EXISTS for an absent rule -- the
 * descriptor's Code is then OK and it carries no current_limit, :65-83) and desc_remaining =
 * TokenResult.remaining (DescriptorStatus.limit_remaining). */
int sga_rls_should_rate_limit(sga_engine *e, const uint32_t *desc_offsets, size_t n_requests,
                              const int64_t *desc_flow_id, const int32_t *hits_addend, const int64_t *ts,
                              int8_t *desc_status, int32_t *desc_remaining, int32_t *code);
/* The same over DEVICE buffers, asynchronous on `hip_stream` with the stream ordering of
 * sga_request_tokens_device: desc_offsets[n_requests + 1] (offsets[n_requests] = n_descriptors
 * <= max_batch), request times ts_base + ts_off[r].  d_desc_status / d_desc_remaining may be NULL. */
int sga_rls_should_rate_limit_device(sga_engine *e, const uint32_t *d_desc_offsets, size_t n_requests,
                                     size_t n_descriptors, const int64_t *d_desc_flow_id,
                                     const int32_t *d_hits_addend, int64_t ts_base, const uint32_t *d_ts_off,
                                     int8_t *d_desc_status, int32_t *d_desc_remaining, int32_t *d_code,
                                     void *hip_stream);

/* ---------------------------------------------------------------------------
 * Local path: resources are dense ids 0..n_resources-1 (the host keeps the
 * name table, like CtSph's chain map keys).  One ClusterNode per resource
 * (single default context, limitApp "default", strategy DIRECT).
 * ------------------------------------------------------------------------- */

/* Coalescing queue of single local events (SphU.entry / Entry.exit from many application threads, one
 * synchronous call each: CtSph.entryWithPriority, CORE/CtSph.java:117-168).  sga_event_submit enqueues one
 * event (lock-free, any thread; kind, flags, param as in sga_submit_events_ex, param_values holding this
 * event's argument words only, at most 64 of them -- SGA_ERANGE otherwise) and returns a ticket;
 * sga_event_poll returns SGA_OK with its decision and wait once decided, SGA_EAGAIN before (a poller that
 * finds no batch running decides every queued event as ONE batch, so concurrent callers share a launch);
 * each ticket is polled to SGA_OK exactly once.  Decisions equal one sga_submit_events_ex call per event in
 * ticket order.  A batch that fails answers decision -1 and SGA_EIO.  sga_event_one = submit + poll until
 * decided (an event with more argument words than a slot holds is decided on its own). */
int sga_event_submit(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                     int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, uint64_t *ticket);
int sga_event_poll(sga_engine *e, uint64_t ticket, int8_t *decision, int32_t *wait_ms);
int sga_event_one(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                  int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, int8_t *decision,
                  int32_t *wait_ms);
/* An event whose caller needs no decision -- Entry.exit, a block counted by a slot before the engine, a revoke
 * (kinds 1-3; an entry is refused with SGA_EINVAL) -- queued like sga_event_submit and returned at once: nobody
 * polls its ticket (written to *ticket when not NULL, ~0 for an event decided on its own), the combining round
 * that decides it frees its slot.  Ticket order holds: it is decided before every event this thread queues later,
 * and every other call on the engine (batches, queries, snapshots, rule loads) first waits for the events queued
 * before it.  A round that failed holding posted events makes the next sga_event_post return SGA_EIO. */
int sga_event_post(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                   int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, uint64_t *ticket);

/* decision codes of sga_submit_events.  wait_ms of an entry: the sleep of a pass (RateLimiter pacing,
 * SHOULD_WAIT, parameter throttle) or of SGA_PASS_WAIT; for a block, the block detail the exception
 * carries: SGA_BLOCK_FLOW the blocking FlowRule's index in the resource's rules (FlowRuleComparator
 * order), SGA_BLOCK_PARAM the ParamFlowRule's index (list order), SGA_BLOCK_DEGRADE the breaker's
 * index (DegradeRuleManager list order), SGA_BLOCK_SYSTEM the SystemRule check (SystemBlockException
 * limitType: 0 qps, 1 thread, 2 rt, 3 load, 4 cpu). */
#define SGA_PASS 0
#define SGA_BLOCK_FLOW 1     /* FlowException */
#define SGA_BLOCK_PARAM 2    /* ParamFlowException */
#define SGA_BLOCK_DEGRADE 3  /* DegradeException */
#define SGA_PASS_WAIT 4      /* PriorityWaitException: passed after wait_ms, not counted as pass */
#define SGA_BLOCK_SYSTEM 5   /* SystemBlockException (SystemSlot, inbound entries only) */

/* event kinds: 0 entry, 1 exit of a passed entry, 2 an entry blocked by a slot outside the engine
 * (AuthoritySlot or a custom slot ahead of the checks): StatisticSlot's BlockException branch only --
 * increaseBlockQps on the node and, inbound, on ENTRY_NODE (StatisticSlot.java:121-135).  Kind 2 events
 * report SGA_PASS and are decided in arrival order by one lane. */
#define SGA_KIND_ENTRY 0
#define SGA_KIND_EXIT 1
#define SGA_KIND_BLOCKED 2
/* kind 3: an entry the engine passed (decision SGA_PASS) that a slot after the engine's checks then blocked
 * (a custom slot sorted after DegradeSlot).  In the reference StatisticSlot fires those slots before its pass
 * accounting (StatisticSlot.java:71-84), so such an entry only counts a block: the revoke undoes the entry's
 * pass, thread count and parameter thread counts and counts the block (node and, inbound, ENTRY_NODE), at the
 * entry's time, with the entry's flags and arguments.  Decided in arrival order by one lane; reports SGA_PASS. */
#define SGA_KIND_REVOKE 3

/* event flags */
#define SGA_EV_PRIORITIZED 1u
#define SGA_EV_ERROR 2u      /* exit of an entry that recorded a business error (Tracer.traceEntry) */
#define SGA_EV_HAS_PARAM 4u  /* args[0] present (param field) */
#define SGA_EV_INBOUND 8u    /* EntryType.IN (on entries and their exits): Constants.ENTRY_NODE + SystemSlot */
#define SGA_EV_PARAM_LIST 16u /* with HAS_PARAM: args[0] is a Collection / array; param = offset << 32 | count
                               * into sga_submit_events_ex's param_values (every element is checked,
                               * ParamFlowChecker.passLocalCheck, and counted by ParameterMetric) */
#define SGA_EV_ARGS 32u       /* the event's whole argument vector (SphU.entry(..., Object... args)):
                               * param = offset << 32 | nargs into param_values, two words per argument:
                               * param_values[offset + 2k] = kind << 62 | list length, param_values[offset
                               * + 2k + 1] = the argument's 64-bit key (SGA_ARG_SCALAR) or the offset of its
                               * elements in param_values (SGA_ARG_LIST: a Collection / array); SGA_ARG_NULL
                               * is a null argument.  HAS_PARAM / PARAM_LIST are ignored on such events.
                               * Chunks holding them are decided in arrival order by one lane. */
#define SGA_ARG_SCALAR 0u
#define SGA_ARG_NULL 1u
#define SGA_ARG_LIST 2u

/* resource id of Constants.ENTRY_NODE ("__total_inbound_traffic__") in sga_query_node and metric rows */
#define SGA_ENTRY_NODE 0xFFFFFFFFu

/* FlowRule, CORE/slots/block/flow/FlowRule.java:52-95 (limitApp default, strategy DIRECT) */
typedef struct sga_flow_rule {
    uint32_t resource;
    int32_t grade;                 /* FLOW_GRADE_THREAD 0 / QPS 1 */
    double count;
    int32_t control_behavior;      /* 0 default, 1 warm up, 2 rate limiter, 3 warm up + rate limiter */
    int32_t warm_up_period_sec;    /* default 10 */
    int32_t max_queueing_time_ms;  /* default 500 */
    int32_t strategy;              /* STRATEGY_DIRECT 0 only */
    /* FlowRule.clusterMode (FlowRuleChecker.passClusterCheck, FlowRuleChecker.java:168-230): the
     * rule asks the token service; with the embedded server (sga_set_cluster_server) that is this
     * engine's cluster rules (sga_load_cluster_flow_rules, keyed by flowId) */
    int32_t cluster_mode;
    int32_t cluster_fallback;      /* ClusterFlowConfig.fallbackToLocalWhenFail (default 1) */
    int64_t cluster_flow_id;       /* ClusterFlowConfig.flowId (> 0 for a valid cluster rule) */
    int32_t cluster_sample_count;  /* ClusterFlowConfig.sampleCount / windowIntervalMs / strategy: */
    int32_t cluster_window_ms;     /*   validity only (FlowRuleUtil.checkClusterField) */
    int32_t cluster_strategy;
    int32_t reserved;
} sga_flow_rule;

/* ParamFlowRule, PF/slots/block/flow/param/ParamFlowRule.java:45-83 */
typedef struct sga_param_rule {
    uint32_t resource;
    int32_t grade;                 /* QPS 1 / THREAD 0 */
    double count;
    int32_t control_behavior;      /* 0 token bucket, 2 throttle (RATE_LIMITER) */
    int32_t max_queueing_time_ms;  /* default 0 */
    int32_t burst_count;           /* default 0 */
    int32_t param_idx;             /* args index; negative counts from the end, fixed on the rule at its first
                                    * check (ParamFlowSlot.applyRealParamIdx, ParamFlowSlot.java:56-66);
                                    * -64 <= param_idx < 64 */
    int64_t duration_in_sec;       /* default 1 */
    uint32_t n_hot;                /* parsed hot items: value -> threshold */
    uint32_t reserved;
    const uint64_t *hot_values;
    const int32_t *hot_thresholds;
    /* ParamFlowRule.clusterMode + ParamFlowClusterConfig (ParamFlowClusterConfig.java:32-44): with the
     * embedded token server on (sga_set_cluster_server 1) a QPS rule asks this engine's cluster parameter
     * path (TokenService.requestParamToken -> ClusterParamFlowChecker) in event order: OK passes,
     * BLOCKED blocks, anything else falls back (ParamFlowChecker.passClusterCheck, :305-343) */
    int32_t cluster_mode;
    int32_t cluster_fallback;      /* fallbackToLocalWhenFail, default 0 */
    int64_t cluster_flow_id;
    int32_t cluster_sample_count;  /* validity only (ParamFlowRuleUtil.checkCluster): default 10 */
    int32_t cluster_window_ms;     /* default 1000 */
} sga_param_rule;

/* DegradeRule, CORE/slots/block/degrade/DegradeRule.java:59-84 */
typedef struct sga_degrade_rule {
    uint32_t resource;
    int32_t grade;                 /* RT 0, EXCEPTION_RATIO 1, EXCEPTION_COUNT 2 */
    double count;
    int32_t time_window;           /* seconds */
    int32_t min_request_amount;    /* default 5 */
    double slow_ratio_threshold;   /* default 1.0 */
    int32_t stat_interval_ms;      /* default 1000 */
    int32_t reserved;
} sga_degrade_rule;

/* Node view at virtual time `now` (StatisticNode getters; reads rotate windows like the reference). */
typedef struct sga_node_view {
    double pass_qps, block_qps, success_qps, exception_qps, occupied_pass_qps;
    double avg_rt, min_rt, previous_pass_qps;
    int64_t total_pass, total_block, total_success, total_exception;  /* minute window */
    int64_t cur_thread_num;
    int64_t waiting;                                                /* borrowed (occupied) tokens */
    double max_success_qps;     /* StatisticNode.maxSuccessQps (StatisticNode.java:225-230): max bucket success
                                 * of the second window (>= 1) x sampleCount / intervalInSec */
    double previous_block_qps;  /* StatisticNode.previousBlockQps (StatisticNode.java:180-182): the minute
                                 * window's previous bucket's block count */
} sga_node_view;

int sga_flow_set_resources(sga_engine *e, uint32_t n_resources);
int sga_load_flow_rules(sga_engine *e, const sga_flow_rule *rules, size_t n);
/* ClusterStateManager for the local path's cluster-mode FlowRules (FlowRuleChecker.pickClusterService):
 * 0 = neither client nor server (cluster-mode rules fall back: fallbackToLocalOrPass), 1 = embedded
 * token server -- the rule's flowId is decided by this engine's cluster path in event order
 * (DefaultTokenService.requestToken, then applyTokenResult: OK pass, SHOULD_WAIT pass after waitInMs,
 * BLOCKED block, NO_RULE_EXISTS / BAD_REQUEST / FAIL / TOO_MANY_REQUEST fall back).  A cluster
 * flowId must belong to one resource's rules, and its namespace must have no GlobalRequestLimiter
 * (-ENOSYS otherwise). */
int sga_set_cluster_server(sga_engine *e, int32_t mode);
int sga_load_param_rules(sga_engine *e, const sga_param_rule *rules, size_t n);
int sga_load_degrade_rules(sga_engine *e, const sga_degrade_rule *rules, size_t n);

/* A time-ordered stream of entries (kind 0) and exits of passed entries (kind 1),
 * decided as if SphU.entry / Entry.exit were called one by one under a mocked
 * TimeUtil returning ts[i].  acquire = batchCount; rt[i] = exit - entry time
 * (exits); param[i] = args[0] when SGA_EV_HAS_PARAM.  decision[i] / wait_ms[i]
 * for entries (exits report SGA_PASS).  Host buffers, synchronous. */
int sga_submit_events(sga_engine *e, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                      const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                      size_t n, int8_t *decision, int32_t *wait_ms);
/* sga_submit_events with Collection / array arguments: events flagged SGA_EV_PARAM_LIST take their
 * values from param_values[param >> 32 .. (param >> 32) + (param & 0xffffffff)). */
int sga_submit_events_ex(sga_engine *e, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                         const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                         size_t n, const uint64_t *param_values, size_t n_values, int8_t *decision,
                         int32_t *wait_ms);
/* sga_submit_events_ex over DEVICE buffers, asynchronous on `hip_stream` (NULL = engine stream), with
 * the stream ordering of sga_request_tokens_device.  One chunk: n <= max_batch.  Timestamps are
 * ts_base + ts_off[i]; d_flags, d_rt, d_param, d_param_values and d_wait_ms may be NULL (zeros /
 * not written).  The checks the host entry makes by scanning the events (SystemSlot or Collection
 * arguments -> arrival-order replay, inbound statistics, acquire >= 0, value ranges inside
 * param_values) run on the device; a chunk that fails them is not applied and answers -1 for
 * every event.  sga_events_device_status waits for the engine stream and reports SGA_EINVAL for
 * such a chunk or SGA_ENOMEM when a parameter map filled, since its last call. */
int sga_submit_events_device(sga_engine *e, const uint8_t *d_kind, const uint32_t *d_resource, int64_t ts_base,
                             const uint32_t *d_ts_off, const int32_t *d_acquire, const uint8_t *d_flags,
                             const int64_t *d_rt, const uint64_t *d_param, size_t n, const uint64_t *d_param_values,
                             size_t n_values, int8_t *d_decision, int32_t *d_wait_ms, void *hip_stream);
int sga_events_device_status(sga_engine *e);
int sga_query_node(sga_engine *e, uint32_t resource, int64_t now, sga_node_view *out);

/* SystemRule (CORE/slots/system/SystemRule.java:43-50); negative = not set. */
typedef struct sga_system_rule {
    double highest_system_load;
    double highest_cpu_usage;  /* > 1 is ignored as invalid */
    double qps;
    int64_t avg_rt;
    int64_t max_thread;
} sga_system_rule;

/* SystemRuleManager.loadRules (SystemPropertyListener.configUpdate + loadSystemConf,
 * SystemRuleManager.java:191-300): the minimum of every field over the rules; the check is on
 * when the LAST rule sets any field (the reference sets the switch per rule); an empty list turns
 * it off.  While on, inbound entries (SGA_EV_INBOUND) pass SystemRuleManager.checkSystem against
 * ENTRY_NODE before the other slots -- a global order dependency: such batches are decided by
 * one sequential lane (exact).  Returns the number of rules that set a field. */
int sga_load_system_rules(sga_engine *e, const sga_system_rule *rules, size_t n);

/* SystemStatusListener readings (system load average, CPU usage 0..1; -1 = not measured yet). */
int sga_set_system_status(sga_engine *e, double avg_load, double cpu_usage);
/* circuit breaker k of a resource: 0 CLOSED, 1 OPEN, 2 HALF_OPEN (negative = no such breaker) */
int sga_circuit_breaker_state(sga_engine *e, uint32_t resource, uint32_t k);

/* ---------------------------------------------------------------------------
 * Once-per-second metrics
 * ------------------------------------------------------------------------- */

/* MetricNode, CORE/node/metric/MetricNode.java:28-51 (thin-format fields); resource = dense id */
typedef struct sga_metric_node {
    int64_t timestamp;        /* second-window start (minute LeapArray bucket) */
    int64_t pass_qps, block_qps, success_qps, exception_qps;
    int64_t rt;               /* rt sum / success (ArrayMetric.fromBucket, :203-218) */
    int64_t occupied_pass_qps;
    uint32_t resource;
    int32_t concurrency;      /* not filled by StatisticNode.metrics() (0) */
} sga_metric_node;

/* StatisticNode.metrics() of every resource's ClusterNode at `now` (CORE/node/StatisticNode.java:120-157):
 * minute buckets with lastFetchTime < start < now - now % 1000 and a non-zero field, each node's
 * lastFetchTime advanced as in the reference.  Up to `cap` nodes; *n = number written (the order
 * between resources is unspecified, like the reference's ClusterNode map).  -ERANGE if more than
 * `cap` nodes were due (the first `cap` are written, lastFetchTime still advanced). */
int sga_metrics_snapshot(sga_engine *e, int64_t now, sga_metric_node *out, size_t cap, size_t *n);

/* ClusterMetricNodeGenerator.flowToMetricNode for every active cluster flow rule
 * (CS/flow/statistic/ClusterMetricNodeGenerator.java:75-91): passQps / blockQps =
 * ClusterMetric.getAvg(PASS / BLOCK) at `now` (rotation side effect included). */
typedef struct sga_cluster_metric_node {
    int64_t flow_id;
    double pass_qps;
    double block_qps;
    int64_t timestamp;
} sga_cluster_metric_node;

int sga_cluster_metric_nodes(sga_engine *e, int64_t now, sga_cluster_metric_node *out, size_t cap, size_t *n);
/* Same into DEVICE memory on `hip_stream` (NULL = engine stream), count into *d_n (uint32, device):
 * the input of the once-per-second RCCL all-gather across the node's GPUs. */
int sga_cluster_metric_nodes_device(sga_engine *e, int64_t now, sga_cluster_metric_node *d_out, size_t cap,
                                    uint32_t *d_n, void *hip_stream);

/* Optional helper for tools: HIP stream of the engine (hipStream_t as void*). */
void *sga_engine_stream(sga_engine *e);

#ifdef __cplusplus
}
#endif
#endif
