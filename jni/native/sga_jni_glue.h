/* Plain-C glue between the JNI entry points (sentinel_amd_jni.c) and the engine's C ABI
 * (include/sentinel_amd.h).  No JNI types: the JNI layer only converts Java arrays / direct
 * buffers to pointers and calls these, so this half compiles and links without a JDK
 * (tests/test_jni_glue.py). */
#ifndef SGA_JNI_GLUE_H
#define SGA_JNI_GLUE_H

#include <stddef.h>
#include <stdint.h>

#include "sentinel_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GpuEngine.create: one engine per device (DefaultTokenService / the slot chain share it). */
int sgaj_create(int32_t device, uint32_t max_batch, uint32_t max_rules, sga_engine **out);

/* ClusterFlowRuleManager.loadRules(namespace, rules) (ClusterFlowRuleManager.java:254-260): the
 * cluster-mode FlowRules of a namespace as parallel arrays (flowId, count, thresholdType,
 * sampleCount, windowIntervalMs); other fields take the reference defaults. */
int sgaj_load_cluster_flow_rules(sga_engine *e, const char *ns, const int64_t *flow_id, const double *count,
                                 const int32_t *threshold_type, const int32_t *sample_count,
                                 const int32_t *window_interval_ms, size_t n);

/* TokenService.requestToken (TokenService.java:36): out3 = {status, remaining, waitInMs}. */
int sgaj_request_token(sga_engine *e, int64_t flow_id, int32_t acquire, int32_t prioritized, int64_t now_ms,
                       int32_t out3[3]);
/* Asynchronous form: submit returns a ticket, poll answers 0 with out3 filled or SGA_EAGAIN. */
int sgaj_submit(sga_engine *e, int64_t flow_id, int32_t acquire, int32_t prioritized, int64_t now_ms,
                uint64_t *ticket);
int sgaj_poll(sga_engine *e, uint64_t ticket, int32_t out3[3]);

/* TokenService.requestParamToken (TokenService.java:46): params already mapped to 64-bit keys
 * (Integer/Long as the value, String by a stable 64-bit hash on the Java side). */
int sgaj_request_param_token(sga_engine *e, int64_t flow_id, int32_t acquire, const int64_t *values,
                             uint32_t n_values, int64_t now_ms, int32_t out3[3]);

/* TokenService.requestConcurrentToken / releaseConcurrentToken (TokenService.java:55-61):
 * op 0 acquire (id = ruleId) / 1 release (id = tokenId); out = {status, tokenId}. */
int sgaj_concurrent(sga_engine *e, int32_t op, uint32_t client, int64_t id, int32_t acquire, int64_t now_ms,
                    int64_t out2[2]);

/* ProcessorSlot.entry / exit of GpuStatisticSlot (ProcessorSlot.java:41-76): one event through the
 * local slot chain.  entry: dec_wait = {decision (0 pass, 1 FlowException, 2 ParamFlowException,
 * 3 DegradeException, 4 PriorityWaitException, 5 SystemBlockException), waitMs}. */
int sgaj_entry(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, uint64_t param,
               int32_t dec_wait[2]);
int sgaj_exit(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, int64_t rt_ms,
              uint64_t param);

/* SphU.entry / Entry.exit with the whole `Object... args` vector (SGA_EV_ARGS): words = the argument
 * pairs and list elements as include/sentinel_amd.h lays them out (offset 0), nwords their count. */
int sgaj_entry_args(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags,
                    const uint64_t *words, uint32_t nargs, uint32_t nwords, int32_t dec_wait[2]);
int sgaj_exit_args(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, int64_t rt_ms,
                   const uint64_t *words, uint32_t nargs, uint32_t nwords);
/* StatisticSlot's BlockException branch for a block thrown by a slot outside the engine (AuthoritySlot):
 * event kind SGA_KIND_BLOCKED. */
int sgaj_blocked(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags);
/* a passed entry that a slot after the engine's checks blocked (SGA_KIND_REVOKE): the entry's time, flags, args */
int sgaj_revoke_args(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags,
                     const uint64_t *words, uint32_t nargs, uint32_t nwords);

/* ParamFlowRuleManager.loadRules (ParamFlowRuleManager.java:52): parallel arrays; rule i's hot items are
 * hot_values / hot_counts [hot_off[i], hot_off[i + 1]); cluster_* may be NULL (local rules). */
int sgaj_load_param_rules(sga_engine *e, size_t n, const uint32_t *resource, const int32_t *grade,
                          const double *count, const int32_t *behavior, const int32_t *max_queue,
                          const int32_t *burst, const int32_t *param_idx, const int64_t *duration_sec,
                          const uint32_t *hot_off, const int64_t *hot_values, const int32_t *hot_counts,
                          const int32_t *cluster_mode, const int32_t *cluster_fallback,
                          const int64_t *cluster_flow_id, const int32_t *cluster_sample_count,
                          const int32_t *cluster_window_ms);
/* DegradeRuleManager.loadRules (DegradeRuleManager.java:108). */
int sgaj_load_degrade_rules(sga_engine *e, size_t n, const uint32_t *resource, const int32_t *grade,
                            const double *count, const int32_t *time_window, const int32_t *min_request,
                            const double *slow_ratio, const int32_t *stat_interval_ms);
/* SystemRuleManager.loadRules (SystemRuleManager.java:114) and SystemStatusListener readings. */
int sgaj_load_system_rules(sga_engine *e, size_t n, const double *load, const double *cpu, const double *qps,
                           const int64_t *avg_rt, const int64_t *max_thread);
int sgaj_set_system_status(sga_engine *e, double avg_load, double cpu_usage);
/* ClusterParamFlowRuleManager.loadRules(namespace, rules) (ClusterParamFlowRuleManager.java:270-276). */
int sgaj_load_cluster_param_rules(sga_engine *e, const char *ns, size_t n, const int64_t *flow_id,
                                  const double *count, const int32_t *threshold_type, const int32_t *sample_count,
                                  const int32_t *window_ms, const uint32_t *hot_off, const int64_t *hot_values,
                                  const int32_t *hot_counts);
/* ConnectionManager connected count of a namespace (AVG_LOCAL thresholds) and GlobalRequestLimiter. */
int sgaj_set_connected_count(sga_engine *e, const char *ns, int32_t connected);
int sgaj_set_namespace_limit(sga_engine *e, const char *ns, double max_qps);
/* ClusterStateManager: 1 embedded token server (cluster-mode rules decided by this engine), 0 none. */
int sgaj_set_cluster_server(sga_engine *e, int32_t mode);
/* Node getters (Node.java:40-203) of a resource's ClusterNode at now_ms (reads rotate windows):
 * d10 = {passQps, blockQps, successQps, exceptionQps, occupiedPassQps, avgRt, minRt, previousPassQps,
 *        maxSuccessQps, previousBlockQps},
 * l6 = {totalPass, totalBlock, totalSuccess, totalException, curThreadNum, waiting}. */
int sgaj_query_node(sga_engine *e, uint32_t resource, int64_t now_ms, double d10[10], int64_t l6[6]);
/* StatisticNode.metrics() of every resource (MetricTimerListener.run's input): up to cap rows of 8
 * longs {timestamp, resource, pass, block, success, exception, rt, occupiedPass}; *n rows written. */
int sgaj_metrics_snapshot(sga_engine *e, int64_t now_ms, int64_t *rows8, size_t cap, size_t *n);

#ifdef __cplusplus
}
#endif
#endif
