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

#ifdef __cplusplus
}
#endif
#endif
