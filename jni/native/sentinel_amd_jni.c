/* JNI entry points of com.alibaba.csp.sentinel.gpu.GpuEngine (the native methods the Java shim
 * declares).  Each converts Java arrays / strings to plain pointers and calls the C glue
 * (sga_jni_glue.c), which calls the engine's C ABI.  Build with the JDK's include directories:
 *   cc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude -Ijni/native \
 *      jni/native/sentinel_amd_jni.c jni/native/sga_jni_glue.c -Lsentinel_amd -lsentinel_amd \
 *      -o libsentinel_amd_jni.so */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "sga_jni_glue.h"

#define ENGINE(h) ((sga_engine *)(intptr_t)(h))

JNIEXPORT jlong JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_create(JNIEnv *env, jclass cls, jint device,
                                                                          jint max_batch, jint max_rules) {
    (void)env;
    (void)cls;
    sga_engine *e = NULL;
    const int rc = sgaj_create(device, (uint32_t)max_batch, (uint32_t)max_rules, &e);
    return rc == SGA_OK ? (jlong)(intptr_t)e : (jlong)rc;  /* a negative value is the error code */
}

JNIEXPORT void JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_destroy(JNIEnv *env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    sga_destroy(ENGINE(h));
}

JNIEXPORT jstring JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_lastError(JNIEnv *env, jclass cls, jlong h) {
    (void)cls;
    const char *m = sga_last_error(ENGINE(h));
    return (*env)->NewStringUTF(env, m ? m : "");
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_loadClusterFlowRules(
    JNIEnv *env, jclass cls, jlong h, jstring ns, jlongArray flow_ids, jdoubleArray counts, jintArray threshold_types,
    jintArray sample_counts, jintArray window_ms) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, flow_ids);
    const char *nss = (*env)->GetStringUTFChars(env, ns, NULL);
    jlong *f = (*env)->GetLongArrayElements(env, flow_ids, NULL);
    jdouble *c = (*env)->GetDoubleArrayElements(env, counts, NULL);
    jint *tt = (*env)->GetIntArrayElements(env, threshold_types, NULL);
    jint *sc = (*env)->GetIntArrayElements(env, sample_counts, NULL);
    jint *w = (*env)->GetIntArrayElements(env, window_ms, NULL);
    const int rc = sgaj_load_cluster_flow_rules(ENGINE(h), nss, (const int64_t *)f, (const double *)c,
                                                (const int32_t *)tt, (const int32_t *)sc, (const int32_t *)w,
                                                (size_t)n);
    (*env)->ReleaseIntArrayElements(env, window_ms, w, JNI_ABORT);
    (*env)->ReleaseIntArrayElements(env, sample_counts, sc, JNI_ABORT);
    (*env)->ReleaseIntArrayElements(env, threshold_types, tt, JNI_ABORT);
    (*env)->ReleaseDoubleArrayElements(env, counts, c, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, flow_ids, f, JNI_ABORT);
    (*env)->ReleaseStringUTFChars(env, ns, nss);
    return rc;
}

/* requestToken: out = int[3] {status, remaining, waitInMs} */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_requestToken(JNIEnv *env, jclass cls, jlong h,
                                                                               jlong flow_id, jint acquire,
                                                                               jboolean prioritized, jlong now_ms,
                                                                               jintArray out) {
    (void)cls;
    int32_t o[3] = {0, 0, 0};
    const int rc = sgaj_request_token(ENGINE(h), flow_id, acquire, prioritized ? 1 : 0, now_ms, o);
    if (rc == SGA_OK) (*env)->SetIntArrayRegion(env, out, 0, 3, (const jint *)o);
    return rc;
}

JNIEXPORT jlong JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_submit(JNIEnv *env, jclass cls, jlong h,
                                                                          jlong flow_id, jint acquire,
                                                                          jboolean prioritized, jlong now_ms) {
    (void)env;
    (void)cls;
    uint64_t t = 0;
    const int rc = sgaj_submit(ENGINE(h), flow_id, acquire, prioritized ? 1 : 0, now_ms, &t);
    return rc == SGA_OK ? (jlong)t : (jlong)rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_poll(JNIEnv *env, jclass cls, jlong h,
                                                                       jlong ticket, jintArray out) {
    (void)cls;
    int32_t o[3] = {0, 0, 0};
    const int rc = sgaj_poll(ENGINE(h), (uint64_t)ticket, o);
    if (rc == SGA_OK) (*env)->SetIntArrayRegion(env, out, 0, 3, (const jint *)o);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_requestParamToken(JNIEnv *env, jclass cls,
                                                                                    jlong h, jlong flow_id,
                                                                                    jint acquire, jlongArray values,
                                                                                    jlong now_ms, jintArray out) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, values);
    jlong *v = (*env)->GetLongArrayElements(env, values, NULL);
    int32_t o[3] = {0, 0, 0};
    const int rc = sgaj_request_param_token(ENGINE(h), flow_id, acquire, (const int64_t *)v, (uint32_t)n, now_ms, o);
    (*env)->ReleaseLongArrayElements(env, values, v, JNI_ABORT);
    if (rc == SGA_OK) (*env)->SetIntArrayRegion(env, out, 0, 3, (const jint *)o);
    return rc;
}

/* requestConcurrentToken (op 0, id = ruleId) / releaseConcurrentToken (op 1, id = tokenId):
 * out = long[2] {status, tokenId} */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_concurrent(JNIEnv *env, jclass cls, jlong h,
                                                                             jint op, jint client, jlong id,
                                                                             jint acquire, jlong now_ms,
                                                                             jlongArray out) {
    (void)cls;
    int64_t o[2] = {0, 0};
    const int rc = sgaj_concurrent(ENGINE(h), op, (uint32_t)client, id, acquire, now_ms, o);
    if (rc == SGA_OK) (*env)->SetLongArrayRegion(env, out, 0, 2, (const jlong *)o);
    return rc;
}

/* GpuStatisticSlot.entry: out = int[2] {decision, waitMs} */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_entry(JNIEnv *env, jclass cls, jlong h,
                                                                        jint resource, jlong now_ms, jint count,
                                                                        jint flags, jlong param, jintArray out) {
    (void)cls;
    int32_t o[2] = {0, 0};
    const int rc = sgaj_entry(ENGINE(h), (uint32_t)resource, now_ms, count, (uint32_t)flags, (uint64_t)param, o);
    if (rc == SGA_OK) (*env)->SetIntArrayRegion(env, out, 0, 2, (const jint *)o);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_exit(JNIEnv *env, jclass cls, jlong h,
                                                                       jint resource, jlong now_ms, jint count,
                                                                       jint flags, jlong rt_ms, jlong param) {
    (void)env;
    (void)cls;
    return sgaj_exit(ENGINE(h), (uint32_t)resource, now_ms, count, (uint32_t)flags, rt_ms, (uint64_t)param);
}

/* SlotChain resources: resource names are mapped to dense ids on the Java side (like CtSph's chain
 * map); the engine is told how many exist. */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_setResources(JNIEnv *env, jclass cls, jlong h,
                                                                               jint n) {
    (void)env;
    (void)cls;
    return sga_flow_set_resources(ENGINE(h), (uint32_t)n);
}

/* FlowRuleManager.loadRules forwarded as packed sga_flow_rule records (direct ByteBuffer). */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_loadFlowRules(JNIEnv *env, jclass cls, jlong h,
                                                                                jobject packed, jint n) {
    (void)cls;
    return sga_load_flow_rules(ENGINE(h), (const sga_flow_rule *)(*env)->GetDirectBufferAddress(env, packed),
                               (size_t)n);
}

/* ---- Java array access helpers (NULL arrays pass through as NULL) ----------------------------------- */
#define GET_I(a) ((a) ? (*env)->GetIntArrayElements(env, (a), NULL) : NULL)
#define GET_L(a) ((a) ? (*env)->GetLongArrayElements(env, (a), NULL) : NULL)
#define GET_D(a) ((a) ? (*env)->GetDoubleArrayElements(env, (a), NULL) : NULL)
#define REL_I(a, p) do { if (a) (*env)->ReleaseIntArrayElements(env, (a), (p), JNI_ABORT); } while (0)
#define REL_L(a, p) do { if (a) (*env)->ReleaseLongArrayElements(env, (a), (p), JNI_ABORT); } while (0)
#define REL_D(a, p) do { if (a) (*env)->ReleaseDoubleArrayElements(env, (a), (p), JNI_ABORT); } while (0)

/* GpuStatisticSlot.entry with the whole args vector: words = GpuArgs encoding (SGA_EV_ARGS pairs + list
 * elements), out = int[2] {decision, waitMs} */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_entryArgs(JNIEnv *env, jclass cls, jlong h,
                                                                            jint resource, jlong now_ms, jint count,
                                                                            jint flags, jlongArray words, jint nargs,
                                                                            jintArray out) {
    (void)cls;
    const jsize nw = (*env)->GetArrayLength(env, words);
    jlong *w = GET_L(words);
    int32_t o[2] = {0, 0};
    const int rc = sgaj_entry_args(ENGINE(h), (uint32_t)resource, now_ms, count, (uint32_t)flags, (const uint64_t *)w,
                                   (uint32_t)nargs, (uint32_t)nw, o);
    REL_L(words, w);
    if (rc == SGA_OK) (*env)->SetIntArrayRegion(env, out, 0, 2, (const jint *)o);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_exitArgs(JNIEnv *env, jclass cls, jlong h,
                                                                           jint resource, jlong now_ms, jint count,
                                                                           jint flags, jlong rt_ms, jlongArray words,
                                                                           jint nargs) {
    (void)cls;
    const jsize nw = (*env)->GetArrayLength(env, words);
    jlong *w = GET_L(words);
    const int rc = sgaj_exit_args(ENGINE(h), (uint32_t)resource, now_ms, count, (uint32_t)flags, rt_ms,
                                  (const uint64_t *)w, (uint32_t)nargs, (uint32_t)nw);
    REL_L(words, w);
    return rc;
}

/* GpuStatisticSlot: a slot sorted after DegradeSlot blocked an entry the engine passed (SGA_KIND_REVOKE) */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_revokedArgs(JNIEnv *env, jclass cls, jlong h,
                                                                              jint resource, jlong now_ms,
                                                                              jint count, jint flags,
                                                                              jlongArray words, jint nargs) {
    (void)cls;
    const jsize nw = (*env)->GetArrayLength(env, words);
    jlong *w = GET_L(words);
    const int rc = sgaj_revoke_args(ENGINE(h), (uint32_t)resource, now_ms, count, (uint32_t)flags,
                                    (const uint64_t *)w, (uint32_t)nargs, (uint32_t)nw);
    REL_L(words, w);
    return rc;
}

/* a BlockException thrown by a slot the engine does not run (AuthoritySlot): counted as a block */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_blocked(JNIEnv *env, jclass cls, jlong h,
                                                                          jint resource, jlong now_ms, jint count,
                                                                          jint flags) {
    (void)env;
    (void)cls;
    return sgaj_blocked(ENGINE(h), (uint32_t)resource, now_ms, count, (uint32_t)flags);
}

/* ParamFlowRuleManager.loadRules: parallel arrays (GpuRuleSync.pushParamRules) */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_loadParamRules(
    JNIEnv *env, jclass cls, jlong h, jintArray resource, jintArray grade, jdoubleArray count, jintArray behavior,
    jintArray max_queue, jintArray burst, jintArray param_idx, jlongArray duration, jintArray hot_off,
    jlongArray hot_values, jintArray hot_counts, jintArray cluster_mode, jintArray cluster_fallback,
    jlongArray cluster_flow_id, jintArray cluster_sample, jintArray cluster_window) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, resource);
    jint *r = GET_I(resource), *g = GET_I(grade), *b = GET_I(behavior), *mq = GET_I(max_queue), *bu = GET_I(burst);
    jint *pi = GET_I(param_idx), *ho = GET_I(hot_off), *hc = GET_I(hot_counts), *cm = GET_I(cluster_mode);
    jint *cf = GET_I(cluster_fallback), *cs = GET_I(cluster_sample), *cw = GET_I(cluster_window);
    jdouble *c = GET_D(count);
    jlong *du = GET_L(duration), *hv = GET_L(hot_values), *cid = GET_L(cluster_flow_id);
    const int rc = sgaj_load_param_rules(ENGINE(h), (size_t)n, (const uint32_t *)r, (const int32_t *)g,
                                         (const double *)c, (const int32_t *)b, (const int32_t *)mq,
                                         (const int32_t *)bu, (const int32_t *)pi, (const int64_t *)du,
                                         (const uint32_t *)ho, (const int64_t *)hv, (const int32_t *)hc,
                                         (const int32_t *)cm, (const int32_t *)cf, (const int64_t *)cid,
                                         (const int32_t *)cs, (const int32_t *)cw);
    REL_I(resource, r); REL_I(grade, g); REL_I(behavior, b); REL_I(max_queue, mq); REL_I(burst, bu);
    REL_I(param_idx, pi); REL_I(hot_off, ho); REL_I(hot_counts, hc); REL_I(cluster_mode, cm);
    REL_I(cluster_fallback, cf); REL_I(cluster_sample, cs); REL_I(cluster_window, cw);
    REL_D(count, c);
    REL_L(duration, du); REL_L(hot_values, hv); REL_L(cluster_flow_id, cid);
    return rc;
}

/* DegradeRuleManager.loadRules */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_loadDegradeRules(
    JNIEnv *env, jclass cls, jlong h, jintArray resource, jintArray grade, jdoubleArray count, jintArray time_window,
    jintArray min_request, jdoubleArray slow_ratio, jintArray stat_interval) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, resource);
    jint *r = GET_I(resource), *g = GET_I(grade), *tw = GET_I(time_window), *mr = GET_I(min_request);
    jint *si = GET_I(stat_interval);
    jdouble *c = GET_D(count), *sr = GET_D(slow_ratio);
    const int rc = sgaj_load_degrade_rules(ENGINE(h), (size_t)n, (const uint32_t *)r, (const int32_t *)g,
                                           (const double *)c, (const int32_t *)tw, (const int32_t *)mr,
                                           (const double *)sr, (const int32_t *)si);
    REL_I(resource, r); REL_I(grade, g); REL_I(time_window, tw); REL_I(min_request, mr); REL_I(stat_interval, si);
    REL_D(count, c); REL_D(slow_ratio, sr);
    return rc;
}

/* SystemRuleManager.loadRules */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_loadSystemRules(
    JNIEnv *env, jclass cls, jlong h, jdoubleArray load, jdoubleArray cpu, jdoubleArray qps, jlongArray avg_rt,
    jlongArray max_thread) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, load);
    jdouble *l = GET_D(load), *c = GET_D(cpu), *q = GET_D(qps);
    jlong *a = GET_L(avg_rt), *m = GET_L(max_thread);
    const int rc = sgaj_load_system_rules(ENGINE(h), (size_t)n, (const double *)l, (const double *)c,
                                          (const double *)q, (const int64_t *)a, (const int64_t *)m);
    REL_D(load, l); REL_D(cpu, c); REL_D(qps, q); REL_L(avg_rt, a); REL_L(max_thread, m);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_setSystemStatus(JNIEnv *env, jclass cls,
                                                                                  jlong h, jdouble load,
                                                                                  jdouble cpu) {
    (void)env;
    (void)cls;
    return sgaj_set_system_status(ENGINE(h), load, cpu);
}

/* ClusterParamFlowRuleManager.loadRules(namespace, rules) */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_loadClusterParamRules(
    JNIEnv *env, jclass cls, jlong h, jstring ns, jlongArray flow_id, jdoubleArray count, jintArray threshold_type,
    jintArray sample_count, jintArray window_ms, jintArray hot_off, jlongArray hot_values, jintArray hot_counts) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, flow_id);
    const char *nss = (*env)->GetStringUTFChars(env, ns, NULL);
    jlong *f = GET_L(flow_id), *hv = GET_L(hot_values);
    jdouble *c = GET_D(count);
    jint *tt = GET_I(threshold_type), *sc = GET_I(sample_count), *w = GET_I(window_ms), *ho = GET_I(hot_off);
    jint *hc = GET_I(hot_counts);
    const int rc = sgaj_load_cluster_param_rules(ENGINE(h), nss, (size_t)n, (const int64_t *)f, (const double *)c,
                                                 (const int32_t *)tt, (const int32_t *)sc, (const int32_t *)w,
                                                 (const uint32_t *)ho, (const int64_t *)hv, (const int32_t *)hc);
    REL_L(flow_id, f); REL_L(hot_values, hv); REL_D(count, c);
    REL_I(threshold_type, tt); REL_I(sample_count, sc); REL_I(window_ms, w); REL_I(hot_off, ho); REL_I(hot_counts, hc);
    (*env)->ReleaseStringUTFChars(env, ns, nss);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_setConnectedCount(JNIEnv *env, jclass cls,
                                                                                    jlong h, jstring ns, jint n) {
    (void)cls;
    const char *nss = (*env)->GetStringUTFChars(env, ns, NULL);
    const int rc = sgaj_set_connected_count(ENGINE(h), nss, n);
    (*env)->ReleaseStringUTFChars(env, ns, nss);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_setNamespaceLimit(JNIEnv *env, jclass cls,
                                                                                    jlong h, jstring ns,
                                                                                    jdouble qps) {
    (void)cls;
    const char *nss = (*env)->GetStringUTFChars(env, ns, NULL);
    const int rc = sgaj_set_namespace_limit(ENGINE(h), nss, qps);
    (*env)->ReleaseStringUTFChars(env, ns, nss);
    return rc;
}

JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_setClusterServer(JNIEnv *env, jclass cls,
                                                                                   jlong h, jint mode) {
    (void)env;
    (void)cls;
    return sgaj_set_cluster_server(ENGINE(h), mode);
}

/* GpuNode: d8 / l6 as sgaj_query_node */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_queryNode(JNIEnv *env, jclass cls, jlong h,
                                                                            jint resource, jlong now_ms,
                                                                            jdoubleArray d10, jlongArray l6) {
    (void)cls;
    double d[10];
    int64_t l[6];
    const int rc = sgaj_query_node(ENGINE(h), (uint32_t)resource, now_ms, d, l);
    if (rc == SGA_OK) {
        (*env)->SetDoubleArrayRegion(env, d10, 0, 10, (const jdouble *)d);
        (*env)->SetLongArrayRegion(env, l6, 0, 6, (const jlong *)l);
    }
    return rc;
}

/* GpuMetricTimerListener: rows of 8 longs into `rows` (length 8 * cap); returns the row count or an error */
JNIEXPORT jint JNICALL Java_com_alibaba_csp_sentinel_gpu_GpuEngine_metricsSnapshot(JNIEnv *env, jclass cls, jlong h,
                                                                                  jlong now_ms, jlongArray rows) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, rows);
    const size_t cap = (size_t)len / 8;
    int64_t *buf = (int64_t *)malloc((cap ? cap : 1) * 8 * sizeof(int64_t));
    if (!buf) return SGA_ENOMEM;
    size_t n = 0;
    const int rc = sgaj_metrics_snapshot(ENGINE(h), now_ms, buf, cap, &n);
    if (n) (*env)->SetLongArrayRegion(env, rows, 0, (jsize)(8 * n), (const jlong *)buf);
    free(buf);
    return rc == SGA_OK ? (jint)n : rc;
}
