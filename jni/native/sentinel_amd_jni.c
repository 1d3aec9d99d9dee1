/* JNI entry points of com.alibaba.csp.sentinel.gpu.GpuEngine (the native methods the Java shim
 * declares).  Each converts Java arrays / strings to plain pointers and calls the C glue
 * (sga_jni_glue.c), which calls the engine's C ABI.  Build with the JDK's include directories:
 *   cc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude -Ijni/native \
 *      jni/native/sentinel_amd_jni.c jni/native/sga_jni_glue.c -Lsentinel_amd -lsentinel_amd \
 *      -o libsentinel_amd_jni.so */
#include <jni.h>
#include <stdint.h>

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
