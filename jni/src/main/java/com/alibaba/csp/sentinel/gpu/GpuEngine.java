package com.alibaba.csp.sentinel.gpu;

import java.nio.ByteBuffer;

/**
 * Native methods of the MI355X engine (jni/native/sentinel_amd_jni.c over include/sentinel_amd.h).
 * One engine per process and device, shared by {@link GpuTokenService} and {@link GpuStatisticSlot}.
 */
public final class GpuEngine {

    static {
        System.loadLibrary("sentinel_amd_jni");
    }

    /** sga_* error codes (include/sentinel_amd.h). */
    public static final int OK = 0;
    public static final int EAGAIN = -11;

    private static volatile long instance;

    private GpuEngine() {}

    /** The process-wide engine on device 0 (created on first use). */
    public static long get() {
        long h = instance;
        if (h != 0) {
            return h;
        }
        synchronized (GpuEngine.class) {
            if (instance == 0) {
                long e = create(Integer.getInteger("csp.sentinel.gpu.device", 0),
                                Integer.getInteger("csp.sentinel.gpu.maxBatch", 1 << 20),
                                Integer.getInteger("csp.sentinel.gpu.maxRules", 1 << 20));
                if (e <= 0) {
                    throw new IllegalStateException("sga_create failed: " + e);
                }
                instance = e;
            }
            return instance;
        }
    }

    static native long create(int device, int maxBatch, int maxRules);

    static native void destroy(long engine);

    static native String lastError(long engine);

    /** ClusterFlowRuleManager.loadRules(namespace, rules): cluster-mode rules as parallel arrays. */
    static native int loadClusterFlowRules(long engine, String namespace, long[] flowIds, double[] counts,
                                           int[] thresholdTypes, int[] sampleCounts, int[] windowIntervalMs);

    /** TokenService.requestToken through the engine's coalescing queue: out = {status, remaining, waitInMs}. */
    static native int requestToken(long engine, long flowId, int acquireCount, boolean prioritized, long nowMs,
                                   int[] out);

    /** Asynchronous requestToken: a ticket (>= 0) or an error code (< 0). */
    static native long submit(long engine, long flowId, int acquireCount, boolean prioritized, long nowMs);

    /** OK with out filled, or EAGAIN while the ticket's batch is not decided. */
    static native int poll(long engine, long ticket, int[] out);

    /** TokenService.requestParamToken with the parameters mapped to 64-bit keys. */
    static native int requestParamToken(long engine, long flowId, int acquireCount, long[] values, long nowMs,
                                        int[] out);

    /** requestConcurrentToken (op 0, id = ruleId) / releaseConcurrentToken (op 1, id = tokenId): out = {status, tokenId}. */
    static native int concurrent(long engine, int op, int client, long id, int acquireCount, long nowMs, long[] out);

    /** One entry event through the local slot chain: out = {decision, waitMs}. */
    static native int entry(long engine, int resource, long nowMs, int count, int flags, long param, int[] out);

    /** The exit event of an entry that passed. */
    static native int exit(long engine, int resource, long nowMs, int count, int flags, long rtMs, long param);

    static native int setResources(long engine, int n);

    /** FlowRuleManager.loadRules: packed sga_flow_rule records in a direct buffer (little endian). */
    static native int loadFlowRules(long engine, ByteBuffer packed, int n);
}
