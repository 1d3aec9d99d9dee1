package com.alibaba.csp.sentinel.gpu;

import java.nio.ByteBuffer;

/**
 * Native methods of the MI355X engine (jni/native/sentinel_amd_jni.c over include/sentinel_amd.h).
 * One engine per process and device, shared by {@link GpuTokenService}, {@link GpuStatisticSlot},
 * {@link GpuRuleSync}, {@link GpuNode} and {@link GpuMetricTimerListener}.
 */
public final class GpuEngine {

    static {
        System.loadLibrary("sentinel_amd_jni");
    }

    /** sga_* error codes (include/sentinel_amd.h). */
    public static final int OK = 0;
    public static final int EAGAIN = -11;

    /** sga_submit_events flags / kinds (include/sentinel_amd.h SGA_EV_*, SGA_KIND_*). */
    static final int EV_PRIORITIZED = 1, EV_ERROR = 2, EV_INBOUND = 8, EV_ARGS = 32;

    /** Resource table size: names get dense ids (like CtSph's chain map), fixed once the engine exists. */
    static final int MAX_RESOURCES = Integer.getInteger("csp.sentinel.gpu.maxResources", 1 << 16);

    private static volatile long instance;

    private GpuEngine() {}

    /** The process-wide engine on device 0 (created on first use, with its resource table). */
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
                int rc = setResources(e, MAX_RESOURCES);
                if (rc != OK) {
                    throw new IllegalStateException("sga_flow_set_resources failed: " + rc + " " + lastError(e));
                }
                instance = e;
            }
            return instance;
        }
    }

    static native long create(int device, int maxBatch, int maxRules);

    static native void destroy(long engine);

    static native String lastError(long engine);

    // ---- cluster token server (TokenService SPI, ClusterFlowRuleManager / ClusterParamFlowRuleManager)

    /** ClusterFlowRuleManager.loadRules(namespace, rules): cluster-mode rules as parallel arrays. */
    static native int loadClusterFlowRules(long engine, String namespace, long[] flowIds, double[] counts,
                                           int[] thresholdTypes, int[] sampleCounts, int[] windowIntervalMs);

    /** ClusterParamFlowRuleManager.loadRules(namespace, rules): hot items of rule i at [hotOff[i], hotOff[i+1]). */
    static native int loadClusterParamRules(long engine, String namespace, long[] flowIds, double[] counts,
                                            int[] thresholdTypes, int[] sampleCounts, int[] windowIntervalMs,
                                            int[] hotOff, long[] hotValues, int[] hotCounts);

    /** ConnectionManager: connected clients of a namespace (AVG_LOCAL thresholds). */
    static native int setConnectedCount(long engine, String namespace, int connected);

    /** GlobalRequestLimiter.initIfAbsent / applyMaxQpsChange of a namespace. */
    static native int setNamespaceLimit(long engine, String namespace, double maxAllowedQps);

    /** TokenService.requestToken through the engine's coalescing queue: out = {status, remaining, waitInMs}. */
    static native int requestToken(long engine, long flowId, int acquireCount, boolean prioritized, long nowMs,
                                   int[] out);

    /** Asynchronous requestToken: a ticket (>= 0) or an error code (< 0). */
    static native long submit(long engine, long flowId, int acquireCount, boolean prioritized, long nowMs);

    /** OK with out filled, or EAGAIN while the ticket's batch is not decided. */
    static native int poll(long engine, long ticket, int[] out);

    /** TokenService.requestParamToken with the parameters mapped to 64-bit keys ({@link GpuArgs#key}). */
    static native int requestParamToken(long engine, long flowId, int acquireCount, long[] values, long nowMs,
                                        int[] out);

    /** requestConcurrentToken (op 0, id = ruleId) / releaseConcurrentToken (op 1, id = tokenId): out = {status, tokenId}. */
    static native int concurrent(long engine, int op, int client, long id, int acquireCount, long nowMs, long[] out);

    // ---- local slot chain (GpuStatisticSlot) and the rule managers (GpuRuleSync)

    /** One entry with its whole args vector ({@link GpuArgs#encode}): out = {decision, waitMs or block detail}. */
    static native int entryArgs(long engine, int resource, long nowMs, int count, int flags, long[] words, int nargs,
                                int[] out);

    /** The exit of an entry that passed, with the exit's args. */
    static native int exitArgs(long engine, int resource, long nowMs, int count, int flags, long rtMs, long[] words,
                               int nargs);

    /** StatisticSlot's BlockException branch for a block thrown outside the engine (AuthoritySlot). */
    static native int blocked(long engine, int resource, long nowMs, int count, int flags);

    /** A passed entry blocked by a slot after the engine's checks (SGA_KIND_REVOKE, the entry's time,
     * flags and arguments). */
    static native int revokedArgs(long engine, int resource, long nowMs, int count, int flags, long[] words,
                                  int nargs);

    /** Round-2 single-parameter forms (flags EV_HAS_PARAM = 4: args = [param]). */
    static native int entry(long engine, int resource, long nowMs, int count, int flags, long param, int[] out);

    static native int exit(long engine, int resource, long nowMs, int count, int flags, long rtMs, long param);

    static native int setResources(long engine, int n);

    /** FlowRuleManager.loadRules: packed sga_flow_rule records in a direct buffer (little endian). */
    static native int loadFlowRules(long engine, ByteBuffer packed, int n);

    /** ParamFlowRuleManager.loadRules: parallel arrays; cluster* may be null for local-only lists. */
    static native int loadParamRules(long engine, int[] resource, int[] grade, double[] count, int[] behavior,
                                     int[] maxQueueingTimeMs, int[] burstCount, int[] paramIdx, long[] durationInSec,
                                     int[] hotOff, long[] hotValues, int[] hotCounts, int[] clusterMode,
                                     int[] clusterFallback, long[] clusterFlowId, int[] clusterSampleCount,
                                     int[] clusterWindowMs);

    /** DegradeRuleManager.loadRules. */
    static native int loadDegradeRules(long engine, int[] resource, int[] grade, double[] count, int[] timeWindow,
                                       int[] minRequestAmount, double[] slowRatioThreshold, int[] statIntervalMs);

    /** SystemRuleManager.loadRules (negative = field not set). */
    static native int loadSystemRules(long engine, double[] highestSystemLoad, double[] highestCpuUsage,
                                      double[] qps, long[] avgRt, long[] maxThread);

    /** SystemStatusListener readings. */
    static native int setSystemStatus(long engine, double avgLoad, double cpuUsage);

    /** ClusterStateManager: 1 = embedded token server (cluster-mode rules decided by this engine), 0 = none. */
    static native int setClusterServer(long engine, int mode);

    /**
     * Node getters of a resource's ClusterNode at nowMs: d10 = {passQps, blockQps, successQps, exceptionQps,
     * occupiedPassQps, avgRt, minRt, previousPassQps, maxSuccessQps, previousBlockQps}, l6 = {totalPass, totalBlock,
     * totalSuccess, totalException, curThreadNum, waiting}.
     */
    static native int queryNode(long engine, int resource, long nowMs, double[] d10, long[] l6);

    /**
     * StatisticNode.metrics() of every resource: rows of 8 longs {timestamp, resource, pass, block, success,
     * exception, rt, occupiedPass} into rows (capacity rows.length / 8); returns the row count or an error.
     */
    static native int metricsSnapshot(long engine, long nowMs, long[] rows);
}
