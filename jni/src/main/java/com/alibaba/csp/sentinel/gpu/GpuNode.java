package com.alibaba.csp.sentinel.gpu;

import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.function.Predicate;

import com.alibaba.csp.sentinel.node.Node;
import com.alibaba.csp.sentinel.node.metric.MetricNode;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * {@link Node} view (Node.java:40-203, OccupySupport.java:40-69) of a resource's ClusterNode, which lives in the
 * engine: every getter is sga_query_node at TimeUtil's now (reads rotate the windows, as ArrayMetric's do).  The
 * statistics are written only by the engine's events (GpuStatisticSlot), so the mutators are unsupported.
 */
public final class GpuNode implements Node {

    /** Constants.ENTRY_NODE (include/sentinel_amd.h SGA_ENTRY_NODE). */
    public static final int ENTRY_NODE = 0xFFFFFFFF;

    private final int resource;

    public GpuNode(String resourceName) {
        this.resource = GpuStatisticSlot.resourceId(resourceName);
    }

    private GpuNode(int resource) {
        this.resource = resource;
    }

    public static GpuNode entryNode() {
        return new GpuNode(ENTRY_NODE);
    }

    private static final class View {
        final double[] d = new double[10];
        final long[] l = new long[6];
    }

    private View view() {
        View v = new View();
        int rc = GpuEngine.queryNode(GpuEngine.get(), resource, TimeUtil.currentTimeMillis(), v.d, v.l);
        if (rc != GpuEngine.OK) {
            throw new IllegalStateException("sga_query_node: " + rc);
        }
        return v;
    }

    @Override public long totalRequest() { View v = view(); return v.l[0] + v.l[1]; }
    @Override public long totalPass() { return view().l[0]; }
    @Override public long totalSuccess() { return view().l[2]; }
    @Override public long blockRequest() { return view().l[1]; }
    @Override public long totalException() { return view().l[3]; }
    @Override public double passQps() { return view().d[0]; }
    @Override public double blockQps() { return view().d[1]; }
    @Override public double totalQps() { View v = view(); return v.d[0] + v.d[1]; }
    @Override public double successQps() { return view().d[2]; }
    @Override public double exceptionQps() { return view().d[3]; }
    @Override public double avgRt() { return view().d[5]; }
    @Override public double minRt() { return view().d[6]; }
    @Override public int curThreadNum() { return (int) view().l[4]; }
    @Override public double previousPassQps() { return view().d[7]; }
    @Override public double occupiedPassQps() { return view().d[4]; }
    @Override public long waiting() { return view().l[5]; }

    @Override
    public double maxSuccessQps() { return view().d[8]; }

    @Override
    public double previousBlockQps() { return view().d[9]; }

    /** StatisticNode.metrics() of this node: the engine's snapshot (it advances every node's lastFetchTime). */
    @Override
    public Map<Long, MetricNode> metrics() {
        Map<Long, MetricNode> out = new HashMap<>();
        for (MetricNode m : GpuMetricTimerListener.snapshot(TimeUtil.currentTimeMillis(), resource)) {
            out.put(m.getTimestamp(), m);
        }
        return out;
    }

    @Override
    public List<MetricNode> rawMetricsInMin(Predicate<Long> timePredicate) {
        List<MetricNode> out = new ArrayList<>();
        for (MetricNode m : metrics().values()) {
            if (timePredicate.test(m.getTimestamp())) {
                out.add(m);
            }
        }
        return out;
    }

    private static UnsupportedOperationException engineOwned() {
        return new UnsupportedOperationException("node statistics are written by the engine's events only");
    }

    @Override public void addPassRequest(int count) { throw engineOwned(); }
    @Override public void addRtAndSuccess(long rt, int success) { throw engineOwned(); }
    @Override public void increaseBlockQps(int count) { throw engineOwned(); }
    @Override public void increaseExceptionQps(int count) { throw engineOwned(); }
    @Override public void increaseThreadNum() { throw engineOwned(); }
    @Override public void decreaseThreadNum() { throw engineOwned(); }
    @Override public void reset() { throw engineOwned(); }
    @Override public long tryOccupyNext(long currentTime, int acquireCount, double threshold) { throw engineOwned(); }
    @Override public void addWaitingRequest(long futureTime, int acquireCount) { throw engineOwned(); }
    @Override public void addOccupiedPass(int acquireCount) { throw engineOwned(); }

    @Override
    public void debug() {
        View v = view();
        System.out.println("GpuNode(" + resource + "): passQps=" + v.d[0] + " blockQps=" + v.d[1] + " threads=" + v.l[4]);
    }
}
