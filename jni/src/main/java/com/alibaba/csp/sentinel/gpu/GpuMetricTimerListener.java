package com.alibaba.csp.sentinel.gpu;

import java.util.ArrayList;
import java.util.List;
import java.util.Map;
import java.util.TreeMap;

import com.alibaba.csp.sentinel.Constants;
import com.alibaba.csp.sentinel.config.SentinelConfig;
import com.alibaba.csp.sentinel.log.RecordLog;
import com.alibaba.csp.sentinel.node.metric.MetricNode;
import com.alibaba.csp.sentinel.node.metric.MetricWriter;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * MetricTimerListener (MetricTimerListener.java:34-81) over the engine: once a second (schedule it like the
 * reference, SCHEDULER.scheduleAtFixedRate(listener, 0, 1, SECONDS)) every resource's StatisticNode.metrics()
 * comes from one sga_metrics_snapshot, grouped by second and written by MetricWriter in time order.  The
 * reference listener keeps running over ClusterBuilderSlot's nodes, which the GPU chain leaves empty.
 */
public class GpuMetricTimerListener implements Runnable {

    private static final MetricWriter METRIC_WRITER = new MetricWriter(SentinelConfig.singleMetricFileSize(),
        SentinelConfig.totalMetricFileCount());
    private static final int CAP = Integer.getInteger("csp.sentinel.gpu.metricRows", 1 << 16);

    /** MetricNodes of one snapshot; resource = -2 for every resource. */
    static List<MetricNode> snapshot(long now, int resource) {
        long[] rows = new long[8 * CAP];
        int n = GpuEngine.metricsSnapshot(GpuEngine.get(), now, rows);
        List<MetricNode> out = new ArrayList<>();
        for (int i = 0; i < Math.max(n, 0); i++) {
            int rid = (int) rows[8 * i + 1];
            if (resource != -2 && rid != resource) {
                continue;
            }
            MetricNode m = new MetricNode();
            m.setTimestamp(rows[8 * i]);
            String name = rid == GpuNode.ENTRY_NODE ? Constants.TOTAL_IN_RESOURCE_NAME : GpuStatisticSlot.resourceName(rid);
            m.setResource(name);
            m.setPassQps(rows[8 * i + 2]);
            m.setBlockQps(rows[8 * i + 3]);
            m.setSuccessQps(rows[8 * i + 4]);
            m.setExceptionQps(rows[8 * i + 5]);
            m.setRt(rows[8 * i + 6]);
            m.setOccupiedPassQps(rows[8 * i + 7]);
            out.add(m);
        }
        return out;
    }

    @Override
    public void run() {
        Map<Long, List<MetricNode>> maps = new TreeMap<>();
        for (MetricNode m : snapshot(TimeUtil.currentTimeMillis(), -2)) {
            maps.computeIfAbsent(m.getTimestamp(), k -> new ArrayList<MetricNode>()).add(m);
        }
        for (Map.Entry<Long, List<MetricNode>> e : maps.entrySet()) {
            try {
                METRIC_WRITER.write(e.getKey(), e.getValue());
            } catch (Exception ex) {
                RecordLog.warn("[GpuMetricTimerListener] Write metric error", ex);
            }
        }
    }
}
