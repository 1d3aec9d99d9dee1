package com.alibaba.csp.sentinel.gpu;

import java.lang.reflect.Field;
import java.lang.reflect.Method;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Collections;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.function.Function;

import com.alibaba.csp.sentinel.cluster.flow.rule.ClusterFlowRuleManager;
import com.alibaba.csp.sentinel.cluster.flow.rule.ClusterParamFlowRuleManager;
import com.alibaba.csp.sentinel.property.PropertyListener;
import com.alibaba.csp.sentinel.property.SentinelProperty;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleUtil;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowClusterConfig;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleUtil;
import com.alibaba.csp.sentinel.slots.system.SystemRule;
import com.alibaba.csp.sentinel.slots.system.SystemRuleManager;

/**
 * The rule managers' updates forwarded to the engine.  {@link #install()} adds a PropertyListener to the
 * SentinelProperty each manager holds (FlowRuleManager.java:56, ParamFlowRuleManager.java:52, DegradeRuleManager.java:49,
 * SystemRuleManager.java:114 -- DynamicSentinelProperty.addListener replays the current rules at once), so
 * FlowRuleManager.loadRules / ParamFlowRuleManager.loadRules / DegradeRuleManager.loadRules /
 * SystemRuleManager.loadRules -- and datasources writing those properties -- reach the GPU unchanged.  Call it
 * again after a manager's register2Property (which moves the manager to another property).  Cluster namespaces
 * go through the managers' property suppliers (ClusterFlowRuleManager.setPropertySupplier,
 * ClusterParamFlowRuleManager.setPropertySupplier): every namespace property the server registers carries a
 * listener that loads the namespace's rules into the engine.
 *
 * The per-resource rule lists are kept in the engine's order, so a block's detail (the blocking rule's index)
 * maps back to the rule object for FlowException / ParamFlowException / DegradeException.
 */
public final class GpuRuleSync {

    private static volatile Map<String, List<FlowRule>> flowByResource = Collections.emptyMap();
    private static volatile Map<String, List<ParamFlowRule>> paramByResource = Collections.emptyMap();
    private static volatile Map<String, List<DegradeRule>> degradeByResource = Collections.emptyMap();

    private GpuRuleSync() {}

    static FlowRule flowRule(String resource, int k) {
        List<FlowRule> l = flowByResource.get(resource);
        return l != null && k >= 0 && k < l.size() ? l.get(k) : null;
    }

    static ParamFlowRule paramRule(String resource, int k) {
        List<ParamFlowRule> l = paramByResource.get(resource);
        return l != null && k >= 0 && k < l.size() ? l.get(k) : null;
    }

    static DegradeRule degradeRule(String resource, int k) {
        List<DegradeRule> l = degradeByResource.get(resource);
        return l != null && k >= 0 && k < l.size() ? l.get(k) : null;
    }

    /** Attaches the engine listeners to the rule managers' current properties and the cluster suppliers. */
    public static synchronized void install() {
        attach(FlowRuleManager.class, new FlowListener());
        attach(ParamFlowRuleManager.class, new ParamListener());
        attach(DegradeRuleManager.class, new DegradeListener());
        attach(SystemRuleManager.class, new SystemListener());
        final Function<String, SentinelProperty<List<FlowRule>>> fs = ClusterFlowRuleManager.DEFAULT_PROPERTY_SUPPLIER;
        ClusterFlowRuleManager.setPropertySupplier(ns -> {
            SentinelProperty<List<FlowRule>> p = fs.apply(ns);
            p.addListener(new ClusterFlowListener(ns));
            return p;
        });
        final Function<String, SentinelProperty<List<ParamFlowRule>>> ps =
            ClusterParamFlowRuleManager.DEFAULT_PROPERTY_SUPPLIER;
        ClusterParamFlowRuleManager.setPropertySupplier(ns -> {
            SentinelProperty<List<ParamFlowRule>> p = ps.apply(ns);
            p.addListener(new ClusterParamListener(ns));
            return p;
        });
    }

    /** ClusterStateManager.setToServer / stop on the engine's local path (embedded token server). */
    public static void setEmbeddedServer(boolean on) {
        check(GpuEngine.setClusterServer(GpuEngine.get(), on ? 1 : 0), "setClusterServer");
    }

    /** ConnectionManager's connected count of a namespace (AVG_LOCAL cluster thresholds). */
    public static void setConnectedCount(String namespace, int connected) {
        check(GpuEngine.setConnectedCount(GpuEngine.get(), namespace, connected), "setConnectedCount");
    }

    /** GlobalRequestLimiter.initIfAbsent / applyMaxQpsChange (ServerFlowConfig.maxAllowedQps of a namespace). */
    public static void setNamespaceLimit(String namespace, double maxAllowedQps) {
        check(GpuEngine.setNamespaceLimit(GpuEngine.get(), namespace, maxAllowedQps), "setNamespaceLimit");
    }

    /** SystemStatusListener readings (system load average, CPU usage 0..1). */
    public static void setSystemStatus(double avgLoad, double cpuUsage) {
        check(GpuEngine.setSystemStatus(GpuEngine.get(), avgLoad, cpuUsage), "setSystemStatus");
    }

    @SuppressWarnings("unchecked")
    private static <T> void attach(Class<?> manager, PropertyListener<T> l) {
        try {
            Field f = manager.getDeclaredField("currentProperty");
            f.setAccessible(true);
            ((SentinelProperty<T>) f.get(null)).addListener(l);
        } catch (ReflectiveOperationException e) {
            throw new IllegalStateException("cannot attach to " + manager.getName(), e);
        }
    }

    private static void check(int rc, String what) {
        if (rc < 0) {
            throw new IllegalStateException(what + ": " + rc + " " + GpuEngine.lastError(GpuEngine.get()));
        }
    }

    private abstract static class Listener<T> implements PropertyListener<T> {
        @Override
        public void configLoad(T value) {
            configUpdate(value);
        }
    }

    /** FlowRuleManager: per resource in FlowRuleComparator order (FlowRuleUtil.buildFlowRuleMap), as packed sga_flow_rule. */
    private static final class FlowListener extends Listener<List<FlowRule>> {
        @Override
        public void configUpdate(List<FlowRule> value) {
            Map<String, List<FlowRule>> m = FlowRuleUtil.buildFlowRuleMap(value == null ? new ArrayList<>() : value);
            List<FlowRule> flat = new ArrayList<>();
            for (List<FlowRule> l : m.values()) {
                flat.addAll(l);
            }
            ByteBuffer b = ByteBuffer.allocateDirect(64 * Math.max(1, flat.size())).order(ByteOrder.LITTLE_ENDIAN);
            for (FlowRule r : flat) {  // sga_flow_rule, 64 bytes (include/sentinel_amd.h)
                int base = b.position();
                b.putInt(GpuStatisticSlot.resourceId(r.getResource())).putInt(r.getGrade()).putDouble(r.getCount());
                b.putInt(r.getControlBehavior()).putInt(r.getWarmUpPeriodSec()).putInt(r.getMaxQueueingTimeMs());
                b.putInt(r.getStrategy());
                boolean cm = r.isClusterMode() && r.getClusterConfig() != null;
                b.putInt(cm ? 1 : 0).putInt(cm && r.getClusterConfig().isFallbackToLocalWhenFail() ? 1 : 0);
                b.putLong(cm && r.getClusterConfig().getFlowId() != null ? r.getClusterConfig().getFlowId() : 0L);
                b.putInt(cm ? r.getClusterConfig().getSampleCount() : 0);
                b.putInt(cm ? r.getClusterConfig().getWindowIntervalMs() : 0);
                b.putInt(cm ? r.getClusterConfig().getStrategy() : 0).putInt(0);
                b.position(base + 64);
            }
            b.flip();
            check(GpuEngine.loadFlowRules(GpuEngine.get(), b, flat.size()), "FlowRuleManager.loadRules");
            flowByResource = m;
        }
    }

    /** The parsed hot items of a rule (ParamFlowRuleUtil.fillExceptionFlowItems + getParsedHotItems). */
    @SuppressWarnings("unchecked")
    private static Map<Object, Integer> hotItems(ParamFlowRule r) {
        try {
            ParamFlowRuleUtil.fillExceptionFlowItems(r);
            Method m = ParamFlowRule.class.getDeclaredMethod("getParsedHotItems");
            m.setAccessible(true);
            Map<Object, Integer> h = (Map<Object, Integer>) m.invoke(r);
            return h == null ? Collections.<Object, Integer>emptyMap() : h;
        } catch (ReflectiveOperationException e) {
            throw new IllegalStateException("ParamFlowRule hot items", e);
        }
    }

    /** ParamFlowRuleManager: per resource in list order (ParamFlowRuleUtil.buildParamRuleMap). */
    private static final class ParamListener extends Listener<List<ParamFlowRule>> {
        @Override
        public void configUpdate(List<ParamFlowRule> value) {
            Map<String, List<ParamFlowRule>> m =
                ParamFlowRuleUtil.buildParamRuleMap(value == null ? new ArrayList<>() : value);
            List<ParamFlowRule> flat = new ArrayList<>();
            for (List<ParamFlowRule> l : m.values()) {
                flat.addAll(l);
            }
            int n = flat.size(), nh = 0;
            List<Map<Object, Integer>> hots = new ArrayList<>();
            for (ParamFlowRule r : flat) {
                Map<Object, Integer> h = hotItems(r);
                hots.add(h);
                nh += h.size();
            }
            int[] res = new int[n], grade = new int[n], beh = new int[n], mq = new int[n], burst = new int[n];
            int[] idx = new int[n], hotOff = new int[n + 1], hotCnt = new int[nh], cm = new int[n], cf = new int[n];
            int[] cs = new int[n], cw = new int[n];
            double[] count = new double[n];
            long[] dur = new long[n], hotVal = new long[nh], cid = new long[n];
            for (int i = 0, h = 0; i < n; i++) {
                ParamFlowRule r = flat.get(i);
                res[i] = GpuStatisticSlot.resourceId(r.getResource());
                grade[i] = r.getGrade();
                count[i] = r.getCount();
                beh[i] = r.getControlBehavior();
                mq[i] = r.getMaxQueueingTimeMs();
                burst[i] = r.getBurstCount();
                idx[i] = r.getParamIdx() == null ? 0 : r.getParamIdx();
                dur[i] = r.getDurationInSec();
                hotOff[i] = h;
                for (Map.Entry<Object, Integer> e : hots.get(i).entrySet()) {
                    hotVal[h] = GpuArgs.key(e.getKey());
                    hotCnt[h++] = e.getValue();
                }
                hotOff[i + 1] = h;
                ParamFlowClusterConfig cc = r.getClusterConfig();
                if (r.isClusterMode() && cc != null) {
                    cm[i] = 1;
                    cf[i] = cc.isFallbackToLocalWhenFail() ? 1 : 0;
                    cid[i] = cc.getFlowId() == null ? 0L : cc.getFlowId();
                    cs[i] = cc.getSampleCount();
                    cw[i] = cc.getWindowIntervalMs();
                }
            }
            check(GpuEngine.loadParamRules(GpuEngine.get(), res, grade, count, beh, mq, burst, idx, dur, hotOff, hotVal,
                                           hotCnt, cm, cf, cid, cs, cw), "ParamFlowRuleManager.loadRules");
            paramByResource = m;
        }
    }

    /** DegradeRuleManager: per resource in list order (buildCircuitBreakers). */
    private static final class DegradeListener extends Listener<List<DegradeRule>> {
        @Override
        public void configUpdate(List<DegradeRule> value) {
            Map<String, List<DegradeRule>> m = new HashMap<>();
            List<DegradeRule> flat = new ArrayList<>();
            for (DegradeRule r : value == null ? new ArrayList<DegradeRule>() : value) {
                if (!DegradeRuleManager.isValidRule(r)) {
                    continue;
                }
                m.computeIfAbsent(r.getResource(), k -> new ArrayList<>()).add(r);
            }
            for (List<DegradeRule> l : m.values()) {
                flat.addAll(l);
            }
            int n = flat.size();
            int[] res = new int[n], grade = new int[n], tw = new int[n], minReq = new int[n], stat = new int[n];
            double[] count = new double[n], slow = new double[n];
            for (int i = 0; i < n; i++) {
                DegradeRule r = flat.get(i);
                res[i] = GpuStatisticSlot.resourceId(r.getResource());
                grade[i] = r.getGrade();
                count[i] = r.getCount();
                tw[i] = r.getTimeWindow();
                minReq[i] = r.getMinRequestAmount();
                slow[i] = r.getSlowRatioThreshold();
                stat[i] = r.getStatIntervalMs();
            }
            check(GpuEngine.loadDegradeRules(GpuEngine.get(), res, grade, count, tw, minReq, slow, stat),
                  "DegradeRuleManager.loadRules");
            degradeByResource = m;
        }
    }

    /** SystemRuleManager (the engine keeps the per-field minimum and the last rule's switch, as the reference). */
    private static final class SystemListener extends Listener<List<SystemRule>> {
        @Override
        public void configUpdate(List<SystemRule> value) {
            List<SystemRule> l = value == null ? new ArrayList<SystemRule>() : value;
            int n = l.size();
            double[] load = new double[n], cpu = new double[n], qps = new double[n];
            long[] rt = new long[n], thr = new long[n];
            for (int i = 0; i < n; i++) {
                SystemRule r = l.get(i);
                load[i] = r.getHighestSystemLoad();
                cpu[i] = r.getHighestCpuUsage();
                qps[i] = r.getQps();
                rt[i] = r.getAvgRt();
                thr[i] = r.getMaxThread();
            }
            check(GpuEngine.loadSystemRules(GpuEngine.get(), load, cpu, qps, rt, thr), "SystemRuleManager.loadRules");
        }
    }

    /** A cluster namespace's FlowRules (ClusterFlowRuleManager.loadRules(namespace, rules)). */
    private static final class ClusterFlowListener extends Listener<List<FlowRule>> {
        private final String ns;

        ClusterFlowListener(String ns) {
            this.ns = ns;
        }

        @Override
        public void configUpdate(List<FlowRule> value) {
            List<FlowRule> l = new ArrayList<>();
            for (FlowRule r : value == null ? new ArrayList<FlowRule>() : value) {
                if (r.isClusterMode() && r.getClusterConfig() != null && r.getClusterConfig().getFlowId() != null) {
                    l.add(r);
                }
            }
            int n = l.size();
            long[] id = new long[n];
            double[] count = new double[n];
            int[] tt = new int[n], sc = new int[n], w = new int[n];
            for (int i = 0; i < n; i++) {
                FlowRule r = l.get(i);
                id[i] = r.getClusterConfig().getFlowId();
                count[i] = r.getCount();
                tt[i] = r.getClusterConfig().getThresholdType();
                sc[i] = r.getClusterConfig().getSampleCount();
                w[i] = r.getClusterConfig().getWindowIntervalMs();
            }
            check(GpuEngine.loadClusterFlowRules(GpuEngine.get(), ns, id, count, tt, sc, w),
                  "ClusterFlowRuleManager.loadRules");
        }
    }

    /** A cluster namespace's ParamFlowRules (ClusterParamFlowRuleManager.loadRules(namespace, rules)). */
    private static final class ClusterParamListener extends Listener<List<ParamFlowRule>> {
        private final String ns;

        ClusterParamListener(String ns) {
            this.ns = ns;
        }

        @Override
        public void configUpdate(List<ParamFlowRule> value) {
            List<ParamFlowRule> l = new ArrayList<>();
            for (ParamFlowRule r : value == null ? new ArrayList<ParamFlowRule>() : value) {
                if (r.isClusterMode() && r.getClusterConfig() != null && r.getClusterConfig().getFlowId() != null) {
                    l.add(r);
                }
            }
            int n = l.size(), nh = 0;
            List<Map<Object, Integer>> hots = new ArrayList<>();
            for (ParamFlowRule r : l) {
                Map<Object, Integer> h = hotItems(r);
                hots.add(h);
                nh += h.size();
            }
            long[] id = new long[n], hv = new long[nh];
            double[] count = new double[n];
            int[] tt = new int[n], sc = new int[n], w = new int[n], off = new int[n + 1], hc = new int[nh];
            for (int i = 0, h = 0; i < n; i++) {
                ParamFlowRule r = l.get(i);
                id[i] = r.getClusterConfig().getFlowId();
                count[i] = r.getCount();
                tt[i] = r.getClusterConfig().getThresholdType();
                sc[i] = r.getClusterConfig().getSampleCount();
                w[i] = r.getClusterConfig().getWindowIntervalMs();
                off[i] = h;
                for (Map.Entry<Object, Integer> e : hots.get(i).entrySet()) {
                    hv[h] = GpuArgs.key(e.getKey());
                    hc[h++] = e.getValue();
                }
                off[i + 1] = h;
            }
            check(GpuEngine.loadClusterParamRules(GpuEngine.get(), ns, id, count, tt, sc, w, off, hv, hc),
                  "ClusterParamFlowRuleManager.loadRules");
        }
    }
}
