package com.alibaba.csp.sentinel.gpu;

import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.TimeUnit;

import com.alibaba.csp.sentinel.EntryType;
import com.alibaba.csp.sentinel.context.Context;
import com.alibaba.csp.sentinel.node.DefaultNode;
import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.ResourceWrapper;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowException;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowException;
import com.alibaba.csp.sentinel.slots.system.SystemBlockException;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * One slot in place of StatisticSlot, ParamFlowSlot, FlowSlot, DegradeSlot and SystemSlot
 * (ProcessorSlot.java:41-76): entry and exit become events of the engine's local path
 * (sga_submit_events), which keeps the nodes' statistics, the controllers, the parameter maps and the
 * breakers on the GPU and answers the decision the reference's slots would have thrown.
 */
public class GpuStatisticSlot extends AbstractLinkedProcessorSlot<DefaultNode> {

    /** sga_submit_events flags (include/sentinel_amd.h SGA_EV_*). */
    static final int EV_PRIORITIZED = 1, EV_ERROR = 2, EV_HAS_PARAM = 4, EV_INBOUND = 8;

    private static final Map<String, Integer> RESOURCE_IDS = new ConcurrentHashMap<>();
    private final long engine = GpuEngine.get();

    /** Dense resource id of a resource name (like CtSph's chain map); grows the engine's table. */
    static int resourceId(String name) {
        Integer id = RESOURCE_IDS.get(name);
        if (id != null) {
            return id;
        }
        synchronized (RESOURCE_IDS) {
            id = RESOURCE_IDS.get(name);
            if (id == null) {
                id = RESOURCE_IDS.size();
                RESOURCE_IDS.put(name, id);
                GpuEngine.setResources(GpuEngine.get(), RESOURCE_IDS.size());
            }
            return id;
        }
    }

    @Override
    public void entry(Context context, ResourceWrapper resourceWrapper, DefaultNode node, int count,
                      boolean prioritized, Object... args) throws Throwable {
        int flags = prioritized ? EV_PRIORITIZED : 0;
        long param = 0;
        if (args != null && args.length > 0 && args[0] != null) {  // ParamFlowRule.paramIdx 0
            flags |= EV_HAS_PARAM;
            param = GpuTokenService.paramKey(args[0]);
        }
        if (resourceWrapper.getEntryType() == EntryType.IN) {
            flags |= EV_INBOUND;
        }
        String name = resourceWrapper.getName();
        int[] o = new int[2];
        int rc = GpuEngine.entry(engine, resourceId(name), TimeUtil.currentTimeMillis(), count, flags, param, o);
        if (rc != GpuEngine.OK) {
            throw new IllegalStateException("sga_submit_events: " + rc + " " + GpuEngine.lastError(engine));
        }
        switch (o[0]) {
            case 0:
                break;
            case 1:
                throw new FlowException(context.getOrigin());
            case 2:
                throw new ParamFlowException(name, String.valueOf(args[0]));
            case 3:
                throw new DegradeException(context.getOrigin());
            case 4:  // DefaultController.canPass slept and threw PriorityWaitException, which StatisticSlot
                     // counts as passed (the engine has counted it); the slots after FlowSlot do not run
                TimeUnit.MILLISECONDS.sleep(o[1]);
                return;
            case 5:
                throw new SystemBlockException(name, "gpu");
            default:
                throw new IllegalStateException("unknown decision " + o[0]);
        }
        fireEntry(context, resourceWrapper, node, count, prioritized, args);
    }

    @Override
    public void exit(Context context, ResourceWrapper resourceWrapper, int count, Object... args) {
        long now = TimeUtil.currentTimeMillis();
        long rt = now - context.getCurEntry().getCreateTimestamp();
        int flags = context.getCurEntry().getError() != null ? EV_ERROR : 0;
        long param = 0;
        if (args != null && args.length > 0 && args[0] != null) {
            flags |= EV_HAS_PARAM;
            param = GpuTokenService.paramKey(args[0]);
        }
        if (resourceWrapper.getEntryType() == EntryType.IN) {
            flags |= EV_INBOUND;
        }
        if (context.getCurEntry().getBlockError() == null) {  // only entries that passed exit
            GpuEngine.exit(engine, resourceId(resourceWrapper.getName()), now, count, flags, rt, param);
        }
        fireExit(context, resourceWrapper, count, args);
    }
}
