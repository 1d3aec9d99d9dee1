package com.alibaba.csp.sentinel.gpu;

import java.util.ArrayList;
import java.util.List;
import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.TimeUnit;

import com.alibaba.csp.sentinel.EntryType;
import com.alibaba.csp.sentinel.context.Context;
import com.alibaba.csp.sentinel.node.DefaultNode;
import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.DefaultProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.ResourceWrapper;
import com.alibaba.csp.sentinel.slots.block.BlockException;
import com.alibaba.csp.sentinel.slots.block.RuleConstant;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeException;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowException;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.system.SystemBlockException;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * One slot in place of StatisticSlot, SystemSlot, ParamFlowSlot, FlowSlot and DegradeSlot (ProcessorSlot.java:41-76).
 * As StatisticSlot (StatisticSlot.java:64-145) it first fires the checks that precede the engine's -- the "pre"
 * chain (AuthoritySlot and the custom slots sorted before DegradeSlot, GpuSlotChainBuilder) -- and then decides:
 * the engine's local path (sga_submit_events) runs SystemSlot, ParamFlowSlot, FlowSlot and DegradeSlot and the
 * StatisticSlot accounting on the GPU in one event; the "post" chain (slots sorted after DegradeSlot) runs only
 * for an entry the engine passed, as in the reference.  A BlockException from the pre chain is counted as a block
 * (event kind 2) and rethrown; one from the post chain revokes the engine's pass (event kind 3: pass, thread and
 * parameter thread counts undone, the block counted) and is rethrown; an engine block becomes the reference's
 * exception with the blocking rule ({@link GpuRuleSync} keeps the per-resource lists in engine order), and its
 * block error is set on the entry so that exit records nothing.  Passes sleep the engine's wait (RateLimiter
 * pacing, cluster SHOULD_WAIT, parameter throttle) as the reference controllers do before returning.
 */
public class GpuStatisticSlot extends AbstractLinkedProcessorSlot<DefaultNode> {

    private static final Map<String, Integer> RESOURCE_IDS = new ConcurrentHashMap<>();
    private static final List<String> NAMES = new ArrayList<>();
    private final long engine = GpuEngine.get();
    private final ProcessorSlotChain pre, post;

    public GpuStatisticSlot() {
        this(new DefaultProcessorSlotChain(), new DefaultProcessorSlotChain());
    }

    GpuStatisticSlot(ProcessorSlotChain pre, ProcessorSlotChain post) {
        this.pre = pre;
        this.post = post;
    }

    /** Dense resource id of a resource name (like CtSph's chain map); at most csp.sentinel.gpu.maxResources. */
    static int resourceId(String name) {
        Integer id = RESOURCE_IDS.get(name);
        if (id != null) {
            return id;
        }
        synchronized (NAMES) {
            id = RESOURCE_IDS.get(name);
            if (id == null) {
                if (NAMES.size() >= GpuEngine.MAX_RESOURCES) {
                    throw new IllegalStateException("more than " + GpuEngine.MAX_RESOURCES + " resources "
                                                    + "(csp.sentinel.gpu.maxResources)");
                }
                id = NAMES.size();
                NAMES.add(name);
                RESOURCE_IDS.put(name, id);
            }
            return id;
        }
    }

    /** The name of a dense resource id (metric rows), or null. */
    static String resourceName(int id) {
        synchronized (NAMES) {
            return id >= 0 && id < NAMES.size() ? NAMES.get(id) : null;
        }
    }

    private static int flags(ResourceWrapper r, boolean prioritized) {
        return (prioritized ? GpuEngine.EV_PRIORITIZED : 0) | (r.getEntryType() == EntryType.IN ? GpuEngine.EV_INBOUND : 0);
    }

    @Override
    public void entry(Context context, ResourceWrapper resourceWrapper, DefaultNode node, int count,
                      boolean prioritized, Object... args) throws Throwable {
        final String name = resourceWrapper.getName();
        final int rid = resourceId(name);
        final int fl = flags(resourceWrapper, prioritized);
        try {
            // StatisticSlot.java:71: the checks before the engine's (AuthoritySlot, custom slots sorted before DegradeSlot)
            pre.entry(context, resourceWrapper, node, count, prioritized, args);
        } catch (BlockException e) {
            // StatisticSlot.java:121-135: the block is counted (node + ENTRY_NODE when inbound)
            context.getCurEntry().setBlockError(e);
            GpuEngine.blocked(engine, rid, TimeUtil.currentTimeMillis(), count, fl);
            throw e;
        }
        long[] words = GpuArgs.encode(args);
        int[] o = new int[2];
        final long now = TimeUtil.currentTimeMillis();
        int rc = GpuEngine.entryArgs(engine, rid, now, count, fl, words, args == null ? 0 : args.length, o);
        if (rc != GpuEngine.OK) {
            throw new IllegalStateException("sga_submit_events: " + rc + " " + GpuEngine.lastError(engine));
        }
        BlockException block;
        switch (o[0]) {
            case 0:  // passed; RateLimiter / SHOULD_WAIT / throttle waits sleep like the controllers
                if (o[1] > 0) {
                    TimeUnit.MILLISECONDS.sleep(o[1]);
                }
                try {  // the slots sorted after DegradeSlot, which the reference reaches only on a pass
                    post.entry(context, resourceWrapper, node, count, prioritized, args);
                } catch (BlockException e) {
                    // the reference counts no pass and no thread for it (StatisticSlot.java:71-84 run after
                    // fireEntry) but a block (:121-135): the revoke event undoes the engine's pass accounting
                    // (node, ENTRY_NODE, parameter thread counts) and counts the block, at the entry's time
                    context.getCurEntry().setBlockError(e);
                    GpuEngine.revokedArgs(engine, rid, now, count, fl, words, args == null ? 0 : args.length);
                    throw e;
                }
                fireEntry(context, resourceWrapper, node, count, prioritized, args);
                return;
            case 4:  // PriorityWaitException (FlowSlot): DefaultController slept; StatisticSlot counted a thread
                     // and returned -- no slot after FlowSlot sees the entry (StatisticSlot.java:86-100)
                if (o[1] > 0) {
                    TimeUnit.MILLISECONDS.sleep(o[1]);
                }
                return;
            case 1: {
                FlowRule r = GpuRuleSync.flowRule(name, o[1]);
                block = new FlowException(r != null ? r.getLimitApp() : RuleConstant.LIMIT_APP_DEFAULT, r);
                break;
            }
            case 2: {
                ParamFlowRule r = GpuRuleSync.paramRule(name, o[1]);
                Object v = null;
                if (r != null && args != null && r.getParamIdx() != null && r.getParamIdx() >= 0
                    && r.getParamIdx() < args.length) {
                    v = args[r.getParamIdx()];
                }
                block = new ParamFlowException(name, v == null ? "" : String.valueOf(v), r);
                break;
            }
            case 3: {
                DegradeRule r = GpuRuleSync.degradeRule(name, o[1]);
                block = new DegradeException(r != null ? r.getLimitApp() : RuleConstant.LIMIT_APP_DEFAULT, r);
                break;
            }
            case 5:
                block = new SystemBlockException(name, SYSTEM_LIMIT_TYPES[Math.min(Math.max(o[1], 0), 4)]);
                break;
            default:
                throw new IllegalStateException("unknown decision " + o[0]);
        }
        context.getCurEntry().setBlockError(block);  // exit then records nothing (StatisticSlot.java:150)
        throw block;
    }

    /** SystemRuleManager.checkSystem's limitType of each check (block detail 0..4). */
    private static final String[] SYSTEM_LIMIT_TYPES = {"qps", "thread", "rt", "load", "cpu"};

    @Override
    public void exit(Context context, ResourceWrapper resourceWrapper, int count, Object... args) {
        if (context.getCurEntry().getBlockError() == null) {  // StatisticSlot.exit: only entries that passed
            long now = TimeUtil.currentTimeMillis();
            long rt = now - context.getCurEntry().getCreateTimestamp();
            int fl = flags(resourceWrapper, false) | (context.getCurEntry().getError() != null ? GpuEngine.EV_ERROR : 0);
            GpuEngine.exitArgs(engine, resourceId(resourceWrapper.getName()), now, count, fl, rt,
                               GpuArgs.encode(args), args == null ? 0 : args.length);
        }
        // StatisticSlot.exit accounts first, then the later slots' exits in chain order
        pre.exit(context, resourceWrapper, count, args);
        post.exit(context, resourceWrapper, count, args);
        fireExit(context, resourceWrapper, count, args);
    }
}
