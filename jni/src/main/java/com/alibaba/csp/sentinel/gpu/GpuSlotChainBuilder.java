package com.alibaba.csp.sentinel.gpu;

import java.util.List;

import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.DefaultProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.SlotChainBuilder;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeSlot;
import com.alibaba.csp.sentinel.slots.block.flow.FlowSlot;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowSlot;
import com.alibaba.csp.sentinel.slots.statistic.StatisticSlot;
import com.alibaba.csp.sentinel.slots.system.SystemSlot;
import com.alibaba.csp.sentinel.spi.Spi;
import com.alibaba.csp.sentinel.spi.SpiLoader;

/**
 * {@link SlotChainBuilder} (SlotChainProvider.java:28-60 resolves the first SPI instance) that builds the
 * default SPI-sorted chain (DefaultSlotChainBuilder) but puts one {@link GpuStatisticSlot} where
 * StatisticSlot was and drops the slots the engine runs: SystemSlot, ParamFlowSlot, FlowSlot, DegradeSlot.
 * NodeSelectorSlot, ClusterBuilderSlot and LogSlot stay in front of it.  The slots sorted between
 * StatisticSlot and DegradeSlot (AuthoritySlot, custom slots ordered before -1000) become the GPU slot's
 * "pre" chain, fired before the engine decides; the slots sorted after DegradeSlot become its "post" chain,
 * fired only when the engine passed the entry -- the reference's order (a custom slot after DegradeSlot runs
 * only once System / ParamFlow / Flow / Degrade have passed).  A custom slot sorted between SystemSlot and
 * DegradeSlot cannot run between the engine's checks (the engine decides them in one event): it runs before
 * all of them.  The engine's rules arrive through {@link GpuRuleSync#install()}, called here, so no rule
 * manager is left without a path into the engine; {@link GpuMetricTimerListener} writes the metric log from
 * the engine.
 */
@Spi(order = -100)
public class GpuSlotChainBuilder implements SlotChainBuilder {

    @Override
    public ProcessorSlotChain build() {
        GpuRuleSync.install();
        ProcessorSlotChain chain = new DefaultProcessorSlotChain();
        ProcessorSlotChain pre = new DefaultProcessorSlotChain(), post = new DefaultProcessorSlotChain();
        List<ProcessorSlot> sorted = SpiLoader.of(ProcessorSlot.class).loadInstanceListSorted();
        int phase = 0;  // 0 before StatisticSlot, 1 up to DegradeSlot, 2 after it
        for (ProcessorSlot slot : sorted) {
            if (!(slot instanceof AbstractLinkedProcessorSlot)) {
                continue;
            }
            if (slot instanceof StatisticSlot) {
                chain.addLast(new GpuStatisticSlot(pre, post));
                phase = Math.max(phase, 1);
            } else if (slot instanceof DegradeSlot) {
                phase = 2;  // decided by the engine inside GpuStatisticSlot
            } else if (slot instanceof ParamFlowSlot || slot instanceof FlowSlot || slot instanceof SystemSlot) {
                continue;  // decided by the engine inside GpuStatisticSlot
            } else if (phase == 0) {
                chain.addLast((AbstractLinkedProcessorSlot<?>) slot);
            } else if (phase == 1) {
                pre.addLast((AbstractLinkedProcessorSlot<?>) slot);
            } else {
                post.addLast((AbstractLinkedProcessorSlot<?>) slot);
            }
        }
        return chain;
    }
}
