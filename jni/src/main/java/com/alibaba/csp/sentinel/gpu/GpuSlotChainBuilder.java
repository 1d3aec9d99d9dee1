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
 * NodeSelectorSlot, ClusterBuilderSlot, LogSlot and AuthoritySlot stay; GpuStatisticSlot fires AuthoritySlot
 * (and any custom slot) before the engine decides, as StatisticSlot fires the checks before accounting.
 * The engine's rules arrive through {@link GpuRuleSync#install()}, called here, so no rule manager is left
 * without a path into the engine; {@link GpuMetricTimerListener} writes the metric log from the engine.
 */
@Spi(order = -100)
public class GpuSlotChainBuilder implements SlotChainBuilder {

    @Override
    public ProcessorSlotChain build() {
        GpuRuleSync.install();
        ProcessorSlotChain chain = new DefaultProcessorSlotChain();
        List<ProcessorSlot> sorted = SpiLoader.of(ProcessorSlot.class).loadInstanceListSorted();
        for (ProcessorSlot slot : sorted) {
            if (!(slot instanceof AbstractLinkedProcessorSlot)) {
                continue;
            }
            if (slot instanceof StatisticSlot) {
                chain.addLast(new GpuStatisticSlot());
            } else if (slot instanceof ParamFlowSlot || slot instanceof FlowSlot || slot instanceof DegradeSlot
                       || slot instanceof SystemSlot) {
                continue;  // decided by the engine inside GpuStatisticSlot
            } else {
                chain.addLast((AbstractLinkedProcessorSlot<?>) slot);
            }
        }
        return chain;
    }
}
