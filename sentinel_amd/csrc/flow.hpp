// Local flow path (StatisticSlot + FlowSlot controllers) -- device engine.
#pragma once
#include "../../include/sentinel_amd.h"
#include "common.hpp"

namespace sga {

struct FlowEngine {
    void init(const sga_config &, hipStream_t) {}
    void release() {}
};

}  // namespace sga
