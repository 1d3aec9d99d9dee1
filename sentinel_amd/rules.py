"""Rule entities of the decision path, with the reference's field names and defaults.

  FlowRule         CORE/slots/block/flow/FlowRule.java:52-95 (+ ClusterFlowConfig, CORE/slots/block/flow/ClusterFlowConfig.java:34-74)
  ParamFlowRule    PF/slots/block/flow/param/ParamFlowRule.java:45-83, ParamFlowItem.java:28-40,
                   ParamFlowClusterConfig.java:32-44
  DegradeRule      CORE/slots/block/degrade/DegradeRule.java:59-84
  RuleConstant     CORE/slots/block/RuleConstant.java:24-61
"""
from dataclasses import dataclass, field
from typing import List, Optional


class RuleConstant:
    FLOW_GRADE_THREAD = 0
    FLOW_GRADE_QPS = 1
    DEGRADE_GRADE_RT = 0
    DEGRADE_GRADE_EXCEPTION_RATIO = 1
    DEGRADE_GRADE_EXCEPTION_COUNT = 2
    DEGRADE_DEFAULT_SLOW_REQUEST_AMOUNT = 5
    DEGRADE_DEFAULT_MIN_REQUEST_AMOUNT = 5
    STRATEGY_DIRECT = 0
    STRATEGY_RELATE = 1
    STRATEGY_CHAIN = 2
    CONTROL_BEHAVIOR_DEFAULT = 0
    CONTROL_BEHAVIOR_WARM_UP = 1
    CONTROL_BEHAVIOR_RATE_LIMITER = 2
    CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER = 3
    LIMIT_APP_DEFAULT = "default"


class ClusterRuleConstant:
    FLOW_CLUSTER_STRATEGY_NORMAL = 0
    FLOW_THRESHOLD_AVG_LOCAL = 0
    FLOW_THRESHOLD_GLOBAL = 1
    DEFAULT_CLUSTER_SAMPLE_COUNT = 10


@dataclass
class ClusterFlowConfig:
    flow_id: Optional[int] = None
    threshold_type: int = ClusterRuleConstant.FLOW_THRESHOLD_AVG_LOCAL
    sample_count: int = ClusterRuleConstant.DEFAULT_CLUSTER_SAMPLE_COUNT
    window_interval_ms: int = 1000
    strategy: int = ClusterRuleConstant.FLOW_CLUSTER_STRATEGY_NORMAL
    resource_timeout: int = 2000     # ClusterFlowConfig.resourceTimeout (concurrency tokens)
    client_offline_time: int = 2000  # ClusterFlowConfig.clientOfflineTime
    fallback_to_local_when_fail: bool = True  # ClusterFlowConfig.fallbackToLocalWhenFail


@dataclass
class FlowRule:
    resource: str = ""
    count: float = 0.0
    grade: int = RuleConstant.FLOW_GRADE_QPS
    limit_app: str = RuleConstant.LIMIT_APP_DEFAULT
    strategy: int = RuleConstant.STRATEGY_DIRECT
    control_behavior: int = RuleConstant.CONTROL_BEHAVIOR_DEFAULT
    warm_up_period_sec: int = 10
    max_queueing_time_ms: int = 500
    cluster_mode: bool = False
    cluster_config: ClusterFlowConfig = field(default_factory=ClusterFlowConfig)


@dataclass
class ParamFlowItem:
    object: object = None
    count: int = 0
    class_type: str = "int"


@dataclass
class ParamFlowClusterConfig:
    """PF/slots/block/flow/param/ParamFlowClusterConfig.java:32-44"""
    flow_id: Optional[int] = None
    threshold_type: int = ClusterRuleConstant.FLOW_THRESHOLD_AVG_LOCAL
    fallback_to_local_when_fail: bool = False
    sample_count: int = ClusterRuleConstant.DEFAULT_CLUSTER_SAMPLE_COUNT
    window_interval_ms: int = 1000


@dataclass
class ParamFlowRule:
    resource: str = ""
    grade: int = RuleConstant.FLOW_GRADE_QPS
    param_idx: int = 0
    count: float = 0.0
    control_behavior: int = RuleConstant.CONTROL_BEHAVIOR_DEFAULT
    max_queueing_time_ms: int = 0
    burst_count: int = 0
    duration_in_sec: int = 1
    param_flow_item_list: List[ParamFlowItem] = field(default_factory=list)
    cluster_mode: bool = False
    cluster_config: Optional[ParamFlowClusterConfig] = None


@dataclass
class DegradeRule:
    resource: str = ""
    grade: int = RuleConstant.DEGRADE_GRADE_RT
    count: float = 0.0
    time_window: int = 0
    min_request_amount: int = RuleConstant.DEGRADE_DEFAULT_MIN_REQUEST_AMOUNT
    slow_ratio_threshold: float = 1.0
    stat_interval_ms: int = 1000
