"""Host-side mirror of the reference's local (in-process) decision path.

Same names and argument meaning as the Java API the engine replaces:
  SphU.entry(resource, EntryType, batchCount, args...)  CORE/SphU.java:84-208  -> LocalSentinel.entry / submit
  Entry.exit(count, args...)                              CORE/Entry.java:86-111  -> Entry.exit
  Tracer.traceEntry(Throwable, Entry)                     CORE/Tracer.java:86-110 -> Entry.trace_error
  FlowRuleManager.loadRules       CORE/slots/block/flow/FlowRuleManager.java:125-127
  ParamFlowRuleManager.loadRules  PF/slots/block/flow/param/ParamFlowRuleManager.java:52
  DegradeRuleManager.loadRules    CORE/slots/block/degrade/DegradeRuleManager.java:108
  SystemRuleManager.loadRules     CORE/slots/system/SystemRuleManager.java:114-300 (SystemSlot, inbound only)
  Constants.ENTRY_NODE            CORE/Constants.java:66 -> LocalSentinel.node(ENTRY_NODE), metrics rows
  ClusterNode statistics          CORE/node/StatisticNode.java:185-250 -> LocalSentinel.node
BlockException subclasses as in CORE/slots/block/BlockException.java and its subclasses.

Every decision is computed by the HIP engine (libsentinel_amd.so).  The mocked
TimeUtil clock of the reference tests is the explicit `now` / `ts` argument.
Resources are registered up front (dense ids), like CtSph's chain map keys.
"""
import ctypes as C
import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import SgaDegradeRule, SgaFlowRule, SgaNodeView, SgaParamRule, check
from .cluster import Engine  # noqa: F401  (one engine serves both paths)
from .rules import DegradeRule, FlowRule, ParamFlowRule, RuleConstant  # noqa: F401


class Decision:
    PASS = 0
    BLOCK_FLOW = 1
    BLOCK_PARAM = 2
    BLOCK_DEGRADE = 3
    PASS_WAIT = 4
    BLOCK_SYSTEM = 5


EV_PRIORITIZED = 1
EV_ERROR = 2
EV_HAS_PARAM = 4
EV_INBOUND = 8          # EntryType.IN
EV_PARAM_LIST = 16      # args[0] is a Collection / array (param = offset << 32 | count into param_values)
EV_ARGS = 32            # the whole argument vector (param = offset << 32 | nargs into param_values)
ARG_SCALAR, ARG_NULL, ARG_LIST = 0, 1, 2
ENTRY_NODE = 0xFFFFFFFF  # resource id of Constants.ENTRY_NODE
TOTAL_IN_RESOURCE_NAME = "__total_inbound_traffic__"  # Constants.TOTAL_IN_RESOURCE_NAME
KIND_ENTRY = 0
KIND_EXIT = 1


class BlockException(Exception):
    def __init__(self, resource: str):
        super().__init__(resource)
        self.resource = resource


class FlowException(BlockException):
    pass


class ParamFlowException(BlockException):
    pass


class DegradeException(BlockException):
    pass


class SystemBlockException(BlockException):
    pass


_EXC = {Decision.BLOCK_FLOW: FlowException, Decision.BLOCK_PARAM: ParamFlowException,
        Decision.BLOCK_DEGRADE: DegradeException, Decision.BLOCK_SYSTEM: SystemBlockException}


def param_value(x) -> int:
    """64-bit key of a hot parameter (ParameterMetric maps compare args[idx] by equals()).

    Integral values (Java byte/short/int/long, boolean) map to their two's-complement
    long bits, floats to their IEEE-754 bits, strings to a 64-bit hash of the UTF-8 bytes
    (distinct strings that collide would share a counter: documented divergence)."""
    if isinstance(x, bool):
        return 1 if x else 0
    if isinstance(x, (int, np.integer)):
        return int(x) & 0xFFFFFFFFFFFFFFFF
    if isinstance(x, (float, np.floating)):
        return struct.unpack("<Q", struct.pack("<d", float(x)))[0]
    if isinstance(x, str):
        import xxhash
        return xxhash.xxh64_intdigest(x.encode("utf-8"), seed=0x5E47)
    raise TypeError(f"unsupported parameter type {type(x).__name__}")


def encode_args(args, pvals: List[int]) -> int:
    """SGA_EV_ARGS encoding of SphU.entry's `Object... args` appended to `pvals` (include/sentinel_amd.h):
    two words per argument -- kind << 62 | list length, then the scalar's key or the offset of the
    list's elements in pvals.  None is a null argument; a list / tuple is a Collection or array (its
    elements in iteration order; ParamFlowChecker.passLocalCheck checks every one).  Returns the event's
    param word, offset << 32 | nargs."""
    off = len(pvals)
    pvals.extend([0] * (2 * len(args)))
    for k, a in enumerate(args):
        if a is None:
            pvals[off + 2 * k] = ARG_NULL << 62
        elif isinstance(a, (list, tuple)):
            vals = [param_value(x) for x in a]
            pvals[off + 2 * k] = (ARG_LIST << 62) | len(vals)
            pvals[off + 2 * k + 1] = len(pvals)
            pvals.extend(vals)
        else:
            pvals[off + 2 * k] = ARG_SCALAR << 62
            pvals[off + 2 * k + 1] = param_value(a)
    return (off << 32) | len(args)


@dataclass
class NodeView:
    pass_qps: float
    block_qps: float
    success_qps: float
    exception_qps: float
    occupied_pass_qps: float
    avg_rt: float
    min_rt: float
    previous_pass_qps: float
    total_pass: int
    total_block: int
    total_success: int
    total_exception: int
    cur_thread_num: int
    waiting: int
    max_success_qps: float
    previous_block_qps: float


@dataclass
class MetricNode:
    """CORE/node/metric/MetricNode.java:28-51 (one resource, one second)."""
    timestamp: int
    resource: str
    pass_qps: int
    block_qps: int
    success_qps: int
    exception_qps: int
    rt: int
    occupied_pass_qps: int
    concurrency: int = 0
    classification: int = 0

    def to_thin_string(self) -> str:
        """MetricNode.toThinString (:160-176): the metric log line the dashboard reads."""
        return "|".join(str(x) for x in (self.timestamp, self.resource.replace("|", "_"), self.pass_qps,
                                         self.block_qps, self.success_qps, self.exception_qps, self.rt,
                                         self.occupied_pass_qps, self.concurrency, self.classification))


class Entry:
    """A passed entry; exit() records RT / success (StatisticSlot.exit) and breaker completion."""

    def __init__(self, owner: "LocalSentinel", rid: int, create_ts: int, count: int, param: Optional[int],
                 wait_ms: int, inbound: bool = False, args=()):
        self._owner = owner
        self.args = tuple(args)
        self.inbound = inbound
        self.rid = rid
        self.create_timestamp = create_ts
        self.count = count
        self.param = param
        self.wait_ms = wait_ms
        self.error = False
        self.exited = False

    def trace_error(self):
        self.error = True

    def exit(self, now: int):
        if self.exited:
            return
        self.exited = True
        # Entry.exit(count, args): ParamFlowStatisticExitCallback decreases the thread counts of the args
        pvals: List[int] = []
        word = encode_args(self.args, pvals)
        fl = (EV_ERROR if self.error else 0) | EV_ARGS | (EV_INBOUND if self.inbound else 0)
        self._owner.submit([KIND_EXIT], [self.rid], [now], [self.count], [fl], [now - self.create_timestamp],
                           [word], pvals)


class LocalSentinel:
    """The local slot chain (StatisticSlot, ParamFlowSlot, FlowSlot, DegradeSlot) on one engine."""

    def __init__(self, engine: Engine, resources: Sequence[str]):
        self.engine = engine
        self.resources: List[str] = list(resources)
        self.ids: Dict[str, int] = {r: i for i, r in enumerate(self.resources)}
        if len(self.ids) != len(self.resources):
            raise ValueError("duplicate resource names")
        check(_lib.load().sga_flow_set_resources(engine.handle, len(self.resources)), engine.handle, "setResources")

    def resource_id(self, name: str) -> int:
        return self.ids[name]

    # ---- batched form: the engine's native interface
    def submit(self, kind, resource, ts, acquire, flags=None, rt=None, param=None, param_values=None):
        """Events in arrival order.  param_values: the values of Collection / array arguments
        (events flagged SGA_EV_PARAM_LIST = 16 carry param = offset << 32 | count into it)."""
        k = np.ascontiguousarray(kind, dtype=np.uint8)
        r = np.ascontiguousarray(resource, dtype=np.uint32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        a = np.ascontiguousarray(acquire, dtype=np.int32)
        n = len(k)
        if not (len(r) == len(t) == len(a) == n):
            raise ValueError("event arrays differ in length")
        f = np.ascontiguousarray(flags, dtype=np.uint8) if flags is not None else None
        rtv = np.ascontiguousarray(rt, dtype=np.int64) if rt is not None else None
        pv = np.ascontiguousarray(param, dtype=np.uint64) if param is not None else None
        for x in (f, rtv, pv):
            if x is not None and len(x) != n:
                raise ValueError("event arrays differ in length")
        dec = np.zeros(n, dtype=np.int8)
        wait = np.zeros(n, dtype=np.int32)
        vals = np.ascontiguousarray(param_values, dtype=np.uint64) if param_values is not None else None
        rc = _lib.load().sga_submit_events_ex(
            self.engine.handle, k.ctypes.data, r.ctypes.data, t.ctypes.data, a.ctypes.data,
            f.ctypes.data if f is not None else None, rtv.ctypes.data if rtv is not None else None,
            pv.ctypes.data if pv is not None else None, n,
            vals.ctypes.data if vals is not None and len(vals) else None, len(vals) if vals is not None else 0,
            dec.ctypes.data, wait.ctypes.data)
        check(rc, self.engine.handle, "submitEvents")
        return dec, wait

    # ---- one event at a time through the coalescing queue (sga_event_submit / sga_event_poll): what a
    # synchronous SphU.entry / Entry.exit of one application thread calls; concurrent callers share a batch
    def event_submit(self, kind, resource, ts, acquire, flags=0, rt=0, param=0, param_values=None) -> int:
        """Enqueue one event (kind, flags, param as in submit; param_values: this event's argument words only).
        Returns a ticket for event_poll."""
        pv = None if param_values is None else np.ascontiguousarray(param_values, dtype=np.uint64)
        t = C.c_uint64()
        rc = _lib.load().sga_event_submit(self.engine.handle, int(kind), int(resource), int(ts), int(acquire),
                                          int(flags), int(rt), int(param), pv.ctypes.data if pv is not None else None,
                                          0 if pv is None else len(pv), C.byref(t))
        check(rc, self.engine.handle, "eventSubmit")
        return int(t.value)

    def event_poll(self, ticket):
        """(decision, wait_ms) once the ticket's event is decided (each ticket answers once), else None."""
        d, w = C.c_int8(), C.c_int32()
        rc = _lib.load().sga_event_poll(self.engine.handle, int(ticket), C.byref(d), C.byref(w))
        if rc == -11:  # SGA_EAGAIN
            return None
        check(rc, self.engine.handle, "eventPoll")
        return int(d.value), int(w.value)

    def event_post(self, kind, resource, ts, acquire, flags=0, rt=0, param=0, param_values=None) -> int:
        """Queue an exit / block / revoke (kinds 1-3) without waiting (sga_event_post): decided in ticket order
        before anything queued or called later.  Returns its ticket (~0: decided on its own)."""
        pv = None if param_values is None else np.ascontiguousarray(param_values, dtype=np.uint64)
        t = C.c_uint64()
        rc = _lib.load().sga_event_post(self.engine.handle, int(kind), int(resource), int(ts), int(acquire), int(flags),
                                        int(rt), int(param), pv.ctypes.data if pv is not None else None,
                                        0 if pv is None else len(pv), C.byref(t))
        check(rc, self.engine.handle, "eventPost")
        return int(t.value)

    def event_one(self, kind, resource, ts, acquire, flags=0, rt=0, param=0, param_values=None):
        """event_submit + event_poll until decided: (decision, wait_ms)."""
        pv = None if param_values is None else np.ascontiguousarray(param_values, dtype=np.uint64)
        d, w = C.c_int8(), C.c_int32()
        rc = _lib.load().sga_event_one(self.engine.handle, int(kind), int(resource), int(ts), int(acquire), int(flags),
                                       int(rt), int(param), pv.ctypes.data if pv is not None else None,
                                       0 if pv is None else len(pv), C.byref(d), C.byref(w))
        check(rc, self.engine.handle, "eventOne")
        return int(d.value), int(w.value)

    def submit_device(self, kind, resource, ts_base, ts_off, acquire, flags=None, rt=None, param=None,
                      param_values=None, decision=None, wait=None, stream=None):
        """submit over device tensors (torch, on the engine's GPU), asynchronous on `stream` (torch stream or
        None = the engine stream): one chunk of at most max_batch events with timestamps ts_base + ts_off.
        Returns (decision int8, wait int32) device tensors; device_status() reports a chunk the device
        checks rejected (rc -EINVAL) or a full parameter map (rc -ENOMEM) as EngineError."""
        import torch
        n = kind.numel()
        for x in (resource, ts_off, acquire) + tuple(v for v in (flags, rt, param) if v is not None):
            if x.numel() != n or not x.is_cuda or not x.is_contiguous():
                raise ValueError("event tensors must be contiguous device tensors of one length")
        want = {"kind": (kind, torch.uint8), "resource": (resource, torch.int32), "ts_off": (ts_off, torch.int32),
                "acquire": (acquire, torch.int32), "flags": (flags, torch.uint8), "rt": (rt, torch.int64),
                "param": (param, torch.int64), "param_values": (param_values, torch.int64)}
        for name, (x, dt) in want.items():
            if x is not None and x.element_size() != torch.empty(0, dtype=dt).element_size():
                raise ValueError(f"{name}: element size of {dt} expected")
        if decision is None:
            decision = torch.empty(n, dtype=torch.int8, device=kind.device)
        if wait is None:
            wait = torch.empty(n, dtype=torch.int32, device=kind.device)
        ptr = (lambda x: x.data_ptr() if x is not None else None)
        rc = _lib.load().sga_submit_events_device(
            self.engine.handle, kind.data_ptr(), resource.data_ptr(), int(ts_base), ts_off.data_ptr(),
            acquire.data_ptr(), ptr(flags), ptr(rt), ptr(param), n, ptr(param_values),
            param_values.numel() if param_values is not None else 0, decision.data_ptr(), wait.data_ptr(),
            stream.cuda_stream if stream is not None else None)
        check(rc, self.engine.handle, "submitEventsDevice")
        return decision, wait

    def device_status(self):
        """Waits for the engine stream; EngineError for a rejected device chunk or a full parameter map."""
        check(_lib.load().sga_events_device_status(self.engine.handle), self.engine.handle, "submitEventsDevice")

    # ---- SphU-style single entry
    def entry(self, resource: str, now: int, batch_count: int = 1, prioritized: bool = False, args=(),
              entry_type: str = "OUT") -> Entry:
        """SphU.entry(resource, entryType, batchCount, args); entry_type "IN" marks inbound traffic."""
        rid = self.ids[resource]
        inbound = entry_type == "IN"
        # the whole argument vector (SGA_EV_ARGS): ParamFlowSlot indexes args by each rule's paramIdx
        pvals: List[int] = []
        word = encode_args(tuple(args), pvals)
        fl = (EV_PRIORITIZED if prioritized else 0) | EV_ARGS | (EV_INBOUND if inbound else 0)
        dec, wait = self.submit([KIND_ENTRY], [rid], [now], [batch_count], [fl], None, [word], pvals)
        d = int(dec[0])
        if d in _EXC:
            raise _EXC[d](resource)
        param = param_value(args[0]) if len(args) > 0 and args[0] is not None and \
            not isinstance(args[0], (list, tuple)) else None
        return Entry(self, rid, now, batch_count, param, int(wait[0]), inbound, args)

    def node(self, resource, now: int) -> NodeView:
        """ClusterNode views; resource ENTRY_NODE (or TOTAL_IN_RESOURCE_NAME) is Constants.ENTRY_NODE."""
        if resource == TOTAL_IN_RESOURCE_NAME:
            resource = ENTRY_NODE
        rid = resource if isinstance(resource, int) else self.ids[resource]
        v = SgaNodeView()
        check(_lib.load().sga_query_node(self.engine.handle, rid, now, C.byref(v)), self.engine.handle, "node")
        return NodeView(*[getattr(v, f) for f, _ in SgaNodeView._fields_])

    def metrics(self, now: int, cap: int = 1 << 16) -> List[MetricNode]:
        """MetricTimerListener.run (CORE/node/metric/MetricTimerListener.java:44-65): StatisticNode.metrics()
        of every resource at `now`, ordered by timestamp then resource (the TreeMap the reference writes)."""
        buf = (_lib.SgaMetricNode * max(1, cap))()
        n = C.c_size_t()
        rc = _lib.load().sga_metrics_snapshot(self.engine.handle, now, buf, cap, C.byref(n))
        _lib.check(rc, self.engine.handle, "metrics")
        def name(r):
            return TOTAL_IN_RESOURCE_NAME if r == ENTRY_NODE else self.resources[r]

        out = [MetricNode(b.timestamp, name(b.resource), b.pass_qps, b.block_qps, b.success_qps,
                          b.exception_qps, b.rt, b.occupied_pass_qps, b.concurrency)
               for b in buf[:n.value]]
        out.sort(key=lambda m: (m.timestamp, self.ids.get(m.resource, ENTRY_NODE)))
        return out

    def circuit_breaker_state(self, resource, k: int = 0) -> int:
        rid = resource if isinstance(resource, int) else self.ids[resource]
        return _lib.load().sga_circuit_breaker_state(self.engine.handle, rid, k)


class ClusterStateManager:
    """ClusterStateManager (CORE/cluster/ClusterStateManager.java) as the local path sees it:
    CLUSTER_SERVER = the embedded token server is this engine (sga_set_cluster_server 1);
    CLUSTER_NOT_STARTED = no token service, cluster-mode rules fall back.  The client mode (a
    remote token server over the network) is outside the decision path."""
    CLUSTER_NOT_STARTED, CLUSTER_SERVER = 0, 1

    def __init__(self, sentinel: "LocalSentinel"):
        self.s = sentinel

    def set_to_server(self):
        check(_lib.load().sga_set_cluster_server(self.s.engine.handle, 1), self.s.engine.handle, "setToServer")

    def stop(self):
        check(_lib.load().sga_set_cluster_server(self.s.engine.handle, 0), self.s.engine.handle, "stop")


class FlowRuleManager:
    def __init__(self, sentinel: LocalSentinel):
        self.s = sentinel

    def load_rules(self, rules: List[FlowRule]) -> int:
        """FlowRuleManager.loadRules.  Cluster-mode rules ask the token service when checked
        (FlowRuleChecker.passClusterCheck): with ClusterStateManager set to server the engine's own
        cluster rules (ClusterFlowRuleManager on the same Engine) decide their flowId, otherwise
        they fall back (fallbackToLocalWhenFail: the local rater, else pass)."""
        rules = [r for r in rules if r.resource in self.s.ids]
        arr = (SgaFlowRule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            a = arr[i]
            a.resource = self.s.ids[r.resource]
            a.grade = r.grade
            a.count = r.count
            a.control_behavior = r.control_behavior
            a.warm_up_period_sec = r.warm_up_period_sec
            a.max_queueing_time_ms = r.max_queueing_time_ms
            # non-default limitApp / RELATE / CHAIN are not served by the engine: rejected as invalid
            a.strategy = r.strategy if r.limit_app == RuleConstant.LIMIT_APP_DEFAULT else -1
            if r.cluster_mode:
                cc = r.cluster_config
                a.cluster_mode = 1
                a.cluster_fallback = 1 if cc is None or cc.fallback_to_local_when_fail else 0
                a.cluster_flow_id = -1 if cc is None or cc.flow_id is None else int(cc.flow_id)
                a.cluster_sample_count = 0 if cc is None else cc.sample_count
                a.cluster_window_ms = 0 if cc is None else cc.window_interval_ms
                a.cluster_strategy = 0 if cc is None else cc.strategy
        return check(_lib.load().sga_load_flow_rules(self.s.engine.handle, arr, len(rules)), self.s.engine.handle,
                     "FlowRuleManager.loadRules")


class ParamFlowRuleManager:
    def __init__(self, sentinel: LocalSentinel):
        self.s = sentinel
        self._keep = []

    def load_rules(self, rules: List[ParamFlowRule]) -> int:
        rules = [r for r in rules if r.resource in self.s.ids]
        arr = (SgaParamRule * max(1, len(rules)))()
        keep = []
        for i, r in enumerate(rules):
            a = arr[i]
            a.resource = self.s.ids[r.resource]
            a.grade = r.grade
            a.count = r.count
            a.control_behavior = r.control_behavior
            a.max_queueing_time_ms = r.max_queueing_time_ms
            a.burst_count = r.burst_count
            a.param_idx = r.param_idx
            a.duration_in_sec = r.duration_in_sec
            if r.cluster_mode:  # ParamFlowRule.clusterMode + ParamFlowClusterConfig
                cc = r.cluster_config
                a.cluster_mode = 1
                a.cluster_flow_id = cc.flow_id if cc and cc.flow_id is not None else 0
                a.cluster_fallback = 1 if cc and cc.fallback_to_local_when_fail else 0
                a.cluster_sample_count = cc.sample_count if cc else 0
                a.cluster_window_ms = cc.window_interval_ms if cc else 0
            # ParamFlowRuleUtil.parseHotItems: later items with the same value win
            hot: Dict[int, int] = {}
            for it in r.param_flow_item_list:
                hot[param_value(it.object)] = int(it.count)
            hv = (C.c_uint64 * max(1, len(hot)))(*hot.keys())
            ht = (C.c_int32 * max(1, len(hot)))(*hot.values())
            keep += [hv, ht]
            a.n_hot = len(hot)
            a.hot_values = C.cast(hv, C.POINTER(C.c_uint64))
            a.hot_thresholds = C.cast(ht, C.POINTER(C.c_int32))
        rc = _lib.load().sga_load_param_rules(self.s.engine.handle, arr, len(rules))
        self._keep = keep
        return check(rc, self.s.engine.handle, "ParamFlowRuleManager.loadRules")


class DegradeRuleManager:
    def __init__(self, sentinel: LocalSentinel):
        self.s = sentinel

    def load_rules(self, rules: List[DegradeRule]) -> int:
        rules = [r for r in rules if r.resource in self.s.ids]
        arr = (SgaDegradeRule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            a = arr[i]
            a.resource = self.s.ids[r.resource]
            a.grade = r.grade
            a.count = r.count
            a.time_window = r.time_window
            a.min_request_amount = r.min_request_amount
            a.slow_ratio_threshold = r.slow_ratio_threshold
            a.stat_interval_ms = r.stat_interval_ms
        return check(_lib.load().sga_load_degrade_rules(self.s.engine.handle, arr, len(rules)), self.s.engine.handle,
                     "DegradeRuleManager.loadRules")


@dataclass
class SystemRule:
    """CORE/slots/system/SystemRule.java:43-50 (negative = not set)."""
    highest_system_load: float = -1.0
    highest_cpu_usage: float = -1.0
    qps: float = -1.0
    avg_rt: int = -1
    max_thread: int = -1


class SystemRuleManager:
    """SystemRuleManager.loadRules + the SystemStatusListener readings the host measures."""

    def __init__(self, sentinel: LocalSentinel):
        self.s = sentinel

    def load_rules(self, rules: List[SystemRule]) -> int:
        arr = (_lib.SgaSystemRule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            arr[i].highest_system_load = r.highest_system_load
            arr[i].highest_cpu_usage = r.highest_cpu_usage
            arr[i].qps = r.qps
            arr[i].avg_rt = r.avg_rt
            arr[i].max_thread = r.max_thread
        return check(_lib.load().sga_load_system_rules(self.s.engine.handle, arr, len(rules)), self.s.engine.handle,
                     "SystemRuleManager.loadRules")

    def set_system_status(self, avg_load: float, cpu_usage: float):
        check(_lib.load().sga_set_system_status(self.s.engine.handle, avg_load, cpu_usage), self.s.engine.handle)
