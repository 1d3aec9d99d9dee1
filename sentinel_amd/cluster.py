"""Host-side mirror of the reference's cluster token-server interface.

Same names and argument meaning as the Java API the engine replaces:
  TokenService.requestToken(Long ruleId, int acquireCount, boolean prioritized)
      CORE/cluster/TokenService.java:36  -> DefaultTokenService.request_token / request_tokens
  ClusterFlowRuleManager.loadRules(String namespace, List<FlowRule> rules)
      CS/flow/rule/ClusterFlowRuleManager.java:254-260 -> ClusterFlowRuleManager.load_rules
  TokenService.requestParamToken(Long ruleId, int acquireCount, Collection<Object> params)
      CORE/cluster/TokenService.java:46 -> DefaultTokenService.request_param_token(s)
  ClusterParamFlowRuleManager.loadRules(String namespace, List<ParamFlowRule> rules)
      CS/flow/rule/ClusterParamFlowRuleManager.java:270-276 -> ClusterParamFlowRuleManager.load_rules
  TokenResult / TokenResultStatus  CORE/cluster/TokenResult.java, CORE/cluster/TokenResultStatus.java:27-60
Every decision is computed by the HIP engine (libsentinel_amd.so); the mocked
TimeUtil clock of the reference tests is the explicit `now`/`ts` argument.
"""
import ctypes as C
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import SgaClusterFlowRule, SgaClusterParamRule, SgaConfig, SgaTokenResult, check
from .rules import (ClusterFlowConfig, ClusterRuleConstant, FlowRule, ParamFlowClusterConfig,  # noqa: F401
                    ParamFlowItem, ParamFlowRule)


class TokenResultStatus:
    BAD_REQUEST = -4
    TOO_MANY_REQUEST = -2
    FAIL = -1
    OK = 0
    BLOCKED = 1
    SHOULD_WAIT = 2
    NO_RULE_EXISTS = 3
    NO_REF_RULE_EXISTS = 4
    NOT_AVAILABLE = 5
    RELEASE_OK = 6
    ALREADY_RELEASE = 7


CONCURRENT_ACQUIRE, CONCURRENT_RELEASE = 0, 1
CLIENT_NONE = 0xFFFFFFFF


class ClusterFlowEvent:
    PASS, BLOCK, PASS_REQUEST, BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK, WAITING = range(7)


@dataclass
class TokenResult:
    status: int
    remaining: int = 0
    wait_in_ms: int = 0
    token_id: int = 0


class Engine:
    """Owns one sga_engine (one GPU / one shard)."""

    def __init__(self, device: int = 0, max_batch: int = 1 << 20, max_rules: int = 1 << 16,
                 exceed_count: float = 1.0, max_occupy_ratio: float = 1.0, max_param_keys: int = 0,
                 hot_rules: bool = True, hot_min_requests: int = 64, small_batch: int = 4096):
        L = _lib.load()
        cfg = SgaConfig()
        L.sga_config_default(C.byref(cfg))
        cfg.device = device
        cfg.max_batch = max_batch
        cfg.max_rules = max_rules
        cfg.exceed_count = exceed_count
        cfg.max_occupy_ratio = max_occupy_ratio
        cfg.max_param_keys = max_param_keys
        h = C.c_void_p()
        rc = L.sga_create(C.byref(cfg), C.byref(h))
        if rc < 0:
            raise _lib.EngineError(f"sga_create failed rc={rc}")
        self._h = h
        self.max_batch = max_batch
        self.set_hot_rules(hot_rules, hot_min_requests)
        self.set_small_batch(small_batch)
        self.clients: dict = {}  # client address -> dense id (concurrency tokens)

    def client_id(self, address: Optional[str]) -> int:
        """Dense id of a client address; null or "" -> SGA_CLIENT_NONE (a BAD_REQUEST)."""
        if not address:
            return CLIENT_NONE
        c = self.clients.get(address)
        if c is None:
            c = self.clients[address] = len(self.clients)
        return c

    def set_hot_rules(self, enabled: bool = True, min_requests: int = 64):
        """Engine tuning (sga_set_hot_rules): the hottest rules (at most 4096, each with at least
        `min_requests` requests in the previous batch) are decided in input order without being
        sorted (the hot path; on by default).  Decisions do not depend on it;
        tests use min_requests=1 to send nearly every rule down the hot path."""
        _lib.check(_lib.load().sga_set_hot_rules(self._h, 1 if enabled else 0, int(min_requests)), self._h,
                   "sga_set_hot_rules")

    def set_small_batch(self, max_requests: int = 4096):
        """Engine tuning (sga_set_small_batch): token batches of at most `max_requests` (<= 4096,
        0 = off) are ordered by one workgroup -- the latency path of a single requestToken."""
        _lib.check(_lib.load().sga_set_small_batch(self._h, int(max_requests)), self._h, "sga_set_small_batch")

    def batch_info(self) -> dict:
        """Path of the last token batch (sga_cluster_batch_info)."""
        v = (C.c_uint32 * 11)()
        _lib.check(_lib.load().sga_cluster_batch_info(self._h, v, 11), self._h, "sga_cluster_batch_info")
        keys = ("hot_mode", "flags", "n_sort", "n_cold", "n_prio", "n_hot_next", "bd_lo", "bd_hi", "hot_err",
                "n_pre", "lane_order_ok")
        return dict(zip(keys, [int(x) for x in v]))

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            _lib.load().sga_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# sga_cluster_flow_rule as a numpy record (bulk loads; the oracle's orc_cluster_rule has the same layout)
CLUSTER_RULE_DTYPE = np.dtype([("flow_id", "<i8"), ("count", "<f8"), ("threshold_type", "<i4"), ("sample_count", "<i4"),
                               ("window_interval_ms", "<i4"), ("grade", "<i4"), ("strategy", "<i4"),
                               ("reserved", "<i4"), ("resource_timeout_ms", "<i8"),
                               ("client_offline_time_ms", "<i8")])


def _rules_array(rules: List[FlowRule]):
    arr = (SgaClusterFlowRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        cc = r.cluster_config
        arr[i].flow_id = cc.flow_id if cc.flow_id is not None else 0
        arr[i].count = r.count
        arr[i].threshold_type = cc.threshold_type
        arr[i].sample_count = cc.sample_count
        arr[i].window_interval_ms = cc.window_interval_ms
        arr[i].grade = r.grade
        arr[i].strategy = cc.strategy
        arr[i].resource_timeout_ms = cc.resource_timeout
        arr[i].client_offline_time_ms = cc.client_offline_time
    return arr


class ClusterFlowRuleManager:
    """CS/flow/rule/ClusterFlowRuleManager.java mirror bound to one engine."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def load_rules(self, namespace: str, rules: List[FlowRule]) -> int:
        rules = [r for r in rules if r.cluster_mode]  # applyClusterFlowRule skips !isClusterMode
        arr = _rules_array(rules)
        rc = _lib.load().sga_load_cluster_flow_rules(self.engine.handle, namespace.encode(), arr, len(rules))
        return check(rc, self.engine.handle, "loadRules")

    def load_rule_arrays(self, namespace: str, flow_id, count, threshold_type=1, sample_count=10,
                         window_interval_ms=1000) -> int:
        """Bulk form for large rule sets (numpy arrays)."""
        n = len(flow_id)
        a = np.zeros(n, dtype=CLUSTER_RULE_DTYPE)
        a["flow_id"] = flow_id
        a["count"] = count
        a["threshold_type"] = threshold_type
        a["sample_count"] = sample_count
        a["window_interval_ms"] = window_interval_ms
        a["grade"] = 1
        a["resource_timeout_ms"] = 2000
        a["client_offline_time_ms"] = 2000
        ptr = a.ctypes.data_as(C.POINTER(SgaClusterFlowRule))
        rc = _lib.load().sga_load_cluster_flow_rules(self.engine.handle, namespace.encode(), ptr, n)
        return check(rc, self.engine.handle, "loadRules")

    def set_connected_count(self, namespace: str, n: int):
        check(_lib.load().sga_set_connected_count(self.engine.handle, namespace.encode(), n), self.engine.handle)


def param_value_key(v) -> int:
    """64-bit stand-in the engine uses for a Java parameter Object, the same mapping as the wire
    decoder (include/sga_wire.h): integers as themselves, bool as Boolean.hashCode (1231 / 1237),
    float by its IEEE-754 double bits, str by FNV-1a 64 of its UTF-8 bytes.  Distinct Objects with
    equal keys would share a counter; callers with such domains pass their own keys."""
    if isinstance(v, bool):
        return 1231 if v else 1237
    if isinstance(v, (int, np.integer)):
        return int(v)
    if isinstance(v, float):
        import struct
        return struct.unpack("<q", struct.pack("<d", v))[0]
    if isinstance(v, str):
        h = 0xcbf29ce484222325
        for b in v.encode():
            h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
        return h - (1 << 64) if h >= (1 << 63) else h
    raise TypeError(f"unsupported parameter type {type(v).__name__}")


def _hot_items(rule: ParamFlowRule):
    """ParamFlowRuleUtil.parseHotItems (PF/.../ParamFlowRuleUtil.java:193-214): items with a null
    object or a missing / negative count are skipped; later items win."""
    hot = {}
    for it in rule.param_flow_item_list:
        if it.object is None or it.count is None or it.count < 0:
            continue
        obj = it.object
        ct = it.class_type
        if isinstance(obj, str) and ct in ("int", "java.lang.Integer", "long", "java.lang.Long"):
            obj = int(obj)
        hot[param_value_key(obj)] = int(it.count)
    return hot


class ClusterParamFlowRuleManager:
    """CS/flow/rule/ClusterParamFlowRuleManager.java mirror bound to one engine."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def load_rules(self, namespace: str, rules: List[ParamFlowRule]) -> int:
        rules = [r for r in rules if r.cluster_mode]  # applyClusterParamRules skips !isClusterMode
        arr = (SgaClusterParamRule * max(1, len(rules)))()
        keep = []
        for i, r in enumerate(rules):
            cc = r.cluster_config
            a = arr[i]
            a.flow_id = cc.flow_id if (cc is not None and cc.flow_id is not None) else 0
            a.count = r.count
            a.threshold_type = cc.threshold_type if cc is not None else 0
            a.sample_count = cc.sample_count if cc is not None else 0
            a.window_interval_ms = cc.window_interval_ms if cc is not None else 0
            a.grade = r.grade
            a.burst_count = r.burst_count
            a.control_behavior = r.control_behavior
            a.max_queueing_time_ms = r.max_queueing_time_ms
            a.param_idx_set = 1 if r.param_idx is not None else 0
            a.duration_in_sec = r.duration_in_sec
            hot = _hot_items(r)
            a.n_hot = len(hot)
            if hot:
                hv = (C.c_int64 * len(hot))(*hot.keys())
                hc = (C.c_int32 * len(hot))(*hot.values())
                keep += [hv, hc]
                a.hot_values = C.cast(hv, C.POINTER(C.c_int64))
                a.hot_counts = C.cast(hc, C.POINTER(C.c_int32))
        rc = _lib.load().sga_load_cluster_param_rules(self.engine.handle, namespace.encode(), arr, len(rules))
        return check(rc, self.engine.handle, "loadRules")

    def set_param_capacity(self, capacity: int = 0) -> None:
        """maxCapacity of each bucket map of the ClusterParamMetrics created from now on (0: the default
        ClusterParamMetric.DEFAULT_CLUSTER_MAX_CAPACITY = 4000); a full map evicts its least recently
        accessed value."""
        check(_lib.load().sga_cluster_set_param_capacity(self.engine.handle, capacity))

    def param_sum(self, flow_id: int, value, now: int) -> int:
        """ClusterParamMetric.getSum(value) of the flow's metric at `now`."""
        out = C.c_int64()
        check(_lib.load().sga_cluster_param_sum(self.engine.handle, flow_id, param_value_key(value), now,
                                                C.byref(out)), self.engine.handle, "getSum")
        return out.value

    def top_values(self, flow_id: int, now: int, number: int = 5) -> List[tuple]:
        """ClusterParamMetric.getTopValues(number): [(value key, qps)], largest first -- the
        topParams of ClusterMetricNodeGenerator.paramToMetricNode (ClusterMetricNodeGenerator.java:93-105)."""
        if number <= 0:
            raise ValueError("number must be positive")
        vals = (C.c_int64 * number)()
        qps = (C.c_double * number)()
        n = C.c_uint32()
        check(_lib.load().sga_cluster_param_top_values(self.engine.handle, flow_id, now, number, vals, qps,
                                                       C.byref(n)), self.engine.handle, "getTopValues")
        return [(vals[i], qps[i]) for i in range(n.value)]


class GlobalRequestLimiter:
    """CS/flow/statistic/limit/GlobalRequestLimiter.java:30-80 mirror (per-namespace QPS guard that
    ClusterFlowChecker.allowProceed consults before a rule's metric)."""

    DEFAULT_MAX_ALLOWED_QPS = 30000.0  # ServerFlowConfig.DEFAULT_MAX_ALLOWED_QPS

    def __init__(self, engine: Engine):
        self.engine = engine
        self.limits = {}

    def init_if_absent(self, namespace: str, max_allowed_qps: float = DEFAULT_MAX_ALLOWED_QPS):
        if not namespace:
            raise ValueError("namespace cannot be empty")
        if namespace in self.limits:
            return
        check(_lib.load().sga_set_namespace_limit(self.engine.handle, namespace.encode(), float(max_allowed_qps)),
              self.engine.handle, "initIfAbsent")
        self.limits[namespace] = float(max_allowed_qps)

    def apply_max_qps_change(self, max_allowed_qps: float):
        if not max_allowed_qps >= 0:
            raise ValueError("max allowed QPS should > 0")
        for ns in self.limits:
            check(_lib.load().sga_set_namespace_limit(self.engine.handle, ns.encode(), float(max_allowed_qps)),
                  self.engine.handle, "applyMaxQpsChange")
            self.limits[ns] = float(max_allowed_qps)

    def get_max_allowed_qps(self, namespace: str) -> float:
        return self.limits.get(namespace, 0.0)


TOKEN_DTYPE = np.dtype([("remaining", "<i4"), ("wait_in_ms", "<i2"), ("status", "i1"), ("reserved", "i1")])
CONC_RESULT_DTYPE = np.dtype([("token_id", "<i8"), ("status", "<i4"), ("reserved", "<i4")])  # sga_concurrent_result


class DefaultTokenService:
    """CS/flow/DefaultTokenService.java mirror: requests are decided in order under a mocked clock."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def request_tokens(self, flow_id, acquire, prioritized, ts) -> np.ndarray:
        fid = np.ascontiguousarray(flow_id, dtype=np.int64)
        acq = np.ascontiguousarray(acquire, dtype=np.int32)
        pr = np.ascontiguousarray(prioritized, dtype=np.uint8)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(fid)
        out = np.zeros(n, dtype=TOKEN_DTYPE)
        rc = _lib.load().sga_request_tokens(self.engine.handle, fid.ctypes.data, acq.ctypes.data, pr.ctypes.data,
                                            t.ctypes.data, n, out.ctypes.data)
        check(rc, self.engine.handle, "requestToken")
        return out

    def request_token(self, rule_id: int, acquire_count: int, prioritized: bool, now: int) -> TokenResult:
        """TokenService.requestToken, one call: through the engine's coalescing queue
        (sga_request_token_one), so concurrent callers share one launch."""
        out = np.zeros(1, dtype=TOKEN_DTYPE)
        rc = _lib.load().sga_request_token_one(self.engine.handle, int(rule_id), int(acquire_count),
                                               1 if prioritized else 0, int(now), out.ctypes.data)
        check(rc, self.engine.handle, "requestToken")
        r = out[0]
        return TokenResult(int(r["status"]), int(r["remaining"]), int(r["wait_in_ms"]))

    def submit(self, rule_id: int, acquire_count: int, prioritized: bool, now: int) -> int:
        """Asynchronous requestToken (sga_token_submit): returns a ticket for poll()."""
        t = C.c_uint64()
        rc = _lib.load().sga_token_submit(self.engine.handle, int(rule_id), int(acquire_count),
                                          1 if prioritized else 0, int(now), C.byref(t))
        check(rc, self.engine.handle, "submit")
        return int(t.value)

    def poll(self, ticket: int) -> Optional[TokenResult]:
        """sga_poll: the ticket's TokenResult once decided (each ticket answers once), else None."""
        out = np.zeros(1, dtype=TOKEN_DTYPE)
        rc = _lib.load().sga_poll(self.engine.handle, int(ticket), out.ctypes.data)
        if rc == -11:  # SGA_EAGAIN
            return None
        check(rc, self.engine.handle, "poll")
        r = out[0]
        return TokenResult(int(r["status"]), int(r["remaining"]), int(r["wait_in_ms"]))

    def request_param_tokens(self, flow_id, acquire, params, ts) -> np.ndarray:
        """requestParamToken for a batch: params[i] is the Collection of request i (sequence of ints /
        strings, or already-mapped int64 keys)."""
        fid = np.ascontiguousarray(flow_id, dtype=np.int64)
        acq = np.ascontiguousarray(acquire, dtype=np.int32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(fid)
        off = np.zeros(n + 1, dtype=np.uint32)
        flat = []
        for i, p in enumerate(params):
            vals = [param_value_key(v) for v in (p if p is not None else [])]
            flat += vals
            off[i + 1] = off[i] + len(vals)
        vals = np.ascontiguousarray(flat if flat else [0], dtype=np.int64)
        out = np.zeros(n, dtype=TOKEN_DTYPE)
        rc = _lib.load().sga_request_param_tokens(self.engine.handle, fid.ctypes.data, acq.ctypes.data,
                                                  off.ctypes.data, vals.ctypes.data, t.ctypes.data, n,
                                                  out.ctypes.data)
        check(rc, self.engine.handle, "requestParamToken")
        return out

    def request_param_token(self, rule_id: int, acquire_count: int, params, now: int) -> TokenResult:
        r = self.request_param_tokens([rule_id], [acquire_count], [params], [now])[0]
        return TokenResult(int(r["status"]), int(r["remaining"]), int(r["wait_in_ms"]))

    # ---- concurrency tokens (DefaultTokenService.java:67-86 -> ConcurrentClusterFlowChecker)
    def concurrent_ops(self, op, client, ids, acquire, ts) -> np.ndarray:
        """Acquire (op 0: ids = flowIds) / release (op 1: ids = tokenIds) operations decided in
        order; returns CONC_RESULT_DTYPE records (token_id, status)."""
        o = np.ascontiguousarray(op, dtype=np.uint8)
        cl = np.ascontiguousarray(client, dtype=np.uint32)
        x = np.ascontiguousarray(ids, dtype=np.int64)
        a = np.ascontiguousarray(acquire, dtype=np.int32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(o)
        if not (len(cl) == len(x) == len(a) == len(t) == n):
            raise ValueError("operation arrays differ in length")
        out = np.zeros(max(n, 1), dtype=CONC_RESULT_DTYPE)
        rc = _lib.load().sga_concurrent_ops(self.engine.handle, o.ctypes.data, cl.ctypes.data, x.ctypes.data,
                                            a.ctypes.data, t.ctypes.data, n, out.ctypes.data)
        check(rc, self.engine.handle, "concurrentOps")
        return out[:n]

    def request_concurrent_token(self, client_address: Optional[str], rule_id: int, acquire_count: int,
                                 now: int) -> TokenResult:
        r = self.concurrent_ops([CONCURRENT_ACQUIRE], [self.engine.client_id(client_address)], [rule_id],
                                [acquire_count], [now])[0]
        return TokenResult(int(r["status"]), token_id=int(r["token_id"]))

    def release_concurrent_token(self, token_id: int, now: int = 0) -> int:
        """ConcurrentClusterFlowChecker.releaseConcurrentToken status (the SPI method returns void)."""
        return int(self.concurrent_ops([CONCURRENT_RELEASE], [CLIENT_NONE], [token_id], [0], [now])[0]["status"])

    def expire_concurrent_tokens(self, now: int, online_addresses=()) -> int:
        """One RegularExpireStrategy pass; online_addresses = ConnectionManager's connected clients."""
        n = len(self.engine.clients)
        bits = np.zeros(max((n + 31) // 32, 1), dtype=np.uint32)
        for a in online_addresses:
            c = self.engine.clients.get(a)
            if c is not None:
                bits[c >> 5] |= np.uint32(1 << (c & 31))
        removed = C.c_uint64()
        check(_lib.load().sga_concurrent_expire(self.engine.handle, now, bits.ctypes.data, n, C.byref(removed)),
              self.engine.handle, "expire")
        return removed.value

    def concurrent_now_calls(self, flow_id: int) -> Optional[int]:
        """CurrentConcurrencyManager.get(flowId).get(), None when absent."""
        v = C.c_int32()
        rc = check(_lib.load().sga_concurrent_now_calls(self.engine.handle, flow_id, C.byref(v)), self.engine.handle)
        return v.value if rc == 1 else None

    def concurrent_token_count(self) -> int:
        n = C.c_uint64()
        check(_lib.load().sga_concurrent_token_count(self.engine.handle, C.byref(n)), self.engine.handle)
        return n.value

    def get_token_cache_node(self, token_id: int):
        node = _lib.SgaTokenCacheNode()
        rc = check(_lib.load().sga_concurrent_get_token(self.engine.handle, token_id, C.byref(node)),
                   self.engine.handle)
        return node if rc == 1 else None

    def metric_sums(self, flow_id: int, now: int) -> List[int]:
        out = (C.c_int64 * 7)()
        check(_lib.load().sga_cluster_metric_sums(self.engine.handle, flow_id, now, out), self.engine.handle)
        return list(out)


class EnvoyRlsService:
    """RLS/SentinelEnvoyRlsServiceImpl.shouldRateLimit mirror over batches of requests."""

    OK = 1
    OVER_LIMIT = 2

    def __init__(self, engine: Engine):
        self.engine = engine

    @staticmethod
    def generate_flow_id(key: str) -> int:
        # EnvoySentinelRuleConverter.generateFlowId: -1 for a blank key, else
        # (long) Integer.MAX_VALUE + key.hashCode()
        from .javautil import is_blank, string_hash_code
        return -1 if is_blank(key) else 2147483647 + string_hash_code(key)

    def should_rate_limit(self, desc_offsets, desc_flow_id, hits_addend, ts, with_remaining: bool = False):
        """Returns (code per request, TokenResult status per descriptor[, remaining per descriptor])."""
        off = np.ascontiguousarray(desc_offsets, dtype=np.uint32)
        fid = np.ascontiguousarray(desc_flow_id, dtype=np.int64)
        hits = np.ascontiguousarray(hits_addend, dtype=np.int32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        nreq = len(hits)
        if len(off) != nreq + 1 or len(t) != nreq or (nreq and int(off[-1]) != len(fid)):
            raise ValueError("desc_offsets must have n_requests + 1 entries ending at len(desc_flow_id)")
        st = np.zeros(max(len(fid), 1), dtype=np.int8)
        rem = np.zeros(max(len(fid), 1), dtype=np.int32)
        code = np.zeros(max(nreq, 1), dtype=np.int32)
        rc = _lib.load().sga_rls_should_rate_limit(self.engine.handle, off.ctypes.data, nreq, fid.ctypes.data,
                                                   hits.ctypes.data, t.ctypes.data, st.ctypes.data, rem.ctypes.data,
                                                   code.ctypes.data)
        check(rc, self.engine.handle, "shouldRateLimit")
        n = len(fid)
        return (code[:nreq], st[:n], rem[:n]) if with_remaining else (code[:nreq], st[:n])

    def should_rate_limit_device(self, desc_offsets, desc_flow_id, hits_addend, ts_base, ts_off, stream=None):
        """shouldRateLimit over device tensors (uint32/int32 offsets [n+1], int64 flowIds, int32 hits,
        request times ts_base + ts_off), asynchronous on `stream` (torch stream or None = engine
        stream).  Returns device tensors (code int32 per request, status int8 and remaining int32 per
        descriptor)."""
        import torch
        nreq = hits_addend.numel()
        nd = desc_flow_id.numel()
        if desc_offsets.numel() != nreq + 1 or ts_off.numel() != nreq:
            raise ValueError("desc_offsets must have n_requests + 1 entries; ts_off one per request")
        for x in (desc_offsets, desc_flow_id, hits_addend, ts_off):
            if not x.is_cuda or not x.is_contiguous():
                raise ValueError("inputs must be contiguous device tensors")
        dev = hits_addend.device
        code = torch.empty(nreq, dtype=torch.int32, device=dev)
        st = torch.empty(max(nd, 1), dtype=torch.int8, device=dev)
        rem = torch.empty(max(nd, 1), dtype=torch.int32, device=dev)
        rc = _lib.load().sga_rls_should_rate_limit_device(
            self.engine.handle, desc_offsets.data_ptr(), nreq, nd, desc_flow_id.data_ptr(), hits_addend.data_ptr(),
            int(ts_base), ts_off.data_ptr(), st.data_ptr(), rem.data_ptr(), code.data_ptr(),
            stream.cuda_stream if stream is not None else None)
        check(rc, self.engine.handle, "shouldRateLimit")
        return code, st[:nd], rem[:nd]
