"""Envoy RLS front end: gRPC ShouldRateLimit (v2 and v3) batched into one engine call.

Mirrors (RLS = sentinel-cluster/sentinel-cluster-server-envoy-rls/src/main/java/com/alibaba/csp/
sentinel/cluster/server/envoy/rls):
  RLS/SentinelRlsGrpcServer.java:30-40          one gRPC server, the v2 and v3 RateLimitService
  RLS/SentinelEnvoyRlsConstants.java:23         default port 10245
  RLS/SentinelEnvoyRlsServiceImpl.java:33-101   shouldRateLimit (v2); service/v3/... the same for v3
  RLS/rule/EnvoyRlsRule.java                    domain -> descriptors {Set<key/value>, count}
  RLS/rule/EnvoyRlsRuleManager.java:70-140      validity, one rule per domain, "default" namespace
  RLS/rule/EnvoySentinelRuleConverter.java      descriptor -> cluster FlowRule (GLOBAL, sampleCount 1)

The request / response messages are the vendored protos' (src/main/proto/envoy/service/ratelimit/
v{2,3}/rls.proto and the descriptor protos), restated as descriptors built at import time -- the
image has no protoc -- with the same package names, message names and field numbers, so the bytes
on the wire are Envoy's.  Fields the reference never reads or writes (descriptor limit overrides,
headers, quota, raw_body, dynamic_metadata) are left out: protobuf keeps them as unknown fields on
parse and the reference never sets them.

Every gRPC call is queued; a batching thread drains the queue every `window_us` (or when
`max_requests` are waiting) and decides all descriptors of all queued calls in ONE
sga_rls_should_rate_limit launch, in arrival order (the reference's per-call checkToken loop is
the same sequence of SimpleClusterFlowChecker.acquireClusterToken calls).
"""
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .javautil import is_blank, string_hash_code

DEFAULT_GRPC_PORT = 10245  # SentinelEnvoyRlsConstants.DEFAULT_GRPC_PORT
SEPARATOR = "|"            # EnvoySentinelRuleConverter.SEPARATOR
CODE_UNKNOWN, CODE_OK, CODE_OVER_LIMIT = 0, 1, 2
UNIT_SECOND = 1
TOKEN_OK, TOKEN_NO_RULE_EXISTS = 0, 3


# ---------------------------------------------------------------- protobuf messages
def _build_messages():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    pool = descriptor_pool.DescriptorPool()

    def fld(name, num, typ, label=F.LABEL_OPTIONAL, type_name=None):
        f = F(name=name, number=num, type=typ, label=label)
        if type_name:
            f.type_name = type_name
        return f

    def descriptor_file(fname, pkg):
        fd = descriptor_pb2.FileDescriptorProto(name=fname, package=pkg, syntax="proto3")
        d = fd.message_type.add(name="RateLimitDescriptor")
        e = d.nested_type.add(name="Entry")
        e.field.extend([fld("key", 1, F.TYPE_STRING), fld("value", 2, F.TYPE_STRING)])
        d.field.extend([fld("entries", 1, F.TYPE_MESSAGE, F.LABEL_REPEATED, f".{pkg}.RateLimitDescriptor.Entry")])
        return fd

    def rls_file(fname, pkg, desc_type, with_name):
        fd = descriptor_pb2.FileDescriptorProto(name=fname, package=pkg, syntax="proto3")
        fd.dependency.append(desc_type[0])
        rq = fd.message_type.add(name="RateLimitRequest")
        rq.field.extend([fld("domain", 1, F.TYPE_STRING),
                         fld("descriptors", 2, F.TYPE_MESSAGE, F.LABEL_REPEATED, desc_type[1]),
                         fld("hits_addend", 3, F.TYPE_UINT32)])
        rs = fd.message_type.add(name="RateLimitResponse")
        code = rs.enum_type.add(name="Code")
        for n, v in (("UNKNOWN", 0), ("OK", 1), ("OVER_LIMIT", 2)):
            code.value.add(name=n, number=v)
        rl = rs.nested_type.add(name="RateLimit")
        unit = rl.enum_type.add(name="Unit")
        for n, v in (("UNKNOWN", 0), ("SECOND", 1), ("MINUTE", 2), ("HOUR", 3), ("DAY", 4)):
            unit.value.add(name=n, number=v)
        rl.field.extend([fld("requests_per_unit", 1, F.TYPE_UINT32),
                         fld("unit", 2, F.TYPE_ENUM, type_name=f".{pkg}.RateLimitResponse.RateLimit.Unit")])
        if with_name:
            rl.field.append(fld("name", 3, F.TYPE_STRING))
        ds = rs.nested_type.add(name="DescriptorStatus")
        ds.field.extend([fld("code", 1, F.TYPE_ENUM, type_name=f".{pkg}.RateLimitResponse.Code"),
                         fld("current_limit", 2, F.TYPE_MESSAGE, type_name=f".{pkg}.RateLimitResponse.RateLimit"),
                         fld("limit_remaining", 3, F.TYPE_UINT32)])
        rs.field.extend([fld("overall_code", 1, F.TYPE_ENUM, type_name=f".{pkg}.RateLimitResponse.Code"),
                         fld("statuses", 2, F.TYPE_MESSAGE, F.LABEL_REPEATED,
                             f".{pkg}.RateLimitResponse.DescriptorStatus")])
        svc = fd.service.add(name="RateLimitService")
        svc.method.add(name="ShouldRateLimit", input_type=f".{pkg}.RateLimitRequest",
                       output_type=f".{pkg}.RateLimitResponse")
        return fd

    v2d = "envoy/api/v2/ratelimit/ratelimit.proto"
    v3d = "envoy/extensions/common/ratelimit/v3/ratelimit.proto"
    pool.Add(descriptor_file(v2d, "envoy.api.v2.ratelimit"))
    pool.Add(descriptor_file(v3d, "envoy.extensions.common.ratelimit.v3"))
    pool.Add(rls_file("envoy/service/ratelimit/v2/rls.proto", "envoy.service.ratelimit.v2",
                      (v2d, ".envoy.api.v2.ratelimit.RateLimitDescriptor"), False))
    pool.Add(rls_file("envoy/service/ratelimit/v3/rls.proto", "envoy.service.ratelimit.v3",
                      (v3d, ".envoy.extensions.common.ratelimit.v3.RateLimitDescriptor"), True))
    out = {}
    for ver in ("v2", "v3"):
        pkg = f"envoy.service.ratelimit.{ver}"
        out[ver] = (message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{pkg}.RateLimitRequest")),
                    message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{pkg}.RateLimitResponse")))
    dpk = {"v2": "envoy.api.v2.ratelimit", "v3": "envoy.extensions.common.ratelimit.v3"}
    for ver, pkg in dpk.items():
        out[ver + "_descriptor"] = message_factory.GetMessageClass(
            pool.FindMessageTypeByName(f"{pkg}.RateLimitDescriptor"))
    return out


_MSGS = None


def messages(version: str = "v3"):
    """(RateLimitRequest, RateLimitResponse) classes of envoy.service.ratelimit.<version>."""
    global _MSGS
    if _MSGS is None:
        _MSGS = _build_messages()
    return _MSGS[version]


def service_name(version: str) -> str:
    return f"envoy.service.ratelimit.{version}.RateLimitService"


# ---------------------------------------------------------------- rules
@dataclass(frozen=True)
class KeyValueResource:
    key: str
    value: str

    def java_hash(self) -> int:
        """Objects.hash(key, value) (EnvoyRlsRule.java:135-137), i32 arithmetic."""
        h = (31 * (31 + string_hash_code(self.key)) + string_hash_code(self.value)) & 0xFFFFFFFF
        return h - (1 << 32) if h >= (1 << 31) else h


def java_hash_set(items: Sequence[KeyValueResource]) -> List[KeyValueResource]:
    """A java.util.HashSet filled by add() in this order, in iteration order: equal items collapse,
    buckets by (h ^ h >>> 16) & (n - 1) with the table doubling past 0.75 n from 16, insertion order
    inside a bucket.  This is the order EnvoySentinelRuleConverter.generateKey walks a descriptor's
    resource Set in (a JSON-decoded Set<KeyValueResource> is such a HashSet)."""
    uniq: List[KeyValueResource] = []
    seen = set()
    for it in items:
        if it not in seen:
            seen.add(it)
            uniq.append(it)
    n = 16
    while len(uniq) > 0.75 * n:
        n *= 2

    def bucket(it):
        h = it.java_hash() & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (n - 1)

    order = sorted(range(len(uniq)), key=lambda i: (bucket(uniq[i]), i))
    return [uniq[i] for i in order]


@dataclass
class ResourceDescriptor:
    resources: Optional[List[KeyValueResource]] = None  # a Java Set (see java_hash_set)
    count: Optional[float] = None


@dataclass
class EnvoyRlsRule:
    domain: Optional[str] = None
    descriptors: Optional[List[ResourceDescriptor]] = None


def generate_flow_id(key: str) -> int:
    """EnvoySentinelRuleConverter.generateFlowId: -1 for a blank key, else MAX_INT + key.hashCode()."""
    return -1 if is_blank(key) else 2147483647 + string_hash_code(key)


def generate_key(domain: str, entries: Sequence[Tuple[str, str]]) -> str:
    """SentinelEnvoyRlsServiceImpl.generateKey / EnvoySentinelRuleConverter.generateKey."""
    parts = [domain]
    for k, v in entries:
        parts.append(k)
        parts.append(v)
    return SEPARATOR.join(parts)


def is_valid_rule(rule: Optional[EnvoyRlsRule]) -> bool:
    """EnvoyRlsRuleManager.isValidRule (RLS/rule/EnvoyRlsRuleManager.java:114-137)."""
    if rule is None or is_blank(rule.domain):
        return False
    if not rule.descriptors:
        return False
    for d in rule.descriptors:
        if d is None or d.count is None or d.count < 0:
            return False
        if not d.resources:
            return False
        for r in d.resources:
            if r is None or is_blank(r.key) or is_blank(r.value):
                return False
    return True


def to_sentinel_flow_rules(rule: EnvoyRlsRule):
    """EnvoySentinelRuleConverter.toSentinelFlowRules: one GLOBAL cluster rule per descriptor."""
    from .rules import ClusterFlowConfig, FlowRule
    if not is_valid_rule(rule):
        raise ValueError("Not a valid RLS rule")
    out = []
    for d in rule.descriptors:
        res = java_hash_set(d.resources)
        ident = generate_key(rule.domain, [(r.key, r.value) for r in res])
        out.append(FlowRule(resource=ident, count=float(d.count), cluster_mode=True,
                            cluster_config=ClusterFlowConfig(flow_id=generate_flow_id(ident), threshold_type=1,
                                                             sample_count=1)))
    return out


class EnvoyRlsRuleManager:
    """EnvoyRlsRuleManager bound to one engine: loadRules replaces the "default" namespace's
    cluster flow rules with the converted descriptors (EnvoyRlsRulePropertyListener.configUpdate)."""

    def __init__(self, engine):
        self.engine = engine
        self.rule_map: Dict[str, EnvoyRlsRule] = {}
        self.flow_rules: Dict[int, object] = {}  # flowId -> FlowRule (ClusterFlowRuleManager.getFlowRuleById)

    def load_rules(self, rules: Optional[List[EnvoyRlsRule]]) -> List:
        m: Dict[str, EnvoyRlsRule] = {}
        for r in rules or []:
            if not is_valid_rule(r) or r.domain in m:  # invalid or duplicate domain: ignored
                continue
            m[r.domain] = r
        flow = [fr for r in m.values() for fr in to_sentinel_flow_rules(r)]
        self.rule_map = m
        self.flow_rules = {fr.cluster_config.flow_id: fr for fr in flow}
        self._push(flow)
        return flow

    def _push(self, flow):
        from .cluster import ClusterFlowRuleManager
        ClusterFlowRuleManager(self.engine).load_rules("default", flow)  # ServerConstants.DEFAULT_NAMESPACE

    def get_rules(self) -> List[EnvoyRlsRule]:
        return list(self.rule_map.values())

    def get_flow_rule_by_id(self, flow_id: int):
        return self.flow_rules.get(flow_id)


def java_int(x: float) -> int:
    """Java (int) of a double: NaN -> 0, saturating, truncation toward zero."""
    if x != x:
        return 0
    if x >= 2147483647:
        return 2147483647
    if x <= -2147483648:
        return -2147483648
    return int(x)


# ---------------------------------------------------------------- batching service
class _Call:
    __slots__ = ("domain", "entries", "hits", "event", "result")

    def __init__(self, domain, entries, hits):
        self.domain, self.entries, self.hits = domain, entries, hits
        self.event = threading.Event()
        self.result = None


class RlsBatcher:
    """Queues ShouldRateLimit calls; one thread decides each drained batch with one engine call.

    `decide(offsets, flow_ids, hits, ts)` -> (code per request, status per descriptor, remaining
    per descriptor); by default EnvoyRlsService(engine).should_rate_limit(..., with_remaining=True).
    The mocked TimeUtil of the tests is `clock` (default wall-clock milliseconds)."""

    def __init__(self, rule_manager: EnvoyRlsRuleManager, window_us: int = 200, max_requests: int = 1 << 14,
                 clock: Optional[Callable[[], int]] = None, decide=None):
        self.rm = rule_manager
        if decide is None:
            from .cluster import EnvoyRlsService
            svc = EnvoyRlsService(rule_manager.engine)
            decide = lambda o, f, h, t: svc.should_rate_limit(o, f, h, t, with_remaining=True)  # noqa: E731
        self.decide = decide
        self.window = window_us / 1e6
        self.max_requests = max_requests
        self.clock = clock or (lambda: int(time.time() * 1000))
        self._q: List[_Call] = []
        self._cv = threading.Condition()
        self._stop = False
        self._fid_cache: Dict[str, int] = {}
        self.batches = 0
        self.trace: Optional[list] = None  # set to [] to record (offsets, flow_ids, hits, now) per batch
        self._t = threading.Thread(target=self._loop, name="rls-batcher", daemon=True)
        self._t.start()

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._t.join()

    def submit(self, domain: str, entries: List[List[Tuple[str, str]]], hits: int):
        c = _Call(domain, entries, hits)
        with self._cv:
            self._q.append(c)
            if len(self._q) == 1 or len(self._q) >= self.max_requests:
                self._cv.notify()
        c.event.wait()
        if isinstance(c.result, BaseException):
            raise c.result
        return c.result

    def _flow_id(self, key: str) -> int:
        f = self._fid_cache.get(key)
        if f is None:
            if len(self._fid_cache) > (1 << 20):
                self._fid_cache.clear()
            f = self._fid_cache[key] = generate_flow_id(key)
        return f

    def _loop(self):
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if self._stop and not self._q:
                    return
            time.sleep(self.window)  # gather the window's calls
            with self._cv:
                batch, self._q = self._q[:self.max_requests], self._q[self.max_requests:]
            try:
                self._decide(batch)
            except BaseException as e:  # every waiter sees the failure
                for c in batch:
                    c.result = e
            for c in batch:
                c.event.set()

    def _decide(self, batch: List[_Call]):
        off = [0]
        fids: List[int] = []
        for c in batch:
            for ent in c.entries:
                fids.append(self._flow_id(generate_key(c.domain, ent)))
            off.append(len(fids))
        now = self.clock()
        o, f, h = np.asarray(off, np.uint32), np.asarray(fids, np.int64), np.asarray([c.hits for c in batch], np.int32)
        if self.trace is not None:
            self.trace.append((o, f, h, now))
        code, st, rem = self.decide(o, f, h, np.full(len(batch), now, np.int64))
        self.batches += 1
        for r, c in enumerate(batch):
            stats = []
            for d in range(off[r], off[r + 1]):
                s = int(st[d])
                rule = None if s == TOKEN_NO_RULE_EXISTS else self.rm.get_flow_rule_by_id(fids[d])
                limit = None if rule is None else java_int(rule.count)
                ok = s in (TOKEN_OK, TOKEN_NO_RULE_EXISTS)
                stats.append((CODE_OK if ok else CODE_OVER_LIMIT, limit, int(rem[d])))
            c.result = (int(code[r]), stats)


def build_response(version: str, overall: int, statuses) -> object:
    """RateLimitResponse of SentinelEnvoyRlsServiceImpl.java:70-94: current_limit {SECOND,
    (int) count} and limit_remaining only for descriptors whose rule exists."""
    _, Resp = messages(version)
    resp = Resp(overall_code=overall)
    for code, limit, remaining in statuses:
        s = resp.statuses.add(code=code)
        if limit is not None:
            s.current_limit.unit = UNIT_SECOND
            s.current_limit.requests_per_unit = limit & 0xFFFFFFFF
            s.limit_remaining = remaining & 0xFFFFFFFF
    return resp


class SentinelRlsGrpcServer:
    """SentinelRlsGrpcServer: the v2 and v3 RateLimitService on one port."""

    def __init__(self, rule_manager: EnvoyRlsRuleManager, port: int = DEFAULT_GRPC_PORT, host: str = "127.0.0.1",
                 window_us: int = 200, max_workers: int = 256, clock: Optional[Callable[[], int]] = None,
                 decide=None):
        import grpc
        self.batcher = RlsBatcher(rule_manager, window_us=window_us, clock=clock, decide=decide)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                                   options=[("grpc.so_reuseport", 0)])
        for ver in ("v2", "v3"):
            Req, Resp = messages(ver)
            h = grpc.unary_unary_rpc_method_handler(self._handler(ver), request_deserializer=Req.FromString,
                                                    response_serializer=Resp.SerializeToString)
            self._server.add_generic_rpc_handlers(
                (grpc.method_handlers_generic_handler(service_name(ver), {"ShouldRateLimit": h}),))
        self.port = self._server.add_insecure_port(f"{host}:{port}")
        self.host = host

    def _handler(self, version: str):
        import grpc

        def should_rate_limit(req, ctx):
            hits = req.hits_addend
            if hits >= 1 << 31:
                hits -= 1 << 32  # getHitsAddend() is a Java int
            if hits < 0:  # responseObserver.onError(IllegalArgumentException) -> UNKNOWN
                ctx.abort(grpc.StatusCode.UNKNOWN, f"acquireCount should be positive, but actual: {hits}")
            entries = [[(e.key, e.value) for e in d.entries] for d in req.descriptors]
            overall, stats = self.batcher.submit(req.domain, entries, hits)
            return build_response(version, overall, stats)

        return should_rate_limit

    def start(self):
        self._server.start()
        return self

    def shutdown(self):
        self._server.stop(grace=None)
        self.batcher.close()


def make_request(version: str, domain: str, descriptors: Sequence[Sequence[Tuple[str, str]]], hits: int = 0):
    Req, _ = messages(version)
    D = _MSGS[version + "_descriptor"]
    return Req(domain=domain, hits_addend=hits & 0xFFFFFFFF,
               descriptors=[D(entries=[D.Entry(key=k, value=v) for k, v in d]) for d in descriptors])


def stub(channel, version: str = "v3"):
    """Client callable for ShouldRateLimit on `channel` (tests, tools)."""
    Req, Resp = messages(version)
    return channel.unary_unary(f"/{service_name(version)}/ShouldRateLimit", request_serializer=Req.SerializeToString,
                               response_deserializer=Resp.FromString)
