"""Envoy RLS front end, host side (no GPU): the restated protos against hand-encoded Envoy wire
bytes, the rule conversion (EnvoySentinelRuleConverterTest, EnvoyRlsRuleManager validity), the
HashSet order of a descriptor's resources, and the gRPC server + batcher end to end with the
oracle's SimpleClusterFlowChecker standing in for the engine call (the GPU run of the same server
is tests/test_rls_server_gpu.py)."""
import threading

import numpy as np
import pytest

from sentinel_amd import rls_server as R
from sentinel_amd.javautil import string_hash_code
from tests import oracle_harness as H

T0 = 1_700_000_000_000


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _ld(field, payload):
    return bytes([(field << 3) | 2]) + _varint(len(payload)) + payload


@pytest.mark.parametrize("ver", ["v2", "v3"])
def test_request_wire_bytes(ver):
    """RateLimitRequest{domain=1, descriptors=2{entries=1{key=1, value=2}}, hits_addend=3}."""
    req = R.make_request(ver, "dom", [[("k1", "v1"), ("k2", "v2")], [("a", "b")]], hits=3)
    ent = lambda k, v: _ld(1, _ld(1, k.encode()) + _ld(2, v.encode()))  # noqa: E731
    want = _ld(1, b"dom") + _ld(2, ent("k1", "v1") + ent("k2", "v2")) + _ld(2, ent("a", "b")) + bytes([0x18, 3])
    assert req.SerializeToString() == want
    Req, _ = R.messages(ver)
    back = Req.FromString(want + _ld(9, b"unknown-field"))  # unknown fields are tolerated
    assert back.domain == "dom" and back.hits_addend == 3
    assert [[(e.key, e.value) for e in d.entries] for d in back.descriptors] == [[("k1", "v1"), ("k2", "v2")],
                                                                                  [("a", "b")]]


@pytest.mark.parametrize("ver", ["v2", "v3"])
def test_response_wire_bytes(ver):
    """RateLimitResponse{overall_code=1, statuses=2{code=1, current_limit=2{rpu=1, unit=2},
    limit_remaining=3}}: a descriptor with a rule carries current_limit, one without does not."""
    resp = R.build_response(ver, R.CODE_OVER_LIMIT, [(R.CODE_OVER_LIMIT, 10, 0), (R.CODE_OK, None, 0),
                                                     (R.CODE_OK, 7, 5)])
    s1 = bytes([0x08, 2]) + _ld(2, bytes([0x08, 10, 0x10, 1]))
    s2 = bytes([0x08, 1])
    s3 = bytes([0x08, 1]) + _ld(2, bytes([0x08, 7, 0x10, 1])) + bytes([0x18, 5])
    assert resp.SerializeToString() == bytes([0x08, 2]) + _ld(2, s1) + _ld(2, s2) + _ld(2, s3)


def test_hash_set_order_matches_converter_test():
    """EnvoySentinelRuleConverterTest.testConvertToSentinelFlowRules: HashSet{k2/v2, k3/v3} walks
    k2 then k3; the flowIds are MAX_INT + key.hashCode()."""
    kv = R.KeyValueResource
    assert string_hash_code("k2") == 3367 and kv("k2", "v2").java_hash() == 109046
    dom = "testConvertToSentinelFlowRules"
    rule = R.EnvoyRlsRule(dom, [R.ResourceDescriptor([kv("k1", "v1")], 10.0),
                                R.ResourceDescriptor([kv("k2", "v2"), kv("k3", "v3")], 20.0)])
    fr = R.to_sentinel_flow_rules(rule)
    by_res = {f.resource: f for f in fr}
    k2 = f"{dom}|k2|v2|k3|v3"
    assert set(by_res) == {f"{dom}|k1|v1", k2}
    assert by_res[k2].count == 20.0 and by_res[f"{dom}|k1|v1"].count == 10.0
    for f in fr:
        cc = f.cluster_config
        assert f.cluster_mode and cc.threshold_type == 1 and cc.sample_count == 1
        assert cc.flow_id == 2147483647 + string_hash_code(f.resource)
    # duplicates collapse; many items spread over buckets by (h ^ h >>> 16) & (n - 1)
    many = [kv(f"key{i}", f"val{i}") for i in range(40)]
    out = R.java_hash_set(many + many[:5])
    assert len(out) == 40 and set(out) == set(many)
    b = [((x.java_hash() & 0xFFFFFFFF) ^ ((x.java_hash() & 0xFFFFFFFF) >> 16)) & 63 for x in out]
    assert b == sorted(b)


def test_rule_validity_and_manager():
    kv, D, Rule = R.KeyValueResource, R.ResourceDescriptor, R.EnvoyRlsRule
    ok = Rule("d", [D([kv("k", "v")], 1.0)])
    assert R.is_valid_rule(ok)
    for bad in (None, Rule(" ", ok.descriptors), Rule("d", []), Rule("d", [D([kv("k", "v")], None)]),
                Rule("d", [D([kv("k", "v")], -1.0)]), Rule("d", [D([], 1.0)]), Rule("d", [D([kv("k", " ")], 1)])):
        assert not R.is_valid_rule(bad)
    with pytest.raises(ValueError):
        R.to_sentinel_flow_rules(Rule("d", []))

    class Mgr(R.EnvoyRlsRuleManager):
        pushed = None

        def _push(self, flow):
            self.pushed = flow

    m = Mgr(None)
    flow = m.load_rules([ok, Rule("d", [D([kv("x", "y")], 9.0)]), Rule("e", [D([kv("k", "v")], 2.5)]), None])
    assert [r.domain for r in m.get_rules()] == ["d", "e"]  # duplicate domain and invalid rule ignored
    assert m.pushed == flow and len(flow) == 2
    assert m.get_flow_rule_by_id(R.generate_flow_id("e|k|v")).count == 2.5
    assert R.generate_flow_id("   ") == -1 and R.generate_flow_id("") == -1
    assert R.java_int(2.9) == 2 and R.java_int(1e12) == 2147483647 and R.java_int(float("nan")) == 0


class _OracleDecide:
    """SimpleClusterFlowChecker per descriptor through the C oracle (the test's stand-in engine)."""

    def __init__(self, flow):
        L = H.lib()
        self.L = L
        self.h = L.orc_cluster_new(1.0, 1.0)
        rs = [{"flow_id": f.cluster_config.flow_id, "count": f.count, "threshold_type": 1, "sample_count": 1,
               "window_interval_ms": 1000} for f in flow]
        L.orc_cluster_load_rules(self.h, b"default", H.cluster_rules_array(rs), len(rs))

    def __call__(self, off, fid, hits, ts):
        n = len(hits)
        code = np.zeros(n, np.int32)
        st = np.full(len(fid), 3, np.int8)
        rem = np.zeros(len(fid), np.int32)
        for r in range(n):
            if hits[r] < 0:
                code[r] = -1
                continue
            a = max(1, int(hits[r]))
            blocked = False
            for d in range(off[r], off[r + 1]):
                res = self.L.orc_cluster_request_token_simple(self.h, int(fid[d]), a, int(ts[r]))
                st[d], rem[d] = res.status, res.remaining
                blocked |= res.status not in (0, 3)
            code[r] = 2 if blocked else 1
        return code, st, rem

    def close(self):
        self.L.orc_cluster_free(self.h)


def test_grpc_server_end_to_end_cpu():
    """v2 and v3 clients against one server: statuses, current_limit/limit_remaining, negative
    hits_addend -> UNKNOWN error, concurrent callers batched into few decide calls."""
    import grpc
    kv, D, Rule = R.KeyValueResource, R.ResourceDescriptor, R.EnvoyRlsRule

    class Mgr(R.EnvoyRlsRuleManager):
        def _push(self, flow):
            pass

    m = Mgr(None)
    flow = m.load_rules([Rule("web", [D([kv("path", "/a")], 3.0), D([kv("path", "/b"), kv("user", "u")], 2.7)])])
    dec = _OracleDecide(flow)
    now = [T0]
    srv = R.SentinelRlsGrpcServer(m, port=0, window_us=2000, clock=lambda: now[0], decide=dec).start()
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{srv.port}")
        v3, v2 = R.stub(ch, "v3"), R.stub(ch, "v2")
        r = v3(R.make_request("v3", "web", [[("path", "/a")], [("nope", "x")]]))
        assert r.overall_code == R.CODE_OK
        assert [s.code for s in r.statuses] == [1, 1]
        assert r.statuses[0].current_limit.requests_per_unit == 3 and r.statuses[0].current_limit.unit == 1
        assert r.statuses[0].limit_remaining == 2
        assert not r.statuses[1].HasField("current_limit") and r.statuses[1].limit_remaining == 0
        r = v2(R.make_request("v2", "web", [[("path", "/a")]], hits=2))
        assert r.overall_code == R.CODE_OK and r.statuses[0].limit_remaining == 0
        r = v2(R.make_request("v2", "web", [[("path", "/a")], [("path", "/b"), ("user", "u")]]))
        assert r.overall_code == R.CODE_OVER_LIMIT
        assert [s.code for s in r.statuses] == [2, 1]
        assert r.statuses[1].current_limit.requests_per_unit == 2  # (int) 2.7
        with pytest.raises(grpc.RpcError) as ei:
            v3(R.make_request("v3", "web", [[("path", "/a")]], hits=-5))
        assert ei.value.code() == grpc.StatusCode.UNKNOWN
        # concurrent callers: 40 requests on /b (limit 2.7 per second) at one instant -> 2 pass
        now[0] = T0 + 5000
        srv.batcher.trace = []
        out = []
        lock = threading.Lock()

        def call():
            x = v3(R.make_request("v3", "web", [[("path", "/b"), ("user", "u")]]))
            with lock:
                out.append(x.overall_code)

        ts = [threading.Thread(target=call) for _ in range(40)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert sorted(out) == [1] * 2 + [2] * 38
        assert len(srv.batcher.trace) < 40  # batched
        ch.close()
    finally:
        srv.shutdown()
        dec.close()
