"""GPU: the Envoy RLS gRPC server (sentinel_amd/rls_server.py) on the HIP engine.  Concurrent v2
and v3 clients; every batch the server hands to sga_rls_should_rate_limit is recorded with the
engine's per-descriptor results and replayed through the oracle's
SimpleClusterFlowChecker.acquireClusterToken in the same order -- statuses, remaining and codes
bit-exact -- and each client's response is checked against its slice of those results."""
import threading

import numpy as np
import pytest

from sentinel_amd import rls_server as R
from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def test_rls_grpc_server_parity():
    import grpc
    from sentinel_amd import cluster
    kv, D, Rule = R.KeyValueResource, R.ResourceDescriptor, R.EnvoyRlsRule
    eng = cluster.Engine(max_batch=1 << 14)
    rm = R.EnvoyRlsRuleManager(eng)
    paths = [f"/p{i}" for i in range(12)]
    flow = rm.load_rules([
        Rule("web", [D([kv("path", p)], float(3 + i % 5)) for i, p in enumerate(paths[:10])]
             + [D([kv("path", "/p0"), kv("user", "vip")], 40.0)]),
        Rule("api", [D([kv("method", "GET")], 25.5)]),
        Rule("bad", [D([kv("k", "v")], None)]),  # invalid: ignored
    ])
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    rs = [{"flow_id": f.cluster_config.flow_id, "count": f.count, "threshold_type": 1, "sample_count": 1,
           "window_interval_ms": 1000} for f in flow]
    L.orc_cluster_load_rules(oh, b"default", H.cluster_rules_array(rs), len(rs))

    svc = cluster.EnvoyRlsService(eng)
    log = []

    def decide(off, fid, hits, ts):
        out = svc.should_rate_limit(off, fid, hits, ts, with_remaining=True)
        log.append((off.copy(), fid.copy(), hits.copy(), ts.copy()) + tuple(x.copy() for x in out))
        return out

    clock = [T0]
    srv = R.SentinelRlsGrpcServer(rm, port=0, window_us=500, clock=lambda: clock[0], decide=decide).start()
    ch = grpc.insecure_channel(f"127.0.0.1:{srv.port}")
    errors, got = [], []
    lock = threading.Lock()

    def client(tid):
        rng = np.random.default_rng(100 + tid)
        ver = "v3" if tid % 2 else "v2"
        call = R.stub(ch, ver)
        for i in range(60):
            descs = []
            for _ in range(int(rng.integers(1, 4))):
                u = rng.random()
                if u < 0.7:
                    descs.append([("path", paths[int(rng.integers(0, 12))])])
                elif u < 0.8:
                    descs.append([("path", "/p0"), ("user", "vip")])
                else:
                    descs.append([("method", "GET")])
            dom = "api" if descs[0][0][0] == "method" else "web"
            hits = int(rng.integers(0, 3))
            try:
                r = call(R.make_request(ver, dom, descs, hits))
                with lock:
                    got.append((dom, descs, hits, r.overall_code, [(s.code, s.HasField("current_limit"),
                                                                    s.current_limit.requests_per_unit,
                                                                    s.limit_remaining) for s in r.statuses]))
            except grpc.RpcError as e:  # noqa: PERF203
                errors.append(e)
            if tid == 0 and i % 10 == 9:
                clock[0] += 350  # time moves under the callers

    try:
        ts = [threading.Thread(target=client, args=(t,)) for t in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not errors
        assert len(got) == 8 * 60
        assert len(log) < len(got)  # calls were batched
        # replay every engine batch on the oracle in order
        for off, fid, hits, tsv, code, st, rem in log:
            for r in range(len(hits)):
                a = max(1, int(hits[r]))
                blocked = False
                for d in range(off[r], off[r + 1]):
                    res = L.orc_cluster_request_token_simple(oh, int(fid[d]), a, int(tsv[r]))
                    assert (st[d], rem[d]) == (res.status, res.remaining)
                    blocked |= res.status not in (0, 3)
                assert code[r] == (2 if blocked else 1)
        # responses: codes per descriptor and (int) count limits match the rules
        for dom, descs, hits, overall, stats in got:
            assert len(stats) == len(descs)
            assert overall == (2 if any(c == 2 for c, *_ in stats) else 1)
            for ent, (c, has, rpu, rem) in zip(descs, stats):
                fr = rm.get_flow_rule_by_id(R.generate_flow_id(R.generate_key(dom, ent)))
                assert has == (fr is not None)
                if fr is not None:
                    assert rpu == int(fr.count)
                else:
                    assert c == 1 and rem == 0
        n_ok = sum(1 for *_, o, _s in got if o == 1)
        assert 0 < n_ok < len(got)
    finally:
        ch.close()
        srv.shutdown()
        L.orc_cluster_free(oh)
        eng.close()
