"""GPU parity: cluster concurrency tokens (sga_concurrent_ops / sga_concurrent_expire) against the
oracle's sequential ConcurrentClusterFlowChecker + TokenCacheNodeManager + RegularExpireStrategy.
Statuses, nowCalls of every rule, cache sizes and cached node fields must be identical; the oracle
is handed the token ids the engine issued (the reference draws random UUID bits)."""
import ctypes as C

import numpy as np
import pytest

from tests import oracle_harness as H

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


@pytest.fixture(scope="module")
def cl():
    from sentinel_amd import cluster
    return cluster


def _rule(cl, r):
    return cl.FlowRule(resource=f"r{r['flow_id']}", count=r["count"], grade=0, cluster_mode=True,
                       cluster_config=cl.ClusterFlowConfig(flow_id=r["flow_id"], threshold_type=r["threshold_type"],
                                                           resource_timeout=r["resource_timeout"],
                                                           client_offline_time=r["client_offline_time"]))


def _load(cl, eng, L, oh, ns, rules):
    cl.ClusterFlowRuleManager(eng).load_rules(ns, [_rule(cl, r) for r in rules])
    L.orc_cluster_load_rules(oh, ns.encode(), H.cluster_rules_array(rules), len(rules))


def test_concurrent_kat_sequences(cl):
    """ConcurrentClusterFlowCheckerTest.testEasyAcquireAndRelease / testReleaseExpiredToken on the engine."""
    eng = cl.Engine(max_batch=1 << 12)
    svc = cl.DefaultTokenService(eng)
    rule = {"flow_id": 111, "count": 10, "threshold_type": 1, "resource_timeout": 500, "client_offline_time": 1000}
    cl.ClusterFlowRuleManager(eng).load_rules("1-name", [_rule(cl, rule)])
    toks = []
    for _ in range(10):
        r = svc.request_concurrent_token("127.0.0.1", 111, 1, T0)
        assert r.status == 0 and r.token_id != 0
        toks.append(r.token_id)
    assert len(set(toks)) == 10
    for _ in range(10):
        assert svc.request_concurrent_token("127.0.0.1", 111, 1, T0).status == 1
    for t in toks:
        assert svc.release_concurrent_token(t) == 6
    assert svc.concurrent_now_calls(111) == 0 and svc.concurrent_token_count() == 0
    assert svc.release_concurrent_token(toks[0]) == 7
    assert svc.request_concurrent_token("", 111, 1, T0).status == -4
    assert svc.request_concurrent_token("127.0.0.1", 5, 1, T0).status == 3
    # testReleaseExpiredToken: online client, 2 x resourceTimeout
    for i in range(10):
        assert svc.request_concurrent_token("127.0.0.1", 111, 1, T0 + i).status == 0
    assert svc.request_concurrent_token("10.0.0.9", 111, 0, T0).status == -4
    assert svc.get_token_cache_node(12345) is None
    assert svc.expire_concurrent_tokens(T0 + 1005, ["127.0.0.1"]) == 5
    assert svc.expire_concurrent_tokens(T0 + 3000, ["127.0.0.1"]) == 5
    assert svc.concurrent_now_calls(111) == 0 and svc.concurrent_token_count() == 0
    eng.close()


@pytest.mark.parametrize("dense", [True, False], ids=["dense", "hash"])
def test_concurrent_random_parity(cl, dense):
    rng = np.random.default_rng(7 if dense else 8)
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    eng = cl.Engine(max_batch=1 << 12)
    svc = cl.DefaultTokenService(eng)
    base = 0 if dense else 10 ** 12
    ids = [base + 1 + k * (1 if dense else 7919) for k in range(60)]

    def mk(fid):
        return {"flow_id": fid, "count": float(rng.integers(1, 25)) + (0.5 if rng.random() < 0.3 else 0.0),
                "threshold_type": int(rng.random() < 0.7), "resource_timeout": int(rng.integers(200, 3000)),
                "client_offline_time": int(rng.integers(100, 2000))}

    rules = {fid: mk(fid) for fid in ids[:50]}
    mgr = cl.ClusterFlowRuleManager(eng)
    mgr.set_connected_count("ns", 3)
    L.orc_cluster_set_connected_count(oh, b"ns", 3)
    _load(cl, eng, L, oh, "ns", list(rules.values()))
    clients = [f"10.0.0.{i}:{4000 + i}" for i in range(8)]
    cids = [eng.client_id(a) for a in clients]
    outstanding = []
    seen_tokens = set()
    now = T0
    for batch in range(36):
        n = int(rng.integers(500, 2500))
        op = np.zeros(n, np.uint8)
        cli = np.zeros(n, np.uint32)
        x = np.zeros(n, np.int64)
        a = np.zeros(n, np.int32)
        ts = now + np.sort(rng.integers(0, 300, size=n))
        for i in range(n):
            u = rng.random()
            if u < 0.5 or not outstanding:
                op[i] = 0
                cli[i] = cids[int(rng.integers(0, 8))] if rng.random() > 0.01 else cl.CLIENT_NONE
                x[i] = ids[int(rng.integers(0, 60))] if rng.random() > 0.02 else int(rng.integers(-1, 2))
                a[i] = int(rng.integers(1, 4)) if rng.random() > 0.01 else 0
            elif u < 0.95:
                op[i] = 1
                x[i] = outstanding[int(rng.integers(0, len(outstanding)))]  # may repeat: ALREADY_RELEASE
            else:
                op[i] = 1
                x[i] = int(rng.integers(-(1 << 62), 1 << 62))
        got = svc.concurrent_ops(op, cli, x, a, ts)
        for i in range(n):
            if op[i] == 0:
                tok = int(got["token_id"][i])
                r = L.orc_cluster_concurrent_acquire(oh, int(cli[i]), int(x[i]), int(a[i]), int(ts[i]), tok)
                assert got["status"][i] == r.status, (batch, i, got["status"][i], r.status)
                if r.status == 0:
                    assert tok not in seen_tokens
                    seen_tokens.add(tok)
                    outstanding.append(tok)
            else:
                s = L.orc_cluster_concurrent_release(oh, int(x[i]))
                assert got["status"][i] == s, (batch, i, got["status"][i], s)
        for fid in ids:
            v = C.c_int32()
            has = L.orc_cluster_concurrent_now_calls(oh, fid, C.byref(v))
            assert svc.concurrent_now_calls(fid) == (v.value if has else None), (batch, fid)
        assert svc.concurrent_token_count() == L.orc_cluster_concurrent_tokens(oh)
        for tok in rng.choice(outstanding, size=min(5, len(outstanding)), replace=False) if outstanding else []:
            node = svc.get_token_cache_node(int(tok))
            f, cd, rd, aq = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32()
            present = L.orc_cluster_concurrent_get(oh, int(tok), C.byref(f), C.byref(cd), C.byref(rd), C.byref(aq))
            assert (node is not None) == bool(present)
            if node is not None:
                assert (node.flow_id, node.client_timeout, node.resource_timeout, node.acquire_count) == \
                    (f.value, cd.value, rd.value, aq.value)
        now = int(ts[-1]) + 1
        if batch % 4 == 3:  # RegularExpireStrategy pass with some clients offline
            now += int(rng.integers(0, 2500))
            online = [i for i in range(8) if rng.random() < 0.6]
            bits = np.zeros(1, np.uint32)
            for c in online:
                bits[0] |= np.uint32(1 << cids[c])
            removed = svc.expire_concurrent_tokens(now, [clients[c] for c in online])
            assert removed == L.orc_cluster_concurrent_expire(oh, now, bits.ctypes.data, len(cids))
        if batch % 9 == 8:  # reload: drop some rules, add others, change thresholds
            keep = [f for f in rules if rng.random() < 0.8]
            rules = {f: dict(rules[f], count=float(rng.integers(1, 25))) for f in keep}
            for f in ids:
                if f not in rules and rng.random() < 0.3:
                    rules[f] = mk(f)
            _load(cl, eng, L, oh, "ns", list(rules.values()))
        if batch == 20:  # clear-all, then back
            _load(cl, eng, L, oh, "ns", [])
            _load(cl, eng, L, oh, "ns", list(rules.values()))
    assert len(seen_tokens) > 1000
    L.orc_cluster_free(oh)
    eng.close()
