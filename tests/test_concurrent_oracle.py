"""Concurrency tokens, the C oracle against the reference's own tests:
ConcurrentClusterFlowCheckerTest (testEasyAcquireAndRelease, testReleaseExpiredToken) and the
semantics around them (validation, AVG_LOCAL threshold, client-offline expiry, rule reloads and
CurrentConcurrencyManager, double release, release after the rule is gone)."""
import ctypes as C

import numpy as np

from tests import oracle_harness as H

T0 = 1_700_000_000_000
NONE = 0xFFFFFFFF
OK, BLOCKED, NO_RULE, BAD, RELEASE_OK, ALREADY = 0, 1, 3, -4, 6, 7


def _cluster(rules, ns="1-name"):
    L = H.lib()
    h = L.orc_cluster_new(1.0, 1.0)
    L.orc_cluster_load_rules(h, ns.encode(), H.cluster_rules_array(rules), len(rules))
    return L, h


def _now_calls(L, h, fid):
    v = C.c_int32()
    return v.value if L.orc_cluster_concurrent_now_calls(h, fid, C.byref(v)) else None


def _bits(online):
    b = np.zeros(4, np.uint32)
    for c in online:
        b[c >> 5] |= np.uint32(1 << (c & 31))
    return b


RULE = {"flow_id": 111, "count": 10, "threshold_type": 1, "grade": 0, "resource_timeout": 500,
        "client_offline_time": 1000}


def test_easy_acquire_and_release():
    # ConcurrentClusterFlowCheckerTest.testEasyAcquireAndRelease
    L, h = _cluster([RULE])
    toks = []
    for i in range(10):
        r = L.orc_cluster_concurrent_acquire(h, 0, 111, 1, T0, 1000 + i)
        assert r.status == OK and r.token_id == 1000 + i
        toks.append(r.token_id)
    for i in range(10):
        assert L.orc_cluster_concurrent_acquire(h, 0, 111, 1, T0, 2000 + i).status == BLOCKED
    assert _now_calls(L, h, 111) == 10 and L.orc_cluster_concurrent_tokens(h) == 10
    for t in toks:
        assert L.orc_cluster_concurrent_release(h, t) == RELEASE_OK
    assert _now_calls(L, h, 111) == 0 and L.orc_cluster_concurrent_tokens(h) == 0
    assert L.orc_cluster_concurrent_release(h, toks[0]) == ALREADY  # already released
    L.orc_cluster_free(h)


def test_release_expired_token():
    # ConcurrentClusterFlowCheckerTest.testReleaseExpiredToken: client online, resourceTimeout 500 ->
    # a token is dropped once it is older than 2 x 500 ms
    L, h = _cluster([RULE])
    for i in range(10):
        assert L.orc_cluster_concurrent_acquire(h, 0, 111, 1, T0 + i, 1000 + i).status == OK
    on = _bits([0])
    assert L.orc_cluster_concurrent_expire(h, T0 + 1000, on.ctypes.data, 1) == 0  # now - (t + 500) = 500: kept
    assert L.orc_cluster_concurrent_expire(h, T0 + 1005, on.ctypes.data, 1) == 5  # t = T0 .. T0 + 4
    assert L.orc_cluster_concurrent_expire(h, T0 + 3000, on.ctypes.data, 1) == 5
    assert _now_calls(L, h, 111) == 0 and L.orc_cluster_concurrent_tokens(h) == 0
    L.orc_cluster_free(h)


def test_client_offline_expiry_and_node_fields():
    L, h = _cluster([dict(RULE, resource_timeout=10_000)])
    assert L.orc_cluster_concurrent_acquire(h, 3, 111, 2, T0, 77).status == OK
    f, cd, rd, a = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32()
    assert L.orc_cluster_concurrent_get(h, 77, C.byref(f), C.byref(cd), C.byref(rd), C.byref(a)) == 1
    assert (f.value, cd.value, rd.value, a.value) == (111, T0 + 1000, T0 + 10_000, 2)
    on = _bits([3])
    assert L.orc_cluster_concurrent_expire(h, T0 + 5000, on.ctypes.data, 4) == 0  # online: only resource timeout
    off = _bits([])
    assert L.orc_cluster_concurrent_expire(h, T0 + 1000, off.ctypes.data, 4) == 0  # clientTimeout - now == 0
    assert L.orc_cluster_concurrent_expire(h, T0 + 1001, off.ctypes.data, 4) == 1
    assert _now_calls(L, h, 111) == 0
    L.orc_cluster_free(h)


def test_validation_threshold_and_reloads():
    L, h = _cluster([dict(RULE, threshold_type=0, count=2.5)], ns="ns")  # AVG_LOCAL: count x connected
    assert L.orc_cluster_concurrent_acquire(h, NONE, 111, 1, T0, 1).status == BAD
    assert L.orc_cluster_concurrent_acquire(h, 0, 0, 1, T0, 1).status == BAD
    assert L.orc_cluster_concurrent_acquire(h, 0, 111, 0, T0, 1).status == BAD
    assert L.orc_cluster_concurrent_acquire(h, 0, 999, 1, T0, 1).status == NO_RULE
    assert L.orc_cluster_concurrent_acquire(h, 0, 111, 1, T0, 1).status == BLOCKED  # 0 connected
    L.orc_cluster_set_connected_count(h, b"ns", 2)  # threshold 5
    st = [L.orc_cluster_concurrent_acquire(h, 0, 111, 2, T0, 10 + i).status for i in range(3)]
    assert st == [OK, OK, BLOCKED]
    assert L.orc_cluster_concurrent_acquire(h, 0, 111, 1, T0, 20).status == OK
    assert _now_calls(L, h, 111) == 5
    # reload keeping 111: nowCalls persists; adding 222 starts at 0
    rs = [dict(RULE, threshold_type=0, count=2.5), dict(RULE, flow_id=222)]
    L.orc_cluster_load_rules(h, b"ns", H.cluster_rules_array(rs), 2)
    assert _now_calls(L, h, 111) == 5 and _now_calls(L, h, 222) == 0
    # 111 dropped: rule and counter gone, its tokens stay cached, release answers NO_RULE_EXISTS
    L.orc_cluster_load_rules(h, b"ns", H.cluster_rules_array(rs[1:]), 1)
    assert _now_calls(L, h, 111) is None
    assert L.orc_cluster_concurrent_release(h, 10) == NO_RULE
    assert L.orc_cluster_concurrent_tokens(h) == 3
    # 111 back: a fresh counter; releasing an old token now drives it negative, as in the reference
    L.orc_cluster_load_rules(h, b"ns", H.cluster_rules_array(rs), 2)
    assert _now_calls(L, h, 111) == 0
    assert L.orc_cluster_concurrent_release(h, 10) == RELEASE_OK
    assert _now_calls(L, h, 111) == -2
    # clear-all of the namespace: counters removed, rules gone
    L.orc_cluster_load_rules(h, b"ns", H.cluster_rules_array([]), 0)
    assert _now_calls(L, h, 222) is None
    assert L.orc_cluster_concurrent_acquire(h, 0, 222, 1, T0, 99).status == NO_RULE
    L.orc_cluster_free(h)


def test_int_overflow_of_now_calls_plus_acquire():
    """nowCalls.get() + acquireCount is int arithmetic: it wraps before the double comparison."""
    L, h = _cluster([dict(RULE, count=3e9)])
    assert L.orc_cluster_concurrent_acquire(h, 0, 111, 2_000_000_000, T0, 1).status == OK
    # 2e9 + 2e9 wraps to a negative int, which is below the threshold: passes
    assert L.orc_cluster_concurrent_acquire(h, 0, 111, 2_000_000_000, T0, 2).status == OK
    assert _now_calls(L, h, 111) == (4_000_000_000 - (1 << 32))
    L.orc_cluster_free(h)
