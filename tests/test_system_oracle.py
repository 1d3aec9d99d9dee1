"""SystemSlot and Constants.ENTRY_NODE in the C oracle: the reference's
SystemRuleManagerTest threshold semantics, and hand-derived checkSystem sequences (qps, thread,
avg RT, BBR under load, CPU usage) for inbound entries; outbound entries never touch
ENTRY_NODE nor the system check (SystemRuleManager.java:298-353, StatisticSlot.java:54-137)."""
import ctypes as C

from tests import local_trace as lt
from tests import oracle_harness as H

T0 = 1_700_000_000_000
ENTRY = 0xFFFFFFFF
PASS, BLOCK_FLOW, BLOCK_SYSTEM, PASS_WAIT = 0, 1, 5, 4


def _entry(o, r, t, a=1, inbound=True):
    w = C.c_int64()
    return o.L.orc_flow_entry_x(o.h, r, t, a, 0, 0, 0, 1 if inbound else 0, C.byref(w))


def _exit(o, r, t, rt, a=1, inbound=True, err=0):
    o.L.orc_flow_exit_x(o.h, r, t, rt, a, err, 0, 0, 1 if inbound else 0)


def _view(o, r, now):
    return dict(zip(lt.NODE_GETTERS, o.node(r, now)))


def test_rule_loading_semantics():
    o = lt.Oracle(2)
    # SystemRuleManagerTest.testLoadInvalidRules: load -0.9 and cpu 2.7 set nothing -> no check
    assert o.system([{"highest_system_load": -0.9}, {"highest_cpu_usage": 2.7}]) == 0
    assert _entry(o, 0, T0) == PASS
    # the switch follows the LAST rule: a trailing rule with no field turns the check off
    assert o.system([{"qps": 0}, {}]) == 1
    assert _entry(o, 0, T0 + 1) == PASS
    assert o.system([{}, {"qps": 0}]) == 1
    assert _entry(o, 0, T0 + 2) == BLOCK_SYSTEM
    assert _entry(o, 0, T0 + 2, inbound=False) == PASS  # outbound: never checked
    # testLoadDuplicateTypeOfRules: the minimum wins
    o.system([{"qps": 3}, {"qps": 2}, {"qps": 7}])
    got = [_entry(o, 1, T0 + 5000 + i) for i in range(4)]
    assert got == [PASS, PASS, BLOCK_SYSTEM, BLOCK_SYSTEM]
    o.close()


def test_entry_node_statistics_inbound_only():
    o = lt.Oracle(3)
    for i in range(5):
        assert _entry(o, i % 3, T0 + i) == PASS
    assert _entry(o, 0, T0 + 10, a=4, inbound=False) == PASS
    _exit(o, 0, T0 + 20, 7)
    _exit(o, 1, T0 + 21, 3, err=1)
    _exit(o, 0, T0 + 22, 5, a=4, inbound=False)
    v = _view(o, ENTRY, T0 + 30)
    assert (v["pass_qps"], v["success_qps"], v["exception_qps"], v["cur_thread_num"]) == (5.0, 2.0, 1.0, 3)
    assert (v["avg_rt"], v["min_rt"]) == (5.0, 3.0)
    assert _view(o, 0, T0 + 30)["pass_qps"] == 6.0  # the resource node counts both
    o.close()


def test_thread_rt_bbr_and_cpu_checks():
    o = lt.Oracle(2)
    o.system([{"max_thread": 2}])
    assert [_entry(o, 0, T0 + i) for i in range(3)] == [PASS, PASS, PASS]  # 0, 1, 2 threads: 2 > 2 is false
    assert _entry(o, 0, T0 + 3) == BLOCK_SYSTEM                           # 3 > 2
    assert _view(o, 0, T0 + 3)["block_qps"] == 1.0 and _view(o, ENTRY, T0 + 3)["block_qps"] == 1.0
    _exit(o, 0, T0 + 4, 100)
    assert _entry(o, 0, T0 + 5) == PASS
    # avg RT: rt sum / success of the second window (one exit, rt 100)
    o.system([{"avg_rt": 60}])
    assert _entry(o, 1, T0 + 6) == BLOCK_SYSTEM  # 100 > 60
    _exit(o, 0, T0 + 7, 10)
    assert _entry(o, 1, T0 + 8) == PASS  # (100 + 10) / 2 = 55
    # BBR: load above the threshold blocks only when threads > maxSuccessQps * minRt / 1000
    o.system([{"highest_system_load": 1.0}], load=0.5, cpu=-1)
    assert _entry(o, 1, T0 + 9) == PASS  # load below threshold
    o.L.orc_flow_set_system_status(o.h, 2.0, -1)
    # threads now 4; maxSuccess 2 (x2 / 1 s = 4 qps), minRt 10 -> 4 * 10 / 1000 = 0.04 < 4: blocked
    assert _entry(o, 1, T0 + 10) == BLOCK_SYSTEM
    # CPU usage: 0 allowed, reading 0.3 -> blocked (SystemRuleManagerTest.testCheckMaxCpuUsageNotBBR)
    o.system([{"highest_cpu_usage": 0.0}], load=-1, cpu=0.3)
    assert _entry(o, 0, T0 + 11) == BLOCK_SYSTEM
    o.L.orc_flow_set_system_status(o.h, -1, 0.0)
    assert _entry(o, 0, T0 + 12) == PASS
    o.close()


def test_qps_window_rolls():
    o = lt.Oracle(1)
    o.system([{"qps": 2.5}])
    got = [_entry(o, 0, T0 + i * 100) for i in range(5)]
    assert got == [PASS, PASS, BLOCK_SYSTEM, BLOCK_SYSTEM, BLOCK_SYSTEM]  # 2 + 1 > 2.5
    assert _entry(o, 0, T0 + 1500) == PASS  # the 1 s window moved on
    o.close()
