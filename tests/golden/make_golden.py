#!/usr/bin/env python3
"""Writes tests/golden/kat_*.json: known-answer scenarios TRANSCRIBED from the
reference's own JUnit suites (inputs + the expected values those tests assert).

The reference is Java and no JDK exists in this image, so the reference cannot
be executed here (DESIGN.md "Oracle").  These fixtures are therefore data
transcribed by hand from the assertions of the cited test methods; the
generating script is this file.  Where a reference test used the wall clock
(System.currentTimeMillis / Thread.sleep) the scenario replays it under the
mocked TimeUtil clock at several base times (aligned and misaligned to bucket
boundaries); the asserted values do not depend on the base.

Op vocabulary: see tests/oracle_harness.py.  Times `t` are relative to `base`.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CORET = "sentinel-core/src/test/java/com/alibaba/csp/sentinel"
CST = "sentinel-cluster/sentinel-cluster-server-default/src/test/java/com/alibaba/csp/sentinel/cluster"
PFT = "sentinel-extension/sentinel-parameter-flow-control/src/test/java/com/alibaba/csp/sentinel"
CORET_DEG = CORET + "/slots/block/degrade/circuitbreaker"
BASES = [1_700_000_000_000, 1_700_000_000_123, 1_700_000_000_499, 1_700_000_000_999, 1_700_000_059_950]

SCENARIOS = []


def scenario(name, source, ops, bases=BASES):
    SCENARIOS.append({"name": name, "source": source, "bases": bases, "ops": ops})


# ---------------------------------------------------------------- leap arrays
scenario("OccupiableBucketLeapArray.testNewWindow",
         CORET + "/slots/statistic/metric/OccupiableBucketLeapArrayTest.java:28-42",
         [{"op": "set_time", "t": 0},
          {"op": "leap_new", "id": "a", "kind": "occupiable", "sample_count": 10, "interval_ms": 2000},
          {"op": "leap_add", "id": "a", "t": 0, "event": "PASS", "n": 1},
          {"op": "leap_current_get", "id": "a", "t": 0, "event": "PASS", "expect": 1},
          {"op": "leap_add_waiting", "id": "a", "t": 200, "n": 1},
          {"op": "leap_current_waiting", "id": "a", "expect": 1},
          {"op": "leap_current_get", "id": "a", "t": 0, "event": "PASS", "expect": 1}])

scenario("OccupiableBucketLeapArray.testWindowInOneInterval",
         CORET + "/slots/statistic/metric/OccupiableBucketLeapArrayTest.java:44-67",
         [{"op": "set_time", "t": 0},
          {"op": "leap_new", "id": "a", "kind": "occupiable", "sample_count": 10, "interval_ms": 2000},
          {"op": "leap_add", "id": "a", "t": 0, "event": "PASS", "n": 1},
          {"op": "leap_current_get", "id": "a", "t": 0, "event": "PASS", "expect": 1},
          {"op": "leap_add_waiting", "id": "a", "t": 200, "n": 2},
          {"op": "leap_current_waiting", "id": "a", "expect": 2},
          {"op": "leap_current_get", "id": "a", "t": 0, "event": "PASS", "expect": 1},
          {"op": "leap_current_window", "id": "a", "t": 200},
          {"op": "leap_values_sum", "id": "a", "t": 200, "event": "PASS", "expect": 3, "expect_count": 2}])

_ops = [{"op": "set_time", "t": 0},
        {"op": "leap_new", "id": "a", "kind": "occupiable", "sample_count": 10, "interval_ms": 2000}]
for i in range(10):
    _ops.append({"op": "leap_add", "id": "a", "t": i * 200, "event": "PASS", "n": 1})
    _ops.append({"op": "leap_add_waiting", "id": "a", "t": (i + 1) * 200, "n": 1})
_ops.append({"op": "leap_values_sum", "id": "a", "t": {"aligned_plus": 2000, "window": 200}, "event": "PASS",
             "expect": 19, "expect_count": 10})
_ops.append({"op": "leap_current_waiting", "id": "a", "expect": 10})
scenario("OccupiableBucketLeapArray.testWindowAfterOneInterval",
         CORET + "/slots/statistic/metric/OccupiableBucketLeapArrayTest.java:104-138", _ops)

scenario("BucketLeapArray.testNewWindow+testLeapArrayWindowStart",
         CORET + "/slots/statistic/metric/BucketLeapArrayTest.java:44-66",
         [{"op": "leap_new", "id": "a", "kind": "bucket", "sample_count": 2, "interval_ms": 2000},
          {"op": "leap_current_window", "id": "a", "t": 0, "expect_start": {"aligned_plus": 0, "window": 1000}},
          {"op": "leap_current_get", "id": "a", "t": 0, "event": "PASS", "expect": 0}])

scenario("BucketLeapArray.testWindowAfterOneInterval",
         CORET + "/slots/statistic/metric/BucketLeapArrayTest.java:68-111",
         [{"op": "leap_new", "id": "a", "kind": "bucket", "sample_count": 2, "interval_ms": 2000},
          {"op": "leap_current_window", "id": "a", "t": {"aligned_plus": 0, "window": 1000},
           "expect_start": {"aligned_plus": 0, "window": 1000}},
          {"op": "leap_add", "id": "a", "t": {"aligned_plus": 0, "window": 1000}, "event": "PASS", "n": 1},
          {"op": "leap_add", "id": "a", "t": {"aligned_plus": 0, "window": 1000}, "event": "BLOCK", "n": 1},
          {"op": "leap_current_get", "id": "a", "t": {"aligned_plus": 500, "window": 1000}, "event": "PASS", "expect": 1},
          {"op": "leap_add", "id": "a", "t": {"aligned_plus": 500, "window": 1000}, "event": "PASS", "n": 1},
          {"op": "leap_current_get", "id": "a", "t": {"aligned_plus": 500, "window": 1000}, "event": "PASS", "expect": 2},
          {"op": "leap_current_get", "id": "a", "t": {"aligned_plus": 500, "window": 1000}, "event": "BLOCK", "expect": 1},
          {"op": "leap_current_window", "id": "a", "t": {"aligned_plus": 1000, "window": 1000},
           "expect_start": {"aligned_plus": 1000, "window": 1000}},
          {"op": "leap_current_get", "id": "a", "t": {"aligned_plus": 1000, "window": 1000}, "event": "PASS", "expect": 0},
          {"op": "leap_current_get", "id": "a", "t": {"aligned_plus": 1000, "window": 1000}, "event": "BLOCK", "expect": 0}])

scenario("BucketLeapArray.testGetPreviousWindow",
         CORET + "/slots/statistic/metric/BucketLeapArrayTest.java:149-161",
         [{"op": "set_time", "t": 0},
          {"op": "leap_new", "id": "a", "kind": "bucket", "sample_count": 2, "interval_ms": 2000},
          {"op": "leap_current_window", "id": "a", "t": 0},
          {"op": "leap_previous_window", "id": "a", "t": 0, "expect_null": True},
          {"op": "leap_previous_window", "id": "a", "t": 1000, "expect_start": {"aligned_plus": 0, "window": 1000}},
          {"op": "leap_previous_window", "id": "a", "t": 11000, "expect_null": True}])

scenario("BucketLeapArray.testListWindowsResetOld (mocked clock)",
         CORET + "/slots/statistic/metric/BucketLeapArrayTest.java:163-186",
         [{"op": "leap_new", "id": "a", "kind": "bucket", "sample_count": 10, "interval_ms": 1000},
          {"op": "leap_current_window", "id": "a", "t": 0},
          {"op": "leap_current_window", "id": "a", "t": 100},
          {"op": "leap_values_sum", "id": "a", "t": 100, "event": "PASS", "expect": 0, "expect_count": 2},
          {"op": "leap_add", "id": "a", "t": 1100, "event": "PASS", "n": 1},
          {"op": "leap_values_sum", "id": "a", "t": 1100, "event": "PASS", "expect": 1, "expect_count": 1}])

_ops = [{"op": "set_time", "t": 0},
        {"op": "leap_new", "id": "a", "kind": "unary", "sample_count": 10, "interval_ms": 1000},
        {"op": "leap_add", "id": "a", "t": "now", "event": 0, "n": 1},
        {"op": "sleep", "ms": 100},
        {"op": "leap_add", "id": "a", "t": "now", "event": 0, "n": 2}]
for i in range(8):
    _ops += [{"op": "sleep", "ms": 100}, {"op": "leap_add", "id": "a", "t": "now", "event": 0, "n": i + 3}]
_ops += [{"op": "leap_valid_head", "id": "a", "expect_start": {"aligned_plus": 0, "window": 100}},
         {"op": "sleep", "ms": 100},
         {"op": "leap_valid_head", "id": "a", "expect_start": {"aligned_plus": 100, "window": 100}}]
scenario("LeapArray.testGetValidHead", CORET + "/slots/statistic/base/LeapArrayTest.java:31-63", _ops)

_ops = [{"op": "leap_new", "id": "a", "kind": "future", "sample_count": 10, "interval_ms": 2000}]
for i in range(0, 2000, 200):
    _ops += [{"op": "leap_add", "id": "a", "t": i, "event": "PASS", "n": 1},
             {"op": "leap_values_sum", "id": "a", "t": i, "event": "PASS", "expect": 0, "expect_count": 0}]
scenario("FutureBucketLeapArray.testFutureMetricLeapArray",
         CORET + "/slots/statistic/metric/FutureBucketLeapArrayTest.java:20-30", _ops)

# ------------------------------------------------------------- controllers
scenario("DefaultController.testCanPassForQps",
         CORET + "/slots/block/flow/controller/DefaultControllerTest.java:30-39",
         [{"op": "ctrl_new", "id": "c", "behavior": 0, "grade": 1, "count": 10},
          {"op": "node_mock", "id": "n", "pass_qps": 9.0, "prev_pass_qps": 0.0, "threads": 0},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS"},
          {"op": "node_mock", "id": "n", "pass_qps": 10.0, "prev_pass_qps": 0.0, "threads": 0},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"}], bases=BASES[:1])

scenario("DefaultController.testCanPassForThreadCount",
         CORET + "/slots/block/flow/controller/DefaultControllerTest.java:41-51",
         [{"op": "ctrl_new", "id": "c", "behavior": 0, "grade": 0, "count": 8},
          {"op": "node_mock", "id": "n", "pass_qps": 0.0, "prev_pass_qps": 0.0, "threads": 7},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS"},
          {"op": "node_mock", "id": "n", "pass_qps": 0.0, "prev_pass_qps": 0.0, "threads": 8},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"}], bases=BASES[:1])

_ops = [{"op": "set_time", "t": 0},
        {"op": "ctrl_new", "id": "c", "behavior": 1, "grade": 1, "count": 10, "warm_up_period_sec": 10,
         "cold_factor": 3},
        {"op": "node_mock", "id": "n", "pass_qps": 8.0, "prev_pass_qps": 1.0, "threads": 0},
        {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"},
        {"op": "node_mock", "id": "n", "pass_qps": 1.0, "prev_pass_qps": 1.0, "threads": 0},
        {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS"},
        {"op": "node_mock", "id": "n", "pass_qps": 1.0, "prev_pass_qps": 10.0, "threads": 0}]
for i in range(100):
    _ops += [{"op": "sleep", "ms": 100}, {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1}]
_ops += [{"op": "node_mock", "id": "n", "pass_qps": 8.0, "prev_pass_qps": 10.0, "threads": 0},
         {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS"},
         {"op": "node_mock", "id": "n", "pass_qps": 10.0, "prev_pass_qps": 10.0, "threads": 0},
         {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"}]
scenario("WarmUpController.testWarmUp", CORET + "/slots/block/flow/controller/WarmUpControllerTest.java:35-61",
         _ops)

_ops = [{"op": "set_time", "t": 0},
        {"op": "ctrl_new", "id": "c", "behavior": 2, "grade": 1, "count": 10, "max_queueing_time_ms": 500},
        {"op": "node_mock", "id": "n", "pass_qps": 0.0, "prev_pass_qps": 0.0, "threads": 0}]
# six acquisitions back to back: the first passes immediately, the next five queue 100 ms apart
# ("(end - start) > 400" in the reference); under the mocked clock the sleep is reported as wait_ms.
for i in range(6):
    _ops.append({"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS",
                 "expect_wait": 0 if i == 0 else 100, "sleep_wait": True})
scenario("RateLimiterController.testPaceController_normal",
         CORET + "/slots/block/flow/controller/RateLimiterControllerTest.java:36-47", _ops)

scenario("RateLimiterController.testPaceController_zeroattack",
         CORET + "/slots/block/flow/controller/RateLimiterControllerTest.java:88-97",
         [{"op": "set_time", "t": 0},
          {"op": "ctrl_new", "id": "c", "behavior": 2, "grade": 1, "count": 0, "max_queueing_time_ms": 500},
          {"op": "node_mock", "id": "n", "pass_qps": 0.0, "prev_pass_qps": 0.0, "threads": 0},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 0, "expect": "PASS"},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 0, "expect": "PASS"}])

_ops = [{"op": "set_time", "t": 0},
        {"op": "ctrl_new", "id": "c", "behavior": 3, "grade": 1, "count": 10, "warm_up_period_sec": 10,
         "max_queueing_time_ms": 1000, "cold_factor": 3},
        {"op": "node_mock", "id": "n", "pass_qps": 100.0, "prev_pass_qps": 100.0, "threads": 0},
        {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS", "sleep_wait": True}]
for i in range(10):  # "cost ~ 100 ms per request": each request queues one more 100 ms slot
    _ops.append({"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS",
                 "expect_wait": 100, "sleep_wait": True})
scenario("WarmUpRateLimiterController.testPace",
         CORET + "/slots/block/flow/controller/WarmUpRateLimiterControllerTest.java:42-56", _ops)

scenario("WarmUpRateLimiterController.testPaceCanNotPass",
         CORET + "/slots/block/flow/controller/WarmUpRateLimiterControllerTest.java:58-68",
         [{"op": "set_time", "t": 0},
          {"op": "ctrl_new", "id": "c", "behavior": 3, "grade": 1, "count": 10, "warm_up_period_sec": 10,
           "max_queueing_time_ms": 10, "cold_factor": 3},
          {"op": "node_mock", "id": "n", "pass_qps": 100.0, "prev_pass_qps": 100.0, "threads": 0},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "PASS"},
          {"op": "ctrl_can_pass", "id": "c", "node": "n", "acquire": 1, "expect": "BLOCK"}])

# ------------------------------------------------------- local flow engine
scenario("FlowPartialIntegrationTest.testQPSGrade",
         CORET + "/slots/block/flow/FlowPartialIntegrationTest.java:50-72",
         [{"op": "set_time", "t": 0},
          {"op": "flow_new", "id": "f", "n_resources": 1},
          {"op": "flow_load", "id": "f", "rules": [{"resource": 0, "grade": 1, "count": 1}]},
          {"op": "flow_entry", "id": "f", "resource": 0, "acquire": 1, "expect": "PASS"},
          {"op": "flow_exit", "id": "f", "resource": 0, "rt": 0, "count": 1},
          {"op": "flow_entry", "id": "f", "resource": 0, "acquire": 1, "expect": "BLOCK"}])

# README.md:75-116 HelloWorld: QPS rule count=20; a tight loop sees 20 passes every second.
_ops = [{"op": "flow_new", "id": "f", "n_resources": 1},
        {"op": "flow_load", "id": "f", "rules": [{"resource": 0, "grade": 1, "count": 20}]},
        {"op": "flow_loop", "id": "f", "resource": 0, "per_ms": 20, "ms": 5000, "expect_pass_per_second": [20] * 5}]
scenario("README HelloWorld (count=20 => 20 pass/s)", "README.md:75-116", _ops, bases=[1_700_000_000_000])

# -------------------------------------------------- cluster token server
scenario("ClusterParamMetricTest.testClusterParamMetric",
         CST + "/flow/statistic/metric/ClusterParamMetricTest.java:27-49 (getTopValues asserts not restated)",
         [{"op": "set_time", "t": 0},
          {"op": "pm_new", "id": "m", "sample_count": 5, "interval_ms": 25},
          {"op": "pm_add", "id": "m", "value": "e1", "n": -1},
          {"op": "pm_add", "id": "m", "value": "e1", "n": -2},
          {"op": "pm_add", "id": "m", "value": "e2", "n": 100},
          {"op": "pm_add", "id": "m", "value": "e2", "n": 23},
          {"op": "pm_add", "id": "m", "value": "e3", "n": 100},
          {"op": "pm_add", "id": "m", "value": "e3", "n": 230},
          {"op": "pm_sum", "id": "m", "value": "e1", "expect": -3},
          {"op": "pm_avg", "id": "m", "value": "e1", "expect": -120, "tol": 0.01},
          {"op": "pm_avg", "id": "m", "value": "e3", "expect": 13200, "tol": 0.01},
          {"op": "pm_avg", "id": "m", "value": "e2", "expect": 4920, "tol": 0.01},
          {"op": "pm_add", "id": "m", "value": "e2", "n": 100},
          {"op": "pm_add", "id": "m", "value": "e2", "n": 23},
          {"op": "pm_sum", "id": "m", "value": "e2", "expect": 246},
          {"op": "pm_avg", "id": "m", "value": "e2", "expect": 9840, "tol": 0.01}])

scenario("ClusterMetricTest.testTryOccupyNext",
         CST + "/flow/statistic/metric/ClusterMetricTest.java:25-45",
         [{"op": "set_time", "t": 0},
          {"op": "cm_new", "id": "m", "sample_count": 5, "interval_ms": 25},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 1},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 2},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 1},
          {"op": "cm_add", "id": "m", "event": "BLOCK", "n": 1},
          {"op": "cm_sum", "id": "m", "event": "PASS", "expect": 4},
          {"op": "cm_sum", "id": "m", "event": "BLOCK", "expect": 1},
          {"op": "cm_avg", "id": "m", "event": "PASS", "expect": 160, "tol": 0.01},
          {"op": "cm_try_occupy_next", "id": "m", "acquire": 111, "threshold": 900, "expect": 200},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 1},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 2},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 1},
          {"op": "cm_try_occupy_next", "id": "m", "acquire": 222, "threshold": 900, "expect": 200},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 1},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 2},
          {"op": "cm_add", "id": "m", "event": "PASS", "n": 1},
          {"op": "cm_try_occupy_next", "id": "m", "acquire": 333, "threshold": 900, "expect": 0}])

scenario("RequestLimiterTest.testRequestLimiter",
         CST + "/flow/statistic/limit/RequestLimiterTest.java:25-42",
         [{"op": "set_time", "t": 0},
          {"op": "lim_new", "id": "l", "qps": 10},
          {"op": "lim_add", "id": "l", "n": 3}, {"op": "lim_add", "id": "l", "n": 3},
          {"op": "lim_add", "id": "l", "n": 3},
          {"op": "lim_can_pass", "id": "l", "expect": True},
          {"op": "lim_sum", "id": "l", "expect": 9},
          {"op": "lim_add", "id": "l", "n": 3},
          {"op": "lim_can_pass", "id": "l", "expect": False},
          {"op": "sleep", "ms": 1000},
          {"op": "lim_add", "id": "l", "n": 3},
          {"op": "lim_try_pass", "id": "l", "expect": True},
          {"op": "lim_can_pass", "id": "l", "expect": True},
          {"op": "lim_sum", "id": "l", "expect": 4}])

scenario("GlobalRequestLimiterTest.testPass",
         CST + "/flow/statistic/limit/GlobalRequestLimiterTest.java:33-49",
         [{"op": "set_time", "t": 0},
          {"op": "lim_new", "id": "l", "qps": 3},
          {"op": "lim_try_pass", "id": "l", "expect": True},
          {"op": "lim_try_pass", "id": "l", "expect": True},
          {"op": "lim_try_pass", "id": "l", "expect": True},
          {"op": "lim_try_pass", "id": "l", "expect": False},
          {"op": "lim_qps", "id": "l", "expect": 3, "tol": 0.01},
          {"op": "sleep", "ms": 1000},
          {"op": "lim_try_pass", "id": "l", "expect": True},
          {"op": "lim_try_pass", "id": "l", "expect": True},
          {"op": "lim_qps", "id": "l", "expect": 2, "tol": 0.01}])

# ClusterFlowCheckerTest is disabled upstream (//@Test) and used real sleeps; its
# asserted pass/block/wait sequence is replayed here under the mocked clock.
_R = {"flow_id": 98765, "count": 5, "threshold_type": 1, "sample_count": 5, "window_interval_ms": 1000}
_ops = [{"op": "set_time", "t": 0},
        {"op": "cl_new", "id": "s"},
        {"op": "cl_load", "id": "s", "namespace": "default", "rules": [_R]}]


def _acq(prio, status, wait=0):
    return {"op": "cl_request", "id": "s", "flow_id": 98765, "acquire": 1, "prio": prio,
            "expect_status": status, "expect_wait": wait}


_ops += [_acq(False, "OK"), _acq(False, "OK"), {"op": "sleep", "ms": 200}, _acq(False, "OK"),
         {"op": "sleep", "ms": 200}, _acq(True, "OK"), _acq(False, "OK"), _acq(True, "BLOCKED"),
         {"op": "sleep", "ms": 200}, _acq(False, "BLOCKED"), _acq(False, "BLOCKED"),
         {"op": "sleep", "ms": 200}, _acq(False, "BLOCKED"), _acq(True, "SHOULD_WAIT", 200), _acq(False, "BLOCKED"),
         {"op": "sleep", "ms": 200}, _acq(False, "OK")]
scenario("ClusterFlowCheckerTest.testAcquireClusterTokenOccupyPass (disabled upstream, mocked clock)",
         CST + "/flow/ClusterFlowCheckerTest.java:37-75", _ops)

scenario("DefaultTokenService request validation",
         "sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/flow/"
         "DefaultTokenService.java:39-50,87-89",
         [{"op": "set_time", "t": 0},
          {"op": "cl_new", "id": "s"},
          {"op": "cl_load", "id": "s", "namespace": "default", "rules": [_R]},
          {"op": "cl_request", "id": "s", "flow_id": 0, "acquire": 1, "prio": False, "expect_status": "BAD_REQUEST"},
          {"op": "cl_request", "id": "s", "flow_id": 98765, "acquire": 0, "prio": False,
           "expect_status": "BAD_REQUEST"},
          {"op": "cl_request", "id": "s", "flow_id": 12345, "acquire": 1, "prio": False,
           "expect_status": "NO_RULE_EXISTS"},
          {"op": "cl_request", "id": "s", "flow_id": 98765, "acquire": 1, "prio": False, "expect_status": "OK",
           "expect_remaining": 4}], bases=BASES[:1])

# ------------------------------------------------------------ param flow
def _prule(**kw):
    r = {"grade": 1, "count": 5, "control_behavior": 0, "max_queueing_time_ms": 0, "burst_count": 0,
         "param_idx": 0, "duration_in_sec": 1}
    r.update(kw)
    return r


def _pp(expect, n=1):
    return [{"op": "prule_pass", "id": "p", "value": 0x76616C756541, "acquire": 1, "expect": expect}] * n


_ops = [{"op": "set_time", "t": 0}, {"op": "prule_new", "id": "p", "rule": _prule(count=25000)}]
_ops += _pp(True, 2) + [{"op": "sleep", "ms": 1000 * 60 * 60 * 24}] + _pp(True, 2) + \
    [{"op": "sleep", "ms": 1000 * 60 * 60 * 48}] + _pp(True, 2)
scenario("ParamFlowDefaultCheckerTest.testCheckQpsWithLongIntervalAndHighThreshold",
         PFT + "/slots/block/flow/param/ParamFlowDefaultCheckerTest.java:46-82", _ops)

_ops = [{"op": "set_time", "t": 0}, {"op": "prule_new", "id": "p", "rule": _prule(count=5)}]
_ops += _pp(True, 5) + _pp(False) + [{"op": "sleep", "ms": 3000}] + _pp(True, 5) + _pp(False)
scenario("ParamFlowDefaultCheckerTest.testParamFlowDefaultCheckSingleQps",
         PFT + "/slots/block/flow/param/ParamFlowDefaultCheckerTest.java:84-116", _ops)

_ops = [{"op": "set_time", "t": 0}, {"op": "prule_new", "id": "p", "rule": _prule(count=5, burst_count=3)}]
_ops += _pp(True, 8) + _pp(False) + [{"op": "sleep", "ms": 1002}] + _pp(True, 5) + _pp(False) + \
    [{"op": "sleep", "ms": 1002}] + _pp(True, 5) + _pp(False) + [{"op": "sleep", "ms": 2000}] + _pp(True, 8) + \
    _pp(False) + [{"op": "sleep", "ms": 1002}] + _pp(True, 5) + _pp(False)
scenario("ParamFlowDefaultCheckerTest.testParamFlowDefaultCheckSingleQpsWithBurst",
         PFT + "/slots/block/flow/param/ParamFlowDefaultCheckerTest.java:118-171", _ops)

_ops = [{"op": "set_time", "t": 0}, {"op": "prule_new", "id": "p", "rule": _prule(count=5, duration_in_sec=60)}]
_ops += _pp(True, 5) + _pp(False) + [{"op": "sleep", "ms": 1000}] + _pp(False) + [{"op": "sleep", "ms": 10000}] + \
    _pp(False) + [{"op": "sleep", "ms": 30000}] + _pp(False) + [{"op": "sleep", "ms": 30000}] + _pp(True, 5) + \
    _pp(False)
scenario("ParamFlowDefaultCheckerTest.testParamFlowDefaultCheckQpsInDifferentDuration",
         PFT + "/slots/block/flow/param/ParamFlowDefaultCheckerTest.java:173-213", _ops)

# --------------------------------------------------------- circuit breakers
def _deg(**kw):
    r = {"resource": 0, "grade": 0, "count": 0, "time_window": 1, "min_request_amount": 5,
         "slow_ratio_threshold": 1.0, "stat_interval_ms": 1000}
    r.update(kw)
    return r


def _es(ms, expect):  # AbstractTimeBasedTest.entryAndSleepFor
    return {"op": "flow_entry_sleep", "id": "f", "resource": 0, "ms": ms, "expect": expect}


def _ee(expect, ms=7):  # entryWithErrorIfPresent(res, exception): sleep 5..10 ms (fixed 7 here)
    return {"op": "flow_entry_error", "id": "f", "resource": 0, "ms": ms, "expect": expect}


_ops = [{"op": "set_time", "t": 0}, {"op": "flow_new", "id": "f", "n_resources": 1},
        {"op": "flow_load_degrade", "id": "f", "rules": [_deg(grade=1, count=0.2, stat_interval_ms=20000,
                                                              time_window=10, min_request_amount=1)]},
        _es(10, True), _ee(True), _ee(False), _es(100, False), {"op": "sleep", "ms": 5000}, _es(100, False),
        {"op": "sleep", "ms": 5000}, _ee(True), _es(100, False), _es(100, False), {"op": "sleep", "ms": 10000}]
_ops += [_es(100, True)] * 7 + [_ee(True), _es(100, True)]
scenario("ExceptionCircuitBreakerTest.testRecordErrorOrSuccess",
         CORET_DEG + "/ExceptionCircuitBreakerTest.java:50-83", _ops)

_ops = [{"op": "set_time", "t": 0}, {"op": "flow_new", "id": "f", "n_resources": 1},
        {"op": "flow_load_degrade", "id": "f", "rules": [_deg(grade=0, count=10, min_request_amount=3,
                                                              slow_ratio_threshold=1, stat_interval_ms=5000,
                                                              time_window=5)]},
        _es(20, True), _es(20, True), _es(20, True), _es(20, False), {"op": "sleep", "ms": 1000}, _es(20, False),
        {"op": "sleep", "ms": 4000}, _es(20, True)]
# the reference test implicitly assumes its first 60 ms do not straddle a 5 s stat-bucket boundary
# (statIntervalMs 5000, one bucket): bases with t % 5000 > 4940 would roll the bucket between the
# three slow exits in the reference too, so only non-straddling bases are used.
scenario("ResponseTimeCircuitBreakerTest.testMaxSlowRatioThreshold",
         CORET_DEG + "/ResponseTimeCircuitBreakerTest.java:33-55", _ops, bases=BASES[:4])


def main():
    for sc in SCENARIOS:
        safe = "".join(ch if ch.isalnum() else "_" for ch in sc["name"]).strip("_")
        while "__" in safe:
            safe = safe.replace("__", "_")
        path = os.path.join(HERE, "kat_" + safe[:80] + ".json")
        with open(path, "w") as f:
            json.dump(sc, f, indent=1)
    print(f"wrote {len(SCENARIOS)} scenarios")


if __name__ == "__main__":
    main()
