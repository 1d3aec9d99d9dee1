"""ctypes binding to the ORACLE (oracle/build/liboracle.so) and the interpreter
for the transcribed known-answer scenarios in tests/golden/kat_*.json.

Test infrastructure only: the oracle is the checker, never the thing measured
or shipped.
"""
import ctypes as C
import glob
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

EV = {"PASS": 0, "BLOCK": 1, "EXCEPTION": 2, "SUCCESS": 3, "RT": 4, "OCCUPIED_PASS": 5}
CEV = {"PASS": 0, "BLOCK": 1, "PASS_REQUEST": 2, "BLOCK_REQUEST": 3, "OCCUPIED_PASS": 4, "OCCUPIED_BLOCK": 5,
       "WAITING": 6}
LEAP_KIND = {"bucket": 0, "occupiable": 1, "future": 2, "cluster": 3, "unary": 4}
DECISION = {"PASS": 0, "BLOCK": 1, "BLOCK_PARAM": 2, "BLOCK_DEGRADE": 3, "PASS_WAIT": 4}
TOKEN_STATUS = {"BAD_REQUEST": -4, "TOO_MANY_REQUEST": -2, "FAIL": -1, "OK": 0, "BLOCKED": 1, "SHOULD_WAIT": 2,
                "NO_RULE_EXISTS": 3}


class OrcFlowRule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double),
                ("control_behavior", C.c_int32), ("warm_up_period_sec", C.c_int32),
                ("max_queueing_time_ms", C.c_int32), ("strategy", C.c_int32),
                ("cluster_mode", C.c_int32), ("cluster_fallback", C.c_int32), ("cluster_flow_id", C.c_int64),
                ("cluster_sample_count", C.c_int32), ("cluster_window_ms", C.c_int32),
                ("cluster_strategy", C.c_int32), ("reserved", C.c_int32)]


class OrcClusterRule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32), ("grade", C.c_int32),
                ("strategy", C.c_int32), ("reserved", C.c_int32), ("resource_timeout_ms", C.c_int64),
                ("client_offline_time_ms", C.c_int64)]


class OrcSystemRule(C.Structure):
    _fields_ = [("highest_system_load", C.c_double), ("highest_cpu_usage", C.c_double), ("qps", C.c_double),
                ("avg_rt", C.c_int64), ("max_thread", C.c_int64)]


class OrcConcResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("reserved", C.c_int32), ("token_id", C.c_int64)]


class OrcParamRule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double),
                ("control_behavior", C.c_int32), ("max_queueing_time_ms", C.c_int32), ("burst_count", C.c_int32),
                ("param_idx", C.c_int32), ("duration_in_sec", C.c_int64), ("n_hot", C.c_uint32),
                ("hot_values", C.POINTER(C.c_uint64)), ("hot_thresholds", C.POINTER(C.c_int32)),
                ("cluster_mode", C.c_int32), ("cluster_fallback", C.c_int32), ("cluster_flow_id", C.c_int64),
                ("cluster_sample_count", C.c_int32), ("cluster_window_ms", C.c_int32)]


class OrcDegradeRule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double), ("time_window", C.c_int32),
                ("min_request_amount", C.c_int32), ("slow_ratio_threshold", C.c_double),
                ("stat_interval_ms", C.c_int32)]


class OrcTokenResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("remaining", C.c_int32), ("wait_in_ms", C.c_int32)]


_lib = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        build_oracle()
    L = C.CDLL(ORACLE_SO)
    P, I64, I32, D, U32 = C.c_void_p, C.c_int64, C.c_int32, C.c_double, C.c_uint32
    sigs = {
        "orc_leap_new": (P, [C.c_int, C.c_int, C.c_int]),
        "orc_leap_free": (None, [P]),
        "orc_leap_current_window": (I64, [P, I64]),
        "orc_leap_add": (None, [P, I64, C.c_int, I64]),
        "orc_leap_current_get": (I64, [P, I64, C.c_int]),
        "orc_leap_values_sum": (I64, [P, I64, C.c_int, C.POINTER(C.c_int)]),
        "orc_leap_previous_window": (C.c_int, [P, I64, I64, C.POINTER(I64), C.POINTER(I64)]),
        "orc_leap_valid_head": (C.c_int, [P, I64, C.POINTER(I64), C.POINTER(I64)]),
        "orc_leap_add_waiting": (None, [P, I64, C.c_int]),
        "orc_leap_current_waiting": (I64, [P, I64]),
        "orc_node_new": (P, []),
        "orc_node_new_mock": (P, [D, D, I32]),
        "orc_node_set_mock": (None, [P, D, D, I32]),
        "orc_node_free": (None, [P]),
        "orc_node_pass_qps": (D, [P, I64]),
        "orc_node_total_pass": (I64, [P, I64]),
        "orc_ctrl_new": (P, [C.c_int, C.c_int, D, C.c_int, C.c_int, C.c_int]),
        "orc_ctrl_free": (None, [P]),
        "orc_ctrl_can_pass": (C.c_int, [P, P, I64, C.c_int, C.c_int, C.POINTER(I64)]),
        "orc_flow_new": (P, [U32, C.c_int]),
        "orc_flow_free": (None, [P]),
        "orc_flow_load_rules": (C.c_int, [P, C.POINTER(OrcFlowRule), C.c_size_t]),
        "orc_flow_set_cluster": (None, [P, P, C.c_int]),
        "orc_flow_entry": (C.c_int, [P, U32, I64, C.c_int, C.c_int, C.POINTER(I64)]),
        "orc_flow_exit": (None, [P, U32, I64, I64, C.c_int, C.c_int]),
        "orc_flow_replay": (None, [P, C.c_size_t, P, P, P, P, P, P, P, P]),
        "orc_flow_node": (P, [P, U32]),
        "orc_cluster_new": (P, [D, D]),
        "orc_cluster_free": (None, [P]),
        "orc_cluster_load_rules": (C.c_int, [P, C.c_char_p, C.POINTER(OrcClusterRule), C.c_size_t]),
        "orc_cluster_set_namespace_limit": (None, [P, C.c_char_p, D]),
        "orc_cluster_set_connected_count": (None, [P, C.c_char_p, I32]),
        "orc_cluster_request_token": (OrcTokenResult, [P, I64, I32, C.c_int, I64]),
        "orc_cluster_request_token_simple": (OrcTokenResult, [P, I64, I32, I64]),
        "orc_cluster_replay": (None, [P, C.c_size_t, P, P, P, P, P]),
        "orc_cluster_replay_simple": (None, [P, C.c_size_t, P, P, P, P]),
        "orc_cluster_metric_sum": (I64, [P, I64, C.c_int, I64]),
        "orc_cmetric_new": (P, [C.c_int, C.c_int]),
        "orc_cmetric_free": (None, [P]),
        "orc_cmetric_add": (None, [P, I64, C.c_int, I64]),
        "orc_cmetric_sum": (I64, [P, I64, C.c_int]),
        "orc_cmetric_avg": (D, [P, I64, C.c_int]),
        "orc_cmetric_try_occupy_next": (I32, [P, I64, C.c_int, I32, D]),
        "orc_flow_metrics": (C.c_size_t, [P, I64, P, C.c_size_t]),
        "orc_pmetric_new": (P, [C.c_int, C.c_int]),
        "orc_pmetric_free": (None, [P]),
        "orc_pmetric_add": (None, [P, I64, I64, I32]),
        "orc_pmetric_sum": (I64, [P, I64, I64]),
        "orc_pmetric_avg": (D, [P, I64, I64]),
        "orc_cluster_load_param_rules": (C.c_int, [P, C.c_char_p, C.POINTER(OrcClusterParamRule), C.c_size_t]),
        "orc_cluster_request_param_token": (OrcTokenResult, [P, I64, I32, P, C.c_size_t, I64]),
        "orc_cluster_param_replay": (None, [P, C.c_size_t, P, P, P, P, P, P]),
        "orc_cluster_param_sum": (I64, [P, I64, I64, I64]),
        "orc_cluster_set_param_capacity": (None, [C.c_size_t]),
        "orc_flow_load_system_rules": (C.c_int, [P, C.POINTER(OrcSystemRule), C.c_size_t]),
        "orc_flow_set_system_status": (None, [P, D, D]),
        "orc_flow_entry_x": (C.c_int, [P, U32, I64, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.POINTER(I64)]),
        "orc_flow_exit_x": (None, [P, U32, I64, I64, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int]),
        "orc_flow_entry_node": (P, [P]),
        "orc_node_max_success_qps": (D, [P, I64]),
        "orc_cluster_param_top_values": (C.c_size_t, [P, I64, I64, C.c_size_t, P, P]),
        "orc_cluster_concurrent_acquire": (OrcConcResult, [P, U32, I64, I32, I64, I64]),
        "orc_cluster_concurrent_release": (I32, [P, I64]),
        "orc_cluster_concurrent_expire": (C.c_uint64, [P, I64, P, U32]),
        "orc_cluster_concurrent_now_calls": (C.c_int, [P, I64, C.POINTER(I32)]),
        "orc_cluster_concurrent_tokens": (C.c_size_t, [P]),
        "orc_cluster_concurrent_get": (C.c_int, [P, I64, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64),
                                                 C.POINTER(I32)]),
        "orc_limiter_new": (P, [D]),
        "orc_limiter_free": (None, [P]),
        "orc_limiter_add": (None, [P, I64, C.c_int]),
        "orc_limiter_sum": (I64, [P, I64]),
        "orc_limiter_qps": (D, [P, I64]),
        "orc_limiter_can_pass": (C.c_int, [P, I64]),
        "orc_limiter_try_pass": (C.c_int, [P, I64]),
        "orc_flow_load_param_rules": (C.c_int, [P, C.POINTER(OrcParamRule), C.c_size_t]),
        "orc_flow_load_degrade_rules": (C.c_int, [P, C.POINTER(OrcDegradeRule), C.c_size_t]),
        "orc_flow_entry_p": (C.c_int, [P, U32, I64, C.c_int, C.c_int, C.c_int, C.c_uint64, C.POINTER(I64)]),
        "orc_flow_exit_p": (None, [P, U32, I64, I64, C.c_int, C.c_int, C.c_int, C.c_uint64]),
        "orc_flow_cb_state": (C.c_int, [P, U32, C.c_int]),
        "orc_flow_replay_p": (None, [P, C.c_size_t, P, P, P, P, P, P, P, P, P]),
        "orc_flow_replay_pl": (None, [P, C.c_size_t, P, P, P, P, P, P, P, P, P, P]),
        "orc_flow_replay_args": (None, [P, C.c_size_t, P, P, P, P, P, P, P, P, P, P]),
        "orc_flow_param_idx": (I32, [P, U32, C.c_int]),
        "orc_prule_new": (P, [C.POINTER(OrcParamRule)]),
        "orc_prule_free": (None, [P]),
        "orc_prule_pass_single": (C.c_int, [P, C.c_uint64, C.c_int, I64, I64, C.POINTER(I64)]),
        "orc_java_round": (I64, [D]),
        "orc_java_next_up": (D, [D]),
        "orc_java_d2i": (I32, [D]),
        "orc_java_d2l": (I64, [D]),
        "orc_java_string_hash": (I32, [C.c_char_p]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def flow_rules_array(rules):
    arr = (OrcFlowRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i].resource = r["resource"]
        arr[i].grade = r.get("grade", 1)
        arr[i].count = r["count"]
        arr[i].control_behavior = r.get("control_behavior", 0)
        arr[i].warm_up_period_sec = r.get("warm_up_period_sec", 10)
        arr[i].max_queueing_time_ms = r.get("max_queueing_time_ms", 500)
        arr[i].strategy = r.get("strategy", 0)
        arr[i].cluster_mode = 1 if r.get("cluster_mode") else 0
        arr[i].cluster_fallback = 1 if r.get("cluster_fallback", True) else 0
        arr[i].cluster_flow_id = r.get("cluster_flow_id", 0)
        arr[i].cluster_sample_count = r.get("cluster_sample_count", 10)
        arr[i].cluster_window_ms = r.get("cluster_window_ms", 1000)
        arr[i].cluster_strategy = r.get("cluster_strategy", 0)
    return arr


def cluster_rules_array(rules):
    arr = (OrcClusterRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i].flow_id = r["flow_id"]
        arr[i].count = r["count"]
        arr[i].threshold_type = r.get("threshold_type", 0)
        arr[i].sample_count = r.get("sample_count", 10)
        arr[i].window_interval_ms = r.get("window_interval_ms", 1000)
        arr[i].grade = r.get("grade", 1)
        arr[i].strategy = r.get("strategy", 0)
        arr[i].resource_timeout_ms = r.get("resource_timeout", 2000)
        arr[i].client_offline_time_ms = r.get("client_offline_time", 2000)
    return arr


def param_rule_struct(r, keep):
    x = OrcParamRule()
    x.resource = r.get("resource", 0)
    x.grade = r.get("grade", 1)
    x.count = r["count"]
    x.control_behavior = r.get("control_behavior", 0)
    x.max_queueing_time_ms = r.get("max_queueing_time_ms", 0)
    x.burst_count = r.get("burst_count", 0)
    x.param_idx = r.get("param_idx", 0)
    x.duration_in_sec = r.get("duration_in_sec", 1)
    x.cluster_mode = 1 if r.get("cluster_mode") else 0
    x.cluster_fallback = 1 if r.get("cluster_fallback") else 0
    x.cluster_flow_id = r.get("cluster_flow_id", 0)
    x.cluster_sample_count = r.get("cluster_sample_count", 10)
    x.cluster_window_ms = r.get("cluster_window_ms", 1000)
    hot = r.get("hot", {})
    x.n_hot = len(hot)
    if hot:
        hv = (C.c_uint64 * len(hot))(*[int(k) for k in hot])
        ht = (C.c_int32 * len(hot))(*[int(v) for v in hot.values()])
        keep += [hv, ht]
        x.hot_values = hv
        x.hot_thresholds = ht
    return x


def param_rules_array(rules, keep):
    arr = (OrcParamRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i] = param_rule_struct(r, keep)
    return arr


def degrade_rules_array(rules):
    arr = (OrcDegradeRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i].resource = r.get("resource", 0)
        arr[i].grade = r.get("grade", 0)
        arr[i].count = r["count"]
        arr[i].time_window = r.get("time_window", 1)
        arr[i].min_request_amount = r.get("min_request_amount", 5)
        arr[i].slow_ratio_threshold = r.get("slow_ratio_threshold", 1.0)
        arr[i].stat_interval_ms = r.get("stat_interval_ms", 1000)
    return arr


def load_scenarios():
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "kat_*.json"))):
        with open(p) as f:
            out.append(json.load(f))
    return out


class ScenarioFailure(AssertionError):
    pass


def java_obj_key(v):
    """64-bit stand-in for a Java parameter Object: Integer/Long values as themselves, Strings by
    String.hashCode (the engine's contract: the caller maps each parameter to a stable int64)."""
    if isinstance(v, str):
        return int(lib().orc_java_string_hash(v.encode()))
    return int(v)


class OrcMetricNode(C.Structure):
    _fields_ = [("timestamp", C.c_int64), ("pass_qps", C.c_int64), ("block_qps", C.c_int64),
                ("success_qps", C.c_int64), ("exception_qps", C.c_int64), ("rt", C.c_int64),
                ("occupied_pass_qps", C.c_int64), ("resource", C.c_uint32), ("concurrency", C.c_int32)]


class OrcClusterParamRule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32), ("grade", C.c_int32),
                ("burst_count", C.c_int32), ("control_behavior", C.c_int32), ("max_queueing_time_ms", C.c_int32),
                ("param_idx_set", C.c_int32), ("duration_in_sec", C.c_int64), ("n_hot", C.c_int32),
                ("reserved", C.c_int32), ("hot_values", C.POINTER(C.c_int64)), ("hot_counts", C.POINTER(C.c_int32))]


def cluster_param_rules_array(rules, keep):
    """rules: dicts {flow_id, count, threshold_type?, sample_count?, window_interval_ms?, hot?: {v: c}}.
    `keep` collects the hot-item buffers so they outlive the call."""
    arr = (OrcClusterParamRule * max(1, len(rules)))()
    for i, r in enumerate(rules):
        a = arr[i]
        a.flow_id = r["flow_id"]
        a.count = float(r["count"])
        a.threshold_type = r.get("threshold_type", 0)
        a.sample_count = r.get("sample_count", 10)
        a.window_interval_ms = r.get("window_interval_ms", 1000)
        a.grade = r.get("grade", 1)
        a.burst_count = r.get("burst_count", 0)
        a.control_behavior = r.get("control_behavior", 0)
        a.max_queueing_time_ms = r.get("max_queueing_time_ms", 0)
        a.param_idx_set = 1 if r.get("param_idx_set", True) else 0
        a.duration_in_sec = r.get("duration_in_sec", 1)
        hot = r.get("hot", {})
        a.n_hot = len(hot)
        if hot:
            hv = (C.c_int64 * len(hot))(*[int(k) for k in hot])
            hc = (C.c_int32 * len(hot))(*[int(v) for v in hot.values()])
            keep.extend([hv, hc])
            a.hot_values = C.cast(hv, C.POINTER(C.c_int64))
            a.hot_counts = C.cast(hc, C.POINTER(C.c_int32))
    return arr


def run_scenario(sc, base):
    """Replays one transcribed scenario against the oracle at virtual base time `base`."""
    L = lib()
    objs = {}
    now = base

    def T(v):
        if v == "now":
            return now
        if isinstance(v, dict):
            b = base - base % v["window"]
            return b + v["aligned_plus"]
        return base + v

    def check(cond, op, got):
        if not cond:
            raise ScenarioFailure(f"{sc['name']} @base={base}: op {op} got {got}")

    frees = []
    try:
        for op in sc["ops"]:
            k = op["op"]
            if k == "set_time":
                now = base + op["t"]
            elif k == "sleep":
                now += op["ms"]
            elif k == "leap_new":
                h = L.orc_leap_new(LEAP_KIND[op["kind"]], op["sample_count"], op["interval_ms"])
                objs[op["id"]] = h
                frees.append((L.orc_leap_free, h))
            elif k == "leap_current_window":
                got = L.orc_leap_current_window(objs[op["id"]], T(op["t"]))
                if "expect_start" in op:
                    check(got == T(op["expect_start"]), op, got)
            elif k == "leap_add":
                ev = op["event"] if isinstance(op["event"], int) else EV[op["event"]]
                L.orc_leap_add(objs[op["id"]], T(op["t"]), ev, op["n"])
            elif k == "leap_current_get":
                got = L.orc_leap_current_get(objs[op["id"]], T(op["t"]), EV[op["event"]])
                check(got == op["expect"], op, got)
            elif k == "leap_values_sum":
                cnt = C.c_int()
                got = L.orc_leap_values_sum(objs[op["id"]], T(op["t"]), EV[op["event"]], C.byref(cnt))
                check(got == op["expect"] and cnt.value == op.get("expect_count", cnt.value), op, (got, cnt.value))
            elif k == "leap_add_waiting":
                L.orc_leap_add_waiting(objs[op["id"]], T(op["t"]), op["n"])
            elif k == "leap_current_waiting":
                got = L.orc_leap_current_waiting(objs[op["id"]], now)
                check(got == op["expect"], op, got)
            elif k == "leap_previous_window":
                st, ps = C.c_int64(), C.c_int64()
                ok = L.orc_leap_previous_window(objs[op["id"]], T(op["t"]), now, C.byref(st), C.byref(ps))
                if op.get("expect_null"):
                    check(ok == 0, op, ok)
                else:
                    check(ok == 1 and st.value == T(op["expect_start"]), op, (ok, st.value))
            elif k == "leap_valid_head":
                st, ps = C.c_int64(), C.c_int64()
                ok = L.orc_leap_valid_head(objs[op["id"]], now, C.byref(st), C.byref(ps))
                if op.get("expect_null"):
                    check(ok == 0, op, ok)
                else:
                    check(ok == 1 and st.value == T(op["expect_start"]), op, (ok, st.value))
            elif k == "ctrl_new":
                h = L.orc_ctrl_new(op["behavior"], op["grade"], float(op["count"]), op.get("warm_up_period_sec", 10),
                                   op.get("max_queueing_time_ms", 500), op.get("cold_factor", 3))
                objs[op["id"]] = h
                frees.append((L.orc_ctrl_free, h))
            elif k == "node_mock":
                if op["id"] not in objs:
                    h = L.orc_node_new_mock(op["pass_qps"], op["prev_pass_qps"], op["threads"])
                    objs[op["id"]] = h
                    frees.append((L.orc_node_free, h))
                else:
                    L.orc_node_set_mock(objs[op["id"]], op["pass_qps"], op["prev_pass_qps"], op["threads"])
            elif k == "ctrl_can_pass":
                w = C.c_int64()
                d = L.orc_ctrl_can_pass(objs[op["id"]], objs[op["node"]], now, op["acquire"],
                                        1 if op.get("prio") else 0, C.byref(w))
                if "expect" in op:
                    want = DECISION[op["expect"]]
                    check(d == want, op, d)
                if "expect_wait" in op:
                    check(w.value == op["expect_wait"], op, w.value)
                if op.get("sleep_wait"):
                    now += w.value
            elif k == "flow_new":
                h = L.orc_flow_new(op["n_resources"], op.get("cold_factor", 3))
                objs[op["id"]] = h
                frees.append((L.orc_flow_free, h))
            elif k == "flow_load":
                arr = flow_rules_array(op["rules"])
                L.orc_flow_load_rules(objs[op["id"]], arr, len(op["rules"]))
            elif k == "flow_entry":
                w = C.c_int64()
                d = L.orc_flow_entry(objs[op["id"]], op["resource"], now, op["acquire"], 1 if op.get("prio") else 0,
                                     C.byref(w))
                check(d == DECISION[op["expect"]], op, d)
            elif k == "flow_exit":
                L.orc_flow_exit(objs[op["id"]], op["resource"], now, op["rt"], op["count"], 1 if op.get("error") else 0)
            elif k == "flow_loop":
                per_sec = {}
                t0 = now
                for ms in range(op["ms"]):
                    t = t0 + ms
                    for _ in range(op["per_ms"]):
                        d = L.orc_flow_entry(objs[op["id"]], op["resource"], t, 1, 0, None)
                        if d == 0:
                            sec = (t - t0) // 1000
                            per_sec[sec] = per_sec.get(sec, 0) + 1
                            L.orc_flow_exit(objs[op["id"]], op["resource"], t, 0, 1, 0)
                got = [per_sec.get(s, 0) for s in range(len(op["expect_pass_per_second"]))]
                check(got == op["expect_pass_per_second"], op, got)
                now = t0 + op["ms"]
            elif k == "cm_new":
                h = L.orc_cmetric_new(op["sample_count"], op["interval_ms"])
                objs[op["id"]] = h
                frees.append((L.orc_cmetric_free, h))
            elif k == "cm_add":
                L.orc_cmetric_add(objs[op["id"]], now, CEV[op["event"]], op["n"])
            elif k == "cm_sum":
                got = L.orc_cmetric_sum(objs[op["id"]], now, CEV[op["event"]])
                check(got == op["expect"], op, got)
            elif k == "cm_avg":
                got = L.orc_cmetric_avg(objs[op["id"]], now, CEV[op["event"]])
                check(abs(got - op["expect"]) <= op.get("tol", 0), op, got)
            elif k == "pm_new":
                h = L.orc_pmetric_new(op["sample_count"], op["interval_ms"])
                objs[op["id"]] = h
                frees.append((L.orc_pmetric_free, h))
            elif k == "pm_add":
                L.orc_pmetric_add(objs[op["id"]], now, java_obj_key(op["value"]), op["n"])
            elif k == "pm_sum":
                got = L.orc_pmetric_sum(objs[op["id"]], now, java_obj_key(op["value"]))
                check(got == op["expect"], op, got)
            elif k == "pm_avg":
                got = L.orc_pmetric_avg(objs[op["id"]], now, java_obj_key(op["value"]))
                check(abs(got - op["expect"]) <= op.get("tol", 0), op, got)
            elif k == "cm_try_occupy_next":
                got = L.orc_cmetric_try_occupy_next(objs[op["id"]], now, CEV["PASS"], op["acquire"],
                                                    float(op["threshold"]))
                check(got == op["expect"], op, got)
            elif k == "lim_new":
                h = L.orc_limiter_new(float(op["qps"]))
                objs[op["id"]] = h
                frees.append((L.orc_limiter_free, h))
            elif k == "lim_add":
                L.orc_limiter_add(objs[op["id"]], now, op["n"])
            elif k == "lim_can_pass":
                got = bool(L.orc_limiter_can_pass(objs[op["id"]], now))
                check(got == op["expect"], op, got)
            elif k == "lim_try_pass":
                got = bool(L.orc_limiter_try_pass(objs[op["id"]], now))
                check(got == op["expect"], op, got)
            elif k == "lim_sum":
                got = L.orc_limiter_sum(objs[op["id"]], now)
                check(got == op["expect"], op, got)
            elif k == "lim_qps":
                got = L.orc_limiter_qps(objs[op["id"]], now)
                check(abs(got - op["expect"]) <= op.get("tol", 0), op, got)
            elif k == "cl_new":
                h = L.orc_cluster_new(op.get("exceed_count", 1.0), op.get("max_occupy_ratio", 1.0))
                objs[op["id"]] = h
                frees.append((L.orc_cluster_free, h))
            elif k == "cl_load":
                arr = cluster_rules_array(op["rules"])
                L.orc_cluster_load_rules(objs[op["id"]], op["namespace"].encode(), arr, len(op["rules"]))
            elif k == "cl_request":
                r = L.orc_cluster_request_token(objs[op["id"]], op["flow_id"], op["acquire"],
                                                1 if op.get("prio") else 0, now)
                check(r.status == TOKEN_STATUS[op["expect_status"]], op, (r.status, r.remaining, r.wait_in_ms))
                if "expect_wait" in op:
                    check(r.wait_in_ms == op["expect_wait"], op, r.wait_in_ms)
                if "expect_remaining" in op:
                    check(r.remaining == op["expect_remaining"], op, r.remaining)
            elif k == "prule_new":
                keep = []
                h = L.orc_prule_new(C.byref(param_rule_struct(op["rule"], keep)))
                objs[op["id"]] = h
                frees.append((L.orc_prule_free, h))
            elif k == "prule_pass":
                w = C.c_int64()
                got = bool(L.orc_prule_pass_single(objs[op["id"]], op["value"], op["acquire"], now,
                                                   op.get("threads", 0), C.byref(w)))
                check(got == op["expect"], op, got)
            elif k == "flow_load_degrade":
                arr = degrade_rules_array(op["rules"])
                L.orc_flow_load_degrade_rules(objs[op["id"]], arr, len(op["rules"]))
            elif k in ("flow_entry_sleep", "flow_entry_error"):
                w = C.c_int64()
                d = L.orc_flow_entry_p(objs[op["id"]], op["resource"], now, 1, 0, 0, 0, C.byref(w))
                passed = d in (0, 4)
                if passed:
                    t_in = now
                    now += op["ms"]
                    L.orc_flow_exit_p(objs[op["id"]], op["resource"], now, now - t_in, 1,
                                      1 if k == "flow_entry_error" else 0, 0, 0)
                check(passed == op["expect"], op, d)
            else:
                raise ScenarioFailure(f"unknown op {k}")
    finally:
        for fn, h in reversed(frees):
            fn(h)


def cluster_replay_sharded(rule_fid, rule_count, batches, threads=16, sample_count=10, interval_ms=1000):
    """The oracle's ClusterFlowChecker replay of whole C3 batches (GLOBAL rules, no namespace limiter):
    rules are independent, so each of `threads` oracle instances replays the requests of the flowIds
    with flowId mod threads == k in arrival order (ctypes releases the GIL: the threads run in parallel).
    batches: [(flowId int64, acquire int32, prio u8, time int64)] in order.  Returns per batch the
    (status, remaining, waitInMs) int32 arrays in request order."""
    import threading

    import numpy as np
    L = lib()
    rule_fid = np.asarray(rule_fid, np.int64)
    rule_count = np.asarray(rule_count, np.float64)
    rdt = np.dtype([("flow_id", np.int64), ("count", np.float64), ("threshold_type", np.int32),
                    ("sample_count", np.int32), ("window_interval_ms", np.int32), ("grade", np.int32),
                    ("strategy", np.int32), ("reserved", np.int32), ("resource_timeout_ms", np.int64),
                    ("client_offline_time_ms", np.int64)])
    assert rdt.itemsize == C.sizeof(OrcClusterRule), "oracle rule layout"
    hs = []
    for k in range(threads):
        sel = (rule_fid % threads) == k
        arr = np.zeros(int(sel.sum()), dtype=rdt)
        arr["flow_id"], arr["count"] = rule_fid[sel], rule_count[sel]
        arr["threshold_type"], arr["sample_count"], arr["window_interval_ms"], arr["grade"] = 1, sample_count, \
            interval_ms, 1
        arr["resource_timeout_ms"], arr["client_offline_time_ms"] = 2000, 2000
        h = L.orc_cluster_new(1.0, 1.0)
        L.orc_cluster_load_rules(h, b"default", arr.ctypes.data_as(C.POINTER(OrcClusterRule)), len(arr))
        hs.append(h)
    results = []
    for f, a, p, ts in batches:
        f = np.ascontiguousarray(f, np.int64)
        shard = np.mod(f, threads).astype(np.uint8 if threads <= 256 else np.int64)
        order = np.argsort(shard, kind="stable")  # radix sort for small integer keys
        bounds = np.concatenate([[0], np.cumsum(np.bincount(shard, minlength=threads))])
        parts = [np.ascontiguousarray(x[order]) for x in (f, np.asarray(a, np.int32), np.asarray(p, np.uint8),
                                                             np.asarray(ts, np.int64))]
        out = np.zeros((len(f), 3), dtype=np.int32)

        def run(k):
            lo, hi = int(bounds[k]), int(bounds[k + 1])
            if hi <= lo:
                return
            buf = (OrcTokenResult * (hi - lo))()
            L.orc_cluster_replay(hs[k], hi - lo, parts[0][lo:].ctypes.data, parts[1][lo:].ctypes.data,
                                 parts[2][lo:].ctypes.data, parts[3][lo:].ctypes.data, buf)
            out[order[lo:hi]] = np.frombuffer(buf, dtype=np.int32).reshape(-1, 3)

        ths = [threading.Thread(target=run, args=(k,)) for k in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        results.append((out[:, 0].copy(), out[:, 1].copy(), out[:, 2].copy()))
    for h in hs:
        L.orc_cluster_free(h)
    return results
