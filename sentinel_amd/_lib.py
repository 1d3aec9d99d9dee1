"""ctypes binding of libsentinel_amd.so (include/sentinel_amd.h).

The HIP library is the only implementation: if it is missing or cannot load,
importing the engine raises -- there is no CPU fallback in the product path.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SGA_LIB_VARIANT=X loads libsentinel_amd_X.so (kernel A/B builds made by tools; the default build
# is the product library)
LIB_PATH = os.path.join(_HERE, "libsentinel_amd" + (("_" + os.environ["SGA_LIB_VARIANT"])
                                                     if os.environ.get("SGA_LIB_VARIANT") else "") + ".so")


class SgaConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_batch", C.c_uint32), ("max_rules", C.c_uint32),
                ("cold_factor", C.c_int32), ("statistic_max_rt", C.c_int32), ("max_param_keys", C.c_uint32),
                ("exceed_count", C.c_double), ("max_occupy_ratio", C.c_double)]


class SgaClusterFlowRule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32), ("grade", C.c_int32),
                ("strategy", C.c_int32), ("reserved", C.c_int32), ("resource_timeout_ms", C.c_int64),
                ("client_offline_time_ms", C.c_int64)]


class SgaSystemRule(C.Structure):
    _fields_ = [("highest_system_load", C.c_double), ("highest_cpu_usage", C.c_double), ("qps", C.c_double),
                ("avg_rt", C.c_int64), ("max_thread", C.c_int64)]


class SgaConcurrentResult(C.Structure):
    _fields_ = [("token_id", C.c_int64), ("status", C.c_int32), ("reserved", C.c_int32)]


class SgaTokenCacheNode(C.Structure):
    _fields_ = [("token_id", C.c_int64), ("flow_id", C.c_int64), ("client_timeout", C.c_int64),
                ("resource_timeout", C.c_int64), ("acquire_count", C.c_int32), ("client", C.c_uint32)]


class SgaClusterParamRule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32), ("grade", C.c_int32),
                ("burst_count", C.c_int32), ("control_behavior", C.c_int32), ("max_queueing_time_ms", C.c_int32),
                ("param_idx_set", C.c_int32), ("duration_in_sec", C.c_int64), ("n_hot", C.c_int32),
                ("reserved", C.c_int32), ("hot_values", C.POINTER(C.c_int64)), ("hot_counts", C.POINTER(C.c_int32))]


class SgaTokenResult(C.Structure):
    _fields_ = [("remaining", C.c_int32), ("wait_in_ms", C.c_int16), ("status", C.c_int8), ("reserved", C.c_int8)]


class SgaFlowRule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double),
                ("control_behavior", C.c_int32), ("warm_up_period_sec", C.c_int32),
                ("max_queueing_time_ms", C.c_int32), ("strategy", C.c_int32),
                ("cluster_mode", C.c_int32), ("cluster_fallback", C.c_int32), ("cluster_flow_id", C.c_int64),
                ("cluster_sample_count", C.c_int32), ("cluster_window_ms", C.c_int32),
                ("cluster_strategy", C.c_int32), ("reserved", C.c_int32)]


class SgaParamRule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double),
                ("control_behavior", C.c_int32), ("max_queueing_time_ms", C.c_int32), ("burst_count", C.c_int32),
                ("param_idx", C.c_int32), ("duration_in_sec", C.c_int64), ("n_hot", C.c_uint32),
                ("reserved", C.c_uint32), ("hot_values", C.POINTER(C.c_uint64)),
                ("hot_thresholds", C.POINTER(C.c_int32)), ("cluster_mode", C.c_int32),
                ("cluster_fallback", C.c_int32), ("cluster_flow_id", C.c_int64),
                ("cluster_sample_count", C.c_int32), ("cluster_window_ms", C.c_int32)]


class SgaDegradeRule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double), ("time_window", C.c_int32),
                ("min_request_amount", C.c_int32), ("slow_ratio_threshold", C.c_double),
                ("stat_interval_ms", C.c_int32), ("reserved", C.c_int32)]


class SgaMetricNode(C.Structure):
    _fields_ = [("timestamp", C.c_int64), ("pass_qps", C.c_int64), ("block_qps", C.c_int64),
                ("success_qps", C.c_int64), ("exception_qps", C.c_int64), ("rt", C.c_int64),
                ("occupied_pass_qps", C.c_int64), ("resource", C.c_uint32), ("concurrency", C.c_int32)]


class SgaClusterMetricNode(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("pass_qps", C.c_double), ("block_qps", C.c_double),
                ("timestamp", C.c_int64)]


class SgaNodeView(C.Structure):
    _fields_ = [("pass_qps", C.c_double), ("block_qps", C.c_double), ("success_qps", C.c_double),
                ("exception_qps", C.c_double), ("occupied_pass_qps", C.c_double), ("avg_rt", C.c_double),
                ("min_rt", C.c_double), ("previous_pass_qps", C.c_double), ("total_pass", C.c_int64),
                ("total_block", C.c_int64), ("total_success", C.c_int64), ("total_exception", C.c_int64),
                ("cur_thread_num", C.c_int64), ("waiting", C.c_int64), ("max_success_qps", C.c_double),
                ("previous_block_qps", C.c_double)]


class SgaWireBatch(C.Structure):  # include/sga_wire.h
    _fields_ = [("cap", C.c_size_t), ("vcap", C.c_size_t), ("n", C.c_size_t), ("nv", C.c_size_t),
                ("xid", C.c_void_p), ("type", C.c_void_p), ("kind", C.c_void_p), ("flow_id", C.c_void_p),
                ("count", C.c_void_p), ("prio", C.c_void_p), ("voff", C.c_void_p), ("values", C.c_void_p),
                ("ns_off", C.c_void_p), ("ns_len", C.c_void_p), ("ns_bytes", C.c_void_p),
                ("ns_cap", C.c_size_t), ("ns_used", C.c_size_t)]


# (restype, argtypes) for every exported symbol; tests check this list against include/*.h
SIGNATURES = {
    "sga_abi_version": (C.c_int, []),
    "sga_config_default": (None, [C.POINTER(SgaConfig)]),
    "sga_create": (C.c_int, [C.POINTER(SgaConfig), C.POINTER(C.c_void_p)]),
    "sga_destroy": (C.c_int, [C.c_void_p]),
    "sga_last_error": (C.c_char_p, [C.c_void_p]),
    "sga_engine_stream": (C.c_void_p, [C.c_void_p]),
    "sga_load_cluster_flow_rules": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(SgaClusterFlowRule), C.c_size_t]),
    "sga_set_namespace_limit": (C.c_int, [C.c_void_p, C.c_char_p, C.c_double]),
    "sga_set_connected_count": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
    "sga_set_hot_rules": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint32]),
    "sga_set_small_batch": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sga_token_submit": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_uint8, C.c_int64, C.POINTER(C.c_uint64)]),
    "sga_poll": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p]),
    "sga_event_submit": (C.c_int, [C.c_void_p, C.c_uint8, C.c_uint32, C.c_int64, C.c_int32, C.c_uint8, C.c_int64,
                                   C.c_uint64, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64)]),
    "sga_event_poll": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_int8), C.POINTER(C.c_int32)]),
    "sga_event_post": (C.c_int, [C.c_void_p, C.c_uint8, C.c_uint32, C.c_int64, C.c_int32, C.c_uint8, C.c_int64,
                                 C.c_uint64, C.c_void_p, C.c_size_t, C.c_void_p]),
    "sga_event_one": (C.c_int, [C.c_void_p, C.c_uint8, C.c_uint32, C.c_int64, C.c_int32, C.c_uint8, C.c_int64,
                                C.c_uint64, C.c_void_p, C.c_size_t, C.POINTER(C.c_int8), C.POINTER(C.c_int32)]),
    "sga_request_token_one": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_uint8, C.c_int64, C.c_void_p]),
    "sga_request_tokens": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                     C.c_void_p]),
    "sga_request_tokens_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                            C.c_size_t, C.c_void_p, C.c_void_p]),
    "sga_request_tokens_packed_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_size_t, C.c_void_p,
                                                   C.c_void_p]),
    "sga_request_tokens_device_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                            C.c_size_t, C.c_void_p, C.c_void_p]),
    "sga_request_tokens_device_pipelined": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                                      C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    "sga_stream_wait": (C.c_int, [C.c_void_p, C.c_void_p]),
    "sga_sync": (C.c_int, [C.c_void_p]),
    "sga_cluster_metric_sums": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.POINTER(C.c_int64)]),
    "sga_cluster_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "sga_cluster_batch_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t]),
    "sga_route_shards": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    "sga_load_cluster_param_rules": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(SgaClusterParamRule), C.c_size_t]),
    "sga_request_param_tokens": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_size_t, C.c_void_p]),
    "sga_cluster_param_sum": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.POINTER(C.c_int64)]),
    "sga_cluster_set_param_capacity": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sga_host_register": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "sga_host_unregister": (C.c_int, [C.c_void_p, C.c_void_p]),
    "sga_rls_should_rate_limit": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p]),
    "sga_cluster_param_top_values": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_uint32, C.c_void_p,
                                               C.c_void_p, C.POINTER(C.c_uint32)]),
    "sga_concurrent_ops": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_size_t, C.c_void_p]),
    "sga_concurrent_expire": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]),
    "sga_concurrent_now_calls": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(C.c_int32)]),
    "sga_concurrent_token_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "sga_concurrent_get_token": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(SgaTokenCacheNode)]),
    "sga_flow_set_resources": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sga_load_system_rules": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "sga_set_system_status": (C.c_int, [C.c_void_p, C.c_double, C.c_double]),
    "sga_load_flow_rules": (C.c_int, [C.c_void_p, C.POINTER(SgaFlowRule), C.c_size_t]),
    "sga_set_cluster_server": (C.c_int, [C.c_void_p, C.c_int32]),
    "sga_load_param_rules": (C.c_int, [C.c_void_p, C.POINTER(SgaParamRule), C.c_size_t]),
    "sga_load_degrade_rules": (C.c_int, [C.c_void_p, C.POINTER(SgaDegradeRule), C.c_size_t]),
    "sga_submit_events": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    "sga_submit_events_ex": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                                       C.c_void_p]),
    "sga_submit_events_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                           C.c_void_p, C.c_void_p, C.c_void_p]),
    "sga_events_device_status": (C.c_int, [C.c_void_p]),
    "sga_rls_should_rate_limit_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                                   C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_void_p, C.c_void_p]),
    "sga_query_node": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int64, C.POINTER(SgaNodeView)]),
    "sga_circuit_breaker_state": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "sga_metrics_snapshot": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "sga_cluster_metric_nodes": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "sga_wire_decode": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(SgaWireBatch)]),
    "sga_wire_decode_sharded": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_uint32,
                                          C.POINTER(SgaWireBatch)]),
    "sga_wire_encode": (C.c_int, [C.c_void_p] * 7 + [C.c_size_t, C.c_void_p, C.c_size_t]),
    "sga_wire_string_key": (C.c_int64, [C.c_char_p, C.c_size_t]),
    "sga_cluster_metric_nodes_device": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_size_t, C.c_void_p,
                                                  C.c_void_p]),
}

_lib = None


class EngineError(RuntimeError):
    pass


def load():
    """Loads the HIP engine library; raises if it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (or `make -C sentinel_amd/csrc`)")
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("SGA_LIB_VARIANT") and not hasattr(L, name):
            continue  # an A/B build older than this symbol; the default build must export all of them
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc, engine=None, what=""):
    if rc < 0:
        msg = ""
        if engine is not None:
            m = load().sga_last_error(engine)
            msg = m.decode() if m else ""
        raise EngineError(f"{what} failed rc={rc} {msg}")
    return rc
