"""The JNI shim's C half (jni/native): the plain-C glue compiles against include/sentinel_amd.h and
links against libsentinel_amd.so, the JNI entry points compile (against a test-only jni.h stand-in,
tests/jni_stub), and the glue reaches the engine: without a GPU, creating an engine answers
SGA_ENODEV through it.  The Java side (jni/src) needs a JDK and is not compiled here."""
import ctypes as C
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def glue(tmp_path_factory):
    out = tmp_path_factory.mktemp("jni") / "libsga_jni_test.so"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-shared", "-fPIC",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "jni", "native"),
           "-I", os.path.join(ROOT, "tests", "jni_stub"),
           os.path.join(ROOT, "jni", "native", "sga_jni_glue.c"), os.path.join(ROOT, "jni", "native", "sentinel_amd_jni.c"),
           os.path.join(ROOT, "tests", "jni_stub", "fake_jvm.c"),
           "-L", os.path.join(ROOT, "sentinel_amd"), "-lsentinel_amd", "-Wl,-rpath," + os.path.join(ROOT, "sentinel_amd"),
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return C.CDLL(str(out))


def test_jni_symbols_exported(glue):
    for name in JAVA_NATIVES:
        assert hasattr(glue, "Java_com_alibaba_csp_sentinel_gpu_GpuEngine_" + name), name
    for name in ("sgaj_create", "sgaj_request_token", "sgaj_submit", "sgaj_poll", "sgaj_entry", "sgaj_exit",
                 "sgaj_request_param_token", "sgaj_concurrent", "sgaj_load_cluster_flow_rules", "sgaj_entry_args",
                 "sgaj_exit_args", "sgaj_blocked", "sgaj_revoke_args", "sgaj_load_param_rules", "sgaj_load_degrade_rules",
                 "sgaj_load_system_rules", "sgaj_set_system_status", "sgaj_load_cluster_param_rules",
                 "sgaj_set_connected_count", "sgaj_set_namespace_limit", "sgaj_set_cluster_server",
                 "sgaj_query_node", "sgaj_metrics_snapshot"):
        assert hasattr(glue, name), name


# every `static native` of GpuEngine.java (the Java half cannot be compiled here: no JDK)
JAVA_NATIVES = ("create", "destroy", "lastError", "loadClusterFlowRules", "loadClusterParamRules", "setConnectedCount",
                "setNamespaceLimit", "requestToken", "submit", "poll", "requestParamToken", "concurrent", "entryArgs",
                "exitArgs", "blocked", "revokedArgs", "entry", "exit", "setResources", "loadFlowRules", "loadParamRules",
                "loadDegradeRules", "loadSystemRules", "setSystemStatus", "setClusterServer", "queryNode",
                "metricsSnapshot")


def test_java_natives_match_the_jni_file():
    import re
    src = open(os.path.join(ROOT, "jni", "src", "main", "java", "com", "alibaba", "csp", "sentinel", "gpu",
                            "GpuEngine.java")).read()
    declared = set(re.findall(r"static native \w+ (\w+)\(", src))
    assert declared == set(JAVA_NATIVES), declared ^ set(JAVA_NATIVES)


def test_glue_calls_reach_the_engine_abi(glue):
    """With no engine (NULL handle) every glue entry answers the engine's SGA_EINVAL: the marshalling reaches
    sga_* (the rule loaders, node view, metric snapshot, argument-vector events)."""
    E = -22
    P, U32, I32, I64, D = C.c_void_p, C.c_uint32, C.c_int32, C.c_int64, C.c_double
    one_u32 = (C.c_uint32 * 2)(0, 0)
    one_i32 = (C.c_int32 * 1)(1)
    one_i64 = (C.c_int64 * 1)(1)
    one_d = (C.c_double * 1)(1.0)
    words = (C.c_uint64 * 2)(0, 7)
    out2 = (C.c_int32 * 2)()
    calls = {
        "sgaj_entry_args": ([P, U32, I64, I32, U32, P, U32, U32, P], [None, 0, 1, 1, 0, words, 1, 2, out2]),
        "sgaj_exit_args": ([P, U32, I64, I32, U32, I64, P, U32, U32], [None, 0, 1, 1, 0, 0, words, 1, 2]),
        "sgaj_blocked": ([P, U32, I64, I32, U32], [None, 0, 1, 1, 0]),
        "sgaj_revoke_args": ([P, U32, I64, I32, U32, P, U32, U32], [None, 0, 1, 1, 0, words, 1, 2]),
        "sgaj_load_degrade_rules": ([P, C.c_size_t, P, P, P, P, P, P, P],
                                    [None, 1, one_u32, one_i32, one_d, one_i32, one_i32, one_d, one_i32]),
        "sgaj_load_system_rules": ([P, C.c_size_t, P, P, P, P, P], [None, 1, one_d, one_d, one_d, one_i64, one_i64]),
        "sgaj_set_system_status": ([P, D, D], [None, 0.5, 0.5]),
        "sgaj_set_connected_count": ([P, C.c_char_p, I32], [None, b"default", 2]),
        "sgaj_set_namespace_limit": ([P, C.c_char_p, D], [None, b"default", 100.0]),
        "sgaj_set_cluster_server": ([P, I32], [None, 1]),
        "sgaj_query_node": ([P, U32, I64, P, P], [None, 0, 1, (C.c_double * 10)(), (C.c_int64 * 6)()]),
    }
    for name, (argt, args) in calls.items():
        fn = getattr(glue, name)
        fn.argtypes = argt
        fn.restype = C.c_int
        assert fn(*args) == E, name
    fn = glue.sgaj_load_param_rules
    fn.restype = C.c_int
    fn.argtypes = [P, C.c_size_t] + [P] * 16
    assert fn(None, 1, one_u32, one_i32, one_d, one_i32, one_i32, one_i32, one_i32, one_i64, None, None, None,
              None, None, None, None, None) == E
    fn = glue.sgaj_load_cluster_param_rules
    fn.restype = C.c_int
    fn.argtypes = [P, C.c_char_p, C.c_size_t] + [P] * 8
    assert fn(None, b"default", 1, one_i64, one_d, None, None, None, None, None, None) == E
    n = C.c_size_t(5)
    fn = glue.sgaj_metrics_snapshot
    fn.restype = C.c_int
    fn.argtypes = [P, I64, P, C.c_size_t, C.POINTER(C.c_size_t)]
    assert fn(None, 1, (C.c_int64 * 8)(), 1, C.byref(n)) == E


def test_glue_reaches_engine_without_gpu(glue):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the no-device answer is not observable")
    glue.sgaj_create.argtypes = [C.c_int32, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p)]
    h = C.c_void_p()
    assert glue.sgaj_create(0, 1 << 16, 1 << 16, C.byref(h)) == -19  # SGA_ENODEV
    assert not h.value


def test_java_entry_points_through_a_fake_jnienv_without_gpu(glue):
    """The Java_* entry points themselves, called with tests/jni_stub/fake_jvm.c's JNIEnv (as
    tests/test_jni_live_gpu.py drives them on a GPU): GpuEngine.create answers SGA_ENODEV here, and
    lastError returns a Java string."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the no-device answer is not observable")
    glue.fake_env.restype = C.c_void_p
    env = C.c_void_p(glue.fake_env())
    create = getattr(glue, "Java_com_alibaba_csp_sentinel_gpu_GpuEngine_create")
    create.restype = C.c_int64
    assert create(env, None, 0, 1 << 14, 1 << 12) == -19
    last = getattr(glue, "Java_com_alibaba_csp_sentinel_gpu_GpuEngine_lastError")
    last.restype = C.c_void_p
    js = last(env, None, C.c_int64(0))
    glue.fake_string_chars.restype = C.c_char_p
    glue.fake_string_chars.argtypes = [C.c_void_p]
    assert isinstance(glue.fake_string_chars(js), bytes)


def test_java_sources_present():
    base = os.path.join(ROOT, "jni", "src", "main", "java", "com", "alibaba", "csp", "sentinel", "gpu")
    for f in ("GpuEngine.java", "GpuTokenService.java", "GpuStatisticSlot.java", "GpuSlotChainBuilder.java",
              "GpuArgs.java", "GpuRuleSync.java", "GpuNode.java", "GpuMetricTimerListener.java"):
        assert os.path.exists(os.path.join(base, f)), f
    svc = os.path.join(ROOT, "jni", "src", "main", "resources", "META-INF", "services")
    assert open(os.path.join(svc, "com.alibaba.csp.sentinel.cluster.TokenService")).read().strip() == \
        "com.alibaba.csp.sentinel.gpu.GpuTokenService"


def test_flow_record_layout_matches_the_c_struct():
    """GpuRuleSync's 64-byte record has sga_flow_rule's size and field offsets (include/sentinel_amd.h)."""
    from sentinel_amd._lib import SgaFlowRule
    # GpuRuleSync.FlowListener: putInt x2, putDouble, putInt x6, putLong, putInt x4 (GpuRuleSync.java:141-154)
    assert struct.calcsize("<iidiiiiiiqiiii") == 64 == C.sizeof(SgaFlowRule)
    java_offsets = [0, 4, 8, 16, 20, 24, 28, 32, 36, 40, 48, 52, 56, 60]
    assert [getattr(SgaFlowRule, f).offset for f, _ in SgaFlowRule._fields_] == java_offsets
