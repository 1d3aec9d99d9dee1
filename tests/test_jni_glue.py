"""The JNI shim's C half (jni/native): the plain-C glue compiles against include/sentinel_amd.h and
links against libsentinel_amd.so, the JNI entry points compile (against a test-only jni.h stand-in,
tests/jni_stub), and the glue reaches the engine: without a GPU, creating an engine answers
SGA_ENODEV through it.  The Java side (jni/src) needs a JDK and is not compiled here."""
import ctypes as C
import os
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
           "-L", os.path.join(ROOT, "sentinel_amd"), "-lsentinel_amd", "-Wl,-rpath," + os.path.join(ROOT, "sentinel_amd"),
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return C.CDLL(str(out))


def test_jni_symbols_exported(glue):
    for name in ("create", "destroy", "lastError", "loadClusterFlowRules", "requestToken", "submit", "poll",
                 "requestParamToken", "concurrent", "entry", "exit", "setResources", "loadFlowRules"):
        assert hasattr(glue, "Java_com_alibaba_csp_sentinel_gpu_GpuEngine_" + name), name
    for name in ("sgaj_create", "sgaj_request_token", "sgaj_submit", "sgaj_poll", "sgaj_entry", "sgaj_exit",
                 "sgaj_request_param_token", "sgaj_concurrent", "sgaj_load_cluster_flow_rules"):
        assert hasattr(glue, name), name


def test_glue_reaches_engine_without_gpu(glue):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the no-device answer is not observable")
    glue.sgaj_create.argtypes = [C.c_int32, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p)]
    h = C.c_void_p()
    assert glue.sgaj_create(0, 1 << 16, 1 << 16, C.byref(h)) == -19  # SGA_ENODEV
    assert not h.value


def test_java_sources_present():
    base = os.path.join(ROOT, "jni", "src", "main", "java", "com", "alibaba", "csp", "sentinel", "gpu")
    for f in ("GpuEngine.java", "GpuTokenService.java", "GpuStatisticSlot.java", "GpuSlotChainBuilder.java"):
        assert os.path.exists(os.path.join(base, f)), f
    svc = os.path.join(ROOT, "jni", "src", "main", "resources", "META-INF", "services")
    assert open(os.path.join(svc, "com.alibaba.csp.sentinel.cluster.TokenService")).read().strip() == \
        "com.alibaba.csp.sentinel.gpu.GpuTokenService"
