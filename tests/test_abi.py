"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/*.h declares, and the Python mirror binds them all."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sentinel_amd", "libsentinel_amd.so")


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(sga\w*)\s*\(", text):
            syms.add(m.group(1))
    return sorted(syms)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import __graft_entry__
        __graft_entry__.build()
    return ctypes.CDLL(LIB)


def test_headers_declare_api():
    syms = declared_symbols()
    assert "sga_request_tokens" in syms and "sga_load_cluster_flow_rules" in syms
    assert len(syms) >= 12


def test_library_exports_every_declared_symbol(lib):
    wl = ctypes.CDLL(os.path.join(ROOT, "sentinel_amd", "libsga_workload.so"))
    missing = [s for s in declared_symbols() if not hasattr(wl if s.startswith("sgaw_") else lib, s)]
    assert not missing, missing


def test_python_mirror_binds_every_symbol():
    from sentinel_amd import _lib
    L = _lib.load()
    decl = {s for s in declared_symbols() if not s.startswith("sgaw_")}
    assert decl <= set(_lib.SIGNATURES), decl - set(_lib.SIGNATURES)
    assert L.sga_abi_version() == 3


def test_struct_layouts_match_header():
    from sentinel_amd import _lib
    assert ctypes.sizeof(_lib.SgaTokenResult) == 8
    assert ctypes.sizeof(_lib.SgaClusterFlowRule) == 56
    assert ctypes.sizeof(_lib.SgaConfig) == 40


_STRUCTS = {"SgaConfig": "sga_config", "SgaClusterFlowRule": "sga_cluster_flow_rule",
            "SgaTokenResult": "sga_token_result", "SgaFlowRule": "sga_flow_rule", "SgaParamRule": "sga_param_rule",
            "SgaDegradeRule": "sga_degrade_rule", "SgaNodeView": "sga_node_view",
            "SgaConcurrentResult": "sga_concurrent_result", "SgaTokenCacheNode": "sga_token_cache_node",
            "SgaSystemRule": "sga_system_rule"}


def test_every_field_offset_matches_the_c_compiler(tmp_path):
    """sizeof / offsetof of every ABI struct as gcc lays it out == the ctypes mirror."""
    from sentinel_amd import _lib
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sentinel_amd.h"', "int main(void) {"]
    expect = []
    for py, c in _STRUCTS.items():
        cls = getattr(_lib, py)
        lines.append(f'printf("%zu\\n", sizeof({c}));')
        expect.append(ctypes.sizeof(cls))
        for f, _ in cls._fields_:
            lines.append(f'printf("%zu\\n", offsetof({c}, {f}));')
            expect.append(getattr(cls, f).offset)
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    import subprocess
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == expect


def test_create_without_gpu_fails_loudly():
    """No GPU here: engine creation must fail with an error code, never fall back to a CPU path."""
    from sentinel_amd import _lib
    L = _lib.load()
    cfg = _lib.SgaConfig()
    L.sga_config_default(ctypes.byref(cfg))
    h = ctypes.c_void_p()
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("GPU present")
    except ImportError:
        pass
    rc = L.sga_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc < 0 and not h.value


def test_java_string_hash_matches_rls_converter():
    # EnvoySentinelRuleConverterTest: flowId = Integer.MAX_VALUE + key.hashCode()
    from sentinel_amd.javautil import rls_key, string_hash_code
    assert string_hash_code("abc") == 96354
    key = rls_key("foo", [("k1", "v1"), ("k2", "v2")])
    assert key == "foo|k1|v1|k2|v2"
    h = 0
    for ch in key:
        h = (h * 31 + ord(ch)) & 0xFFFFFFFF
    h = h - (1 << 32) if h >= (1 << 31) else h
    assert string_hash_code(key) == h
