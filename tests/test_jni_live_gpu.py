"""The JNI shim end to end on a live engine (N1): jni/native/sentinel_amd_jni.c and its C glue, compiled
as the JDK build would compile them (against tests/jni_stub/jni.h plus tests/jni_stub/fake_jvm.c, a JNIEnv
over caller-owned arrays), are driven through their Java_* entry points exactly as GpuEngine.java /
GpuRuleSync.java / GpuStatisticSlot.java call them:

  * GpuEngine.create on the GPU, setResources;
  * FlowRuleManager rules as the 64-byte little-endian records GpuRuleSync.FlowListener writes into a
    direct ByteBuffer (GpuRuleSync.java:141-154), passed to loadFlowRules;
  * ParamFlowRuleManager / DegradeRuleManager / ClusterFlowRuleManager rules as the parallel arrays of
    GpuRuleSync's listeners (loadParamRules, loadDegradeRules, loadClusterFlowRules), the embedded token
    server switched on (setClusterServer);
  * a mixed stream of SphU.entry / Entry.exit with whole argument vectors through entryArgs / exitArgs
    (GpuArgs words), one call per event as GpuStatisticSlot makes them;
  * the node views (queryNode, every Node getter incl. maxSuccessQps and previousBlockQps) and the metric
    rows (metricsSnapshot) afterwards.

Every decision and wait, every node getter and every metric row must equal the oracle's replay of the
same stream."""
import ctypes as C
import os
import struct
import subprocess

import numpy as np
import pytest

from tests import local_trace as lt
from tests.test_local_parity_gpu import T0

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PFX = "Java_com_alibaba_csp_sentinel_gpu_GpuEngine_"
FLOW_RECORD = "<iidiiiiiiqiiii"  # GpuRuleSync.FlowListener's putInt/putDouble/putLong sequence, 64 bytes


@pytest.fixture(scope="module")
def jni(tmp_path_factory):
    out = tmp_path_factory.mktemp("jnilive") / "libsga_jni_live.so"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-shared", "-fPIC",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "jni", "native"),
           "-I", os.path.join(ROOT, "tests", "jni_stub"),
           os.path.join(ROOT, "jni", "native", "sga_jni_glue.c"), os.path.join(ROOT, "jni", "native", "sentinel_amd_jni.c"),
           os.path.join(ROOT, "tests", "jni_stub", "fake_jvm.c"),
           "-L", os.path.join(ROOT, "sentinel_amd"), "-lsentinel_amd", "-Wl,-rpath," + os.path.join(ROOT, "sentinel_amd"),
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    L = C.CDLL(str(out))
    L.fake_env.restype = C.c_void_p
    L.fake_array.restype = C.c_void_p
    L.fake_array.argtypes = [C.c_int32, C.c_void_p]
    L.fake_string.restype = C.c_void_p
    L.fake_string.argtypes = [C.c_char_p]
    L.fake_buffer.restype = C.c_void_p
    L.fake_buffer.argtypes = [C.c_void_p]
    L.fake_free.argtypes = [C.c_void_p]
    return L


class Jvm:
    """Java-side helper: arrays and strings handed to the JNI entry points (kept alive until close)."""

    def __init__(self, L):
        self.L = L
        self.env = C.c_void_p(L.fake_env())
        self.keep, self.objs = [], []

    def arr(self, a, dt):
        if a is None:
            return None
        x = np.ascontiguousarray(a, dtype=dt)
        self.keep.append(x)
        o = self.L.fake_array(len(x), x.ctypes.data if len(x) else None)
        self.objs.append(o)
        return C.c_void_p(o)

    def s(self, txt):
        o = self.L.fake_string(txt.encode())
        return C.c_void_p(o)

    def call(self, name, restype, *args):
        fn = getattr(self.L, PFX + name)
        fn.restype = restype
        return fn(self.env, None, *args)

    def close(self):
        for o in self.objs:
            self.L.fake_free(o)


def flow_records(flow):
    """sga_flow_rule records as GpuRuleSync.FlowListener packs them (per resource, list order)."""
    b = bytearray()
    for r in flow:
        cm = bool(r.get("cluster_mode"))
        b += struct.pack(FLOW_RECORD, r["resource"], r.get("grade", 1), float(r["count"]),
                         r.get("control_behavior", 0), r.get("warm_up_period_sec", 10), r.get("max_queueing_time_ms", 500),
                         0, 1 if cm else 0, 1 if cm and r.get("cluster_fallback", True) else 0,
                         r.get("cluster_flow_id", 0) if cm else 0, 10 if cm else 0, 1000 if cm else 0, 0, 0)
    return bytes(b)


def _rules():
    flow = [{"resource": 0, "count": 5.0},
            {"resource": 1, "count": 10.0, "control_behavior": 2, "max_queueing_time_ms": 200},
            {"resource": 2, "count": 20.0, "control_behavior": 1, "warm_up_period_sec": 2},
            {"resource": 3, "count": 3.0, "cluster_mode": True, "cluster_flow_id": 7003, "cluster_fallback": True},
            {"resource": 4, "grade": 0, "count": 2.0},
            {"resource": 5, "count": 50.0}, {"resource": 5, "count": 8.0}]
    param = [{"resource": 6, "count": 3.0, "param_idx": 0},
             {"resource": 7, "count": 4.0, "param_idx": -1, "control_behavior": 2, "max_queueing_time_ms": 100},
             {"resource": 8, "count": 4.0, "param_idx": 0}, {"resource": 8, "count": 2.0, "param_idx": 1, "hot": {3: 6}},
             {"resource": 3, "count": 6.0, "param_idx": 0}]
    degrade = [{"resource": 9, "grade": 0, "count": 20.0, "slow_ratio_threshold": 0.5, "min_request_amount": 5,
                "time_window": 1, "stat_interval_ms": 1000},
               {"resource": 5, "grade": 1, "count": 0.3, "min_request_amount": 5, "time_window": 1}]
    crules = [{"flow_id": 7003, "count": 4.0, "threshold_type": 1}]
    return flow, param, degrade, crules


def _local_words(st, k):
    """The event's GpuArgs words (pairs at offset 0, then list elements) from the stream's global param_values."""
    pv = st["param_values"]
    p = int(st["param"][k])
    off, nargs = p >> 32, p & 0xFFFFFFFF
    words = [0] * (2 * nargs)
    for a in range(nargs):
        tag, val = int(pv[off + 2 * a]), int(pv[off + 2 * a + 1])
        if tag >> 62 == 2:  # list: re-based element offset
            ln = tag & ((1 << 62) - 1)
            words[2 * a] = tag
            words[2 * a + 1] = len(words)
            words.extend(int(x) for x in pv[val:val + ln])
        else:
            words[2 * a], words[2 * a + 1] = tag, val
    return np.array(words or [0], dtype=np.uint64), nargs


def test_live_engine_through_the_jni_entry_points(jni):
    from tests.test_cluster_parity_gpu import oracle_cluster
    n_res = 10
    flow, param, degrade, crules = _rules()
    L = lt.lib()
    gen = lt.Oracle(n_res, flow, param, degrade)
    ohg = oracle_cluster({"default": crules})
    L.orc_flow_set_cluster(gen.h, ohg, 1)
    st = lt.generate_args(gen, n_res, 2500, seed=5, t0=T0, gap_mean=2.0, acq_max=2, prio_pct=0.05, rt_max=40,
                          domain=5, zipf=False)
    gen.close()
    orc = lt.Oracle(n_res, flow, param, degrade)
    oh = oracle_cluster({"default": crules})
    L.orc_flow_set_cluster(orc.h, oh, 1)
    exp_d, exp_w = orc.replay(st)

    J = Jvm(jni)
    h = J.call("create", C.c_int64, 0, 1 << 14, 1 << 12)
    assert h > 0, J.L
    H = C.c_int64(h)
    I, D, Q = np.int32, np.float64, np.int64
    try:
        assert J.call("setResources", C.c_int32, H, n_res) == 0
        rec = C.create_string_buffer(flow_records(flow))
        buf = C.c_void_p(jni.fake_buffer(C.addressof(rec)))
        J.objs.append(buf.value)
        assert J.call("loadFlowRules", C.c_int32, H, buf, len(flow)) >= 0
        hot_off, hot_v, hot_c = [0], [], []
        for r in param:
            for k, v in r.get("hot", {}).items():
                hot_v.append(k)
                hot_c.append(v)
            hot_off.append(len(hot_v))
        npr = len(param)
        rc = J.call("loadParamRules", C.c_int32, H, J.arr([r["resource"] for r in param], I),
                    J.arr([r.get("grade", 1) for r in param], I), J.arr([r["count"] for r in param], D),
                    J.arr([r.get("control_behavior", 0) for r in param], I),
                    J.arr([r.get("max_queueing_time_ms", 0) for r in param], I),
                    J.arr([r.get("burst_count", 0) for r in param], I), J.arr([r.get("param_idx", 0) for r in param], I),
                    J.arr([r.get("duration_in_sec", 1) for r in param], Q), J.arr(hot_off, I), J.arr(hot_v, Q),
                    J.arr(hot_c, I), J.arr([0] * npr, I), J.arr([0] * npr, I), J.arr([0] * npr, Q),
                    J.arr([0] * npr, I), J.arr([0] * npr, I))
        assert rc >= 0, rc
        rc = J.call("loadDegradeRules", C.c_int32, H, J.arr([r["resource"] for r in degrade], I),
                    J.arr([r["grade"] for r in degrade], I), J.arr([r["count"] for r in degrade], D),
                    J.arr([r["time_window"] for r in degrade], I), J.arr([r["min_request_amount"] for r in degrade], I),
                    J.arr([r.get("slow_ratio_threshold", 1.0) for r in degrade], D),
                    J.arr([r.get("stat_interval_ms", 1000) for r in degrade], I))
        assert rc >= 0, rc
        rc = J.call("loadClusterFlowRules", C.c_int32, H, J.s("default"), J.arr([c["flow_id"] for c in crules], Q),
                    J.arr([c["count"] for c in crules], D), J.arr([c["threshold_type"] for c in crules], I),
                    J.arr([10] * len(crules), I), J.arr([1000] * len(crules), I))
        assert rc >= 0, rc
        assert J.call("setClusterServer", C.c_int32, H, 1) == 0

        n = len(st["kind"])
        got_d = np.zeros(n, np.int8)
        got_w = np.zeros(n, np.int32)
        out2 = np.zeros(2, np.int32)
        o2 = J.arr(out2, I)
        for k in range(n):
            words, nargs = _local_words(st, k)
            w = J.arr(words.view(np.int64), Q)
            fl = int(st["flags"][k]) & ~32  # the JNI layer adds SGA_EV_ARGS itself
            if st["kind"][k] == 0:
                rc = J.call("entryArgs", C.c_int32, H, int(st["resource"][k]), C.c_int64(int(st["ts"][k])),
                            int(st["acquire"][k]), fl, w, nargs, o2)
                assert rc == 0, (k, rc)
                got_d[k], got_w[k] = out2[0], out2[1]  # written through SetIntArrayRegion
            else:
                rc = J.call("exitArgs", C.c_int32, H, int(st["resource"][k]), C.c_int64(int(st["ts"][k])),
                            int(st["acquire"][k]), fl, C.c_int64(int(st["rt"][k])), w, nargs)
                assert rc == 0, (k, rc)
        bad = np.nonzero((got_d != exp_d) | (got_w != exp_w))[0]
        assert len(bad) == 0, (f"{len(bad)} of {n} events differ; first at {bad[0]}: kind={st['kind'][bad[0]]} "
                               f"res={st['resource'][bad[0]]} jni=({got_d[bad[0]]},{got_w[bad[0]]}) "
                               f"oracle=({exp_d[bad[0]]},{exp_w[bad[0]]})")
        ent = st["kind"] == 0
        assert (exp_d[ent] == 0).sum() > 200 and len(set(exp_d[ent].tolist()) - {0}) >= 2  # passes and blocks

        now = int(st["ts"].max()) + 1
        for rid in range(n_res):
            d10, l6 = np.zeros(10, D), np.zeros(6, Q)
            assert J.call("queryNode", C.c_int32, H, rid, C.c_int64(now), J.arr(d10, D), J.arr(l6, Q)) == 0
            v = dict(zip(["pass_qps", "block_qps", "success_qps", "exception_qps", "occupied_pass_qps", "avg_rt",
                          "min_rt", "previous_pass_qps", "max_success_qps", "previous_block_qps"], d10.tolist()))
            v.update(zip(["total_pass", "total_block", "total_success", "total_exception", "cur_thread_num",
                          "waiting"], l6.tolist()))
            assert [v[g] for g in lt.NODE_GETTERS] == orc.node(rid, now), rid
        rows = np.zeros(8 * 4096, Q)
        nrows = J.call("metricsSnapshot", C.c_int32, H, C.c_int64(now), J.arr(rows, Q))
        assert nrows >= 0, nrows
        got_rows = sorted(tuple(int(x) for x in rows[8 * i:8 * i + 8]) for i in range(nrows))
        assert got_rows == [tuple(int(x) for x in r) for r in orc.metrics(now, cap=4096)]
        assert nrows > 0
    finally:
        J.call("destroy", None, H)
        J.close()
        orc.close()
        lt.lib()
        from tests import oracle_harness as OH
        OH.lib().orc_cluster_free(oh)
        OH.lib().orc_cluster_free(ohg)


def test_post_chain_block_revokes_through_the_jni_entry_points(jni):
    """GpuStatisticSlot's post-chain path (a custom slot sorted after DegradeSlot throws BlockException for an
    entry the engine passed): entryArgs, then revokedArgs at the entry's time with its flags and argument
    vector.  The node then holds what the reference's StatisticSlot records (StatisticSlot.java:71-84,121-135):
    no pass, no thread -- node, ENTRY_NODE and the parameter thread map -- and the block; thread-grade flow and
    parameter rules of 1 pass the next entry again.  Node views equal the oracle's (kind 3)."""
    flow = [{"resource": 0, "grade": 0, "count": 1.0}]
    param = [{"resource": 0, "grade": 0, "count": 1.0, "param_idx": 0}]
    J = Jvm(jni)
    h = J.call("create", C.c_int64, 0, 1 << 12, 1 << 10)
    assert h > 0
    H = C.c_int64(h)
    I, D, Q = np.int32, np.float64, np.int64
    orc = lt.Oracle(2, flow, param)
    try:
        assert J.call("setResources", C.c_int32, H, 2) == 0
        rec = C.create_string_buffer(flow_records(flow))
        buf = C.c_void_p(jni.fake_buffer(C.addressof(rec)))
        J.objs.append(buf.value)
        assert J.call("loadFlowRules", C.c_int32, H, buf, 1) >= 0
        z = lambda dt: J.arr([0], dt)
        assert J.call("loadParamRules", C.c_int32, H, J.arr([0], I), J.arr([0], I), J.arr([1.0], D), z(I), z(I), z(I),
                      z(I), J.arr([1], Q), J.arr([0, 0], I), J.arr([], Q), J.arr([], I), z(I), z(I), z(Q), z(I),
                      z(I)) >= 0
        pv = []
        word = lt.encode_args([7], pv)
        w = J.arr(np.array(pv, np.uint64).view(np.int64), Q)
        out2 = np.zeros(2, np.int32)
        o2 = J.arr(out2, I)
        fl = 8  # EntryType.IN
        events = [(0, T0), (0, T0 + 1), (3, T0), (0, T0 + 3)]
        got = []
        for kind, t in events:
            if kind == 0:
                assert J.call("entryArgs", C.c_int32, H, 0, C.c_int64(t), 1, fl, w, 1, o2) == 0
                got.append(int(out2[0]))
            else:
                assert J.call("revokedArgs", C.c_int32, H, 0, C.c_int64(t), 1, fl, w, 1) == 0
        st = {"kind": np.array([k for k, _ in events], np.uint8), "resource": np.zeros(4, np.uint32),
              "ts": np.array([t for _, t in events], np.int64), "acquire": np.ones(4, np.int32),
              "flags": np.full(4, 8 | 32, np.uint8), "rt": np.zeros(4, np.int64),
              "param": np.full(4, word, np.uint64), "param_values": np.array(pv, np.uint64)}
        exp_d, _ = orc.replay(st)
        assert got == [int(exp_d[i]) for i in (0, 1, 3)] and got[0] == 0 and got[1] != 0 and got[2] == 0
        now = T0 + 4
        for rid in (0, 0xFFFFFFFF):  # the resource, ENTRY_NODE
            d10, l6 = np.zeros(10, D), np.zeros(6, Q)
            assert J.call("queryNode", C.c_int32, H, C.c_int32(rid - (1 << 32) if rid >> 31 else rid), C.c_int64(now),
                          J.arr(d10, D), J.arr(l6, Q)) == 0
            v = dict(zip(["pass_qps", "block_qps", "success_qps", "exception_qps", "occupied_pass_qps", "avg_rt",
                          "min_rt", "previous_pass_qps", "max_success_qps", "previous_block_qps"], d10.tolist()))
            v.update(zip(["total_pass", "total_block", "total_success", "total_exception", "cur_thread_num",
                          "waiting"], l6.tolist()))
            assert [v[g] for g in lt.NODE_GETTERS] == orc.node(rid, now), rid
            assert v["total_block"] == 2 and v["total_pass"] == 1 and v["cur_thread_num"] == 1, (rid, v)
    finally:
        J.call("destroy", None, H)
        J.close()
        orc.close()
