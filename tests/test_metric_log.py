"""Metric log files: MetricWriter / MetricSearcher / MetricsReader.

CPU: the reference's MetricWriterTest (file-name comparator with and without pid, fileNameMatches)
and MetricNodeTest (fromFatString) known answers; the fat-line format; the writer's index (big-endian
(second, offset) pairs, written when the second advances), size and day roll-over, the
totalFileCount clean-up, dropped earlier seconds; MetricSearcher.find / findByTimeAndResource.
GPU: MetricTimerListener over the engine's metrics snapshots, read back through MetricSearcher,
equals the oracle's StatisticNode.metrics rows."""
import os
import struct
import time

import numpy as np
import pytest

from sentinel_amd import metric_log as ML
from sentinel_amd.local import MetricNode

T0 = 1_700_000_000_000


@pytest.fixture
def utc():
    old = os.environ.get("TZ")
    os.environ["TZ"] = "UTC"
    time.tzset()
    yield
    if old is None:
        os.environ.pop("TZ", None)
    else:
        os.environ["TZ"] = old
    time.tzset()


def test_file_name_comparator_kat():
    # MetricWriterTest.testFileNameCmp / testFileNamePidCmp
    for pre in ("metrics.log.", "metrics.log.pid1234."):
        arr = [pre + s for s in ("2018-03-06", "2018-03-07", "2018-03-07.51", "2018-03-07.10", "2018-03-06.100")]
        key = [pre + s for s in ("2018-03-06", "2018-03-06.100", "2018-03-07", "2018-03-07.10", "2018-03-07.51")]
        assert sorted(arr, key=ML.metric_file_name_key) == key


def test_file_name_matches_kat():
    # MetricWriterTest.testFileNameMatches
    assert ML.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06", "Sentinel-SDK-Demo-metrics.log")
    assert ML.file_name_matches("Sentinel-Admin-metrics.log.pid22568.2018-12-24", "Sentinel-Admin-metrics.log.pid22568")
    assert ML.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06.11", "Sentinel-SDK-Demo-metrics.log")
    assert not ML.file_name_matches("Sentinel-SDK-Demo-metrics.log.XXX.2018-03-06.11", "Sentinel-SDK-Demo-metrics.log")
    assert not ML.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06.11XXX", "Sentinel-SDK-Demo-metrics.log")
    assert ML.form_metric_file_name("a.b.c", 77) == "a-b-c-metrics.log"
    assert ML.form_metric_file_name("app", 77, use_pid=True) == "app-metrics.log.pid77"


def test_fat_and_thin_strings(utc):
    # MetricNodeTest.testFromFatString
    n = ML.from_fat_string("1564382218000|2019-07-29 14:36:58|/foo/*|1|0|1|0|0|0|2|1")
    assert (n.classification, n.concurrency, n.success_qps, n.resource) == (1, 2, 1, "/foo/*")
    m = MetricNode(1564382218000, "a|b", 5, 1, 4, 0, 12, 2, 3, 1)
    assert ML.to_fat_string(m) == "1564382218000|2019-07-29 06:36:58|a_b|5|1|4|0|12|2|3|1\n"
    assert ML.from_fat_string(ML.to_fat_string(m).rstrip("\n")) == MetricNode(1564382218000, "a_b", 5, 1, 4, 0, 12, 2,
                                                                              3, 1)
    assert ML.from_thin_string(m.to_thin_string()) == MetricNode(1564382218000, "a_b", 5, 1, 4, 0, 12, 2, 3, 1)
    old = ML.from_thin_string("1|r|1|2|3|4|5")  # pre-occupiedPass lines still parse
    assert (old.rt, old.occupied_pass_qps, old.concurrency) == (5, 0, 0)


def _nodes(t, k, tag=""):
    return [MetricNode(0, f"res{tag}{i}", i + 1, i, i + 1, 0, 7, 0) for i in range(k)]


def _read_index(path):
    b = open(path, "rb").read()
    return [struct.unpack_from(">qq", b, i) for i in range(0, len(b), 16)]


def test_writer_index_and_search(tmp_path, utc):
    d = str(tmp_path)
    w = ML.MetricWriter(d, app_name="my.app", pid=1, now_ms=T0 - 5000)
    w.write(T0 - 9000, _nodes(0, 2))        # earlier than the writer's start second: dropped
    for s in range(6):
        w.write(T0 + 1000 * s, _nodes(s, 3))
    w.write(T0 + 5000, _nodes(5, 1, "x"))  # same second again: lines, no new index entry
    w.close()
    files = ML.list_metric_files(d, "my-app-metrics.log")
    assert [os.path.basename(f) for f in files] == ["my-app-metrics.log.2023-11-14"]
    lines = open(files[0]).read().splitlines()
    assert len(lines) == 6 * 3 + 1
    idx = _read_index(files[0] + ".idx")
    assert [s for s, _ in idx] == [T0 // 1000 + s for s in range(6)]
    offs = [o for _, o in idx]
    assert offs[0] == 0 and all(b - a == sum(len(x) + 1 for x in lines[3 * i:3 * i + 3])
                                for i, (a, b) in enumerate(zip(offs, offs[1:])))
    se = ML.MetricSearcher(d, "my-app-metrics.log")
    got = se.find(T0 + 2500, 4)  # from second 2; 4 lines requested, the rest of the last second too
    assert [n.timestamp for n in got] == [T0 + 2000] * 3 + [T0 + 3000] * 3
    got = se.find(T0 + 4000, 1)  # cached position reused
    assert [n.timestamp for n in got] == [T0 + 4000] * 3
    got = se.find_by_time_and_resource(T0 + 1000, T0 + 3999, "res1")
    assert [(n.timestamp, n.resource, n.pass_qps) for n in got] == [(T0 + 1000 * s, "res1", 2) for s in (1, 2, 3)]
    got = se.find_by_time_and_resource(T0 + 5000, T0 + 9000, None)
    assert [n.resource for n in got] == ["res0", "res1", "res2", "resx0"]
    assert se.find(T0 + 60_000, 10) is None


def test_writer_size_roll_and_file_count(tmp_path, utc):
    d = str(tmp_path)
    w = ML.MetricWriter(d, single_file_size=300, total_file_count=3, app_name="app", pid=1, now_ms=T0 - 1000)
    for s in range(12):
        w.write(T0 + 1000 * s, _nodes(s, 2))  # ~130 bytes per second: a new file every 3 seconds
    w.close()
    files = [os.path.basename(f) for f in ML.list_metric_files(d, "app-metrics.log")]
    # a roll after seconds 2, 5, 8 and 11 (the last leaves an empty file); totalFileCount: the oldest
    # files are removed before each new one, so the new one is the third
    assert files == ["app-metrics.log.2023-11-14.2", "app-metrics.log.2023-11-14.3", "app-metrics.log.2023-11-14.4"]
    assert os.path.getsize(os.path.join(d, files[2])) == 0
    assert sorted(os.listdir(d)) == sorted(files + [f + ".idx" for f in files])
    se = ML.MetricSearcher(d, "app-metrics.log")
    got = se.find_by_time_and_resource(T0, T0 + 20_000, "res0")
    assert [n.timestamp for n in got] == [T0 + 1000 * s for s in range(6, 12)]


def test_writer_day_roll(tmp_path, utc):
    d = str(tmp_path)
    day_end = (T0 // 86_400_000 + 1) * 86_400_000
    w = ML.MetricWriter(d, app_name="app", pid=1, now_ms=day_end - 3000)
    for t in (day_end - 2000, day_end - 1000, day_end, day_end + 1000):
        w.write(t, _nodes(0, 1))
    w.close()
    files = [os.path.basename(f) for f in ML.list_metric_files(d, "app-metrics.log")]
    assert files == ["app-metrics.log.2023-11-14", "app-metrics.log.2023-11-15"]
    # the new day's first index entry is written into the old day's index, then the new file starts
    assert [s for s, _ in _read_index(os.path.join(d, files[0] + ".idx"))] == [(day_end - 2000) // 1000,
                                                                                (day_end - 1000) // 1000,
                                                                                day_end // 1000]
    assert [s for s, _ in _read_index(os.path.join(d, files[1] + ".idx"))] == [(day_end + 1000) // 1000]
    assert len(open(os.path.join(d, files[1])).read().splitlines()) == 2


@pytest.mark.gpu
def test_metric_timer_listener_engine_to_file(tmp_path):
    from sentinel_amd.cluster import Engine
    from sentinel_amd.local import FlowRuleManager, LocalSentinel
    from sentinel_amd.rules import FlowRule
    from tests import local_trace as lt
    n_res = 12
    flow = [{"resource": r, "count": float(4 + 3 * r)} for r in range(0, n_res, 2)]
    gen = lt.Oracle(n_res, flow)
    st = lt.generate(gen, n_res, n_entries=8000, seed=9, t0=T0, gap_mean=0.7, err_pct=0.05, rt_max=30)
    gen.close()
    orc = lt.Oracle(n_res, flow)
    eng = Engine(max_batch=1 << 16)
    names = [f"r{i}" for i in range(n_res)]
    s = LocalSentinel(eng, names)
    FlowRuleManager(s).load_rules([FlowRule(resource=f"r{r['resource']}", count=r["count"]) for r in flow])
    w = ML.MetricWriter(str(tmp_path), app_name="gpu-app", pid=7, now_ms=T0 - 1000)
    lis = ML.MetricTimerListener(s, w, classification={"r3": 1})
    ts = st["ts"]
    expect = []
    now, lo = T0 + 250, 0
    while lo < len(ts):
        now += 1000
        hi = int(np.searchsorted(ts, now, side="left"))
        sub = {k: np.ascontiguousarray(v[lo:hi]) for k, v in st.items()}
        if hi > lo:
            s.submit(sub["kind"], sub["resource"], sub["ts"], sub["acquire"], sub["flags"], sub["rt"], sub["param"])
            orc.replay(sub)
        lis.run(now)
        expect += orc.metrics(now)
        lo = hi
    w.close()
    se = ML.MetricSearcher(str(tmp_path), "gpu-app-metrics.log")
    got = se.find_by_time_and_resource(T0, now + 10_000, None)
    assert len(got) == len(expect) > 2 * n_res
    for g, e in zip(got, expect):
        assert (g.timestamp, g.resource, g.pass_qps, g.block_qps, g.success_qps, g.exception_qps, g.rt,
                g.occupied_pass_qps) == (e[0], names[e[1]], *e[2:])
        assert g.classification == (1 if g.resource == "r3" else 0)
    eng.close()
    orc.close()
