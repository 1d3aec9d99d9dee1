"""Metric log files: MetricWriter / MetricSearcher / MetricsReader / MetricTimerListener.

Mirrors (CORE = sentinel-core/src/main/java/com/alibaba/csp/sentinel):
  CORE/node/metric/MetricNode.java:160-250      thin / fat line formats and their parsers
  CORE/node/metric/MetricWriter.java            <app>-metrics.log[.pid<N>].<yyyy-MM-dd>[.<n>] files, one
                                                 line per node per second, a .idx of (second, offset)
                                                 big-endian longs written when the second advances,
                                                 size roll-over, day roll-over, keep totalFileCount
  CORE/node/metric/MetricSearcher.java          index lookup with the cached last position
  CORE/node/metric/MetricsReader.java           line reads, recommendLines / end-time cut-offs
  CORE/node/metric/MetricTimerListener.java:44-65  every second: metrics() of all nodes, by time

The rows come from the engine's once-per-second snapshot (LocalSentinel.metrics ->
sga_metrics_snapshot, the HIP k_metrics kernel); this module is the on-disk format the dashboard
reads.  Dates use the process's local time zone, as SimpleDateFormat uses the JVM's default.
"""
import os
import re
import struct
import time as _time
from typing import Callable, Dict, List, Optional

from .local import MetricNode

METRIC_FILE = "metrics.log"
METRIC_FILE_INDEX_SUFFIX = ".idx"
DEFAULT_SINGLE_METRIC_FILE_SIZE = 1024 * 1024 * 50  # SentinelConfig.DEFAULT_SINGLE_METRIC_FILE_SIZE
DEFAULT_TOTAL_METRIC_FILE_COUNT = 6                  # SentinelConfig.DEFAULT_TOTAL_METRIC_FILE_COUNT
MAX_LINES_RETURN = 100000                            # MetricsReader.MAX_LINES_RETURN
CHARSET = "utf-8"                                    # SentinelConfig.charset() default


def java_split(s: str, sep: str = "|") -> List[str]:
    """String.split(regex) for a literal separator: trailing empty strings are removed."""
    parts = s.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def _fmt_time(ms: int) -> str:
    return _time.strftime("%Y-%m-%d %H:%M:%S", _time.localtime(ms // 1000))


def to_fat_string(n: MetricNode) -> str:
    """MetricNode.toFatString (:200-220): timestamp|yyyy-MM-dd HH:mm:ss|resource|pass|block|success|
    exception|rt|occupiedPass|concurrency|classification\\n, '|' in the resource replaced by '_'."""
    return "|".join(str(x) for x in (n.timestamp, _fmt_time(n.timestamp), n.resource.replace("|", "_"), n.pass_qps,
                                     n.block_qps, n.success_qps, n.exception_qps, n.rt, n.occupied_pass_qps,
                                     n.concurrency, n.classification)) + "\n"


def from_fat_string(line: str) -> MetricNode:
    """MetricNode.fromFatString (:229-250)."""
    s = java_split(line)
    n = MetricNode(int(s[0]), s[2], int(s[3]), int(s[4]), int(s[5]), int(s[6]), int(s[7]), 0)
    if len(s) >= 9:
        n.occupied_pass_qps = int(s[8])
    if len(s) >= 10:
        n.concurrency = int(s[9])
    if len(s) == 11:
        n.classification = int(s[10])
    return n


def from_thin_string(line: str) -> MetricNode:
    """MetricNode.fromThinString (:178-198)."""
    s = java_split(line)
    n = MetricNode(int(s[0]), s[1], int(s[2]), int(s[3]), int(s[4]), int(s[5]), int(s[6]), 0)
    if len(s) >= 8:
        n.occupied_pass_qps = int(s[7])
    if len(s) >= 9:
        n.concurrency = int(s[8])
    if len(s) == 10:
        n.classification = int(s[9])
    return n


def form_metric_file_name(app_name: Optional[str], pid: int, use_pid: bool = False) -> str:
    """MetricWriter.formMetricFileName: dots of the app name become '-'."""
    name = (app_name or "").replace(".", "-") + "-" + METRIC_FILE
    if use_pid:
        name += ".pid" + str(pid)
    return name


def form_index_file_name(metric_file_name: str) -> str:
    return metric_file_name + METRIC_FILE_INDEX_SUFFIX


_MATCH = re.compile(r"\.[0-9]{4}-[0-9]{2}-[0-9]{2}(\.[0-9]*)?")


def file_name_matches(file_name: str, base_file_name: str) -> bool:
    """MetricWriter.fileNameMatches: base + '.yyyy-MM-dd' + optional '.<number>'."""
    return file_name.startswith(base_file_name) and _MATCH.fullmatch(file_name[len(base_file_name):]) is not None


def metric_file_name_key(path: str):
    """Sort key of MetricWriter.MetricFileNameComparator: date part (the one after 'pidN' when
    present), then name length, then the name."""
    name = os.path.basename(path)
    parts = name.split(".")
    date = parts[2]
    if date.startswith("pid"):
        date = parts[3]
    return (date, len(name), name)


def list_metric_files(base_dir: str, base_file_name: str) -> List[str]:
    """MetricWriter.listMetricFiles: sorted absolute paths, index and lock files excluded."""
    if not os.path.isdir(base_dir):
        return []
    out = []
    for f in os.listdir(base_dir):
        p = os.path.join(base_dir, f)
        if (os.path.isfile(p) and file_name_matches(f, base_file_name) and not f.endswith(METRIC_FILE_INDEX_SUFFIX)
                and not f.endswith(".lck")):
            out.append(os.path.abspath(p))
    out.sort(key=metric_file_name_key)
    return out


class MetricWriter:
    """MetricWriter(singleFileSize, totalFileCount) writing under `base_dir`.

    `now_ms` stands for the System.currentTimeMillis() the constructor reads: writes whose second
    is earlier than it are dropped, as in the reference."""

    def __init__(self, base_dir: str, single_file_size: int = DEFAULT_SINGLE_METRIC_FILE_SIZE,
                 total_file_count: int = DEFAULT_TOTAL_METRIC_FILE_COUNT, app_name: str = "",
                 pid: Optional[int] = None, use_pid: bool = False, now_ms: Optional[int] = None):
        if single_file_size <= 0 or total_file_count <= 0:
            raise ValueError("singleFileSize and totalFileCount must be positive")
        self.base_dir = base_dir if base_dir.endswith(os.sep) else base_dir + os.sep
        os.makedirs(self.base_dir, exist_ok=True)
        self.single_file_size = single_file_size
        self.total_file_count = total_file_count
        self.app_name = app_name
        self.pid = os.getpid() if pid is None else pid
        self.use_pid = use_pid
        t = int(_time.time() * 1000) if now_ms is None else now_ms
        self.last_second = t // 1000
        self.time_second_base = -_time.localtime(0).tm_gmtoff  # df.parse("1970-01-01 00:00:00") / 1000
        self.base_file_name: Optional[str] = None
        self.cur_metric_file: Optional[str] = None
        self.cur_index_file: Optional[str] = None
        self._out = None
        self._idx = None

    # -- MetricWriter.write
    def write(self, time_ms: int, nodes: Optional[List[MetricNode]]):
        if nodes is None:
            return
        for n in nodes:
            n.timestamp = time_ms
        if self.cur_metric_file is None:
            self.base_file_name = form_metric_file_name(self.app_name, self.pid, self.use_pid)
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        if not (os.path.exists(self.cur_metric_file) and os.path.exists(self.cur_index_file)):
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        second = time_ms // 1000
        if second < self.last_second:
            return  # the reference ignores an earlier second
        if second == self.last_second:
            self._write_lines(nodes, time_ms)
            return
        self._write_index(second, self._out.tell())
        if self._is_new_day(self.last_second, second):
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        self._write_lines(nodes, time_ms)
        self.last_second = second

    def _write_lines(self, nodes, time_ms):
        self._out.write("".join(to_fat_string(n) for n in nodes).encode(CHARSET))
        self._out.flush()
        if os.fstat(self._out.fileno()).st_size >= self.single_file_size:  # !validSize()
            self._close_and_new_file(self._next_file_name_of_day(time_ms))

    def _write_index(self, second: int, offset: int):
        self._idx.write(struct.pack(">qq", second, offset))  # DataOutputStream.writeLong x2
        self._idx.flush()

    def _is_new_day(self, last_second: int, second: int) -> bool:
        return (second - self.time_second_base) // 86400 > (last_second - self.time_second_base) // 86400

    def _next_file_name_of_day(self, time_ms: int) -> str:
        model = self.base_file_name + "." + _time.strftime("%Y-%m-%d", _time.localtime(time_ms // 1000))
        found = [os.path.abspath(os.path.join(self.base_dir, f)) for f in os.listdir(self.base_dir)
                 if model in f and not f.endswith(METRIC_FILE_INDEX_SUFFIX) and not f.endswith(".lck")]
        found.sort(key=metric_file_name_key)
        if not found:
            return self.base_dir + model
        last = found[-1].split(".")
        n = int(last[-1]) if last and re.fullmatch(r"[0-9]{1,10}", last[-1]) else 0
        return self.base_dir + model + "." + str(n + 1)

    def _remove_more_files(self):
        files = list_metric_files(self.base_dir, self.base_file_name)
        for f in files[:max(0, len(files) - self.total_file_count + 1)]:
            for p in (f, form_index_file_name(f)):
                try:
                    os.remove(p)
                except FileNotFoundError:
                    pass

    def _close_and_new_file(self, file_name: str):
        self._remove_more_files()
        self.close()
        self._out = open(file_name, "wb")  # FileOutputStream(fileName, append = false)
        self.cur_metric_file = file_name
        self.cur_index_file = form_index_file_name(file_name)
        self._idx = open(self.cur_index_file, "wb")

    def close(self):
        if self._out is not None:
            self._out.close()
            self._out = None
        if self._idx is not None:
            self._idx.close()
            self._idx = None


class MetricsReader:
    def __init__(self, charset: str = CHARSET):
        self.charset = charset

    def _lines(self, file_name: str, offset: int):
        with open(file_name, "rb") as f:
            f.seek(offset)
            data = f.read().decode(self.charset, errors="replace")
        return data.splitlines()  # BufferedReader.readLine: \n, \r or \r\n

    def read_in_one_file_by_end_time(self, out, file_name, offset, begin_ms, end_ms, identity) -> bool:
        begin_s, end_s = begin_ms // 1000, end_ms // 1000
        for line in self._lines(file_name, offset):
            node = from_fat_string(line)
            cur = node.timestamp // 1000
            if cur < begin_s:
                return False
            if cur <= end_s:
                if identity is None or node.resource == identity:
                    out.append(node)
            else:
                return False
            if len(out) >= MAX_LINES_RETURN:
                return False
        return True

    def read_in_one_file(self, out, file_name, offset, recommend_lines):
        last = out[-1].timestamp // 1000 if out else -1
        for line in self._lines(file_name, offset):
            node = from_fat_string(line)
            cur = node.timestamp // 1000
            if len(out) < recommend_lines:
                out.append(node)
            elif cur == last:
                out.append(node)
            else:
                break
            last = cur

    def read_metrics_by_end_time(self, files, pos, offset, begin_ms, end_ms, identity):
        out: List[MetricNode] = []
        if self.read_in_one_file_by_end_time(out, files[pos], offset, begin_ms, end_ms, identity):
            pos += 1
            while pos < len(files):
                f = files[pos]
                pos += 1
                if not self.read_in_one_file_by_end_time(out, f, 0, begin_ms, end_ms, identity):
                    break
        return out

    def read_metrics(self, files, pos, offset, recommend_lines):
        out: List[MetricNode] = []
        self.read_in_one_file(out, files[pos], offset, recommend_lines)
        pos += 1
        while len(out) < recommend_lines and pos < len(files):
            self.read_in_one_file(out, files[pos], 0, recommend_lines)
            pos += 1
        return out


class MetricSearcher:
    """MetricSearcher(baseDir, baseFileName): find / findByTimeAndResource with the cached
    position of the last index hit (validPosition)."""

    def __init__(self, base_dir: str, base_file_name: str, charset: str = CHARSET):
        if base_dir is None or base_file_name is None or charset is None:
            raise ValueError("baseDir, baseFileName and charset can't be null")
        self.base_dir = base_dir if base_dir.endswith(os.sep) else base_dir + os.sep
        self.base_file_name = base_file_name
        self.reader = MetricsReader(charset)
        self.pos_metric_file: Optional[str] = None
        self.pos_index_file: Optional[str] = None
        self.pos_offset_in_index = 0
        self.pos_second = 0

    def _valid_position(self, begin_ms: int) -> bool:
        if begin_ms // 1000 < self.pos_second or self.pos_index_file is None:
            return False
        try:
            with open(self.pos_index_file, "rb") as f:
                f.seek(self.pos_offset_in_index)
                b = f.read(8)
            return len(b) == 8 and struct.unpack(">q", b)[0] == self.pos_second
        except OSError:
            return False

    def _find_offset(self, begin_ms: int, metric_file: str, idx_file: str, offset_in_index: int) -> int:
        self.pos_metric_file = None
        self.pos_index_file = None
        if not os.path.exists(idx_file):
            return -1
        begin_s = begin_ms // 1000
        with open(idx_file, "rb") as f:
            f.seek(offset_in_index)
            data = f.read()
        at = 0
        self.pos_offset_in_index = offset_in_index
        while True:
            if at + 8 > len(data):
                return -1  # EOFException
            second = struct.unpack_from(">q", data, at)[0]
            at += 8
            if second >= begin_s:
                break
            if at + 8 > len(data):
                return -1
            at += 8
            self.pos_offset_in_index = offset_in_index + at
        if at + 8 > len(data):
            return -1
        offset = struct.unpack_from(">q", data, at)[0]
        self.pos_metric_file = metric_file
        self.pos_index_file = idx_file
        self.pos_second = second
        return offset

    def _start(self, begin_ms, files):
        i, off_in_idx = 0, 0
        if self._valid_position(begin_ms):
            try:
                i = files.index(self.pos_metric_file)
                off_in_idx = self.pos_offset_in_index
            except ValueError:
                i = 0
        return i, off_in_idx

    def find(self, begin_ms: int, recommend_lines: int) -> Optional[List[MetricNode]]:
        files = list_metric_files(self.base_dir, self.base_file_name)
        i, off_in_idx = self._start(begin_ms, files)
        while i < len(files):
            off = self._find_offset(begin_ms, files[i], form_index_file_name(files[i]), off_in_idx)
            off_in_idx = 0
            if off != -1:
                return self.reader.read_metrics(files, i, off, recommend_lines)
            i += 1
        return None

    def find_by_time_and_resource(self, begin_ms: int, end_ms: int,
                                  identity: Optional[str]) -> Optional[List[MetricNode]]:
        files = list_metric_files(self.base_dir, self.base_file_name)
        i, off_in_idx = self._start(begin_ms, files)
        while i < len(files):
            off = self._find_offset(begin_ms, files[i], form_index_file_name(files[i]), off_in_idx)
            off_in_idx = 0
            if off != -1:
                return self.reader.read_metrics_by_end_time(files, i, off, begin_ms, end_ms, identity)
            i += 1
        return None


class MetricTimerListener:
    """MetricTimerListener.run: the engine's metrics snapshot of every resource, grouped by
    timestamp in ascending order (the TreeMap), one MetricWriter.write per timestamp.
    `classification` maps a resource name to its ResourceTypeConstants value (default COMMON 0)."""

    def __init__(self, sentinel, writer: MetricWriter, classification: Optional[Dict[str, int]] = None):
        self.sentinel = sentinel
        self.writer = writer
        self.classification = classification or {}

    def run(self, now: int):
        by_time: Dict[int, List[MetricNode]] = {}
        for n in self.sentinel.metrics(now):
            n.classification = self.classification.get(n.resource, 0)
            by_time.setdefault(n.timestamp, []).append(n)
        for t in sorted(by_time):
            self.writer.write(t, by_time[t])
