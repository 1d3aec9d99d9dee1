#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration from tools/calib/pmccal under rocprofv3 (tools/pmc_bench.sh).
Prints reported bytes per known access and writes the factors pmc_summary.py applies:
  stream16_fetch_factor  known bytes / FETCH_SIZE bytes for 16 B-per-lane coalesced reads (guide: 2)
  random16_fetch_factor  correction for kernels dominated by random 16 B gathers: a random 16 B read
                         is charged what a whole random 128 B line read costs per request when both
                         report the same bytes per request (the line is fetched either way), else 1
Usage: python3 tools/pmc_cal.py <dir with counters_*.csv and cal.out> [--json out]"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--json", default=None)
a = ap.parse_args()
known = {}
for line in open(os.path.join(a.dir, "cal.out")):
    if line.startswith("{"):
        known = json.loads(line)
v = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(a.dir, "counters_*.csv")):
    for row in csv.DictReader(open(f)):
        m = re.search(r"(k_cal_\w+)", row.get("Kernel_Name", ""))
        if m:
            v[m.group(1)][row["Counter_Name"]].append(float(row["Counter_Value"]) * 1024.0)


def mean(k, c):
    x = v[k][c]
    return sum(x) / len(x) if x else float("nan")


out = {
    "stream16_fetch_factor": known["stream16_bytes"] / mean("k_cal_stream16", "FETCH_SIZE"),
    "stream4_fetch_factor": known["stream4_bytes"] / mean("k_cal_stream4", "FETCH_SIZE"),
    "rand8_fetch_bytes_per_access": mean("k_cal_rand8", "FETCH_SIZE") / known["rand8_accesses"],
    "rand16_fetch_bytes_per_access": mean("k_cal_rand16", "FETCH_SIZE") / known["rand16_accesses"],
    "rand128_fetch_bytes_per_line": mean("k_cal_rand128", "FETCH_SIZE") / known["rand128_lines"],
    "wrand8_write_bytes_per_access": mean("k_cal_wrand8", "WRITE_SIZE") / known["wrand8_accesses"],
    "wstream8_write_factor": known["wstream8_bytes"] / mean("k_cal_wstream8", "WRITE_SIZE"),
}
r16, r128 = out["rand16_fetch_bytes_per_access"], out["rand128_fetch_bytes_per_line"]
out["random16_fetch_factor"] = (128.0 / r128) if abs(r16 - r128) <= 0.1 * r128 else 1.0
for k, x in out.items():
    print(f"{k:32s} {x:10.3f}")
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
