#!/usr/bin/env python3
"""Per-kernel steady-state durations from a rocprofv3 kernel_trace.csv: the mean and median over the
last `--last` dispatches of each kernel (the timed steps of bench.py; warmup and the first, fallback
batches excluded).  `--skip-tail K` drops each kernel's last K dispatches first: a bench run without
--no-e2e ends with E2E_BATCHES host-buffer batches through the same kernels, which are not timed steps.
Usage: python3 tools/ktrace.py kernel_trace.csv [--last 10] [--skip-tail 0]"""
import argparse
import csv
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last", type=int, default=10)
ap.add_argument("--skip-tail", type=int, default=0)
a = ap.parse_args()
d = defaultdict(list)
for row in csv.DictReader(open(a.csv)):
    name = row.get("Kernel_Name", "?")
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    key = m.group(1) if m else name[:40]
    d[key].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
rows = []
for k, v in d.items():
    v.sort()
    if a.skip_tail:
        v = v[:-a.skip_tail] if len(v) > a.skip_tail else []
    if not v:
        continue
    last = v[-a.last:]
    durs = sorted(e - s for s, e in last)
    us = sum(durs) / len(durs) / 1e3
    med = durs[len(durs) // 2] / 1e3
    rows.append((us, med, k, len(v)))
tot = 0.0
for us, med, k, n in sorted(rows, reverse=True):
    if n < a.last:
        continue
    tot += us
    print(f"{k:34s} calls={n:4d} last{a.last}_avg_us={us:9.1f} median_us={med:9.1f}")
print(f"sum over kernels with >= {a.last} calls (per dispatch set): {tot:.1f} us")
