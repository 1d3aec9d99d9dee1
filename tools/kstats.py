#!/usr/bin/env python3
"""Prints a rocprofv3 kernel_stats.csv with short kernel names.

--steps N: also the per-step sum of the cluster pipeline's kernels (classify, radix passes, runs,
flows, results) over N bench steps (warmup + timed + the roofline probe), to compare with the
bench's HIP-event gpu_ms_per_step."""
import csv
import re
import sys

ENGINE = re.compile(r'k_(classify|rs64_|row_scan|runs_|flows|results)')
rows = list(csv.DictReader(open(sys.argv[1])))
total = 0.0
for r in rows:
    m = re.search(r'(k_\w+(<\d+>)?|sgaw_\w+|__amd\w+)', r['Name'])
    nm = m.group(1) if m else r['Name'][:40]
    print(f"{nm:28s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
    if ENGINE.match(nm):
        total += float(r['TotalDurationNs']) / 1e3
if len(sys.argv) > 3 and sys.argv[2] == "--steps":
    print(f"engine kernels per step: {total / int(sys.argv[3]):.1f} us")
