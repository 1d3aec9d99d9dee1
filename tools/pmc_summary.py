#!/usr/bin/env python3
"""Summarise tools/pmc_bench.sh output: per kernel, mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "counters_*.csv"))):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", row.get("Kernel-Name", "?"))
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in agg.items():
    print(k[:70])
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
