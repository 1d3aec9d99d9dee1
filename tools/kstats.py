#!/usr/bin/env python3
"""Prints a rocprofv3 kernel_stats.csv with short kernel names."""
import csv
import re
import sys

for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r'(k_\w+(<\d+>)?|sgaw_\w+|__amd\w+)', r['Name'])
    nm = m.group(1) if m else r['Name'][:40]
    print(f"{nm:28s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
