#!/usr/bin/env python3
"""Summarise tools/pmc_bench.sh output.

Per kernel: mean counter value per dispatch.  Per step: HBM traffic of the
engine pipeline = sum over its kernels of (2 x FETCH_SIZE + WRITE_SIZE) per
dispatch x dispatches per step.  rocprofv3 reports FETCH_SIZE and WRITE_SIZE in
KiB; FETCH_SIZE is doubled because gfx950 tallies 128-B read requests at 64 B
(MI355X_MICROARCH.md, HBM section).  --json writes the per-step figure."""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--steps-from", default=None, help="bench output whose JSON line gives steps+warmup")
ap.add_argument("--json", default=None)
a = ap.parse_args()

agg = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.dir, "counters_*.csv"))):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", row.get("Kernel-Name", "?"))
        m = re.search(r'(k_\w+(<\d+>)?)', name)
        agg[m.group(1) if m else name[:60]][row["Counter_Name"]].append(float(row["Counter_Value"]))

steps = None
if a.steps_from and os.path.exists(a.steps_from):
    for line in open(a.steps_from):
        if line.startswith("{"):
            d = json.loads(line)
            steps = d["steps"] + d["warmup"]
tot_fetch = tot_write = 0.0
for k, cs in sorted(agg.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.6g}  (n={len(v)})")
    if "FETCH_SIZE" in cs:
        tot_fetch += sum(cs["FETCH_SIZE"]) * 1024.0
    if "WRITE_SIZE" in cs:
        tot_write += sum(cs["WRITE_SIZE"]) * 1024.0
if steps:
    per_step = (2 * tot_fetch + tot_write) / steps
    print(f"per step (all engine kernels): FETCH_SIZE {tot_fetch / steps / 1e6:.1f} MB (x2 = {2 * tot_fetch / steps / 1e6:.1f}), "
          f"WRITE_SIZE {tot_write / steps / 1e6:.1f} MB, traffic {per_step / 1e6:.1f} MB")
    if a.json:
        json.dump({"traffic_bytes_per_step": per_step, "fetch_bytes_per_step_raw": tot_fetch / steps,
                   "write_bytes_per_step": tot_write / steps, "dispatch_sets": steps,
                   "run": os.path.basename(os.path.normpath(a.dir)),
                   "note": "2*FETCH_SIZE+WRITE_SIZE (KiB->B) summed over the engine kernels of one step"},
                  open(a.json, "w"), indent=1)
