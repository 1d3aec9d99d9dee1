#!/usr/bin/env python3
"""HBM traffic of the engine pipeline per bench step from rocprofv3 PMC passes (tools/pmc_bench.sh).

Counted: the engine's own dispatches only -- kernels of namespace sga:: that run once per batch.
Excluded: the workload generator's kernels (k_flags / k_emit / k_hist and the exclusive-scan kernels
k_scan_* it runs once per generated batch), one-time set-up kernels (k_init_slots, k_hot_reset,
k_lds_order_probe, k_conc_reset), and torch / runtime kernels.

Corrections (MI355X_MICROARCH.md, HBM section, and tools/calib/pmccal.hip measured on the box):
FETCH_SIZE counts 128-B requests at 64 B, so a wide coalesced streaming read reports half its bytes;
the x2 applies to the kernels whose reads are coalesced streams (STREAMING below).  Kernels whose
reads are dominated by random sector gathers (RANDOM below) get the factor the calibration measured
for random 16-byte reads (--cal JSON; 1.0 without one).  WRITE_SIZE is taken as reported.

Per kernel: calls per step, raw and corrected read MB, write MB, traffic MB per step, and (with
--trace, a kernel_trace.csv of the same bench) the average duration, so the table's time column sums
to the step's kernel time.  --json writes the per-step totals and the table."""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

WORKLOAD = {"k_flags", "k_emit", "k_hist", "k_scan_reduce", "k_scan_apply", "k_scan_partials"}
ONE_TIME = {"k_init_slots", "k_hot_reset", "k_lds_order_probe", "k_conc_reset", "k_lim_init"}
# reads are coalesced streams (input arrays, sort tiles, codes, count rows)
STREAMING = {"k_hot_key_dense<0>", "k_hot_key_dense<1>", "k_hot_final", "k_rs64_hist<7>", "k_rs64_sweep<7>",
             "k_row_scan", "k_hscan_group", "k_hscan_mid", "k_hscan_down", "k_hot_pre", "k_hot_mode",
             "k_prio_rank", "k_prio_results", "k_part_colscan", "k_part_binscan", "k_part_scatter", "k_psort_cols",
             "k_psort_scatter", "k_unpack"}
# reads are dominated by random gathers of rule records / parameters
RANDOM = {"k_cold_fused", "k_hot_flows", "k_hot_precheck", "k_hot_hist", "k_hot_pick", "k_hot_clear", "k_hot_fin",
          "k_cluster_nodes", "k_hot_final_g", "k_hot_final_h", "k_hot_next_a", "k_hot_next_b"}


def base(k):
    """k_cold_fused_t<0> -> k_cold_fused; k_rs64_sweep<7> -> k_rs64_sweep (template instances and the
    _t suffix of templated kernels are classified by their base name)."""
    b = re.sub(r"<.*", "", k)
    return b[:-2] if b.endswith("_t") else b


STREAMING_BASE = {base(k) for k in STREAMING}
RANDOM_BASE = {base(k) for k in RANDOM}


def kind_of(k):
    b = base(k)
    return "stream" if b in STREAMING_BASE else ("random" if b in RANDOM_BASE else "other")


E_DEC = 1  # bench_local.py: one decision byte per entry (the wait word is written only for waits)


def alg_local(k, bl):
    """Local-path lines (bench_local.py): SURVEY.md 8(d)'s bytes per step split over the kernels that move
    them -- the event records in (entries E_in, exits E_exit) to k_lclassify, which reads every event; the
    decisions out (E_DEC per entry) to k_lresults; the touched keys' state (2 * S_k each: node, rule,
    breaker and parameter state) to the synthetic row "(state)", since it is read and written across the
    per-resource kernels.  The three parts sum to the line's roofline.bytes_alg_per_step."""
    rf = bl.get("roofline", {})
    total = rf.get("bytes_alg_per_step")
    io = rf.get("lower_bound_bytes_per_step")
    if total is None or io is None:
        return None
    cfg = bl["config"]
    dec = E_DEC * (cfg["entries_per_step_per_gpu"] if "entries_per_step_per_gpu" in cfg
                   else cfg.get("entries_per_step", 0) / max(1, bl.get("n_gpus", 1)))
    if k == "k_lclassify":
        return io - dec
    if k == "k_lresults":
        return dec
    if k == "(state)":
        return total - io
    return 0.0


def alg_bytes(k, bl):
    """Per-kernel share of SURVEY.md 8(d)'s algorithmic bytes per step, from the bench line `bl`:
    the key kernel reads every request (E_in = 12 B), the cold stage writes the cold results and reads
    + writes the cold touched rules, the hot runs read + write the hot rules, the hot results kernel
    writes the hot results (E_out = 8 B).  Everything else (the sort, scans, next hot set) is 0:
    traffic there is non-algorithmic.  Hot touched rules ~ the hot-set size of the last batch."""
    if bl and ("entries_per_step" in bl.get("config", {}) or "entries_per_step_per_gpu" in bl.get("config", {})):
        return alg_local(k, bl)
    if not bl or "requests_per_step_per_gpu" not in bl.get("config", {}):
        return None
    n = bl["config"]["requests_per_step_per_gpu"]
    touched = bl["roofline"]["touched_rules_per_step_per_gpu"]
    lp = bl.get("last_batch_path") or {}
    n_cold = lp.get("n_cold", n)
    t_hot = min(lp.get("n_hot_next", 0), touched)
    b = base(k)
    if b == "k_hot_key_dense" and re.search(r"<0\s*[,>]", k):  # pass 0 (k_hot_key_dense<0> or <0, true>)
        return n * 12.0
    if b == "k_cold_fused":
        return n_cold * 8.0 + (touched - t_hot) * 2 * 704.0
    if b == "k_hot_flows":
        return t_hot * 2 * 704.0
    if b in ("k_hot_final", "k_hot_final_g", "k_hot_final_h"):
        return (n - n_cold) * 8.0
    return 0.0


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps-from", default=None, help="bench output whose JSON line gives steps+warmup")
    ap.add_argument("--cal", default=None, help="calibration JSON (tools/pmc_cal.py) with random-read factors")
    ap.add_argument("--trace", default=None, help="kernel_trace.csv of the same bench for durations")
    ap.add_argument("--json", default=None)
    ap.add_argument("--all-random", action="store_true",
                    help="local-path lines: every engine kernel's FETCH_SIZE gets the measured random factor")
    ap.add_argument("--relabel", default=None, help="update an existing traffic JSON's alg columns from the "
                    "bench line given by --steps-from (no counters needed)")
    a = ap.parse_args()
    if a.relabel:
        relabel(a.relabel, a.steps_from)
        return

    agg = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(a.dir, "counters_*.csv"))):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", row.get("Kernel-Name", "?"))
            agg[(short(name), "sga::" in name)][row["Counter_Name"]].append(float(row["Counter_Value"]))

    sets, bline = None, None
    if a.steps_from and os.path.exists(a.steps_from):
        for line in open(a.steps_from):
            if line.startswith("{"):
                d = json.loads(line)
                # every batch the bench ran through the engine: warmup + timed steps, plus the host-buffer
                # (end-to-end) batches that follow the timed loop unless the bench ran with --no-e2e
                e2e = d.get("end_to_end_host_buffers") or {}
                sets = d["steps"] + d["warmup"] + int(e2e.get("batches", 0))
                bline = d
    rand_factor = 1.0
    if a.cal and os.path.exists(a.cal):
        rand_factor = float(json.load(open(a.cal)).get("random16_fetch_factor", 1.0))

    durations = defaultdict(list)
    if a.trace and os.path.exists(a.trace):
        for row in csv.DictReader(open(a.trace)):
            durations[short(row.get("Kernel_Name", "?"))].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))

    # every counter of a kernel, averaged per dispatch (diagnostics)
    for (k, eng), cs in sorted(agg.items()):
        print(f"{k}{'' if eng else '  (not engine)'}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.6g}  (n={len(v)})")

    if not sets:
        return
    table = []
    tot = {"fetch_raw": 0.0, "fetch": 0.0, "write": 0.0, "us": 0.0}
    for (k, eng), cs in sorted(agg.items()):
        if not eng or k in WORKLOAD or k in ONE_TIME:
            continue
        if "FETCH_SIZE" not in cs and "WRITE_SIZE" not in cs:
            continue
        n_calls = max(len(cs.get("FETCH_SIZE", [])), len(cs.get("WRITE_SIZE", [])))
        per_step = n_calls / sets
        fr = (sum(cs.get("FETCH_SIZE", [0.0])) / max(1, len(cs.get("FETCH_SIZE", [])))) * 1024.0
        wr = (sum(cs.get("WRITE_SIZE", [0.0])) / max(1, len(cs.get("WRITE_SIZE", [])))) * 1024.0
        kind = "random" if a.all_random else kind_of(k)
        fac = 2.0 if kind == "stream" else (rand_factor if kind == "random" else 1.0)
        us = None
        if durations.get(k):
            dd = sorted(durations[k])  # median dispatch (warmup / fallback batches included)
            us = dd[len(dd) // 2] / 1e3 * per_step
            tot["us"] += us
        row = {"kernel": k, "kind": kind, "calls_per_step": per_step, "fetch_raw_mb": fr * per_step / 1e6,
               "fetch_factor": fac, "fetch_mb": fr * fac * per_step / 1e6, "write_mb": wr * per_step / 1e6,
               "us_per_step": us}
        row["traffic_mb"] = row["fetch_mb"] + row["write_mb"]
        tot["fetch_raw"] += row["fetch_raw_mb"]
        tot["fetch"] += row["fetch_mb"]
        tot["write"] += row["write_mb"]
        table.append(row)
    table.sort(key=lambda r: -r["traffic_mb"])
    alg_total = attach_alg(table, bline) if bline else None
    print(f"\nper step ({sets} dispatch sets; engine kernels only; FETCH x2 for streaming kernels, "
          f"x{rand_factor:.2f} for random-gather kernels)")
    print(f"{'kernel':24s} {'kind':7s} {'calls':>5s} {'fetch_raw':>10s} {'fetch':>10s} {'write':>10s} {'traffic':>10s} "
          f"{'alg':>8s} {'us':>8s}")
    for r in table:
        us = f"{r['us_per_step']:8.1f}" if r["us_per_step"] is not None else "       -"
        al = f"{r['alg_mb']:8.1f}" if r["alg_mb"] is not None else "       -"
        print(f"{r['kernel']:24s} {r['kind']:7s} {r['calls_per_step']:5.2f} {r['fetch_raw_mb']:10.1f} {r['fetch_mb']:10.1f} "
              f"{r['write_mb']:10.1f} {r['traffic_mb']:10.1f} {al} {us}")
    traffic = (tot["fetch"] + tot["write"]) * 1e6
    print(f"{'total':24s} {'':7s} {'':5s} {tot['fetch_raw']:10.1f} {tot['fetch']:10.1f} {tot['write']:10.1f} "
          f"{traffic / 1e6:10.1f} {tot['us']:8.1f}")
    if a.json:
        json.dump({"traffic_bytes_per_step": traffic, "fetch_bytes_per_step": tot["fetch"] * 1e6,
                   "fetch_bytes_per_step_raw": tot["fetch_raw"] * 1e6, "write_bytes_per_step": tot["write"] * 1e6,
                   "kernel_us_per_step": tot["us"], "dispatch_sets": sets, "random_fetch_factor": rand_factor,
                   "run": os.path.basename(os.path.dirname(os.path.normpath(a.dir))), "kernels": table,  # the pmc_configs tag
                   "alg_bytes_per_step": alg_total,
                   "note": "engine kernels only (sga::, per batch); FETCH_SIZE x2 for coalesced streaming kernels, "
                           "x random16_fetch_factor (tools/calib/pmccal.hip) for random-gather kernels; WRITE_SIZE as "
                           "reported"},
                  open(a.json, "w"), indent=1)


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            d = json.loads(line)
    return d


def attach_alg(table, bl):
    """Per-kernel alg_mb / traffic_over_alg and the step total (local lines add the "(state)" row)."""
    local = bl and ("entries_per_step" in bl.get("config", {}) or "entries_per_step_per_gpu" in bl.get("config", {}))
    if local and not any(r["kernel"] == "(state)" for r in table):
        table.append({"kernel": "(state)", "kind": "-", "calls_per_step": 0.0, "fetch_raw_mb": 0.0, "fetch_factor": 0.0,
                      "fetch_mb": 0.0, "write_mb": 0.0, "us_per_step": None, "traffic_mb": 0.0,
                      "note": "2 * S_k per touched key, moved by the per-resource kernels (no single kernel)"})
    for r in table:
        ab = alg_bytes(r["kernel"], bl)
        r["alg_mb"] = None if ab is None else ab / 1e6
        r["traffic_over_alg"] = (r["traffic_mb"] / r["alg_mb"]) if r["alg_mb"] else None
    return sum((r["alg_mb"] or 0.0) for r in table) * 1e6


def relabel(path, steps_from):
    d = json.load(open(path))
    bl = bench_line(steps_from)
    d["alg_bytes_per_step"] = attach_alg(d["kernels"], bl)
    d["alg_source"] = os.path.basename(steps_from)
    tr = d["traffic_bytes_per_step"]
    d["traffic_over_alg"] = tr / d["alg_bytes_per_step"] if d["alg_bytes_per_step"] else None
    json.dump(d, open(path, "w"), indent=1)
    print(f"{path}: alg {d['alg_bytes_per_step'] / 1e6:.1f} MB/step, traffic {tr / 1e6:.1f} MB/step, "
          f"ratio {d['traffic_over_alg']:.2f}")


if __name__ == "__main__":
    main()
