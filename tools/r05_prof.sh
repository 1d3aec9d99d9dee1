#!/bin/bash
# Round 5 profiling (GPU box): parity of the packed C3 path, hot-final A/B, k_cold_fused phase ticks, SQ counters of the
# big kernels, record-access calibration.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05p}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_packed_device_gpu.py > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $out/pytest.log | head; grep -q "Fatal\|core dumped\|Aborted\|Segmentation" $out/pytest.log && exit 1; }
rep=0
for envs in "SGA_FIN_G=0" "SGA_FIN_G=1" "SGA_FIN_G=0" "SGA_FIN_G=1"; do
  rep=$((rep+1)); extra="--no-parity"; [ $rep -le 2 ] && extra=""
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e $extra > $out/ab.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/ab.json').read().strip().splitlines()[-1]); p=d.get('parity_sample') or {}; print('[$envs] ms %.4f gpu_ms %.4f mism %s' % (d['ms_per_step'], d['roofline']['gpu_ms_per_step'], p.get('mismatches')))"
done
SGA_FZ_DEBUG=16 timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-parity --steps 4 --warmup 2 > $out/fz.json 2> $out/fz.err || { tail -5 $out/fz.err; exit 1; }
grep "fz phases" $out/fz.err | tail -4
for wg in 256; do timeout -k 10 120 ./tools/calib/recbench 700000 $wg | tee -a $out/recbench.jsonl || exit 1; done
timeout -k 10 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
grep -o "TA_[A-Z_]*\|TD_[A-Z_]*\|TCP_[A-Z_]*" $out/counters_list.txt | sort -u | head -80 > $out/ta_td_tcp.txt
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_cold_fused|k_hot_key_dense|k_hot_final|k_part_scatter" -d /tmp/pmcp_$i -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-parity --steps 3 --warmup 2 > $out/pmc_$i.out 2>&1 || exit $?
  find /tmp/pmcp_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
python3 - $out <<'PY'
import csv, glob, sys, re, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(out + "/counters_*.csv"):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r.get("Kernel_Name", ""))
        k = re.sub(r"^.*::", "", k)
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", ""))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        n = max(1, len(cnt[(k, c)]))
        print(f"   {c:28s} {v / n:16.1f} per dispatch (n={n})")
PY
