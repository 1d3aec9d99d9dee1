set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 200 python3 bench.py --no-cpu > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || exit 1
cat gpurun_out/r03a/bench.json
bash tools/ab_trace.sh r03a_t "SGA_X=0" || exit 1
python3 tools/timeline.py gpurun_out/r03a_t/trace_1.csv 2 > gpurun_out/r03a_t/timeline.txt
cat gpurun_out/r03a_t/timeline.txt
