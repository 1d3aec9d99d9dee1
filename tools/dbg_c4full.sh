mkdir -p gpurun_out/r03w
SGA_PSEG_DEBUG=1 SGA_SIZE_CHECK=1 SGA_LRU_DEBUG=1 timeout -k 10 300 python3 -u -m pytest "tests/test_param_lru_gpu.py::test_c4_full_mode_10k_rules_unfolded_values[4194304]" -m gpu -x -q -s --timeout 250 --timeout-method thread > gpurun_out/r03w/dbg.log 2>&1
grep -a "size check\|lru_prepare\|pseg m=" gpurun_out/r03w/dbg.log | head -24
