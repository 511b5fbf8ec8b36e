#!/bin/bash
# Key-table mask kernel as a persistent T-table grid (tree) vs a lane per
# record with the byte-wise cipher (prev.so): config-4 GPU tests, config 4 A/B.
set -e
mkdir -p gpurun_out/r4ab
timeout -k 10 500 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config4 or key_table or out_of_range" > gpurun_out/r4ab/pytest.log 2>&1
tail -2 gpurun_out/r4ab/pytest.log
bash tools/gpu_c4_sweep_env.sh r4ab 3 "X=tree" "TLSGPU_LIB=tools/ab/prev.so"
