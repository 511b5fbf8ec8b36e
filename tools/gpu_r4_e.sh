#!/bin/bash
set -e
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_config4.py -m gpu -x -q --timeout 300 --timeout-method thread -k "key_table or config4 or out_of_range or hybrid_kernel" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_c4_sweep_env.sh r4e 2 "X=tree" "TLSGPU_LIB=tools/ab/head.so"
