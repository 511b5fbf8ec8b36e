#!/bin/bash
# Key-table hybrid: tag masks precomputed per plan slot (tree) vs computed per
# record by every wave (nomask.so); then the config-4 GPU tests on the tree.
set -e
bash tools/gpu_c4_sweep_env.sh r4k 3 "X=tree" "TLSGPU_LIB=tools/ab/nomask.so"
timeout -k 10 400 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4k/pytest.log 2>&1
tail -3 gpurun_out/r4k/pytest.log
