#!/bin/bash
# Key-table hybrid: per-job keys precomputed (kth_jobkey_kernel) and a chunk's
# bounds/keys in one round of loads (tree) vs the per-job dependent chain
# (prev.so); then the config-4 GPU tests.
set -e
bash tools/gpu_c4_sweep_env.sh r4n 3 "X=tree" "TLSGPU_LIB=tools/ab/prev.so"
timeout -k 10 400 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n/pytest.log 2>&1
tail -3 gpurun_out/r4n/pytest.log
