#!/bin/bash
# 4-bit table build: basis x^(4j) G by shift + reduction (tree) vs a table-free
# multiply by the monomial (prev.so); then the key-table GPU tests.
set -e
bash tools/gpu_c4_sweep_env.sh r4o 3 "X=tree" "TLSGPU_LIB=tools/ab/prev.so"
timeout -k 10 400 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_kernel_variants.py tests/test_gpu_selftest.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4o/pytest.log 2>&1
tail -3 gpurun_out/r4o/pytest.log
