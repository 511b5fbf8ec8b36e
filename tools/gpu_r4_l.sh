#!/bin/bash
# Single-key hybrid: tag masks precomputed per slot (tree) vs computed per job
# (hynomask.so), 3 alternating rounds; then the AES GPU tests on the tree.
set -e
mkdir -p gpurun_out/r4l
bash tools/gpu_aes_ab.sh r4l 3 -- tools/ab/hynomask.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_variants.py tests/test_gpu_threads.py tests/test_gpu_records.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4l/pytest.log 2>&1
tail -3 gpurun_out/r4l/pytest.log
