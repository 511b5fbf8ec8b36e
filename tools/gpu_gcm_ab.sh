#!/bin/bash
# AES-GCM change check: the AES-GCM GPU tests on the tree's library, then the
# headline bench alternating with the given builds.
# usage: bash tools/gpu_gcm_ab.sh <tag> <rounds> lib.so...
set -e
T=$1; O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_variants.py tests/test_gpu_records.py tests/test_gpu_selftest.py tests/test_gpu_config4.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "gcm or aes or records or ghash or config4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_bench_libs.sh $T/bench $R "$@"
