#!/bin/bash
# AES-128-CCM / CCM_8 row at the headline shape (bench.py --config ccm) with
# its CPU baseline, then the CCM GPU tests.
set -e
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 600 python -u bench.py --config ccm > $O/bench_ccm.json 2> $O/bench_ccm.err
tail -1 $O/bench_ccm.json | cut -c1-600
timeout -k 10 300 python -u -m pytest tests/test_gpu_ccm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
