#!/bin/bash
# Single-key mask kernel: persistent T-table grid (tree) vs a lane per record
# with the byte-wise cipher (prev.so): GPU tests, AES A/B, kernel times.
set -e
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_variants.py tests/test_gpu_records.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
bash tools/gpu_aes_ab.sh r4v 3 -- tools/ab/prev.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/aes_time.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$O/kernel_stats.csv \;
grep -i "mask\|hy_setup" $GRAFT_REPO_ROOT/$O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
