#!/bin/bash
# Precomputed last-block keystream for records whose last batch row holds one
# block (tree) vs HEAD (prev.so): GPU tests first, then headline AES A/B and
# config 5 A/B, alternating on one box.
set -e
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_variants.py tests/test_gpu_records.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
bash tools/gpu_aes_ab.sh r4q 3 -- tools/ab/prev.so
for r in 1 2; do
  for lib in "" tools/ab/prev.so; do
    TLSGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
    python3 -c "
import json; d=json.load(open('$O/c5.json')); print('c5 %-20s %8.2f GiB/s %.3f ms' % ('${lib:-tree}', d['value'], d['ms_per_step']))" | tee -a $O/c5_ab.txt
  done
done
