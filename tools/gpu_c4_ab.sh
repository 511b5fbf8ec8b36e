#!/bin/bash
# Config-4 A/B: the key-table GPU tests on the tree's library, then
# bench.py --config c4 alternating between the tree and the given builds.
# usage: bash tools/gpu_c4_ab.sh <tag> lib.so...
set -e
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_kernel_variants.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "config4 or key_table" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config c4 > $O/tree$r.json 2> $O/tree$r.err
  echo "tree r$r $(python3 -c "import json;d=json.load(open('$O/tree$r.json'));print(d['value'],d['per_op']['seal']['ms'],d['per_op']['open']['ms'])")"
  i=0
  for lib in "$@"; do
    i=$((i+1))
    TLSGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config c4 > $O/lib${i}_$r.json 2> $O/lib${i}_$r.err
    echo "$lib r$r $(python3 -c "import json;d=json.load(open('$O/lib${i}_$r.json'));print(d['value'],d['per_op']['seal']['ms'],d['per_op']['open']['ms'])")"
  done
done
