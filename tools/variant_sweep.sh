#!/bin/bash
# AES-GCM kernel variants (TLSGPU_GCM_VARIANT) through bench.py, one process each.
# usage: tools/variant_sweep.sh "0 1 2 3 4" [extra bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sweep
mkdir -p $OUT
for v in $1; do
  TLSGPU_GCM_VARIANT=$v timeout -k 10 240 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline $2 > $OUT/v$v.json 2> $OUT/v$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/v$v.json').read().strip().splitlines()[-1]); print('variant $v', {k: v['ms'] for k, v in d['per_kernel'].items()})"
done
