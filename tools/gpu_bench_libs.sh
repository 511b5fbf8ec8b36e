#!/bin/bash
# Headline bench (no CPU baseline) alternating between the tree's library and
# alternative builds (TLSGPU_LIB), R rounds; one line per run with the four
# kernel times.   usage: bash tools/gpu_bench_libs.sh <tag> <rounds> lib.so...
set -e
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
line() { python3 -c "
import json,sys; d=json.load(open('$1')); k=d['per_kernel']
print('%-40s %8.2f' % ('$2', d['value']), ' '.join('%s %.3f' % (n.split('_')[0][:6]+'_'+n.split('_')[1], v['ms']) for n, v in k.items()))"; }
for r in $(seq 1 $R); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/tree_$r.json 2> $O/tree_$r.err
  line $O/tree_$r.json "tree r$r"
  i=0
  for lib in "$@"; do
    i=$((i+1))
    TLSGPU_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/lib${i}_$r.json 2> $O/lib${i}_$r.err
    line $O/lib${i}_$r.json "$(basename $lib) r$r"
  done
done
