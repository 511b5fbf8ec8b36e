#!/bin/bash
# Config 4 (bench.py --config c4) under each given environment, alternating, R
# rounds: usage: bash tools/gpu_c4_sweep_env.sh <tag> <rounds> "ENV=.. ENV=.." ...
set -e
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_${i}_$r.json 2> $O/c4_${i}_$r.err
    python3 -c "
import json; d=json.load(open('$O/c4_${i}_$r.json'))
print('%-40s %8.2f GiB/s seal %.3f open %.3f' % ('$e', d['value'], d['per_op']['seal']['ms'], d['per_op']['open']['ms']))" | tee -a $O/c4_sweep.txt
  done
done
