#!/bin/bash
# Config 4 under key-table option settings (environment, read once per process),
# two alternating rounds.  usage: bash tools/gpu_c4_sweep.sh <tag> "ENV=V ..." ...
set -e
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  i=0
  for cfg in "default" "$@"; do
    i=$((i+1))
    if [ "$cfg" = default ]; then e=""; else e="$cfg"; fi
    env $e timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c${i}_${r}.json 2> $O/c${i}_${r}.err
    echo "$cfg r$r $(python3 -c "import json;d=json.load(open('$O/c${i}_${r}.json'));print(d['value'],d['per_op']['seal']['ms'],d['per_op']['open']['ms'])")"
  done
done
