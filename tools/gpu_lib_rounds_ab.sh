#!/bin/bash
# Same-box A/B of the tree's library against another build (e.g. the previous
# round's, tools/ab/r05.so): bench.py --config c4 and the headline, alternating,
# R rounds.   usage: bash tools/gpu_lib_rounds_ab.sh <tag> <lib.so> [rounds]
set -e
T=$1; LIB=$2; R=${3:-2}; O=gpurun_out/$T; mkdir -p $O
for r in $(seq 1 $R); do
  for which in tree other; do
    if [ $which = other ]; then export TLSGPU_LIB=$LIB; else unset TLSGPU_LIB; fi
    timeout -k 10 300 python -u bench.py --config c4 > $O/c4_${which}_$r.json 2> $O/c4_${which}_$r.err
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_${which}_$r.json 2> $O/bench_${which}_$r.err
    python3 -c "import json;c=json.load(open('$O/c4_${which}_$r.json'));b=json.load(open('$O/bench_${which}_$r.json'));print('$which', $r, 'c4', c['value'], 'headline', b['value'], {k:v['ms'] for k,v in b['per_kernel'].items()})" | tee -a $O/ab.txt
  done
done
