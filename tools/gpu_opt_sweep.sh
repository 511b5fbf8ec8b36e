#!/bin/bash
# Same-box sweep of one option over values with tools/aes_time.py, alternating
# the values R rounds (each line carries its TLSGPU_* options).
#   bash tools/gpu_opt_sweep.sh <tag> <rounds> <ENVNAME> "<v1 v2 ...>" [aes_time args]
set -e
T=$1; R=$2; E=$3; V=$4; shift 4; O=gpurun_out/$T; mkdir -p $O
for r in $(seq 1 $R); do
  for v in $V; do
    env "$E=$v" timeout -k 10 120 python -u tools/aes_time.py "$@" | tee -a $O/sweep_$E.txt
  done
done
