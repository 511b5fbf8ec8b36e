#!/bin/bash
# Second half of a round's final measurement (after tools/gpu_check.sh):
# config 4 / config 5 / end-to-end bench lines (CPU baselines on), the N = 2
# launcher rehearsal, the HBM traffic passes and the full-dispatch counters.
# Each GPU step has its own time limit; the first failure ends the script.
#     usage: bash tools/measure_final.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err
cat $O/bench_c4.json
timeout -k 10 400 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
timeout -k 10 400 python -u bench.py --e2e --no-cpu-baseline > $O/bench_e2e.json 2> $O/bench_e2e.err
cat $O/bench_e2e.json
bash tools/gpu_n2_rehearsal.sh $1/n2
bash tools/traffic.sh $1/traffic
bash tools/pmc_full.sh $1/pmc_full
