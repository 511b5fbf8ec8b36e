#!/bin/bash
# Final-tree counters and rows: SQ counters of the headline kernels and of
# config 4's kernels; config 4 and config 5 lines (config 5 with its CPU
# baseline).
set -e
O=gpurun_out/r4t; mkdir -p $O
bash tools/pmc_full.sh r4t/pmc_full > $O/pmc_full.log 2>&1
bash tools/pmc_c4.sh r4t/pmc_c4 > $O/pmc_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 400 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
tail -1 $O/bench_c4.json | cut -c1-300; tail -1 $O/bench_c5.json | cut -c1-300
