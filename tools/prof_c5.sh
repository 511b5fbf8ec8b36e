#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py --config c5 (framing + AEAD
# kernels of tg_seal_records).   usage: bash tools/prof_c5.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats.csv')):
    print(r['Name'][:100], r['Calls'], round(float(r['AverageNs'])/1e6,4), r['Percentage'])
" | head -20
