#!/bin/bash
# Round-4 measurement pass 2: PMC ceilings over full dispatches, the other
# bench rows (config 4, config 5, end to end, ingest, config 1) and the RCCL
# world-1 line.
set -e
O=gpurun_out/r4g; mkdir -p $O
bash tools/pmc_full.sh r4g/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
grep -E "^==|VALU lane|LDS lane|duration|clock" $O/pmc.log | head -40
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 400 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 400 python -u bench.py --e2e --no-cpu-baseline > $O/bench_e2e.json 2> $O/bench_e2e.err
timeout -k 10 400 python -u bench.py --config ingest > $O/bench_ingest.json 2> $O/bench_ingest.err
timeout -k 10 300 python -u bench.py --config c1 > $O/bench_c1.json 2> $O/bench_c1.err
timeout -k 10 400 python -u bench.py --dist-selftest --no-cpu-baseline > $O/bench_dist_selftest.json 2> $O/bench_dist_selftest.err
for f in c4 c5 e2e ingest c1 dist_selftest; do python3 -c "
import json; d=json.load(open('$O/bench_$f.json')); print('$f', d['value'], d.get('unit'), d.get('verified'), d.get('dist_backend', ''))"; done
