#!/bin/bash
set -e
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 python -u bench.py --config c1 > $O/bench_c1.json 2> $O/bench_c1.err
cat $O/bench_c1.json
timeout -k 10 400 python -u bench.py --dist-selftest --no-cpu-baseline > $O/bench_dist_selftest.json 2> $O/bench_dist_selftest.err
python3 -c "
import json; d=json.load(open('$O/bench_dist_selftest.json')); print(d['value'], d['dist_backend'], d['dist_selftest'])"
wc -l $O/bench_dist_selftest.json
