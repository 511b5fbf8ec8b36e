#!/bin/bash
# Round-4 measurement pass: calibrated HBM traffic of the headline, config-4 and
# config-5 kernels (tools/traffic.sh), the RCCL world-1 bench line and test,
# and the config-1 line (device + the host run in full).
set -e
O=gpurun_out/r4d; mkdir -p $O
bash tools/traffic.sh r4d/traffic > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
tail -40 $O/traffic.log | head -60
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 1; }
tail -2 $O/pytest_dist.log
timeout -k 10 400 python -u bench.py --dist-selftest --no-cpu-baseline --traffic-file $O/traffic/traffic.json > $O/bench_dist_selftest.json 2> $O/bench_dist_selftest.err
cat $O/bench_dist_selftest.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['dist_backend'], d['dist_selftest'])"
timeout -k 10 300 python -u bench.py --config c1 > $O/bench_c1.json 2> $O/bench_c1.err
cat $O/bench_c1.json
