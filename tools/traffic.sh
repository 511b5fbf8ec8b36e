#!/bin/bash
# HBM traffic of the headline kernels, per launch, calibrated per access shape:
# separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; no tracing) over
# (1) tools/fetch_calib (4 GiB copies in each access shape the kernels use)
# and (2) one launch of each kernel at bench.py's headline config and one
# config-4 seal + open (bench.py --config c4), and one config-5 record seal
# (bench.py --config c5, in c5_* directories: its AEAD kernel has the
# headline seal kernel's name); then
# tools/traffic_summary.py derives each shape's factor and writes
# <out>/traffic.json.   usage: tools/traffic.sh <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-traffic}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/cal_$c -o pass \
      -- $R/tools/fetch_calib > $OUT/cal_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/bench_$c -o pass \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/bench_c4_$c -o pass \
      -- python3 $R/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_c4_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/c5_$c -o pass \
      -- python3 $R/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c5_$c.log 2>&1
done
python3 $R/tools/traffic_summary.py $OUT > $OUT/traffic.json
cat $OUT/traffic.json
