#!/bin/bash
# HBM traffic of the headline kernels, per launch: two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE: separate passes, no tracing) over one launch of each
# kernel at bench.py's headline config, then tools/traffic_summary.py applies
# the MI355X_MICROARCH.md corrections and writes <out>/traffic.json.
# usage: tools/traffic.sh <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-traffic}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o pass \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$c.log 2>&1
done
python3 $R/tools/traffic_summary.py $OUT > $OUT/traffic.json
cat $OUT/traffic.json
