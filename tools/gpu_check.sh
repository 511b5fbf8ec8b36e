#!/bin/bash
# One GPU pass over the tree: the -m gpu suite, smoke(), the headline bench
# (CPU baseline off unless CPU=1) and a rocprofv3 kernel-trace summary of the
# same bench command.  Each step has its own time limit; the first failure
# ends the script.  usage: bash tools/gpu_check.sh <tag> [pytest -k expr]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
K=${2:+-k "$2"}
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread $K > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
CB=--no-cpu-baseline; [ "$CPU" = 1 ] && CB=
timeout -k 10 600 python -u bench.py $CB > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -12 $O/kernel_stats.csv
