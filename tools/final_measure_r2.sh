# Round-2 measurement refresh, part A (B: tools/final_measure_r2b.sh): the full
# -m gpu suite, HBM traffic passes, the headline bench (roofline.traffic from
# this run's passes), smoke, rocprofv3 kernel stats.  usage: bash tools/final_measure_r2.sh <tag>
set -e
TAG=${1:-r2final}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
bash tools/traffic.sh $TAG/traffic > $O/traffic.log 2>&1
cd $R
timeout -k 10 300 python -u bench.py --traffic-file $O/traffic/traffic.json > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo done
