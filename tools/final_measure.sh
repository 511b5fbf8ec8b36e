# Round measurement refresh: HBM traffic passes, headline bench (roofline.traffic
# from this run's passes), smoke, rocprofv3 kernel stats, configs 4/5, e2e, ingest,
# small-batch crossover probe.  usage: bash tools/final_measure.sh <tag>
set -e
TAG=${1:-v31}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/traffic.sh $TAG/traffic > $O/traffic.log 2>&1
cd $R
timeout -k 10 300 python -u bench.py --traffic-file $O/traffic/traffic.json > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
cd $R
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/c4.err
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/c5.err
timeout -k 10 300 python -u bench.py --e2e --no-cpu-baseline > $O/bench_e2e.json 2> $O/e2e.err
timeout -k 10 300 python -u bench.py --config ingest > $O/bench_ingest.json 2> $O/ingest.err
timeout -k 10 300 python -u tools/smallbatch_probe.py > $O/smallbatch.txt 2>&1
echo done
