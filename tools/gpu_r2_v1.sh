set -e
mkdir -p gpurun_out/r2v1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2v1/pytest.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r2v1/bench.json 2> gpurun_out/r2v1/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2v1/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2v1/prof.log 2>&1
echo done
