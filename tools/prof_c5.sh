set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/v63
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/v63/prof -o c5 -- python3 $R/bench.py --config c5 --steps 3 --warmup 1 > $R/gpurun_out/v63/c5.log 2>&1
echo done
