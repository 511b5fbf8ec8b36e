set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c4prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --config c4 --steps 3 --warmup 1 > $O/c4.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cat $O/kernel_stats.csv | cut -c1-250
