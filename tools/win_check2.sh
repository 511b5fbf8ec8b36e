# Window cache in the wave-per-record and key-table kernels: full GPU suite,
# small-batch probe (wave kernels), config 4 A/B (table variant 6 = full rounds).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/v30
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u tools/smallbatch_probe.py > $O/smallbatch.txt 2>&1
timeout -k 10 200 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/c4.err
TLSGPU_GCM_TABLE_VARIANT=6 timeout -k 10 200 python -u bench.py --config c4 > $O/bench_c4_v6.json 2> $O/c4v6.err
echo done
