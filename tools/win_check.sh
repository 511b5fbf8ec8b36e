# Window-cache GCM lane kernel: parity (forced variants) and A/B bench vs full rounds.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/v29
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_variants.py -x -q --timeout 120 --timeout-method thread > $O/variants.log 2>&1
for v in 5 7 8; do
  TLSGPU_GCM_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_v$v.json 2> $O/bench_v$v.err
done
echo done
