# A/B of alternative library builds with the headline bench (no CPU
# baseline), alternating, plus FETCH/WRITE passes of the B build.
# usage: bash tools/gpu_bench_ab.sh <tag> <lib.so>
set -e
O=gpurun_out/$1; LIB=$2; mkdir -p $O
R=$GRAFT_REPO_ROOT
TLSGPU_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chacha" > $O/pytest.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/a$r.json 2> $O/a$r.err
  TLSGPU_LIB=$LIB timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b$r.json 2> $O/b$r.err
done
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  TLSGPU_LIB=$R/$LIB timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/$O/bench_$c -o pass \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/$O/bench_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $R/$O/cal_$c -o pass \
      -- $R/tools/fetch_calib > $R/$O/cal_$c.log 2>&1
done
echo done
