# GCM kernel probe A/B between the tree's library and alternative builds,
# alternating, plus the AES GPU tests under each alternative.
# usage: bash tools/gpu_lib_ab.sh <tag> <variant-args> lib.so...
set -e
O=gpurun_out/$1; V=$2; shift 2; mkdir -p $O
for lib in "$@"; do
  TLSGPU_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_parity.py tests/test_gpu_records.py -m gpu -x -q --timeout 200 --timeout-method thread >> $O/pytest.log 2>&1
done
for r in 1 2; do
  timeout -k 10 300 python -u tools/gcm_kernel_probe.py $V > $O/tree$r.txt 2>&1
  i=0
  for lib in "$@"; do i=$((i+1)); TLSGPU_LIB=$lib timeout -k 10 300 python -u tools/gcm_kernel_probe.py $V > $O/lib${i}_$r.txt 2>&1; done
done
echo done
