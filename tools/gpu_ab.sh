# A/B of two builds of libtlsgpu on one box: tools/ab/libtlsgpu_a.so (before)
# against the tree's build, alternating, with gcm_kernel_probe (bytes checked
# against the first kernel) and the bench.  usage: bash tools/gpu_ab.sh <tag> [probe args]
set -e
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for r in 1 2; do
  TLSGPU_LIB=tools/ab/libtlsgpu_a.so timeout -k 10 300 python -u tools/gcm_kernel_probe.py "$@" > $O/a$r.txt 2>&1
  timeout -k 10 300 python -u tools/gcm_kernel_probe.py "$@" > $O/b$r.txt 2>&1
done
echo done
