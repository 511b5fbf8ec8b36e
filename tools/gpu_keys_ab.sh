# Hybrid AES-GCM key-plane providers on one box (TLSGPU_HY_KEYS), alternating,
# with the parity/variant GPU tests run under each.  usage: bash tools/gpu_keys_ab.sh <tag> K...
set -e
O=gpurun_out/$1; shift; mkdir -p $O
for k in "$@"; do
  TLSGPU_HY_KEYS=$k timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "15 or gcm or aes" >> $O/pytest.log 2>&1
done
args=""
for k in "$@"; do args="$args 15:TLSGPU_HY_KEYS=$k"; done
timeout -k 10 500 python -u tools/gcm_kernel_probe.py $args $args > $O/probe.txt 2>&1
echo done
