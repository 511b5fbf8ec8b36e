# A/B of the hybrid kernel's key-plane providers (TLSGPU_HY_KEYS 1 = scalar
# loads at use, 3 = scalar loads hoisted to the round start).
set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 120 --timeout-method thread -k "15" > $O/pytest.log 2>&1
TLSGPU_HY_KEYS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread >> $O/pytest.log 2>&1
timeout -k 10 500 python -u tools/gcm_kernel_probe.py 15:TLSGPU_HY_KEYS=1 15:TLSGPU_HY_KEYS=3 15:TLSGPU_HY_KEYS=1 15:TLSGPU_HY_KEYS=3 15:TLSGPU_HY_KEYS=3,TLSGPU_HY_T=6 15:TLSGPU_HY_KEYS=3,TLSGPU_HY_T=7 > $O/probe.txt 2>&1
echo done
