set -e
O=gpurun_out/r2v10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 120 --timeout-method thread -k "14 or 15" > $O/pytest.log 2>&1
TLSGPU_OCT_PF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 120 --timeout-method thread -k "15" >> $O/pytest.log 2>&1
timeout -k 10 400 python -u tools/gcm_kernel_probe.py 0 15:TLSGPU_HY_T=8 15:TLSGPU_HY_T=8,TLSGPU_OCT_PF=1 15:TLSGPU_HY_T=6 15:TLSGPU_HY_T=10 15:TLSGPU_HY_T=6,TLSGPU_OCT_PF=1 15:TLSGPU_HY_T=16,TLSGPU_OCT_PF=1 15:TLSGPU_HY_T=0,TLSGPU_OCT_PF=1 > $O/probe.txt 2>&1
PROBE_KEYLEN=32 timeout -k 10 400 python -u tools/gcm_kernel_probe.py 0 14 15:TLSGPU_HY_T=8 15:TLSGPU_HY_T=6 15:TLSGPU_HY_T=10 >> $O/probe.txt 2>&1
echo done
