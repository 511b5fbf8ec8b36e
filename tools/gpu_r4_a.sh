#!/bin/bash
# Round-4 batch: the new key-table hybrid and bitsliced key-row paths tested,
# then same-box A/Bs (AES headline, config 4, mid-size hybrid calls).
set -e
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_config4.py tests/test_gpu_parity.py tests/test_gpu_keysetup.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hybrid_kernel or config4 or out_of_range or hy_t or full_size or key_table or kat or golden or keysetup or device" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/gpu_aes_ab.sh r4a 3 -- tools/ab/kvec.so tools/ab/base.so
bash tools/gpu_c4_hyb.sh r4a 2 X=1
for lib in tree tools/ab/kvec.so; do
  if [ $lib = tree ]; then timeout -k 10 200 python -u tools/hy_call_time.py | tee -a $O/calltime.txt
  else TLSGPU_LIB=$lib timeout -k 10 200 python -u tools/hy_call_time.py | tee -a $O/calltime.txt; fi
done
