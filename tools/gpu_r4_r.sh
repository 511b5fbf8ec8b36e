#!/bin/bash
# Role splits after the per-record precomputes: hybrid T-table waves 9 / 10 / 11
# of 16 (headline AES-128-GCM) and key-table hybrid 6 / 7 / 8 of 11 (config 4).
set -e
O=gpurun_out/r4r; mkdir -p $O
for r in 1 2 3; do
  for t in 10 9 11; do
    TLSGPU_HY_T=$t timeout -k 10 120 python -u tools/aes_time.py | sed "s/^/hy_t=$t /" | tee -a $O/hy_t.txt
  done
done
bash tools/gpu_c4_sweep_env.sh r4r 2 "TLSGPU_KT_T=7" "TLSGPU_KT_T=6" "TLSGPU_KT_T=8"
