#!/bin/bash
set -e
O=gpurun_out/r4b; mkdir -p $O
bash tools/gpu_aes_ab.sh r4b 3 -- tools/ab/base.so
bash tools/gpu_c4_sweep_env.sh r4b 2 "TLSGPU_KT_T=5" "TLSGPU_KT_T=7" "TLSGPU_KT_T=9" "TLSGPU_KT_T=11" "TLSGPU_KT_HYBRID=-1"
