#!/bin/bash
# Config 4 with the lane kernel at 512 threads and 2 jobs per grab (tree):
# lane kernel 2 / 4 blocks per step, 1 / 4 jobs per grab, split 1024 / 1536.
set -e
bash tools/gpu_c4_sweep_env.sh r4j 2 "X=tree" "TLSGPU_LIB=tools/ab/g2.so" "TLSGPU_LIB=tools/ab/g4.so" \
  "TLSGPU_LIB=tools/ab/ch1.so" "TLSGPU_LIB=tools/ab/ch4.so" "TLSGPU_KT_SPLIT=1024" "TLSGPU_KT_SPLIT=1536"
