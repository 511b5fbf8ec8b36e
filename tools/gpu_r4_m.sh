#!/bin/bash
# Config 4 measurement builds (wrong tags, refused by tlsgpu.load() unless
# TLSGPU_ALLOW_MEASUREMENT_BUILD=1): key-table GHASH multiply removed
# (noghash.so), per-key table build removed (nobuild.so), against the tree.
set -e
bash tools/gpu_c4_sweep_env.sh r4m 2 "X=tree" "TLSGPU_ALLOW_MEASUREMENT_BUILD=1 TLSGPU_LIB=tools/ab/noghash.so" \
  "TLSGPU_ALLOW_MEASUREMENT_BUILD=1 TLSGPU_LIB=tools/ab/nobuild.so"
