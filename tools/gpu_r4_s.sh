#!/bin/bash
# Key-table hybrid occupancy probe: 11 waves (tree) vs the last 1 / 2 bitsliced
# waves idle (10 / 9 working waves).
set -e
bash tools/gpu_c4_sweep_env.sh r4s 2 "X=tree" "TLSGPU_LIB=tools/ab/idle1.so" "TLSGPU_LIB=tools/ab/idle2.so"
