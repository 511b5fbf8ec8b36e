#!/bin/bash
# Same-box A/B of AES-GCM kernel builds: tools/aes_time.py alternating between
# the tree's library and alternative builds (TLSGPU_LIB), R rounds.
# usage: bash tools/gpu_aes_ab.sh <tag> <rounds> [--chacha|--keylen 32] -- lib.so...
set -e
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
EXTRA=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do EXTRA+=("$1"); shift; done
shift
for r in $(seq 1 $R); do
  timeout -k 10 120 python -u tools/aes_time.py "${EXTRA[@]}" | tee -a $O/ab.txt
  for lib in "$@"; do
    TLSGPU_LIB=$lib timeout -k 10 120 python -u tools/aes_time.py "${EXTRA[@]}" | tee -a $O/ab.txt
  done
done
