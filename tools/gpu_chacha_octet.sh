#!/bin/bash
# The octet ChaCha20-Poly1305 kernel (chacha_variant 6): its GPU tests, then a
# same-box alternating A/B against the tile kernel (auto) with
# tools/aes_time.py --chacha, R rounds; LIBS: extra builds timed as octets too.
#   [LIBS="a.so b.so"] bash tools/gpu_chacha_octet.sh <tag> [rounds] [tests-expr]
set -e
T=$1; R=${2:-3}; O=gpurun_out/$T; mkdir -p $O
K=${3:-"selftest or (variants and chacha) or (full_size and octet)"}
if [ "$K" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for r in $(seq 1 $R); do
  timeout -k 10 120 python -u tools/aes_time.py --chacha | sed 's/"lib": "tree"/"lib": "tile (auto)"/' | tee -a $O/ab.txt
  TLSGPU_CHACHA_VARIANT=6 timeout -k 10 120 python -u tools/aes_time.py --chacha | sed 's/"lib": "tree"/"lib": "octet (variant 6)"/' | tee -a $O/ab.txt
  for lib in $LIBS; do
    TLSGPU_LIB=$lib TLSGPU_CHACHA_VARIANT=6 timeout -k 10 120 python -u tools/aes_time.py --chacha | tee -a $O/ab.txt
  done
done
