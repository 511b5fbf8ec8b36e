set -e
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    TLSGPU_LIB=$lib timeout -k 10 120 python -u tools/ccm_latency_ab.py >> $O/ab.txt 2>&1
  done
  timeout -k 10 120 python -u tools/ccm_latency_ab.py >> $O/ab.txt 2>&1
done
echo done
