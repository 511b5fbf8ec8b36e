set -e
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python -u tools/chacha_time_ab.py >> $O/ab.txt 2>&1
  for lib in "$@"; do TLSGPU_LIB=$lib timeout -k 10 120 python -u tools/chacha_time_ab.py >> $O/ab.txt 2>&1; done
done
echo done
