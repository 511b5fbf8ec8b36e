set -e
O=gpurun_out/v68; mkdir -p $O
TLSGPU_LIB=tools/ab/libtlsgpu_cc_defer.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "chacha or Chacha or CHACHA or records or full_size or smoke" > $O/pytest.log 2>&1
for r in 1 2; do
  timeout -k 10 120 python -u tools/chacha_time_ab.py >> $O/ab.txt 2>&1
  TLSGPU_LIB=tools/ab/libtlsgpu_cc_defer.so timeout -k 10 120 python -u tools/chacha_time_ab.py >> $O/ab.txt 2>&1
done
TLSGPU_LIB=tools/ab/libtlsgpu_cc_defer.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_defer.json 2>/dev/null
echo done
