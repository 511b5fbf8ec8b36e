set -e
O=gpurun_out/v67; mkdir -p $O
bash tools/gpu_ab.sh v67 15
for r in 1 2; do
  TLSGPU_LIB=tools/ab/libtlsgpu_a.so timeout -k 10 300 python -u bench.py --config c5 > $O/a_c5_$r.json 2>/dev/null
  timeout -k 10 300 python -u bench.py --config c5 > $O/b_c5_$r.json 2>/dev/null
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_records.py tests/test_gpu_config4.py -m gpu -x -q --timeout 200 --timeout-method thread >> $O/pytest.log 2>&1
echo done
