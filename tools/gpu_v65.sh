set -e
O=gpurun_out/v65; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_variants.py tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_bitsliced.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for r in 1 2; do
  TLSGPU_LIB=tools/ab/libtlsgpu_a.so timeout -k 10 300 python -u bench.py --config c5 > $O/a_c5_$r.json 2>/dev/null
  timeout -k 10 300 python -u bench.py --config c5 > $O/b_c5_$r.json 2>/dev/null
done
TLSGPU_LIB=tools/ab/libtlsgpu_a.so timeout -k 10 300 python -u tools/gcm_kernel_probe.py 15 > $O/a_probe.txt 2>&1
timeout -k 10 300 python -u tools/gcm_kernel_probe.py 15 > $O/b_probe.txt 2>&1
echo done
