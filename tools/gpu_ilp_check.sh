set -e
mkdir -p gpurun_out/ilp1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_variants.py tests/test_gpu_selftest.py tests/test_gpu_records.py -m gpu -x -q --timeout 200 --timeout-method thread -k "chacha or records" > gpurun_out/ilp1/pytest.log 2>&1 || { tail -30 gpurun_out/ilp1/pytest.log; exit 1; }
tail -2 gpurun_out/ilp1/pytest.log
bash tools/gpu_c4_ab.sh c4ilp tools/ab/lib_bs8_ilp.so tools/ab/lib_gcm_ilp.so
