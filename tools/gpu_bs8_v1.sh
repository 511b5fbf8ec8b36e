set -e
O=gpurun_out/r2v2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 120 --timeout-method thread -k "14" > $O/pytest_bs8.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "full_size and bs8" >> $O/pytest_bs8.log 2>&1
TLSGPU_GCM_VARIANT=14 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_bs8.json 2> $O/bench_bs8.err
echo done
