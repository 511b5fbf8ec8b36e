set -e
O=gpurun_out/r2v13; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_selftest.py tests/test_gpu_distributed.py tests/test_gpu_records.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python -u bench.py --e2e > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/c5.err
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/c4.err
bash tools/traffic.sh r2v13/traffic > $O/traffic.log 2>&1
echo done
