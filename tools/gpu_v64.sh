set -e
O=gpurun_out/v64; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/c5.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
