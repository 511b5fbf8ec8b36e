# Round-2 measurement refresh, part B: configs 4 / 5, end-to-end against the
# measured PCIe ceiling, the ingest pipeline, the AES-CCM wave kernel probe.
# usage: bash tools/final_measure_r2b.sh <tag>
set -e
TAG=${1:-r2final}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/c4.err
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/c5.err
timeout -k 10 300 python -u bench.py --e2e --no-cpu-baseline > $O/bench_e2e.json 2> $O/e2e.err
timeout -k 10 300 python -u bench.py --config ingest > $O/bench_ingest.json 2> $O/ingest.err
timeout -k 10 200 python -u tools/ccm_wave_probe.py > $O/ccm_wave.txt 2>&1
echo done
