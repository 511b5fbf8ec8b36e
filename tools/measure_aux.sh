#!/bin/bash
# The round's auxiliary measurements -> gpurun_out/<tag>/: HBM traffic passes
# (tools/traffic.sh: headline + config 4), the PMC role passes of DESIGN.md
# section 4 (tools/pmc_roles.sh), the single-key AES-256-GCM 2^20 x 16 KiB
# ceiling reference for config 4 and the ingest bench line.  Each step has its
# own time limit; the first failure ends the script.
#     usage: bash tools/measure_aux.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd $R
PROBE_KEYLEN=32 timeout -k 10 300 python -u tools/gcm_kernel_probe.py 0 > $O/aes256_single_key.txt 2>&1
cat $O/aes256_single_key.txt
timeout -k 10 300 python -u bench.py --config ingest --no-cpu-baseline > $O/bench_ingest.json 2> $O/bench_ingest.err
cat $O/bench_ingest.json
bash tools/traffic.sh $1/traffic
bash tools/pmc_roles.sh $1/roles
