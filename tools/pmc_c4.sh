#!/bin/bash
# Counters over config 4's dispatches (bench.py --config c4, one timed step):
# the key-table hybrid (gcm_kth_kernel) and the short-record lane kernel.
# Per-16-B figures are normalised to the long records' payload (PROF_LEN).
#     usage: bash tools/pmc_c4.sh <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_c4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -k 10 240 rocprofv3 --pmc $P1 --kernel-trace --stats --output-format csv -d $OUT/c4/p1 -o pass -- python3 $R/bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c4.p1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc $P2 --kernel-trace --stats --output-format csv -d $OUT/c4/p2 -o pass -- python3 $R/bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c4.p2.log 2>&1
PROF_RECORDS=1 PROF_LEN=6103244480 python3 $R/tools/pmc_summary.py $OUT/c4 > $OUT/c4.summary.txt
cat $OUT/c4.summary.txt
