#!/bin/bash
# Counters over FULL headline dispatches (2^20 x 16 KiB records, bench.py's
# layout), two rounds of seal + open per AEAD, with the kernel trace in the
# same runs: effective clock (GRBM_GUI_ACTIVE / 8 / duration), VALU and LDS
# instructions per 16-byte block, LDS bank conflicts.
# One rocprofv3 --pmc run per pass, no system/runtime tracing.
#     usage: [PMC_ALGS="aes128ccm ..."] bash tools/pmc_full.sh <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_full}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
export PROF_RECORDS=1048576 PROF_REPS=2
for alg in ${PMC_ALGS:-aes128gcm chacha20-poly1305}; do
  export PROF_ALGS=$alg
  timeout -k 10 180 rocprofv3 --pmc $P1 --kernel-trace --stats --output-format csv -d $OUT/$alg/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/$alg.p1.log 2>&1
  timeout -k 10 180 rocprofv3 --pmc $P2 --kernel-trace --stats --output-format csv -d $OUT/$alg/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/$alg.p2.log 2>&1
  python3 $R/tools/pmc_summary.py $OUT/$alg > $OUT/$alg.summary.txt
  echo "== $alg"; cat $OUT/$alg.summary.txt
done
