#!/bin/bash
# Counters of the hybrid AES-GCM kernel over full headline dispatches (2^20 x
# 16 KiB, AES-128 seal + open, two rounds) for three role mixes: the default
# (10 T-table + 6 bitsliced waves), T-table waves only (hy_t 16) and bitsliced
# waves only (hy_t -1) -- VERDICT r05 item 1.  Passes 1 and 2 as
# tools/pmc_full.sh; pass 3 the wait counters.  One rocprofv3 --pmc run per
# pass and mix, no other tracing.
#     usage: bash tools/pmc_roles2.sh <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_roles2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
export PROF_RECORDS=1048576 PROF_REPS=2 PROF_ALGS=aes128gcm
for mix in default hy_t=16 hy_t=-1; do
  if [ $mix = default ]; then export PROF_OPTS=""; else export PROF_OPTS=$mix; fi
  d=$OUT/${mix//=/_}
  for p in 1 2 3; do
    eval C=\$P$p
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --stats --output-format csv -d $d/p$p -o pass -- python3 $R/tools/prof_kernels.py > $d.p$p.log 2>&1 || { echo "pass $p of $mix failed"; tail -5 $d.p$p.log; [ $p = 3 ] || exit 1; }
  done
  python3 $R/tools/pmc_summary.py $d > $d.summary.txt
  echo "== $mix"; cat $d.summary.txt
done
