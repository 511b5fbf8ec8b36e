#!/bin/bash
# SQ counter passes over tools/prof_kernels.py (AES-128-GCM only) for the
# hybrid octet kernel at several T-table wave counts.  usage: tools/pmc_hy.sh <outname>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_hy}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export PROF_ALGS=aes128gcm TLSGPU_GCM_VARIANT=15
for t in 0 8 16; do
  TLSGPU_HY_T=$t timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d $OUT/t$t/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/t$t.p1.log 2>&1 || exit 1
  TLSGPU_HY_T=$t timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/t$t/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/t$t.p2.log 2>&1 || exit 1
  echo "#### HY_T=$t" >> $OUT/summary.txt
  python3 $R/tools/pmc_summary.py $OUT/t$t >> $OUT/summary.txt
done
cat $OUT/summary.txt
