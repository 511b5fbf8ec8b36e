#!/bin/bash
# SQ counter passes over tools/prof_kernels.py (AES-128-GCM only) for the
# T-table kernel (variant 0) and the 8-block bitsliced kernel (variant 14).
# usage: tools/pmc_bs8.sh <outname>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_bs8}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export PROF_ALGS=aes128gcm
for v in 0 14; do
  TLSGPU_GCM_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d $OUT/v$v/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/v$v.p1.log 2>&1 || exit 1
  TLSGPU_GCM_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/v$v/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/v$v.p2.log 2>&1 || exit 1
done
python3 $R/tools/pmc_summary.py $OUT/v0 > $OUT/summary.txt
python3 $R/tools/pmc_summary.py $OUT/v14 >> $OUT/summary.txt
cat $OUT/summary.txt
