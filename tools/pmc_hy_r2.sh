#!/bin/bash
# SQ counter passes over tools/prof_kernels.py (AES-128-GCM, 2^18 x 16 KiB) for
# the default hybrid octet kernel.  usage: tools/pmc_hy_r2.sh <outname>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_hy_r2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export PROF_ALGS=aes128gcm
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d $OUT/c/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/c/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT --output-format csv -d $OUT/c/p3 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p3.log 2>&1 || echo "pass 3 failed"
python3 $R/tools/pmc_summary.py $OUT/c > $OUT/summary.txt
cat $OUT/summary.txt
