#!/bin/bash
# SQ counter passes over the bitsliced AES-GCM kernel (TLSGPU_GCM_VARIANT=$2).
# Usage: tools/pmc_bs.sh <outname> <variant>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_bs}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export TLSGPU_GCM_VARIANT=${2:-4} PROF_ALGS=${PROF_ALGS:-aes128gcm}
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p2.log 2>&1 &&
python3 $R/tools/pmc_summary.py $OUT
