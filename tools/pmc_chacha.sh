#!/bin/bash
# SQ counter passes over tools/prof_kernels.py (ChaCha20-Poly1305 only, 2^18 x
# 16 KiB records) for the lane-per-record kernel, plus the VALU issue probe of
# the ChaCha instruction shapes.  usage: tools/pmc_chacha.sh <outname>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_chacha}
mkdir -p $OUT
timeout -k 10 120 $R/tools/issue_probe3 > $OUT/issue_probe3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
export PROF_ALGS=chacha20-poly1305
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d $OUT/c/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/c/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/p2.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c/kt -o kt -- python3 $R/tools/prof_kernels.py > $OUT/kt.log 2>&1
python3 $R/tools/pmc_summary.py $OUT/c > $OUT/summary.txt
cat $OUT/issue_probe3.txt $OUT/summary.txt
