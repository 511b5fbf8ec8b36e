#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per pass, no tracing) and a kernel-trace
# run over tools/prof_kernels.py (2^18 x 16 KiB records) for the hybrid
# AES-GCM kernel and its two roles alone (T-table waves only: hy_t=16;
# bitsliced waves only: hy_t=-1) and the ChaCha20-Poly1305 lane kernel, for
# the issue / LDS ceilings of DESIGN.md section 4 (tools/pmc_summary.py,
# tools/issue_model.py).  usage: tools/pmc_roles.sh <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_roles}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
run() {   # name algs opts
  local name=$1; export PROF_ALGS=$2 PROF_OPTS=$3
  timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/$name/p1 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/$name.p1.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $P2 --output-format csv -d $OUT/$name/p2 -o pass -- python3 $R/tools/prof_kernels.py > $OUT/$name.p2.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name/kt -o kt -- python3 $R/tools/prof_kernels.py > $OUT/$name.kt.log 2>&1
  python3 $R/tools/pmc_summary.py $OUT/$name > $OUT/$name.summary.txt
  echo "== $name"; cat $OUT/$name.summary.txt
}
run hybrid aes128gcm ""
run ttable aes128gcm hy_t=16
run bitsliced aes128gcm hy_t=-1
run chacha chacha20-poly1305 ""
