#!/bin/bash
# One GPU call, any mix of steps, each under its own time limit; the first
# failing step ends the script (set -e).  Output under gpurun_out/<tag>/.
#   bash tools/gpu_run.sh <tag> step [step ...]
# steps:
#   tests[=EXPR]   pytest -m gpu (-k EXPR)            -> pytest.log
#   smoke          __graft_entry__.smoke()             -> smoke.log
#   bench          bench.py (headline, CPU baseline)   -> bench.json
#   bench-nocpu    bench.py --no-cpu-baseline          -> bench.json
#   c4 | c5 | ccm | c1 | e2e | ingest                  -> bench_<step>.json
#   distself       bench.py --dist-selftest: RCCL at world size 1 -> bench_dist_selftest.json
#   n2             bench.py --gpus 2 --config c5 --records 65536 over gloo on
#                  one MI355X (both ranks on the one device), CPU baseline on
#                  -> bench_n2_c5.json; and the headline leg -> bench_n2.json
#   prof           rocprofv3 --kernel-trace --stats of bench.py --no-cpu-baseline
#                  -> kernel_stats.csv
#   pmc            tools/pmc_full.sh passes of the headline kernels
#   traffic        tools/traffic.sh FETCH_SIZE / WRITE_SIZE passes -> traffic.json
#   memprobe       device memory per fresh stream by launch kind -> stream_mem.jsonl
#   roleprobe      per-role cycle accounting of the hybrid AES-GCM kernel -> role_probe.json
#   pmcroles       counters of the hybrid for three role mixes (tools/pmc_roles2.sh)
#   c4fetch        FETCH_SIZE / WRITE_SIZE passes over one config-4 seal + open
#                  -> c4fetch<suffix>.txt (per-dispatch sums by kernel)
#   ab=LIBA,LIBB   alternate two built libraries (tools/gpu_lib_ab.sh) -> ab.txt
# A step may carry its own environment after '@' (comma-separated, e.g.
# ccm@TLSGPU_CCM_VARIANT=4,TLSGPU_CCM_HY_T=-1); its output file then takes the
# suffix after '@' with '=' and ',' replaced.  Environment passes through
# (TLSGPU_* options, BENCH_ARGS for bench steps).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$R/gpurun_out/$T; mkdir -p $O
cd $R
for st0 in "$@"; do
  echo "== $st0 $(date +%T)"
  st=${st0%%@*}; SUF=""; ENVS=""
  if [ "$st" != "$st0" ]; then ENVS=${st0#*@}; SUF=_$(echo "$ENVS" | tr '=,' '-_'); fi
  for kv in ${ENVS//,/ }; do export "$kv"; done
  case $st in
    tests|tests=*)
      K=${st#tests}; K=${K#=}
      if [ -n "$K" ]; then
        timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
      else
        timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
      fi
      tail -3 $O/pytest.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err; cat $O/bench.json ;;
    bench-nocpu)
      timeout -k 10 600 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $O/bench.json 2> $O/bench.err; cat $O/bench.json ;;
    c4|c5|ccm|c1|ingest)
      timeout -k 10 600 python -u bench.py --config $st $BENCH_ARGS > $O/bench_$st$SUF.json 2> $O/bench_$st$SUF.err
      cat $O/bench_$st$SUF.json ;;
    distself)
      timeout -k 10 600 python -u bench.py --dist-selftest --no-cpu-baseline $BENCH_ARGS > $O/bench_dist_selftest.json 2> $O/bench_dist_selftest.err
      cat $O/bench_dist_selftest.json ;;
    e2e)
      timeout -k 10 600 python -u bench.py --e2e --no-cpu-baseline $BENCH_ARGS > $O/bench_e2e.json 2> $O/bench_e2e.err; cat $O/bench_e2e.json ;;
    n2)
      TLSGPU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --config c5 --records 65536 \
        --steps 3 --warmup 1 > $O/bench_n2_c5.json 2> $O/bench_n2_c5.err; cat $O/bench_n2_c5.json
      TLSGPU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --records 65536 \
        --steps 3 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err; cat $O/bench_n2.json ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline $BENCH_ARGS > $O/prof.log 2>&1)
      find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
      head -12 $O/kernel_stats.csv ;;
    pmc)
      bash tools/pmc_full.sh $T/pmc ;;
    fetch)   # FETCH_SIZE / WRITE_SIZE of one seal + open per PROF_ALGS AEAD (2^18 x 16 KiB)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --pmc $c --kernel-trace --stats --output-format csv \
          -d $O/fetch_$c$SUF -o pass -- python3 $R/tools/prof_kernels.py > $O/fetch_$c$SUF.log 2>&1)
      done
      python3 tools/pmc_summary.py $O > $O/fetch$SUF.txt 2>&1 || true; head -40 $O/fetch$SUF.txt ;;
    traffic)
      bash tools/traffic.sh $T ;;
    roleprobe)   # per-role cycle accounting (tools/role_probe.py, tools/ab/role_probe.so) + role PMC passes
      timeout -k 10 900 python -u tools/role_probe.py tools/ab/role_probe.so > $O/role_probe.json 2> $O/role_probe.err; tail -3 $O/role_probe.err ;;
    pmcroles)
      bash tools/pmc_roles2.sh $T/pmc_roles ;;
    memprobe)   # device memory per fresh stream by launch kind (tools/stream_mem_probe.py)
      timeout -k 10 300 python -u tools/stream_mem_probe.py > $O/stream_mem.jsonl 2> $O/stream_mem.err
      timeout -k 10 600 python -u tools/stream_mem_probe.py --torch-pool >> $O/stream_mem.jsonl 2>> $O/stream_mem.err; cat $O/stream_mem.jsonl ;;
    c4fetch)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv \
          -d $O/c4fetch$SUF/p_$c -o pass -- python3 $R/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline \
          > $O/c4fetch_$c$SUF.log 2>&1)
      done
      PROF_RECORDS=1 PROF_LEN=6103244480 python3 tools/pmc_summary.py $O/c4fetch$SUF > $O/c4fetch$SUF.txt 2>&1 || true
      grep -E "==|FETCH|WRITE" $O/c4fetch$SUF.txt | head -40 ;;
    ab=*)
      L=${st#ab=}; bash tools/gpu_lib_ab.sh $T ${L%,*} ${L#*,} ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
  for kv in ${ENVS//,/ }; do unset "${kv%%=*}"; done
done
echo "== done $(date +%T)"
