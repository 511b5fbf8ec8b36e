#!/bin/bash
# Config 4 (bench.py --config c4) alternating the key-table long-record kernels:
# kt_hybrid 0 (T-table + bitsliced, default) and -1 (bitsliced key-grouped).
# usage: bash tools/gpu_c4_hyb.sh <tag> <rounds> [extra env assignments for the default runs]
set -e
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
line() { python3 -c "
import json; d=json.load(open('$1'))
print('%-12s %8.2f GiB/s' % ('$2', d['value']), {k: v.get('ms') for k, v in d.get('per_op', d.get('per_kernel', {})).items()} if isinstance(d.get('per_op', d.get('per_kernel')), dict) else '')"; }
for r in $(seq 1 $R); do
  env "$@" timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/hyb_$r.json 2> $O/hyb_$r.err
  line $O/hyb_$r.json "hybrid r$r"
  TLSGPU_KT_HYBRID=-1 timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/bs_$r.json 2> $O/bs_$r.err
  line $O/bs_$r.json "bitsliced r$r"
done
