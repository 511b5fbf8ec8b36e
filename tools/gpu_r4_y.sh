#!/bin/bash
# Same-box headline A/B: the final tree vs the library of the f1 full check
# (commit 3a17c27), alternating, two rounds each.
set -e
O=gpurun_out/r4y; mkdir -p $O
for r in 1 2; do
  for lib in "" tools/ab/f1.so; do
    TLSGPU_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b.json 2> $O/b.err
    python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('%-16s %8.2f' % ('${lib:-tree}', d['value']), {k: v['ms'] for k, v in d['per_kernel'].items()})" | tee -a $O/ab.txt
  done
done
