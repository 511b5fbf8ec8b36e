#!/bin/bash
# bench.py --config ingest REPS times (default pipeline) -> gpurun_out/<tag>/ingest_<r>.json
set -e
T=$1; REPS=${2:-2}; O=gpurun_out/$T; mkdir -p $O
for r in $(seq 1 $REPS); do
  timeout -k 10 300 python -u bench.py --config ingest $BENCH_ARGS > $O/ingest_$r.json 2> $O/ingest_$r.err
  python3 -c "import json;d=json.load(open('$O/ingest_$r.json'));print({a:(v['write_GiBps'],v['read_GiBps'],v['read_feed_first_GiBps'],v['verified']) for a,v in d['per_alg'].items()}, d['host_copy_to_pinned_GiBps'])"
done
