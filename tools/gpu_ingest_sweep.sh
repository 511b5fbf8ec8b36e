set -e
mkdir -p gpurun_out/${TAG:-x5}
[ -n "$NOTEST" ] || bash tools/gpu_run.sh x5 "tests=ingest"
for cfg in ${CFGS:-"2048 4 512" "4096 4 512" "4096 3 1024" "2048 6 1024" "2048 4 512"}; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --config ingest --ingest-mib 2048 --ingest-batch $1 --ingest-slots $2 --ingest-read-mib $3 > gpurun_out/${TAG:-x5}/ingest_$1_$2_$3.json 2> gpurun_out/${TAG:-x5}/ingest_$1_$2_$3.err
  python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG:-x5}/ingest_$1_$2_$3.json'));print('$cfg', {a:(v['write_GiBps'],v['read_GiBps'],v['read_feed_first_GiBps'],v['verified']) for a,v in d['per_alg'].items()}, d['host_copy_to_pinned_GiBps'])"
done
