# GCM lane-kernel variants with the counter-window cache (TLSGPU_GCM_VARIANT 7-12).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-v32}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-7 9 10 11 12 7}; do
  TLSGPU_GCM_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_v$v.json 2> $O/bench_v$v.err
  python -c "import json; d=json.load(open('$O/bench_v$v.json')); print($v, d['value'], {k: v['ms'] for k, v in d['per_kernel'].items() if 'gcm' in k})" | tee -a $O/sweep.txt
done
