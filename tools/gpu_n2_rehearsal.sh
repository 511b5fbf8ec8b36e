# N = 2 rehearsal of bench.py's multi-GPU path on one MI355X: `bench.py --gpus 2`
# starts its two ranks itself; over gloo (TLSGPU_DIST_BACKEND=gloo: RCCL needs
# one GPU per rank) both ranks share the one device, 65 536 records per rank.
# Under the default nccl backend the same command must refuse (exit 2: fewer
# devices than ranks).   usage: bash tools/gpu_n2_rehearsal.sh <tag>
set -e
O=gpurun_out/$1; mkdir -p $O
TLSGPU_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --records 65536 \
  --no-cpu-baseline > $O/bench2_gloo.json 2> $O/bench2_gloo.err
cat $O/bench2_gloo.json
rc=0
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --records 65536 --no-cpu-baseline \
  > $O/bench2_nccl.json 2> $O/bench2_nccl.err || rc=$?
echo "nccl with one device: exit $rc"; tail -2 $O/bench2_nccl.err
[ $rc -eq 2 ]   # refused before any rank started
