# N = 2 rehearsal of bench.py's multi-GPU path on one MI355X: two ranks over
# gloo (TLSGPU_DIST_BACKEND=gloo; RCCL needs one GPU per rank), 65 536 records
# per rank.  usage: bash tools/gpu_n2_rehearsal.sh <tag>
set -e
O=gpurun_out/$1; mkdir -p $O
TLSGPU_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --records 65536 \
  --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err
echo done
