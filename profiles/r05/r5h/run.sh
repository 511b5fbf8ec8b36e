set -e
O=gpurun_out/r5h; mkdir -p $O
for r in 1 2 3; do
  for t in -1 1; do
    TLSGPU_BS_TOUCH=$t timeout -k 10 120 python -u tools/aes_time.py | sed "s/^/touch=$t /" | tee -a $O/aes_touch.txt
  done
done
bash tools/gpu_c4_sweep_env.sh r5h 2 "TLSGPU_BS_TOUCH=-1" "TLSGPU_BS_TOUCH=1"
