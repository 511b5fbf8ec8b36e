set -e
bash tools/gpu_run.sh r5i "tests=config4 or kt_ or key_table or keysetup"
bash tools/gpu_c4_sweep_env.sh r5i 2 "TLSGPU_KT_XCD=0" "TLSGPU_LIB=$PWD/tools/ab/kth11.so" "TLSGPU_KT_XCD=-1" "TLSGPU_KT_T=8" "TLSGPU_LIB=$PWD/tools/ab/tvg4.so"
bash tools/gpu_run.sh r5i c4fetch c4fetch@TLSGPU_KT_XCD=-1 c4fetch@TLSGPU_LIB=$PWD/tools/ab/tvg4.so
