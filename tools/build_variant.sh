# Build an alternative libtlsgpu.so for A/B runs (TLSGPU_LIB=...): object
# NAME.hip recompiled with extra flags, linked with the tree's other objects.
# usage: bash tools/build_variant.sh NAME OUT.so -DFLAG ...
# SRC=path/to/file.hip compiles that file in place of NAME.hip (an edited copy).
# A build with a measurement-only flag (TG_CHACHA_NO_IO, TG_CHACHA_ILV, TG_KT_NO_GHASH,
# TG_KT_NO_BUILD, TG_NT_IO) marks tg_version() and is refused by tlsgpu.load()
# unless TLSGPU_ALLOW_MEASUREMENT_BUILD=1 (tests/test_measurement_fence.py).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/tlslite-ng_amd/csrc
NAME=$1; OUT=$2; shift 2
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C -Wall -Wno-unused-result \
  -fvisibility=hidden "$@" -c -o $T/$NAME.o ${SRC:-$C/$NAME.hip}
OBJS=$(ls $C/obj/*.o | grep -v "/$NAME.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT $T/$NAME.o $OBJS
rm -rf $T
