# Build libtlsgpu.so from the sources of git revision REV (A/B baseline for
# TLSGPU_LIB), in a scratch checkout; the tree's own build is untouched.
# usage: bash tools/build_rev_lib.sh REV OUT.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; OUT=$(realpath -m "$2")
T=$(mktemp -d)
git -C "$R" archive "$REV" tlslite-ng_amd/csrc include | tar -x -C "$T"
make -s -C "$T/tlslite-ng_amd/csrc" -j8 OUT="$OUT" > /dev/null
rm -rf "$T"
