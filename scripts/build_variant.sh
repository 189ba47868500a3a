#!/bin/bash
# Link an A/B variant of libgr_amd.so: SRC (a csrc file name, or a path to another version of one)
# compiled with extra flags in place of build/obj/<basename>.o, every other object as built (run the
# normal build first).  Output: lib/libgr_amd_TAG.so (git-ignored).
#   scripts/build_variant.sh TAG rq.hip -DSOME_FLAG
#   git show HEAD:.../csrc/score_topk.hip > /tmp/v/score_topk.hip; scripts/build_variant.sh head /tmp/v/score_topk.hip
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/ai-education-generative-recommendation_amd
TAG=$1; SRC=$2; shift 2
case "$SRC" in /*) PATH_SRC=$SRC ;; *) PATH_SRC=$PKG/csrc/$SRC ;; esac
BASE=$(basename "$SRC")
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$PKG/csrc" -I "$ROOT/include" "$@" \
  -x hip -c "$PATH_SRC" -o "$TMP/$BASE.o"
OBJS=$(ls "$ROOT"/build/obj/*.o | grep -v "/$BASE.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS "$TMP/$BASE.o" -o "$PKG/lib/libgr_amd_$TAG.so"
rm -rf "$TMP"
echo "$PKG/lib/libgr_amd_$TAG.so"
