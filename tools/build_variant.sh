#!/bin/bash
# Build libhvk.so from the csrc/ of a git revision (or the working tree with REV=WT plus
# optional extra CXXFLAGS) into abl/<name>.so for A/B runs (tools/gpu_ab_lib.sh).
#   tools/build_variant.sh HEAD base            # committed kernels
#   EXTRA="-DHVK_X=1" tools/build_variant.sh WT probe
#   FROM_REV="HEAD:layernorm.hip" tools/build_variant.sh WT lnold   # one file from a revision
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TT=$(mktemp -d /tmp/hvkvar.XXXX)
T=$TT/pkg/csrc  # csrc/../../include/hvk.h as in the tree
mkdir -p "$T" "$TT/include"
if [ "$REV" = WT ]; then cp -r "$ROOT/hierarchical-vision_amd/csrc/." "$T/"; rm -rf "$T/build"; cp "$ROOT/include/hvk.h" "$TT/include/"
else git -C "$ROOT" archive "$REV" hierarchical-vision_amd/csrc | tar -x -C "$T" --strip-components=2
  git -C "$ROOT" show "$REV:include/hvk.h" > "$TT/include/hvk.h"; fi
for fr in $FROM_REV; do
  git -C "$ROOT" show "${fr%%:*}:hierarchical-vision_amd/csrc/${fr#*:}" > "$T/${fr#*:}"
done
mkdir -p "$ROOT/abl"
make -s -C "$T" -j8 OUT="$ROOT/abl/$NAME.so" CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $EXTRA"
rm -rf "$TT"
echo "built abl/$NAME.so"
