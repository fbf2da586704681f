#!/bin/bash
# Build an A/B variant of libof3d.so from the current sources with extra compile flags:
#   tools/build_variant.sh NAME "-DMACRO=0 ..." ['sed-expr' ...]  ->  tools/variants/NAME.so
# (a copy of csrc/ + include/ under /tmp, so the tree's own objects stay untouched; each sed
# expression is applied to the copy's of3d_dev.hpp — a source A/B without touching the tree)
set -eu
REPO=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=${2:-}; shift; shift || true
D=/tmp/of3d_variant_$NAME
rm -rf "$D"; mkdir -p "$D/opticalflow3d_dev_amd" "$REPO/tools/variants"
cp -r "$REPO/include" "$D/include"
cp -r "$REPO/opticalflow3d_dev_amd/csrc" "$D/opticalflow3d_dev_amd/csrc"
rm -rf "$D/opticalflow3d_dev_amd/csrc/build"
for e in "$@"; do sed -i -e "$e" "$D/opticalflow3d_dev_amd/csrc/of3d_dev.hpp"; done
make -C "$D/opticalflow3d_dev_amd/csrc" -j8 OUT="$REPO/tools/variants/$NAME.so" EXTRA="$FLAGS" > "$D/build.log" 2>&1 \
  || { tail -20 "$D/build.log"; exit 1; }
echo "built tools/variants/$NAME.so ($FLAGS)"
