#!/bin/bash
# run bench once per library variant in tools/variants/ (plus the in-tree build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for lib in opticalflow3d_dev_amd/libof3d.so tools/variants/*.so; do
  OF3D_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/ab.log 2>&1
  rc=$?; echo "$lib rc=$rc $(grep -o '"stage_ms": {[^}]*}' $OUT/ab.log)"
  [ $rc -eq 0 ] || exit $rc
done
