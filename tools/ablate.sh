#!/bin/bash
# run bench once per library variant in tools/variants/*.so, for each config in $CFGS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for cfg in ${CFGS:-c2}; do
  for lib in tools/variants/*.so; do
    OF3D_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $OUT/ab.log 2>&1
    rc=$?; echo "$cfg $(basename $lib) rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/ab.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
