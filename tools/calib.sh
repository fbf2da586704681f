#!/bin/bash
# microbenchmarks + FETCH_SIZE/WRITE_SIZE calibration for 8-B and 16-B lanes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 120 ./tools/microbench > "$OUT/microbench.log" 2>&1; rc=$?; cat "$OUT/microbench.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp; cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/calib_$c" -o run -- "$ROOT/tools/microbench" > "$OUT/calib_$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
