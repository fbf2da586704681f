#!/bin/bash
# Same-box A/B over library arms, interleaved by round: ARMS="name=path ..." (path relative to the
# repo; OF3D_ALLOW_STALE=1 for the variants), TESTS run first against every arm whose name is in
# TEST_ARMS, then ROUNDS rounds of one bench line per config in CFGS ("cfg:steps") per arm.
# Output under gpurun_out/$TAG/.  First failure ends the script (no GPU step after a failed one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for arm in ${TEST_ARMS:-}; do
  for a in $ARMS; do
    [ "${a%%=*}" = "$arm" ] || continue
    OF3D_ALLOW_STALE=1 OF3D_LIB=$PWD/${a#*=} timeout -k 10 ${TTMO:-600} python -u -m pytest $TESTS -m gpu -x -q \
      --timeout 120 --timeout-method thread > $OUT/tests_$arm.log 2>&1
    rc=$?; echo "$arm tests rc=$rc $(tail -1 $OUT/tests_$arm.log)"
    [ $rc -eq 0 ] || { grep -E '^E ' $OUT/tests_$arm.log | head -20; exit $rc; }
  done
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for run in $CFGS; do
    cfg=${run%%:*}; steps=${run#*:}
    for a in $ARMS; do
      name=${a%%=*}
      OF3D_ALLOW_STALE=1 OF3D_LIB=$PWD/${a#*=} timeout -k 10 ${BTMO:-300} python bench.py --config $cfg --steps $steps \
        --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${cfg}_${name}_$r.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$cfg $name bench rc=$rc"; tail -5 $OUT/${cfg}_${name}_$r.log; exit $rc; }
      echo "$cfg r$r $name $(grep -o '"ms_per_step": [0-9.]*' $OUT/${cfg}_${name}_$r.log | head -1) $(grep -o '"stage_ms": {[^}]*}' $OUT/${cfg}_${name}_$r.log | head -1) $(grep -o '"vxyz": "[^"]*"' $OUT/${cfg}_${name}_$r.log | head -1)"
    done
  done
done
echo done
