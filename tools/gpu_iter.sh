#!/bin/bash
# Iteration pass: a chosen set of GPU tests, then bench lines with the plan's K34 candidates listed
# (OF3D_VERBOSE=2).  TESTS (pytest paths, "" skips), CFGS (configs, "" skips).  First failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-it}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TTMO:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc $(tail -1 $OUT/pytest_$TAG.log)"; [ $rc -eq 0 ] || { grep -E '^E ' $OUT/pytest_$TAG.log | head -20; exit $rc; }
fi
for cfg in ${CFGS:-}; do
  OF3D_VERBOSE=2 timeout -k 10 ${BTMO:-300} python bench.py --config $cfg --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_${cfg}_$TAG.log 2>&1 || { tail -5 $OUT/bench_${cfg}_$TAG.log; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${cfg}_$TAG.log | head -1) $(grep -o '"stage_ms": {[^}]*}' $OUT/bench_${cfg}_$TAG.log | head -1) $(grep -o '"vxyz": "[^"]*"' $OUT/bench_${cfg}_$TAG.log | head -1)"
  grep 'K34 tuned' $OUT/bench_${cfg}_$TAG.log | head -2
done
