#!/bin/bash
# fp32 K5c with 128-plane blocks (OF3D_K5C_R=16) vs the default 64: fp32 tests on it, then c3 / c5 fp32 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
OF3D_K5C_R=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_oracle_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/k5r_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/k5r_tests.log)"; [ $rc -eq 0 ] || exit $rc
for cfg in c3 c5; do
  for r in 8 16; do
    OF3D_K5C_R=$r timeout -k 10 300 python bench.py --config $cfg --precision fp32 --steps $([ $cfg = c3 ] && echo 20 || echo 3) --warmup 2 --no-cpu-baseline > $OUT/k5r_${cfg}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$cfg r=$r rc=$rc"; tail -5 $OUT/k5r_${cfg}_$r.log; exit $rc; }
    echo "$cfg r=$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/k5r_${cfg}_$r.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/k5r_${cfg}_$r.log)"
  done
done
