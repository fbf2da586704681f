#!/bin/bash
# K12 z-march length (OF3D_K12_ZC) on the large configs: c5 fp32 and c4 fp64, one bench line each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
OF3D_K12_ZC=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_families.py tests/test_gpu_fp32.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/k12zc_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/k12zc_tests.log)"; [ $rc -eq 0 ] || exit $rc
for spec in c5:0 c5:128 c5:256 c4:0 c4:128; do
  IFS=: read cfg zc <<< "$spec"
  OF3D_K12_ZC=$zc timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline > $OUT/k12zc_${cfg}_$zc.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -5 $OUT/k12zc_${cfg}_$zc.log; exit $rc; }
  echo "$cfg zc=$zc $(grep -o '"ms_per_step": [0-9.]*' $OUT/k12zc_${cfg}_$zc.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/k12zc_${cfg}_$zc.log)"
done
