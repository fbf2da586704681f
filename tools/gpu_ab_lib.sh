#!/bin/bash
# A/B over library variants (tools/variants/*.so): first the fp32 and kernel-family GPU tests
# against each variant (bit-identity with the oracle / golden vectors), then one bench line per
# variant and config in $RUNS (words "cfg:precision:steps").  First failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
RUNS=${RUNS:-c3:fp32:20 c5:fp32:3}
TESTS=${TESTS:-tests/test_gpu_fp32.py tests/test_gpu_oracle_paths.py}
for lib in opticalflow3d_dev_amd/libof3d.so tools/variants/*.so; do
  v=$(basename $lib .so)
  OF3D_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/abt_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 $OUT/abt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for run in $RUNS; do
  IFS=: read cfg prec steps <<< "$run"
  for lib in opticalflow3d_dev_amd/libof3d.so tools/variants/*.so; do
    v=$(basename $lib .so)
    OF3D_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $cfg --precision $prec --steps $steps --warmup 2 --no-cpu-baseline > $OUT/ab_${v}_$cfg$prec.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v $cfg bench rc=$rc"; tail -5 $OUT/ab_${v}_$cfg$prec.log; exit $rc; }
    echo "$cfg $prec $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_$cfg$prec.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/ab_${v}_$cfg$prec.log)"
  done
done
echo done
