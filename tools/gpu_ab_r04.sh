#!/bin/bash
# Round-4 A/B: GPU tests on the tree's library, then bench lines alternating the tree's library
# and tools/variants/*.so (ROUNDS rounds, configs in RUNS as "cfg:precision:steps").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-ab}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/abt_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/abt_$TAG.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/abt_$TAG.log | head; exit $rc; }
fi
# arms: every library (the tree's + tools/variants/*.so), then ENV_ARMS ("name:ENV=V,ENV2=V2" on
# the tree's library)
arms=()
for lib in opticalflow3d_dev_amd/libof3d.so tools/variants/*.so; do
  [ -f "$lib" ] && arms+=("$(basename $lib .so)|$lib|")
done
for a in ${ENV_ARMS:-}; do arms+=("${a%%:*}|opticalflow3d_dev_amd/libof3d.so|${a#*:}"); done
for r in $(seq 1 ${ROUNDS:-2}); do
  for run in ${RUNS:-c3:fp64:20}; do
    IFS=: read cfg prec steps <<< "$run"
    for arm in "${arms[@]}"; do
      IFS='|' read v lib envs <<< "$arm"
      log=$OUT/ab_${TAG}_${v}_$cfg${prec}_$r.log
      ( IFS=','; for e in $envs; do export "$e"; done; unset IFS
        OF3D_ALLOW_STALE=1 OF3D_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $cfg --precision $prec --steps $steps --warmup 3 --no-cpu-baseline --no-parity-sample --no-single-window > $log 2>&1 )
      rc=$?; [ $rc -eq 0 ] || { echo "$v $cfg bench rc=$rc"; tail -5 $log; exit $rc; }
      echo "$r $cfg $prec $v $(grep -o '"ms_per_step": [0-9.]*' $log) $(grep -o '"stage_ms": {[^}]*}' $log)"
    done
  done
done
