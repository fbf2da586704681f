#!/bin/bash
# A/B bench runs: each argument is one arm "name:ENV=V,ENV2=V2" (lib variants via OF3D_LIB=tools/variants/x.so).
# CFGS (default c2) x arms; one line per run with ms/step and stage ms.  Stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for cfg in ${CFGS:-c2}; do
  for arm in "$@"; do
    name=${arm%%:*}; envs=${arm#*:}
    [ "$envs" = "$arm" ] && envs=""
    ( IFS=','; for e in $envs; do export "$e"; done; unset IFS
      timeout -k 10 ${TMO:-150} python bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/ab_${cfg}_$name.log 2>&1 )
    rc=$?; echo "$cfg $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${cfg}_$name.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/ab_${cfg}_$name.log)"
    [ $rc -eq 0 ] || { tail -5 $OUT/ab_${cfg}_$name.log; exit $rc; }
  done
done
