#!/bin/bash
# A/B of plan-time variants by environment (same library): c3 / c2 bench lines, alternating.
# VARIANTS="A:ENV=1,ENV2=0 B:..." ; CFGS="c3 c2"; REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-c3}; do
    for v in $VARIANTS; do
      name=${v%%:*}; envs=${v#*:}
      env $(echo $envs | tr ',' ' ') OF3D_VERBOSE=1 timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 \
        --no-cpu-baseline --no-parity-sample ${BENCH_ARGS:-} > $OUT/${name}_${cfg}_$rep.log 2>&1 || exit $?
      python3 - $OUT/${name}_${cfg}_$rep.log $name $cfg <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], sys.argv[3], "ms/step %.4f" % d["ms_per_step"], "stages", {k: round(v, 4) for k, v in d["roofline"]["stage_ms"].items()})
PY
    done
  done
done
