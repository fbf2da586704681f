#!/bin/bash
# Tests on the in-tree library (TESTS), then the in-tree library vs tools/variants/$VAR.so
# (an EXTRA-flag build of the same sources) on the configs in CFGS, REPS rounds alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_$VAR; mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-c3}; do
    for v in base $VAR; do
      if [ $v = base ]; then unset OF3D_LIB OF3D_ALLOW_STALE; else export OF3D_LIB=$PWD/tools/variants/$VAR.so OF3D_ALLOW_STALE=1; fi
      st=20; [ $cfg = c5 ] && st=6
      timeout -k 10 400 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline \
        > $OUT/${v}_${cfg}_$rep.log 2>&1 || { echo "$v $cfg failed"; tail -8 $OUT/${v}_${cfg}_$rep.log; exit 1; }
      python3 - $OUT/${v}_${cfg}_$rep.log $v $cfg <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], sys.argv[3], "ms/step %.4f" % d["ms_per_step"], {k: round(v, 4) for k, v in d["roofline"]["stage_ms"].items()}, (d.get("parity_sample") or {}).get("vxyz"))
PY
    done
  done
done
unset OF3D_LIB OF3D_ALLOW_STALE
