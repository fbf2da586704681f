#!/bin/bash
# A/B of the in-tree library against tools/variants/$VAR.so (an EXTRA-flag build of the same
# sources): the K34 autotune listing of each (OF3D_VERBOSE=2) and alternating c3 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_$VAR; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in base $VAR; do
    if [ $v = base ]; then unset OF3D_LIB OF3D_ALLOW_STALE; else export OF3D_LIB=$PWD/tools/variants/$VAR.so OF3D_ALLOW_STALE=1; fi
    OF3D_VERBOSE=2 timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps 20 --warmup 5 --no-cpu-baseline \
      > $OUT/${v}_$rep.log 2>&1 || { echo "$v failed"; tail -8 $OUT/${v}_$rep.log; exit 1; }
    python3 - $OUT/${v}_$rep.log $v <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {k: round(v, 4) for k, v in d["roofline"]["stage_ms"].items()}, (d.get("parity_sample") or {}).get("vxyz"))
PY
    grep "K34 tuned" $OUT/${v}_$rep.log
  done
done
