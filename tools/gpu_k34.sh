#!/bin/bash
# K34 geometry A/B: GPU parity tests, then c3/c2 bench lines per forced block shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-k34}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for cfg in c3 c2; do
  for nw in auto 8 4 2; do
    if [ $nw = auto ]; then unset OF3D_K34_NW; else export OF3D_K34_NW=$nw; fi
    OF3D_VERBOSE=1 timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_${TAG}_${cfg}_$nw.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $OUT/b_${TAG}_${cfg}_$nw.log; exit $rc; }
    python - "$OUT/b_${TAG}_${cfg}_$nw.log" "$cfg" "$nw" <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
k = [l for l in lines if l.startswith("of3d: K34")]
j = [json.loads(l) for l in lines if l.startswith("{")][-1]
print(sys.argv[2], "nw", sys.argv[3], "ms/step", j["ms_per_step"], "stages", j["roofline"]["stage_ms"], "|", k[-1] if k else "")
PY
  done
done
