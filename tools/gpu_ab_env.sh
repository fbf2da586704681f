#!/bin/bash
# A/B over environment settings: one bench line per spec (specs separated by ';', each a list of
# VAR=value words, "-" for none); CFG config; prints ms/step, stage times and the K34 pick.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-ab}; CFG=${CFG:-c3}; STEPS=${STEPS:-20}
IFS=';' read -ra SPECS <<< "${SPECS:--}"
i=0
for spec in "${SPECS[@]}"; do
  i=$((i+1))
  env_args=(); [ "$spec" != "-" ] && read -ra env_args <<< "$spec"
  env "${env_args[@]}" OF3D_VERBOSE=1 timeout -k 10 200 python bench.py --config $CFG --steps $STEPS --warmup 5 --no-cpu-baseline > $OUT/ab_${TAG}_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$spec] bench rc=$rc"; tail -5 $OUT/ab_${TAG}_$i.log; exit $rc; }
  python - "$OUT/ab_${TAG}_$i.log" "$spec" <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
k = [l for l in lines if l.startswith("of3d: K34")]
j = [json.loads(l) for l in lines if l.startswith("{")][-1]
print("[%s]" % sys.argv[2], "ms/step", j["ms_per_step"], "stages", j["roofline"]["stage_ms"], "|", k[-1][6:] if k else "")
PY
done
