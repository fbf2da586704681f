#!/bin/bash
# Iteration loop on the GPU box: parity subset -> benches -> rocprof kernel stats.
# TESTS (pytest args), CFGS (bench configs), PROF (config to profile, "" = none), TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-it}; TESTS=${TESTS:-tests/test_gpu_parity.py}; CFGS=${CFGS:-c3}; PROF=${PROF:-}
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 "$OUT/pytest_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_${c}_$TAG.log" 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -1 "$OUT/bench_${c}_$TAG.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline'].get('stage_ms'))" || tail -5 "$OUT/bench_${c}_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp; cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${PROF}_$TAG" -o run \
    -- python3 "$ROOT/bench.py" --config "$PROF" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/rocprof_${PROF}_$TAG.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"
  python3 - "$OUT/prof_${PROF}_$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "anonymous" in r["Name"]:
            print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), r["Name"].split("(")[0][30:110])
PY
  exit $rc
fi
