#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout/abort ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
STEPS=${STEPS:-20}
CFG=${CFG:-c2}

ok_or_stop() {  # $1 = rc; test failures (1) continue, anything else stops
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP rc=$1"; exit "$1"; fi
}

timeout -k 10 600 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu_$TAG.log"; ok_or_stop $rc

timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 300 python bench.py --config "$CFG" --steps "$STEPS" --warmup 5 > "$OUT/bench_${CFG}_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_${CFG}_$TAG.log"; [ $rc -eq 0 ] || exit $rc

export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${CFG}_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --config "$CFG" --steps "$STEPS" --warmup 5 --no-cpu-baseline > "$OUT/rocprof_${CFG}_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/rocprof_${CFG}_$TAG.log"
find "$OUT/prof_${CFG}_$TAG" -name "*stats*" | head
exit $rc
