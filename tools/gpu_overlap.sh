#!/bin/bash
# Overlap-mode check: GPU tests (all), then bench lines per z chunk for c3 and c2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-ov}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for spec in "c3 0" "c3 64" "c3 32" "c3 16" "c2 0" "c2 32" "c2 16" "c2 8"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --overlap $2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/ov_${TAG}_$1_$2.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $spec rc=$rc"; tail -5 $OUT/ov_${TAG}_$1_$2.log; exit $rc; }
  python -c "import json,sys; j=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'ms/step', j['ms_per_step'], 'dom', j['roofline']['kernel'], j['roofline']['avg_launch_ms'])" $OUT/ov_${TAG}_$1_$2.log "$spec"
done
