#!/bin/bash
# End-of-session check: all GPU tests, smoke, c3 (default) and c2 bench lines.  First failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-fin}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit $?
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 400 python bench.py > $OUT/bench_c3_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 5 > $OUT/bench_c2_$TAG.log 2>&1 || exit $?
for c in c3 c2; do tail -1 $OUT/bench_${c}_$TAG.log | cut -c1-200; done
