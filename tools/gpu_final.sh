#!/bin/bash
# End-of-session evidence, part A: all GPU tests, smoke, the c3 (default, with the CPU baseline),
# c2 and c1 bench lines, and the rocprofv3 kernel statistics of the c3 line.  First failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-fin}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $OUT/pytest_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit $?
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 400 python bench.py > $OUT/bench_c3_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 5 > $OUT/bench_c2_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c1 > $OUT/bench_c1_$TAG.log 2>&1 || exit $?
for c in c3 c2 c1; do tail -1 $OUT/bench_${c}_$TAG.log | cut -c1-160; done
CFGS=c3 TAG=$TAG bash tools/gpu_rocprof.sh || exit $?
