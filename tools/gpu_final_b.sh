#!/bin/bash
# End-of-session evidence, part B: the c4 and c5 one-GPU lines, the c3 PMC passes (tools/pmc.sh)
# and the 2-rank gloo rehearsal of the N > 1 line (tools/gpu_nrank_rehearsal.sh).  First failure
# ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-fin}
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline > $OUT/bench_c4_$TAG.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c5_$TAG.log 2>&1 || exit $?
for c in c4 c5; do tail -1 $OUT/bench_${c}_$TAG.log | cut -c1-160; done
CFG=c3 STEPS=5 bash tools/pmc.sh $TAG || exit $?
NS=2 TAG=$TAG bash tools/gpu_nrank_rehearsal.sh || exit $?
