#!/bin/bash
# Scaling model inputs: per-rank compute of a P-way split on one GPU (bench.py OF3D_BENCH_VRANK),
# both split axes, for CFG (default c4).  One line per run: P, axis, ms per step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c4}
timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $OUT/vr_${CFG}_1.log 2>&1 || exit $?
echo "$CFG P=1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/vr_${CFG}_1.log)"
for P in 2 4 8; do
  r=$(( P > 2 ? P / 2 - 1 : 0 ))
  for ax in z y; do
    OF3D_BENCH_VRANK="$r/$P" timeout -k 10 300 python bench.py --config $CFG --split $ax --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $OUT/vr_${CFG}_${P}_$ax.log 2>&1 || exit $?
    echo "$CFG P=$P rank=$r split=$ax $(grep -o '"ms_per_step": [0-9.]*' $OUT/vr_${CFG}_${P}_$ax.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/vr_${CFG}_${P}_$ax.log)"
  done
done
