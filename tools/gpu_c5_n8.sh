#!/bin/bash
# Rehearsal of the driver's N = 8 line (configs[4], c5: 2048^2 x 512 fp32) on ONE GPU, phase by
# phase as bench.py --gpus 8 runs them on every rank: the replica (the whole volume: t1 and the
# one-GPU frame), the z-slab rank (rank 3 of 8, the busiest interior rank) and the row-slab rank,
# each with its device-memory high-water mark ("memory" / device_used_GB in the line) and wall
# time.  Logs under gpurun_out/c5n8_<TAG>_*.log; a summary line per phase.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-r05}
S=${STEPS:-20}; W=${WARMUP:-5}
run() {  # name, env, args
  local name=$1; shift; local envs=$1; shift
  local t0=$SECONDS
  env $envs OF3D_VERBOSE=1 timeout -k 10 ${TMO:-400} python bench.py --config c5 --steps $S --warmup $W --no-cpu-baseline "$@" \
    > $OUT/c5n8_${TAG}_$name.log 2>&1 || { tail -5 $OUT/c5n8_${TAG}_$name.log; exit 1; }
  echo "$name wall_s=$((SECONDS - t0)) $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5n8_${TAG}_$name.log | head -1) $(grep -o '"memory": {[^}]*}' $OUT/c5n8_${TAG}_$name.log) $(grep -o '"stage_ms": {[^}]*}' $OUT/c5n8_${TAG}_$name.log | head -1) $(grep -o '"vxyz": "[^"]*"' $OUT/c5n8_${TAG}_$name.log | head -1)"
}
run replica ""
run zslab_r3of8 "OF3D_BENCH_VRANK=3/8" --split z
run rows_r3of8 "OF3D_BENCH_VRANK=3/8" --split y
