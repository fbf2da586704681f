#!/bin/bash
# Round-4 evidence, bench half: one bench line per config on one GPU (c3 the headline with its
# CPU baseline, parity sample and single-window number; c2; c4 / c5 slab lines with their parity
# samples), then rocprofv3 --kernel-trace --stats of the c3 and c5 bench commands.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04e}
for c in ${CFGS:-c3 c2 c4 c5}; do
  steps=20; [ $c = c5 ] && steps=${C5_STEPS:-20}
  timeout -k 10 420 python bench.py --config $c --steps $steps --warmup 5 > $OUT/${TAG}_${c}_bench.log 2>&1
  rc=$?; echo "bench $c rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/${TAG}_${c}_bench.log | head -1) $(grep -o '"parity_sample": {"ok": [a-z]*' $OUT/${TAG}_${c}_bench.log)"
  [ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_${c}_bench.log; exit $rc; }
done
# per-rank compute of the N > 1 z-slab splits on this one GPU (OF3D_BENCH_VRANK="r/P": rank r of a
# P-way split alone, no exchange): what the driver's 2 / 4 / 8-GPU lines run per rank
for v in ${VRANKS:-}; do
  IFS=: read c rp <<< "$v"
  OF3D_BENCH_VRANK=$rp timeout -k 10 420 python bench.py --config $c --split z --steps 20 --warmup 5 --no-cpu-baseline \
    > $OUT/${TAG}_${c}_vrank_${rp/\//of}.log 2>&1
  rc=$?; echo "vrank $c $rp rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/${TAG}_${c}_vrank_${rp/\//of}.log | head -1)"
  [ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_${c}_vrank_${rp/\//of}.log; exit $rc; }
done
export TMPDIR=/tmp
cd /tmp
for c in ${PROF_CFGS:-c3 c5}; do
  steps=20; [ $c = c5 ] && steps=10
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_$c" -o run \
    -- python3 "$ROOT/bench.py" --config $c --steps $steps --warmup 5 --no-cpu-baseline --no-parity-sample --no-single-window \
    > "$OUT/${TAG}_${c}_bench_under_rocprof.log" 2>&1
  rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/${TAG}_prof_$c" -name "run_kernel_trace.csv" -delete 2>/dev/null
done
exit 0
