#!/bin/bash
# Same-box A/B of configs[4] (c5, fp32, one GPU, 20 steps, whole K0 batches): the round-3 final tree
# (src 0eb4f496, staged under tools/variants/r03tree with its own bench.py and library) against the
# current tree, in the order HEAD, r03, HEAD, r03 (drift shows as a difference between the pairs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-c5ab}
R03=tools/variants/r03tree
for i in 1 2; do
  for arm in head r03; do
    if [ $arm = head ]; then B=bench.py; else B=$R03/bench.py; fi
    timeout -k 10 ${BTMO:-240} python $B --config c5 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline > $OUT/${TAG}_${arm}_$i.log 2>&1; rc=$?
    echo "$arm $i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/${TAG}_${arm}_$i.log | head -1) $(grep -o '"stage_ms": {[^}]*}' $OUT/${TAG}_${arm}_$i.log | head -1) $(grep -o '"src_hash": "[^"]*"' $OUT/${TAG}_${arm}_$i.log | head -1)"
    [ $rc -eq 0 ] || { tail -5 $OUT/${TAG}_${arm}_$i.log; exit $rc; }
  done
done
