#!/bin/bash
# K0 batching over 5 windows (default) vs 4: GPU tests of this tree, then alternating bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/k0m5; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  for cfg in c3 c5; do
    for m in 5 4; do
      st=20
      OF3D_BENCH_K0_BATCH=$m timeout -k 10 400 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline \
        > $OUT/m${m}_${cfg}_$rep.log 2>&1 || { echo "m$m $cfg failed"; tail -8 $OUT/m${m}_${cfg}_$rep.log; exit 1; }
      grep '^{' $OUT/m${m}_${cfg}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('M=$m $cfg ms/step %.4f' % d['ms_per_step'], {k: round(v,4) for k,v in d['roofline']['stage_ms'].items()}, (d.get('parity_sample') or {}).get('vxyz'))"
    done
  done
done
