#!/bin/bash
# Round-4 GPU pass: the given pytest files, then bench lines (c3 single GPU with the
# single-window number; c4 / c5 on one GPU with their parity samples), then the N > 1 line
# rehearsed with gloo ranks sharing the one GPU (default config: c4 z-slabs).
# STEPS: TESTS (pytest args, "" = skip), BENCH ("c3 c4 c5" subset), NS (gloo rank counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest_$TAG.log | head -30; exit $rc; }
fi
for c in ${BENCH:-}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > $OUT/bench_${c}_$TAG.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -c 400 $OUT/bench_${c}_$TAG.log; echo; [ $rc -eq 0 ] || exit $rc
done
export OF3D_BENCH_BACKEND=gloo
for n in ${NS:-}; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29540 + n)) bench.py --gpus $n --steps ${NSTEPS:-5} --warmup 2 ${N_ARGS:-} > $OUT/bench_n${n}_gloo_$TAG.log 2>&1
  rc=$?; echo "gloo n=$n rc=$rc"; [ $rc -eq 0 ] || { tail -30 $OUT/bench_n${n}_gloo_$TAG.log; exit $rc; }
  grep '^{"metric"' $OUT/bench_n${n}_gloo_$TAG.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('N=%d %s value %.1f ms/step %.3f parity %s' % (d['n_gpus'], d['config']['parallelism'], d['value'], d['ms_per_step'], (d.get('parity_sample') or {}).get('ok')))
for k in ('split','replicas','row_slabs'):
    print('  ', k, d.get(k))
"
done
