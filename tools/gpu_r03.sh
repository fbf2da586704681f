#!/bin/bash
# Round-3 evidence pass: GPU tests (incl. the c3-geometry oracle crops), smoke, the default bench
# line (c3 + cpu_baseline + parity sample), a 2-rank gloo rehearsal of the N>1 line (strong split
# with the halo exchange; both ranks on the one GPU), rocprofv3 kernel stats of c3.
# Every GPU step has its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r03a}
STAGES=${STAGES:-tests,smoke,bench,n2,cfgs,prof}
has() { [[ ",$STAGES," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_$TAG.log | tail -3; [ $rc -eq 0 ] || exit $rc
fi
if has smoke; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit $?
  tail -1 $OUT/smoke_$TAG.log
fi
if has bench; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_c3_$TAG.log 2>&1 || exit $?
  tail -1 $OUT/bench_c3_$TAG.log | cut -c1-400
fi
if has n2; then
  OF3D_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > $OUT/bench_n2gloo_$TAG.log 2>&1 || exit $?
  tail -1 $OUT/bench_n2gloo_$TAG.log | cut -c1-300
fi
if has cfgs; then  # the other configs' bench lines (c2: configs[1]; c4: one GPU; c5: fp32, one GPU)
  for cfg in ${BENCH_CFGS:-c2 c4 c5}; do
    timeout -k 10 600 python bench.py --config $cfg --steps 12 --warmup 4 --no-cpu-baseline > $OUT/bench_${cfg}_$TAG.log 2>&1 || exit $?
    tail -1 $OUT/bench_${cfg}_$TAG.log | cut -c1-200
  done
fi
if has prof; then
  export TMPDIR=/tmp
  for cfg in ${PROF_CFGS:-c3}; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${cfg}_$TAG -o run \
      -- python3 $ROOT/bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-parity-sample \
      > $OUT/rocprof_${cfg}_$TAG.log 2>&1) || exit $?
  done
  find $OUT -name "run_kernel_trace.csv" -delete
  echo "rocprof done"
fi
echo done
