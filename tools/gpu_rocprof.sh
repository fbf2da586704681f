#!/bin/bash
# rocprofv3 kernel-trace statistics of bench lines (per-kernel average duration: the figures the
# bench's roofline events must agree with), one pass per config in CFGS; summaries under
# gpurun_out/prof_<cfg>_<TAG>/.  First failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; TAG=${TAG:-r05}
export TMPDIR=/tmp
for cfg in ${CFGS:-c3}; do
  (cd /tmp && timeout -k 10 ${TMO:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${cfg}_$TAG" -o run \
    -- python3 "$ROOT/bench.py" --config $cfg --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$OUT/rocprof_${cfg}_$TAG.log" 2>&1) || exit $?
  find "$OUT/prof_${cfg}_$TAG" -name "run_kernel_trace.csv" -delete 2>/dev/null
  echo "$cfg $(tail -1 "$OUT/rocprof_${cfg}_$TAG.log" | grep -o '"ms_per_step": [0-9.]*')"
done
