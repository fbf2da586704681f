#!/bin/bash
# Round-2 evidence: GPU tests, smoke, PMC (c2, c3), rocprofv3 kernel stats (c2, c3), bench lines
# (c3 headline with cpu_baseline, c2, c4 fp64, c5 fp32).  Every GPU step has its own limit; the
# first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r02}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit $?
tail -1 $OUT/smoke_$TAG.log
for cfg in c2 c3; do
  CFG=$cfg STEPS=3 bash tools/pmc.sh $TAG > $OUT/pmc_${cfg}_$TAG.txt 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/pmc_${cfg}_$TAG $OUT/pmc_${cfg}_$TAG.json --calib profiles/pmc_calibration.json > $OUT/pmc_${cfg}_$TAG.summary 2>&1 || exit $?
done
echo "pmc done"
export TMPDIR=/tmp
for cfg in c2 c3; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${cfg}_$TAG -o run \
    -- python3 $ROOT/bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rocprof_${cfg}_$TAG.log 2>&1) || exit $?
done
echo "rocprof done"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_c3_$TAG.log 2>&1 || exit $?
tail -1 $OUT/bench_c3_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 > $OUT/bench_c2_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_$TAG.log 2>&1 || exit $?
for c in c2 c4 c5; do tail -1 $OUT/bench_${c}_$TAG.log | cut -c1-200; done
# keep the summaries, drop the per-dispatch traces (gpurun copies back at most 64 MiB)
find $OUT -name "run_kernel_trace.csv" -delete; find $OUT -name "run_counter_collection.csv" -size +4M -delete
echo done
