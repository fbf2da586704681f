# Full evidence pass: parity tests, smoke, PMC summaries (c2, c3), bench lines, rocprofv3 kernel stats.
set -u
cd $GRAFT_REPO_ROOT; OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r01s2}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -2 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit $?
for cfg in c2 c3; do
  CFG=$cfg STEPS=3 bash tools/pmc.sh $TAG > $OUT/pmc_${cfg}_$TAG.txt 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/pmc_${cfg}_$TAG $OUT/pmc_${cfg}_$TAG.json > /dev/null || exit $?
done
export TMPDIR=/tmp
for cfg in c2 c3; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_${cfg}_$TAG -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/rocprof_${cfg}_$TAG.log 2>&1) || exit $?
done
echo done
