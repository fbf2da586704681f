# End-to-end streaming benchmarks (tools/bench_e2e.py) for c2 and c3; logs under gpurun_out/.
set -u
cd $GRAFT_REPO_ROOT; OUT=gpurun_out; mkdir -p $OUT
for c in c2 c3; do
  mkdir -p /tmp/e2e_$c && timeout -k 10 400 python tools/bench_e2e.py --config $c --dir /tmp/e2e_$c > $OUT/e2e_${c}_r01s2.log 2>&1 || { tail -5 $OUT/e2e_${c}_r01s2.log; exit 1; }
  grep '^{' $OUT/e2e_${c}_r01s2.log | cut -c1-160
done
