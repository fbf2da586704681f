# Bench lines for every config (c2 with the CPU baseline); logs under gpurun_out/.
set -u
cd $GRAFT_REPO_ROOT; OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-r01s2}
timeout -k 10 300 python bench.py > $OUT/bench_c2_$TAG.log 2>&1 || exit $?
tail -1 $OUT/bench_c2_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --precision fp32 --no-cpu-baseline > $OUT/bench_c2_fp32_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $OUT/bench_c3_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_$TAG.log 2>&1 || exit $?
for f in $OUT/bench_c*_$TAG.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
