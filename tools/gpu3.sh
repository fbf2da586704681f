set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tune.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tune.log; [ $rc -eq 0 ] || exit $rc
export OF3D_VERBOSE=1
CFGS="c2 c3 c4" bash tools/ab.sh tuned: || exit $?
BENCH_ARGS="--precision fp32" CFGS="c2" bash tools/ab.sh f32tuned: || exit $?
grep -h "K34 tuned" gpurun_out/ab_c*.log
