set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k5c.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_k5c.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh nok5c:OF3D_K5C=0 k5c: || exit $?
BENCH_ARGS="--precision fp32" CFGS="c2" bash tools/ab.sh f32nok5c:OF3D_K5C=0 f32k5c: || exit $?
