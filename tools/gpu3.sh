set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k1c.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_k1c.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh nok1c:OF3D_K1C=0 k1c: || exit $?
BENCH_ARGS="--precision fp32" CFGS="c2" bash tools/ab.sh f32k1c: || exit $?
