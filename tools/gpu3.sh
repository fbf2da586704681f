set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k34.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_k34.log; [ $rc -eq 0 ] || exit $rc
export OF3D_VERBOSE=1
CFGS="c2 c3" bash tools/ab.sh base:OF3D_K34=0 k34: || exit $?
BENCH_ARGS="--precision fp32" CFGS="c2" bash tools/ab.sh f32base:OF3D_K34=0 f32k34: || exit $?
grep -h "K34 cw" gpurun_out/ab_c*.log | sort | uniq -c
