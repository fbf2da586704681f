set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k5r.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k5r.log; [ $rc -eq 0 ] || exit $rc
OF3D_K5C_R=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k5r4.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k5r4.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh def: r4:OF3D_K5C_R=4 nyb2:OF3D_K34_NYBX=2 nyb4:OF3D_K34_NYBX=4 || exit $?
