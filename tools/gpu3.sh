set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k2c.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k2c.log; [ $rc -eq 0 ] || exit $rc
OF3D_K2C=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_nok2c.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_nok2c.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3 c4" STEPS=10 bash tools/ab.sh nok2c:OF3D_K2C=0 k2c: || exit $?
