set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_pair.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh pair: || exit $?
