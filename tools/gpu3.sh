set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_eig.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_eig.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh eig: || exit $?
