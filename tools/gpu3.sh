set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_families.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fam.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_fam.log; exit $rc
