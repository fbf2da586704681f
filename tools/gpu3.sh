set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_gpu_process_flow.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k0c.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k0c.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh nok0c:OF3D_K0C=0 k0c: nyc16:OF3D_K1C_NYC=16 nyc64:OF3D_K1C_NYC=64 cw64:OF3D_K1C_CW=64 cw256:OF3D_K1C_CW=256 || exit $?
