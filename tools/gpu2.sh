set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k34.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_k34.log; [ $rc -eq 0 ] || exit $rc
CFGS="c2 c3" bash tools/ab.sh base:OF3D_K34=0 k34: nosb:OF3D_LIB=$PWD/tools/variants/nosb.so
