set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export OF3D_VERBOSE=1
CFGS="c2 c3" bash tools/ab.sh tuned: nw3:OF3D_K34_NW=3 || exit $?
grep -h "K34 tuned" gpurun_out/ab_c*.log
