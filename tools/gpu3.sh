set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
CFGS="c2 c3" bash tools/ab.sh def: occ2pd8:OF3D_LIB=$PWD/tools/variants/occ2pd8.so pd2:OF3D_LIB=$PWD/tools/variants/pd2.so || exit $?
