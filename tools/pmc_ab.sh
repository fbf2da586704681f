#!/bin/bash
# PMC passes for an A/B of one env knob (VAR=OF3D_K34_NW VALS="8 4"), config CFG; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-ab}; CFG=${CFG:-c3}; VAR=${VAR:-OF3D_K34_NW}; VALS=${VALS:-"8 4"}
G1="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
export TMPDIR=/tmp
cd /tmp
for v in $VALS; do
  export $VAR=$v
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}_$v/p$i" -o run \
      -- python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_${TAG}_${v}_p$i.log" 2>&1
    rc=$?; echo "$VAR=$v pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_${TAG}_$v" "$OUT/pmc_${TAG}_$v.json" > /dev/null && \
    python3 "$ROOT/tools/pmc_report.py" "$OUT/pmc_${TAG}_$v.json" 33554432 | grep -E "prod_wyx|wz_solve_c"
done
exit 0
