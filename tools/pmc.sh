#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace; one counter group per pass).
# PMC_GROUPS: ';'-separated counter groups (default below).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r01}; CFG=${CFG:-c2}; STEPS=${STEPS:-5}
DEF="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS;TCC_HIT_sum TCC_MISS_sum"
GROUPS_=${PMC_GROUPS:-$DEF}
export TMPDIR=/tmp
cd /tmp
if [ -n "${LIST:-}" ]; then timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1; echo "list rc=$?"; fi
i=0
IFS=';' read -ra GRP <<< "$GROUPS_"
for grp in "${GRP[@]}"; do
  i=$((i+1))
  # counters only for this library's kernels (torch's input-generation kernels are many and small:
  # collecting on each of them serialises minutes of launches at c5)
  timeout -k 10 ${PASS_LIMIT:-240} rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "k_(tderiv|grad|prod|wz|solve)" \
    --output-format csv -d "$OUT/pmc_${CFG}_$TAG/p$i" -o run \
    -- python3 "$ROOT/bench.py" --config "$CFG" --steps "$STEPS" --warmup 1 --no-cpu-baseline --no-parity-sample > "$OUT/pmc_${CFG}_${TAG}_p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  # the dispatch traces are large (gpurun copies back at most 64 MiB): counters stay
  find "$OUT/pmc_${CFG}_$TAG/p$i" -name "run_kernel_trace.csv" -delete 2>/dev/null
  case $rc in 0|1|2) ;; *) echo "STOP"; exit $rc;; esac
done
exit 0
