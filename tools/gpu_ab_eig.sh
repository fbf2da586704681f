#!/bin/bash
# The polynomial eigenvalue (this tree) vs the acos form (tools/variants/old_eig.so, the same
# sources before the change): GPU test suite on this tree, then alternating bench lines
# c3 (fp64) and c5 (fp32) per library, REPS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-eig}; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
for rep in $(seq 1 ${REPS:-2}); do
  for run in ${RUNS:-c3:20 c5:6}; do
    IFS=: read cfg steps <<< "$run"
    for v in new old; do
      if [ $v = old ]; then export OF3D_LIB=$PWD/tools/variants/old_eig.so OF3D_ALLOW_STALE=1; else unset OF3D_LIB OF3D_ALLOW_STALE; fi
      timeout -k 10 400 python bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline \
        > $OUT/${v}_${cfg}_$rep.log 2>&1 || { echo "$v $cfg failed"; tail -8 $OUT/${v}_${cfg}_$rep.log; exit 1; }
      python3 - $OUT/${v}_${cfg}_$rep.log $v $cfg <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], sys.argv[3], "ms/step %.4f" % d["ms_per_step"], {k: round(v, 4) for k, v in d["roofline"]["stage_ms"].items()}, (d.get("parity_sample") or {}).get("rel_max_err_over_lmax"))
PY
    done
  done
done
unset OF3D_LIB OF3D_ALLOW_STALE
