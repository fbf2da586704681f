#!/bin/bash
# Round-3 session-2 A/B pass: GPU tests (TESTS, default the whole -m gpu suite), then c3 bench
# lines per variant (VARIANTS="name:ENV=1,ENV2=0 ..."), REPS rounds alternating, with the K34
# autotune listing every candidate (OF3D_VERBOSE=2); C5=1 adds one c5 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03g}; mkdir -p $OUT
python -c "from opticalflow3d_dev_amd import _lib; print(_lib.build_info())" > $OUT/build_info.txt 2>&1 || exit $?
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-default:}; do
    name=${v%%:*}; envs=${v#*:}
    env $(echo $envs | tr ',' ' ') OF3D_VERBOSE=2 timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps 20 --warmup 5 \
      --no-cpu-baseline > $OUT/${name}_${CFG:-c3}_$rep.log 2>&1 || { tail -20 $OUT/${name}_${CFG:-c3}_$rep.log; exit 1; }
    python3 - $OUT/${name}_${CFG:-c3}_$rep.log $name <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "stages", {k: round(v, 4) for k, v in d["roofline"]["stage_ms"].items()}, "parity", d.get("parity_sample", {}).get("vxyz"))
PY
    grep "K34 tuned" $OUT/${name}_${CFG:-c3}_$rep.log | head -2
  done
done
if [ -n "${C5:-}" ]; then
  OF3D_VERBOSE=2 timeout -k 10 400 python bench.py --config c5 --steps 8 --warmup 2 --no-cpu-baseline \
    > $OUT/c5.log 2>&1 || { tail -20 $OUT/c5.log; exit 1; }
  grep '^{' $OUT/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 ms/step', d['ms_per_step'], d['roofline']['stage_ms'])"
fi
