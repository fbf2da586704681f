#!/bin/bash
# N>1 rehearsal of bench.py's multi-rank line on ONE GPU (gloo, every rank on the same card):
# N = 4 and 6 ranks — at c3 (128 planes) a 6-way z split leaves 21-22 planes per rank, thinner
# than the 27-plane halo, so the strong split's exchange reaches two neighbours each way (the
# driver's 8-GPU run: 16 planes per rank).  One line per N under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export OF3D_BENCH_BACKEND=gloo
for n in ${NS:-4 6}; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29540 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $OUT/bench_n${n}_gloo_${TAG:-r03i}.log 2>&1 \
    || { tail -20 $OUT/bench_n${n}_gloo_${TAG:-r03i}.log; exit 1; }
  grep '^{"metric"' $OUT/bench_n${n}_gloo_${TAG:-r03i}.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('N=%d value %.1f ms/step %.3f' % (d['n_gpus'], d['value'], d['ms_per_step']))
for k,v in d.get('strong',{}).items():
    if isinstance(v, dict): print('  ', k, {x: v.get(x) for x in ('rank0_part','ms_per_step','compute_ms_max_rank','exchange_ms','outputs_finite_rank0','error')})
"
done
