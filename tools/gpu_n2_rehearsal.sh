# N>1 rehearsal on one GPU: 2 ranks (gloo, sharing the GPU) for the replica and z-slab bench paths.
set -u
cd $GRAFT_REPO_ROOT; OUT=gpurun_out; mkdir -p $OUT
export OF3D_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/bench_n2_gloo.log 2>&1 || { tail -20 $OUT/bench_n2_gloo.log; exit 1; }
grep '^{"metric"' $OUT/bench_n2_gloo.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c4 --steps 3 --warmup 1 > $OUT/bench_n2_c4_gloo.log 2>&1 || { tail -20 $OUT/bench_n2_c4_gloo.log; exit 1; }
grep '^{"metric"' $OUT/bench_n2_c4_gloo.log | cut -c1-300
