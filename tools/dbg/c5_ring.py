"""Diagnostic: c5 ring slots vs their regeneration (which input frames differ)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
import bench
import test_gpu_full_configs as T

dims = tuple(int(v) for v in os.environ.get("DIMS", "512,2048,2048").split(","))
kb = int(os.environ.get("KB", "0"))
sb = T._slab(dims, fp32=True, seed=20260206 + 5, k0_batch=kb, pipeline=kb > 0)
torch.cuda.synchronize()
nz, ny, nx = dims
for sl in range(len(sb.ring)):
    bad = []
    for (z0, z1) in ((0, 4), (nz // 2, nz // 2 + 4), (nz - 4, nz)):
        want = bench.synthetic_slab(1, nz, ny, nx, z0, z1, sb.seed + sl, sb.dev)[0]
        have = sb.ring[sl][z0:z1]
        d = (want != have)
        if bool(d.any()):
            bad.append((z0, int(d.sum())))
    print("slot", sl, "ok" if not bad else bad, flush=True)
