# Experiment: do two frames on two streams overlap usefully? (c2, fp64)
import sys, time, numpy as np, torch
sys.path.insert(0, '/root/repo')
from bench import synthetic_frames
from opticalflow3d_dev_amd import _lib, make_taps, radii
nt, nz, ny, nx, s, t, w = 13, 64, 256, 256, 2, 2, 5
rd, rs, rt, rw = radii(s, t, w)
dev = torch.device('cuda', 0)
fr = synthetic_frames(nt, nz, ny, nx, 1)
d_in = torch.from_numpy(fr.view(np.int16)).to(dev)
vox = nz * ny * nx
for nstreams in (1, 2, 3):
    plans = [_lib.Plan(3, nz, ny, nx, make_taps(s, t, w)) for _ in range(nstreams)]
    outs = [[torch.empty(vox, dtype=torch.float64, device=dev) for _ in range(3)] + [torch.empty(vox, dtype=torch.float32, device=dev)] for _ in range(nstreams)]
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    ptrs = [d_in[i].data_ptr() for i in range(nt)]
    def run(k):
        i = k % nstreams
        plans[i].execute(ptrs, _lib.OF3D_U16, 0, 0, nz, *[o.data_ptr() for o in outs[i]], streams[i].cuda_stream)
    for k in range(6): run(k)
    torch.cuda.synchronize()
    K = 60
    t0 = time.perf_counter()
    for k in range(K): run(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(nstreams, 'streams: ms/frame', round(dt / K * 1e3, 4))
    for p in plans: p.close()
