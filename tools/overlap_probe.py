"""Timing probe: can an HBM-streaming kernel run beside the VALU-bound frame kernels?

The batched K0 (5 windows' temporal derivatives, ~0.56 ms at configs[2], HBM-bound) runs in line
before K12 every 5th step.  This probe times, on one GPU, one c3 output frame through the bench's
plan (K0 + K12 + K34 + K5c) alone, a device copy moving the batched K0's bytes alone (2.9 GB: 23
uint16 frames read, 5 fp64 fields written, as one read + one write stream), and the two launched
together on two streams.  If the pair takes about the frame alone, the K0 batch could hide beside
the frame's VALU-bound kernels on a second stream.  Not a product path; prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from opticalflow3d_dev_amd import _lib, make_taps, radii  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    nt, nz, ny, nx, s, t, w, _ = bench.CONFIGS["c3"]
    rt = radii(s, t, w)[2]
    nwin = 2 * rt + 1
    d_in = bench.synthetic_slab(nwin, nz, ny, nx, 0, nz, 20260206 + 3, dev)
    vox = nz * ny * nx
    outs = [torch.empty(vox, dtype=torch.float64, device=dev) for _ in range(3)] + [torch.empty(vox, dtype=torch.float32, device=dev)]
    plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=0)
    ptrs = [d_in[i].data_ptr() for i in range(nwin)]
    sa = torch.cuda.Stream(dev)
    sb = torch.cuda.Stream(dev)
    nbytes = (23 * 2 + 5 * 8) * vox // 2  # read + write streams of a copy: ~2.9 GB moved
    src = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
    dst = torch.empty_like(src)

    def frame():
        with torch.cuda.stream(sa):
            plan.execute(ptrs, _lib.OF3D_U16, 0, 0, nz, *[o.data_ptr() for o in outs], sa.cuda_stream)

    def copy():
        with torch.cuda.stream(sb):
            dst.copy_(src)

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps * 1e3

    t_frame = timeit(frame)
    t_copy = timeit(copy)
    t_both = timeit(lambda: (frame(), copy()))
    plan.close()
    print(json.dumps({"probe": "frame + concurrent HBM copy", "frame_ms": round(t_frame, 4), "copy_ms": round(t_copy, 4),
                      "copy_GBs": round(2 * nbytes / t_copy / 1e6, 1), "both_two_streams_ms": round(t_both, 4),
                      "sum_ms": round(t_frame + t_copy, 4), "hidden_fraction_of_copy": round((t_frame + t_copy - t_both) / t_copy, 3),
                      "env_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}))


if __name__ == "__main__":
    main()
