"""configs[3] and configs[4] at their full sizes, through the plans bench.py times, against the
oracle (oracle/cpu_ref.py, pinned to the reference's calc_flow3D, calc_flow.py:175-360).

  * c4 = configs[3]: 13 x 256 x 1024 x 1024, xyzSig 2, tSig 2, wSig 5, fp64 — the whole volume
    on one GPU (the driver's t1 / replica line) in the bench's series mode (K0 batching: the
    batched K0 pass, then a window whose dt0 comes from its slot);
  * c5 = configs[4]: 13 x 512 x 2048 x 2048, fp32 — the whole volume on one GPU (~250 GB
    resident: the one-GPU line bench --config c5 runs);
  * one z-slab rank of each split the driver's N > 1 lines time: rank 1 of the 4-way c4 split
    (N = 4) and rank 3 of the 8-way c5 split (N = 8) — the rank's own planes plus the rd + rw
    halo, as bench.SlabBench builds them (tools/gpu_vrank.sh), checked at both of its cuts.

Inputs are bench.synthetic_slab's (values are a function of the global voxel and the frame's
seed), so the oracle's input box of any crop is regenerated, never copied off the device whole.

Crops sit on the seams of the kernels' decompositions at these sizes: K5c's 64-plane z chunks
(planes 64, 128, 192, ...), K12's 256-plane march boundary (c5: plane 256; c4 marches the whole
256 planes at once), K34's column blocks (x ~ 344 / 688 at nx 1024, ~ 512 / 1024 / 1536 at
nx 2048; row chunks do not occur at these sizes: one chunk per column), and the volume
corners / x edges (global clamping).  An output voxel farther than rd + rw from every face
where the crop cuts the volume is exact (tests/test_gpu_bench_geometry.py), so the crop's
input box is the crop plus rd + rw = 21 voxels, clipped into the volume.

Tolerances: fp64 vx, vy, vz bitwise and rel within 1e-6 lambda_max; fp32 within
1e-4 max|v| of the fp64 oracle (bench.parity_check, the checker of every bench line).
"""
import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIG = (2, 2, 5)  # configs[3] / [4]: sigmas as configs[1]


def _free():
    import torch

    from opticalflow3d_dev_amd import _lib

    gc.collect()
    _lib.cache_clear()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _slab(dims, fp32, seed, vrank=None, k0_batch=5, pipeline=True):
    import torch

    import bench

    _free()
    return bench.SlabBench(dims, SIG, 0, 0, 1, torch.device("cuda", 0), fp32=fp32, seed=seed, vrank=vrank,
                           pipeline=pipeline, k0_batch=k0_batch)


def _check(sb, box, fp32):
    """bench.parity_check of one output box of the slab's last computed window: the outputs of
    the rank's own planes vs the oracle of the regenerated input box."""
    import bench

    nz, ny, nx = sb.dims
    z0, z1, y0, y1, x0, x1 = box
    assert sb.a0 <= z0 < z1 <= sb.a1, (box, sb.a0, sb.a1)
    got = [o[:sb.n_out].view(sb.a1 - sb.a0, ny, nx)[z0 - sb.a0:z1 - sb.a0, y0:y1, x0:x1].cpu().numpy()
           for o in sb.outs + [sb.rel]]
    h = sb.rd + sb.rw
    lo = [max(a - h, 0) for a in (z0, y0, x0)]
    hi = [min(b + h, n) for b, n in zip((z1, y1, x1), (nz, ny, nx))]
    sub = np.stack([bench.synthetic_slab(1, nz, ny, nx, lo[0], hi[0], sb.seed + sl, sb.dev, rows=(lo[1], hi[1]))[0]
                    [:, :, lo[2]:hi[2]].cpu().numpy().view(np.uint16) for sl in sb.last_window])
    r = bench.parity_check(sub, lo, box, got, *SIG, fp32=fp32)
    assert r["ok"], (box, r)
    return r


def _run_steps(sb, n):
    import torch

    for _ in range(n):
        sb.step()
    torch.cuda.synchronize(sb.dev)
    assert sb.finite()


C4 = (256, 1024, 1024)
C4_CROPS = [
    (56, 72, 500, 516, 336, 352),       # K5c z chunk 64 x K34 column-block seam (x ~ 344)
    (120, 136, 40, 56, 680, 696),       # z chunk 128 x the next column seam (x ~ 688)
    (184, 200, 1000, 1016, 1008, 1024),  # z chunk 192, far x edge
    (0, 16, 0, 16, 0, 16),              # corner at the origin
    (240, 256, 1008, 1024, 0, 24),      # far z / y corner, x = 0 edge
]


def test_c4_full_volume_bench_plan_vs_oracle():
    """configs[3] as one volume on one GPU through bench.SlabBench (the plan and the series mode
    of the bench's c4 line and of the N > 1 line's replicas): two steps — the first runs the
    batched K0 for five windows, the second takes its dt0 from a slot — then oracle crops."""
    sb = _slab(C4, fp32=False, seed=20260206 + 4)
    try:
        _run_steps(sb, 2)
        ks = sb.plan.kernels()
        assert {"k_tderiv_multi", "k_grad_xyz_c", "k_wz_solve_c"} <= set(ks), ks
        assert any(k.startswith("k_prod_wyx") for k in ks), ks
        for box in C4_CROPS:
            _check(sb, box, fp32=False)
    finally:
        sb.close()
        del sb
        _free()


def test_c4_zslab_rank1_of4_vs_oracle():
    """Rank 1 of the 4-way z split of configs[3] (planes 64..128 plus the 27-plane halo each
    side, the N = 4 line's interior rank): crops at both of its cuts and at the volume edges."""
    sb = _slab(C4, fp32=False, seed=20260206 + 50, vrank=(1, 4))
    try:
        assert (sb.a0, sb.a1) == (64, 128)
        _run_steps(sb, 2)
        for box in ((64, 80, 500, 516, 336, 352), (112, 128, 40, 56, 680, 696), (64, 80, 0, 16, 1000, 1024),
                    (112, 128, 1008, 1024, 0, 16)):
            _check(sb, box, fp32=False)
    finally:
        sb.close()
        del sb
        _free()


C5 = (512, 2048, 2048)


def test_c5_full_volume_fp32_vs_oracle():
    """configs[4] (fp32 path) as one volume on one GPU (~250 GB resident; the plan bench --config
    c5 times): K12's two 256-plane marches, K5c's 64-plane chunks, the packed K34's column
    blocks at nx 2048; a plain series (one K0 per window: the ring of 14 frames fits beside the
    workspace), two windows."""
    sb = _slab(C5, fp32=True, seed=20260206 + 5, k0_batch=0, pipeline=False)
    try:
        _run_steps(sb, 2)
        ks = sb.plan.kernels()
        assert {"k_grad_xyz_c", "k_wz_solve_c"} <= set(ks), ks
        assert any(k.startswith("k_prod_wyx") for k in ks), ks
        for box in ((248, 264, 1016, 1032, 1016, 1032),  # K12 march seam (plane 256), x ~ 1024
                    (56, 72, 200, 216, 504, 520),          # K5c chunk 64, x ~ 512
                    (440, 456, 1800, 1816, 1528, 1544),    # K5c chunk 448, x ~ 1536
                    (0, 16, 0, 16, 0, 16),
                    (496, 512, 2032, 2048, 2024, 2048)):
            _check(sb, box, fp32=True)
    finally:
        sb.close()
        del sb
        _free()


def test_c5_zslab_rank3_of8_fp32_vs_oracle():
    """Rank 3 of the 8-way z split of configs[4] (planes 192..256 plus the halo: the N = 8 line's
    interior rank), fp32, the bench's K0 batching: crops at both cuts."""
    sb = _slab(C5, fp32=True, seed=20260206 + 50, vrank=(3, 8))
    try:
        assert (sb.a0, sb.a1) == (192, 256)
        _run_steps(sb, 2)
        for box in ((192, 208, 1016, 1032, 1016, 1032), (240, 256, 100, 116, 2030, 2048),
                    (192, 208, 2032, 2048, 0, 16)):
            _check(sb, box, fp32=True)
    finally:
        sb.close()
        del sb
        _free()
