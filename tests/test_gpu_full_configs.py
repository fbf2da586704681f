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
    """configs[4] (fp32 path) as one volume on one GPU (~265 GB resident; the plan and the series
    mode bench --config c5 times): K12's two 256-plane marches, K5c's 64-plane chunks, the packed
    K34's column blocks at nx 2048, and the bench's K0 batching — a ring of 18 frames (the 13-frame
    window, 4 lookahead frames, one free slot) beside the 155 GB workspace; the first step runs the
    batched K0 for five windows, the second takes its dt0 from a slot (its outputs are checked)."""
    sb = _slab(C5, fp32=True, seed=20260206 + 5, k0_batch=5, pipeline=True)
    try:
        _run_steps(sb, 2)
        ks = sb.plan.kernels()
        assert {"k_tderiv_multi", "k_grad_xyz_c", "k_wz_solve_c"} <= set(ks), ks
        geo = sb.plan.geometry()
        assert geo["k0_batch"] == 5 and geo["k12"]["march"] == 256, geo
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


# ---- configs[1] at its full size through the bench's series plan (round 6) ----

C2 = dict(nz=64, ny=256, nx=256, s=2, t=2, w=5)


def test_c2_full_volume_bench_plan_vs_oracle():
    """configs[1] (13 x 64 x 256 x 256, xyzSig 2, tSig 2, wSig 5, fp64) as bench.py --config c2 runs
    it: a series of 17 resident frames through one plan with K0 batching (of3d_plan_execute_ahead),
    the first step forming five windows' dt0, the second using its slot.  The plan's cost model
    picks 32-plane K12 marches at this size (one round of 256 blocks: csrc/of3d_host.hip, the K12
    march-length model) — asserted through of3d_plan_geometry — so the crops straddle K12's march
    seam at plane 32, the column-block seams of the K34 shape the autotune kept, and two corners;
    then every K34 candidate gives the default plan's bits at this size."""
    import torch

    import bench
    from opticalflow3d_dev_amd import _lib, make_taps, radii
    from conftest import assert_rel_within, bits_equal, oracle3d

    _free()
    p = C2
    s, t, w = p["s"], p["t"], p["w"]
    nz, ny, nx = p["nz"], p["ny"], p["nx"]
    rd, _, rt, rw = radii(s, t, w)
    nwin, kb = 2 * rt + 1, 5
    dev = torch.device("cuda", 0)
    d_in = bench.synthetic_slab(nwin + kb - 1, nz, ny, nx, 0, nz, 20260206 + 2, dev)
    vox = nz * ny * nx
    outs = [torch.full((vox,), float("nan"), dtype=torch.float64, device=dev) for _ in range(3)]
    outs.append(torch.full((vox,), float("nan"), dtype=torch.float32, device=dev))
    ptrs = [d_in[i].data_ptr() for i in range(nwin + kb - 1)]
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run(plan, j):
        plan.execute(ptrs[j:j + nwin], _lib.OF3D_U16, 0, 0, nz, *[o.data_ptr() for o in outs], stream,
                     ahead_ptrs=ptrs[j + nwin:])

    plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=0, timing=4)
    try:
        run(plan, 0)
        geo0 = plan.geometry()
        run(plan, 1)
        torch.cuda.synchronize(dev)
        ks = set(plan.kernels())
        geo = plan.geometry()
    finally:
        plan.close()
    assert {"k_tderiv_multi", "k_grad_xyz_c", "k_wz_solve_c"} <= ks, ks
    assert geo0["k0_batch"] == kb, geo0
    assert geo["k12"]["march"] == 32 and geo["k12"]["grid"][1] == 2, geo
    tx = geo["k34"]["tx"]
    host = d_in[1:1 + nwin].cpu().numpy().view(np.uint16)  # window 1 (its dt0 from the batch's slot)
    got = [o.view(nz, ny, nx) for o in outs]
    xs = [min(max(tx - 8, 0), nx - 16)] if geo["k34"]["nbx"] > 1 else [nx // 2 - 8]
    crops = [(24, 40, 120, 136, xs[0], xs[0] + 16),   # K12 march seam (plane 32) x a K34 column seam
             (28, 36, 0, 16, 100, 130),             # march seam at the y = 0 edge
             (0, 16, 0, 16, 0, 16),                 # corner at the origin
             (48, 64, 240, 256, 236, 256)]          # far corner
    h = rd + rw
    for box in crops:
        z0, z1, y0, y1, x0, x1 = box
        lo = [max(a - h, 0) for a in (z0, y0, x0)]
        hi = [min(b + h, n) for b, n in zip((z1, y1, x1), (nz, ny, nx))]
        sub = np.ascontiguousarray(host[:, lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]])
        vx, vy, vz, lmin, lmax = oracle3d(sub, s, t, w)
        sl = (slice(z0 - lo[0], z1 - lo[0]), slice(y0 - lo[1], y1 - lo[1]), slice(x0 - lo[2], x1 - lo[2]))
        for g, want, name in zip(got[:3], (vx[sl], vy[sl], vz[sl]), ("vx", "vy", "vz")):
            assert bits_equal(g[z0:z1, y0:y1, x0:x1].cpu().numpy(), want), (box, name)
        assert_rel_within(got[3][z0:z1, y0:y1, x0:x1].cpu().numpy(), lmin[sl], lmax[sl], 1e-6)
    # every K34 candidate at this size (plain execute of window 1), bit-identical to the above
    ref = [o.clone() for o in outs]
    ncand = geo["k34"]["candidates"]
    assert ncand >= 2, geo
    import os
    for i in range(ncand):
        os.environ["OF3D_K34_CAND"] = str(i)
        try:
            pl = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=0)
            try:
                pl.execute(ptrs[1:1 + nwin], _lib.OF3D_U16, 0, 0, nz, *[o.data_ptr() for o in outs], stream)
                torch.cuda.synchronize(dev)
            finally:
                pl.close()
        finally:
            del os.environ["OF3D_K34_CAND"]
        for a, b in zip(ref, outs):
            it = torch.int64 if a.element_size() == 8 else torch.int32
            assert bool(torch.equal(a.view(it), b.view(it))), i
    del d_in, outs, ref
    _free()
