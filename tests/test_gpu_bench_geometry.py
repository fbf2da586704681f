"""The benchmarked geometry pinned to the oracle: bench.py's headline workload (configs[2],
c3: 19 x 128 x 512 x 512, xyzSig 2, tSig 3, wSig 7, fp64) run through the same Plan the
bench times, on the bench's own synthetic input, compared with the oracle
(oracle/cpu_ref.py, pinned to the reference's calc_flow3D, calc_flow.py:175-360) on crops.

Crops: an output voxel further than rd + rw = 6 + 21 = 27 voxels from every face where the
crop cuts the volume sees no clamping the full volume does not (the y, x, z gradient passes
reach rd, the W passes rw further), so the oracle of the crop's input box gives its exact
outputs.  The crops cover the seams of the kernels' decompositions at this size: K12's and
K5c's 64-plane z chunks (plane 64, where K5c's XCD block remap is live: 2 z chunks), K34's
256-row chunks (row 256), and the volume corners and x edge (global clamping).

Every kernel family the plan can pick at this size (the K34 autotune's candidates, the
duplicate / unique / wave-specialised K34 forms, K5c's 4- and 8-wave blocks, K1c + K2c
instead of K12) is forced in turn and must give the same bits.

Tolerances: vx, vy, vz bitwise; rel within 1e-6 * lambda_max of the fp64
eigenvalue; fp32 plans within 1e-4 * max|v| of the fp64 oracle.
"""
import contextlib
import os

import numpy as np
import pytest

from conftest import assert_rel_within, bits_equal, oracle3d

pytestmark = pytest.mark.gpu

C3 = dict(nt=19, nz=128, ny=512, nx=512, s=2, t=3, w=7)
HALO = 6 + 21  # rd + rw at xyzSig 2, wSig 7
# output boxes (z0, z1, y0, y1, x0, x1)
CROPS = {
    "z64_y256_interior": (52, 76, 244, 268, 300, 330),
    "corner_origin": (0, 20, 0, 24, 0, 24),
    "corner_far": (108, 128, 488, 512, 486, 512),
    "x_edge_y256": (30, 48, 248, 264, 0, 28),
}


@contextlib.contextmanager
def env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_plan(d_in, nz, ny, nx, s, t, w, mode=0, geo=None):
    """One output frame through a device plan as bench.py runs it: (vx, vy, vz, rel) device
    tensors and the kernel families the plan launched (and its of3d_plan_geometry into `geo`)."""
    import torch

    from opticalflow3d_dev_amd import _lib, make_taps

    dev = d_in.device
    fp32 = bool(mode & _lib.OF3D_FP32)
    n = nz * ny * nx
    vt = torch.float32 if fp32 else torch.float64
    outs = [torch.full((n,), float("nan"), dtype=vt, device=dev) for _ in range(3)]
    outs.append(torch.full((n,), float("nan"), dtype=torch.float32, device=dev))
    plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=dev.index, timing=4, mode=mode)
    try:
        plan.execute([d_in[i].data_ptr() for i in range(d_in.shape[0])], _lib.OF3D_U16, 0, 0, nz,
                     *[o.data_ptr() for o in outs], torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        kernels = plan.kernels()
        if geo is not None:
            geo.append(plan.geometry())
    finally:
        plan.close()
    return [o.view(nz, ny, nx) for o in outs], kernels


def same_bits(a, b):
    import torch

    it = torch.int64 if a.element_size() == 8 else torch.int32
    return a.shape == b.shape and a.dtype == b.dtype and bool(torch.equal(a.view(it), b.view(it)))


def crop_check(host_in, outs, box, s, t, w, fp32=False):
    """Oracle of the crop's input box vs the outputs in `box` (host copies of the crop only)."""
    nt, nz, ny, nx = host_in.shape
    z0, z1, y0, y1, x0, x1 = box
    lo = [max(a - HALO, 0) for a in (z0, y0, x0)]
    hi = [min(b + HALO, n) for b, n in zip((z1, y1, x1), (nz, ny, nx))]
    sub = np.ascontiguousarray(host_in[:, lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]])
    vx, vy, vz, lmin, lmax = oracle3d(sub, s, t, w)
    sl = (slice(z0 - lo[0], z1 - lo[0]), slice(y0 - lo[1], y1 - lo[1]), slice(x0 - lo[2], x1 - lo[2]))
    got = [o[z0:z1, y0:y1, x0:x1].cpu().numpy() for o in outs]
    if fp32:
        for g, want in zip(got[:3], (vx[sl], vy[sl], vz[sl])):
            assert np.abs(g.astype(np.float64) - want).max() <= 1e-4 * np.abs(want).max()
        assert np.abs(got[3].astype(np.float64) - lmin[sl]).max() <= 1e-4 * np.abs(lmax[sl]).max()
        return
    for g, want, name in zip(got[:3], (vx[sl], vy[sl], vz[sl]), ("vx", "vy", "vz")):
        assert bits_equal(g, want), (box, name)
    assert_rel_within(got[3], lmin[sl], lmax[sl], 1e-6)


@pytest.fixture(scope="module")
def c3():
    """bench.py's c3 input (synthetic_slab, seed 20260206 + 3 as bench.main uses at rank 0),
    resident on the device, and the default plan's outputs."""
    import torch

    import bench
    from opticalflow3d_dev_amd import radii

    p = C3
    rt = radii(p["s"], p["t"], p["w"])[2]
    dev = torch.device("cuda", 0)
    d_in = bench.synthetic_slab(2 * rt + 1, p["nz"], p["ny"], p["nx"], 0, p["nz"], 20260206 + 3, dev)
    outs, kernels = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"])
    host_in = d_in.cpu().numpy().view(np.uint16)
    yield d_in, host_in, outs, kernels
    del d_in, outs
    torch.cuda.empty_cache()


def test_c3_default_plan_kernels(c3):
    """The headline plan runs the fused kernels the bench's roofline names."""
    _, _, outs, kernels = c3
    assert "k_grad_xyz_c" in kernels and "k_wz_solve_c" in kernels, kernels
    assert any(k.startswith("k_prod_wyx") for k in kernels), kernels
    for o in outs[:3]:
        assert bool(o.isfinite().all())


@pytest.mark.parametrize("crop", sorted(CROPS))
def test_c3_full_size_vs_oracle_crops(c3, crop):
    d_in, host_in, outs, _ = c3
    crop_check(host_in, outs, CROPS[crop], C3["s"], C3["t"], C3["w"])


def k34_candidates(d_in, p, mode=0):
    """Number of K34 autotune candidates of this plan shape (OF3D_K34_CAND past the end fails with
    OF3D_K34_CAND_STRICT=1; without it a pin past the end is ignored with a warning)."""
    from opticalflow3d_dev_amd import _lib, make_taps

    n = 0
    while n < 64:
        with env(OF3D_K34_CAND=n, OF3D_K34_CAND_STRICT=1):
            try:
                _lib.Plan(3, p["nz"], p["ny"], p["nx"], make_taps(p["s"], p["t"], p["w"]), device=0,
                          mode=mode).close()
            except RuntimeError as e:
                assert "OF3D_K34_CAND out of range" in str(e)
                return n
        n += 1
    return n


FAMILIES = [dict(OF3D_K34_UQ=0), dict(OF3D_K34_UQ=1), dict(OF3D_K34_UQ=2), dict(OF3D_K5C_NW=8),
            dict(OF3D_K5C_R=4), dict(OF3D_K12=0), dict(OF3D_K34_TUNE=0),
            # both K5c knobs at once: the 8-wave instances are R 8 only, so the host's grid and
            # LDS must follow R 8 too (a 4-plane grid over the 8-plane kernel once gave garbage)
            dict(OF3D_K5C_R=4, OF3D_K5C_NW=8),
            # the W-xy hand-off in plain planes instead of z-tiled (round 5)
            dict(OF3D_WXY_TILE=0)]


def test_c3_every_kernel_family_bit_identical(c3):
    """Each forced family and each K34 autotune candidate at the headline size gives the
    default plan's bits (so the timing-based autotune cannot change a result)."""
    d_in, _, ref, _ = c3
    p = C3
    ncand = k34_candidates(d_in, p)
    assert ncand >= 2
    variants = FAMILIES + [dict(OF3D_K34_CAND=i) for i in range(ncand)]
    seen = set()
    for v in variants:
        with env(**v):
            outs, kernels = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"])
        seen.update(kernels)
        for a, b, name in zip(ref, outs, ("vx", "vy", "vz", "rel")):
            assert same_bits(a, b), (v, name, kernels)
        del outs
    # the families really changed: lockstep, wave-specialised K34, K1c + K2c, 8-wave K5c
    assert {"k_prod_wyx", "k_prod_wyx_ws", "k_grad_xy_c", "k_grad_z_c"} <= seen, seen


def test_c3_fp32_plans_vs_oracle_and_candidates(c3):
    """configs[4]'s fp32 path at the c3 size: every K34 candidate (packed, wave-specialised,
    lockstep fp32 kernels) bit-identical, and the outputs within 1e-4 of the fp64 oracle."""
    from opticalflow3d_dev_amd import _lib

    d_in, host_in, _, _ = c3
    p = C3
    mode = _lib.OF3D_FP32
    ref, _ = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
    ncand = k34_candidates(d_in, p, mode)
    for v in [dict(OF3D_K34_CAND=i) for i in range(ncand)] + [dict(OF3D_K12=0), dict(OF3D_K5C_R=4),
                                                               dict(OF3D_WXY_TILE=1)]:
        with env(**v):
            outs, kernels = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
        for a, b, name in zip(ref, outs, ("vx", "vy", "vz", "rel")):
            assert same_bits(a, b), (v, name, kernels)
        del outs
    crop_check(host_in, ref, CROPS["z64_y256_interior"], p["s"], p["t"], p["w"], fp32=True)
    crop_check(host_in, ref, CROPS["corner_far"], p["s"], p["t"], p["w"], fp32=True)


@pytest.mark.parametrize("variant", [dict(), dict(OF3D_K5C_NW=8), dict(OF3D_K34_UQ=0), dict(OF3D_K34_UQ=2),
                                     dict(OF3D_K12=1), dict(OF3D_WXY_TILE=0), dict(OF3D_K5C_R=8)])
def test_more_than_64_planes_small_xy_vs_oracle(variant):
    """13 x 200 x 41 x 48 (sigma 2, tau 2, omega 5): four K5c z chunks, and a block grid whose
    size is not a multiple of 8 z-chunk sets, so the XCD remap's tail branch runs
    (csrc/of3d_dev.hpp k5c_block); the whole volume against the oracle."""
    import torch

    img = np.random.default_rng(64).integers(0, 4096, size=(13, 200, 41, 48)).astype(np.uint16)
    d_in = torch.from_numpy(np.ascontiguousarray(img[6 - 6:6 + 7]).view(np.int16)).to("cuda")
    with env(**variant):
        outs, kernels = run_plan(d_in, 200, 41, 48, 2, 2, 5)
    vx, vy, vz, lmin, lmax = oracle3d(img, 2, 2, 5)
    for g, want, name in zip(outs[:3], (vx, vy, vz), ("vx", "vy", "vz")):
        assert bits_equal(g.cpu().numpy(), want), (variant, name, kernels)
    assert_rel_within(outs[3].cpu().numpy(), lmin, lmax, 1e-6)


# ---- configs[3] / configs[4] geometry (round 4): the branches only the big volumes take ----

LONG = dict(nt=13, nz=320, ny=40, nx=48, s=2, t=2, w=5)


@pytest.fixture(scope="module")
def long_volume():
    """A >= 300-plane small-xy volume (13 x 320 x 40 x 48, sigma 2, tau 2, omega 5) and its
    full oracle: K12's 128- and 256-plane z marches (what c4 / c5 run: csrc/of3d_host.hip picks
    the longest march that still gives >= 1024 blocks) have whole marches and a tail here."""
    import torch

    p = LONG
    img = np.random.default_rng(320).integers(0, 4096, size=(p["nt"], p["nz"], p["ny"], p["nx"])).astype(np.uint16)
    d_in = torch.from_numpy(np.ascontiguousarray(img).view(np.int16)).to("cuda")
    yield d_in, oracle3d(img, p["s"], p["t"], p["w"])
    del d_in
    torch.cuda.empty_cache()


@pytest.mark.parametrize("fp32", [False, True])
@pytest.mark.parametrize("zc", [32, 128, 256])
def test_k12_long_marches_vs_oracle(long_volume, zc, fp32):
    """OF3D_K12_ZC = 32 / 128 / 256 (the c2 / c4 / c5 marches) against the full oracle: fp64
    bitwise (marches of >= 128 planes on the three-DMA-slot instance), fp32 within 1e-4 max|v|
    and bit-identical to the 16-plane marches of the same plan."""
    from opticalflow3d_dev_amd import _lib

    d_in, (vx, vy, vz, lmin, lmax) = long_volume
    p = LONG
    mode = _lib.OF3D_FP32 if fp32 else 0
    geo = []
    with env(OF3D_K12=1, OF3D_K12_ZC=zc):
        outs, kernels = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode, geo=geo)
    assert "k_grad_xyz_c" in kernels, kernels
    assert geo[0]["k12"]["march"] == zc and geo[0]["k12"]["deep"] == int(not fp32 and zc >= 128), geo
    if not fp32:
        for g, want, name in zip(outs[:3], (vx, vy, vz), ("vx", "vy", "vz")):
            assert bits_equal(g.cpu().numpy(), want), (zc, name)
        assert_rel_within(outs[3].cpu().numpy(), lmin, lmax, 1e-6)
        return
    for g, want in zip(outs[:3], (vx, vy, vz)):
        assert np.abs(g.cpu().numpy().astype(np.float64) - want).max() <= 1e-4 * np.abs(want).max()
    with env(OF3D_K12=1, OF3D_K12_ZC=16):
        short, _ = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
    for a, b, name in zip(outs, short, ("vx", "vy", "vz", "rel")):
        assert same_bits(a, b), (zc, name)


C5S = dict(nt=13, nz=48, ny=64, nx=2048, s=2, t=2, w=5)


def test_c5_shaped_fp32_plan_candidates_and_oracle():
    """configs[4]'s row geometry (nx = 2048, rw 15, fp32: the packed K34 with its 2048-wide
    rows, K34's whole-column row chunks grouped per plane, K12's 256-plane march) on a thin
    slab of c5's own synthetic family: every K34 autotune candidate bit-identical, and oracle
    crops (interior and the far corner) within 1e-4 of the fp64 oracle."""
    import torch

    import bench
    from opticalflow3d_dev_amd import _lib

    p = C5S
    dev = torch.device("cuda", 0)
    d_in = bench.synthetic_slab(p["nt"], p["nz"], p["ny"], p["nx"], 0, p["nz"], 20260206 + 5, dev)
    host_in = d_in.cpu().numpy().view(np.uint16)
    mode = _lib.OF3D_FP32
    with env(OF3D_K12=1, OF3D_K12_ZC=256):
        ref, kernels = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
        assert "k_grad_xyz_c" in kernels, kernels
        ncand = k34_candidates(d_in, p, mode)
        assert ncand >= 2
        seen = set(kernels)
        for i in range(ncand):
            with env(OF3D_K34_CAND=i):
                outs, ks = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
            seen.update(ks)
            for a, b, name in zip(ref, outs, ("vx", "vy", "vz", "rel")):
                assert same_bits(a, b), (i, name, ks)
            del outs
    assert "k_prod_wyx_pk" in seen, seen
    crop_check(host_in, ref, (16, 32, 24, 40, 1016, 1040), p["s"], p["t"], p["w"], fp32=True)
    crop_check(host_in, ref, (32, 48, 44, 64, 2020, 2048), p["s"], p["t"], p["w"], fp32=True)


C4S = dict(nt=13, nz=24, ny=64, nx=1024, s=2, t=2, w=5)


@pytest.mark.parametrize("fp32", [False, True])
def test_c4_shaped_plan_every_k34_candidate(fp32):
    """configs[3]'s row geometry (nx = 1024, rw 15: the K34 autotune's column-block shapes for a
    1024-wide row) on a thin slab of c4's synthetic family: every K34 candidate bit-identical to
    the default plan (the timing-based autotune may pick any of them on the driver's nodes), and
    oracle crops across the candidates' column-block seams and at both x edges."""
    import torch

    import bench
    from opticalflow3d_dev_amd import _lib

    p = C4S
    dev = torch.device("cuda", 0)
    d_in = bench.synthetic_slab(p["nt"], p["nz"], p["ny"], p["nx"], 0, p["nz"], 20260206 + 4, dev)
    host_in = d_in.cpu().numpy().view(np.uint16)
    mode = _lib.OF3D_FP32 if fp32 else 0
    ref, kernels = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
    ncand = k34_candidates(d_in, p, mode)
    assert ncand >= 2
    for i in range(ncand):
        with env(OF3D_K34_CAND=i):
            outs, ks = run_plan(d_in, p["nz"], p["ny"], p["nx"], p["s"], p["t"], p["w"], mode=mode)
        for a, b, name in zip(ref, outs, ("vx", "vy", "vz", "rel")):
            assert same_bits(a, b), (i, name, ks)
        del outs
    for box in ((4, 20, 24, 40, 330, 360), (4, 20, 24, 40, 500, 530), (4, 20, 24, 40, 676, 700),
                (4, 20, 40, 64, 0, 24), (0, 16, 0, 20, 1000, 1024)):
        crop_check(host_in, ref, box, p["s"], p["t"], p["w"], fp32=fp32)


@pytest.mark.parametrize("nz,tiled", [(4096, True), (32768, False)])
def test_wxy_tiled_layout_size_guard(nz, tiled):
    """The z-tiled W-xy hand-off addresses a K34 tile of S rows through one buffer descriptor with
    32-bit offsets: a plan whose S_max * nx * cap_planes * 8 bytes would pass 2^31 keeps the plain
    planes even when tiling is forced (OF3D_WXY_TILE=1), one that fits takes the tiles (ADVICE r05;
    csrc/of3d_host.hip wxy_tile_fits).  Geometry only (fp64, 8 x 1024 planes: 0.5 / 4 GiB per tile)."""
    from opticalflow3d_dev_amd import _lib, make_taps

    with env(OF3D_WXY_TILE=1, OF3D_K34_TUNE=0):
        plan = _lib.Plan(3, nz, 8, 1024, make_taps(2, 2, 5), device=0)
        try:
            geo = plan.geometry()
        finally:
            plan.close()
    span = geo["k34"]["s_max"] * 1024 * geo["cap_planes"] * 8
    assert (span <= 0x7FFFFFFF) == tiled, geo
    assert (geo["wxy_zt"] > 0) == tiled, geo


@pytest.mark.parametrize("shape,knob,r", [((64, 256, 256), None, 4), ((128, 512, 512), None, 8),
                                          ((64, 256, 256), 8, 8), ((128, 512, 512), 4, 4)])
def test_k5c_block_rule_by_workspace(shape, knob, r):
    """K5c takes 32-plane blocks (R 4, three per CU) where the nine fp64 W-xy fields fit 320 MB —
    configs[1]: 302 MB, cache-resident — and 64-plane blocks (R 8) above (configs[2]: 2.4 GB);
    OF3D_K5C_R forces either (csrc/of3d_host.hip k5c_setup; geometry only)."""
    from opticalflow3d_dev_amd import _lib, make_taps

    kv = dict(OF3D_K34_TUNE=0)
    if knob:
        kv["OF3D_K5C_R"] = knob
    with env(**kv):
        plan = _lib.Plan(3, *shape, make_taps(2, 2, 5), device=0)
        try:
            geo = plan.geometry()
        finally:
            plan.close()
    assert geo["k5c"]["r"] == r and geo["k5c"]["nw"] == 4, geo
