"""The column-march kernels (K1c k_grad_xy_c, K34 k_prod_wyx, K5c k_wz_solve_c) against
the earlier kernel family (k_grad_xy, k_prod_wy + k_wx, k_wz_solve_dma / k_wz_solve) on
the same device inputs: every output bit-identical, at sizes beyond the oracle-checked
cases (several column blocks and row chunks, K34 autotune on).  Each family is itself
pinned to the reference's golden vectors (test_gpu_parity.py); this covers the
geometry paths (tail column blocks, partial tiles, XCD grouping) at scale, in fp64 and
in the fp32 mode."""
import os

import numpy as np
import pytest

from opticalflow3d_dev_amd import _lib, make_taps, radii

pytestmark = pytest.mark.gpu

FAMILY_ENV = ("OF3D_K34", "OF3D_K5C", "OF3D_K1C", "OF3D_K12", "OF3D_K5C_NW", "OF3D_K34_UQ", "OF3D_WXY_TILE",
              "OF3D_K12_ZC")


def _run(img, s, t, w, ndim, mode, old, force=None, kernels=None):
    import torch

    saved = {k: os.environ.get(k) for k in FAMILY_ENV}
    try:
        for k in FAMILY_ENV:
            if old:
                os.environ[k] = "0"
            else:
                os.environ.pop(k, None)
        os.environ.update(force or {})
        dev = torch.device("cuda", 0)
        nt = img.shape[0]
        vol = img.shape[1:] if ndim == 3 else (1,) + img.shape[1:]
        nz, ny, nx = vol
        rt = radii(s, t, w)[2]
        c = nt // 2
        win = np.ascontiguousarray(img[c - rt:c + rt + 1]).reshape((2 * rt + 1,) + vol)
        d_in = torch.from_numpy(win.view(np.int16)).to(dev)
        fp32 = bool(mode & _lib.OF3D_FP32)
        vt = torch.float32 if fp32 else torch.float64
        n = nz * ny * nx
        outs = [torch.empty(n, dtype=vt, device=dev) for _ in range(3)]
        rel = torch.empty(n, dtype=torch.float64 if (ndim == 2 and not fp32) else (vt if ndim == 2 else torch.float32),
                          device=dev)
        plan = _lib.Plan(ndim, nz, ny, nx, make_taps(s, t, w), device=0, mode=mode)
        try:
            plan.execute([d_in[i].data_ptr() for i in range(2 * rt + 1)], _lib.OF3D_U16, 0, 0, nz,
                         outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), rel.data_ptr())
            torch.cuda.synchronize(dev)
            if kernels is not None:
                kernels.extend(plan.kernels())
        finally:
            plan.close()
        res = [o.cpu().numpy() for o in outs[:3 if ndim == 3 else 2]] + [rel.cpu().numpy()]
        return res
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


CASES = [
    ((13, 20, 300, 266), (2, 2, 5), 3),   # rw 15: several column blocks, tail block, partial tiles
    ((7, 9, 130, 140), (3, 1, 4), 3),     # reference defaults: rd 9, rw 12
    ((19, 12, 100, 530), (2, 3, 7), 3),   # rw 21 (c3 parameters)
    ((13, 1, 700, 333), (2, 2, 5), 2),    # 2D, five products
]


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("fp32", [False, True])
def test_families_bit_identical(case, fp32):
    shape, (s, t, w), ndim = CASES[case]
    rng = np.random.default_rng(300 + case)
    img = rng.integers(0, 4096, size=shape).astype(np.uint16)
    if ndim == 2:
        img = img[:, 0]
    mode = _lib.OF3D_FP32 if fp32 else 0
    new = _run(img, s, t, w, ndim, mode, old=False)
    ref = _run(img, s, t, w, ndim, mode, old=True)
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("case", range(3))
@pytest.mark.parametrize("fp32", [False, True])
def test_fused_gradients_k12_forced(case, fp32):
    """K12 (fused y/x/z gradient passes) forced on volumes below its size heuristic, against
    K1c + K2c and the older kernels: every output bit-identical."""
    shape, (s, t, w), ndim = CASES[case]
    rng = np.random.default_rng(400 + case)
    img = rng.integers(0, 4096, size=shape).astype(np.uint16)
    mode = _lib.OF3D_FP32 if fp32 else 0
    new = _run(img, s, t, w, ndim, mode, old=False, force={"OF3D_K12": "1"})
    ref = _run(img, s, t, w, ndim, mode, old=True)
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("zc", [0, 16, 40])
@pytest.mark.parametrize("fp32", [False, True])
def test_fused_gradients_k12_xyzsig1(zc, fp32):
    """K12 at xyzSig 1 (rd 3, rs 1: three-plane DMA chunks in fp64 since its A tiles hold one
    copy per row) forced, with whole-volume, 16- and 40-plane marches (chunk tails and march
    tails), against K1c + K2c and the older kernels: every output bit-identical."""
    rng = np.random.default_rng(450 + zc)
    img = rng.integers(0, 4096, size=(13, 45, 70, 232)).astype(np.uint16)  # 16-byte u16 rows
    mode = _lib.OF3D_FP32 if fp32 else 0
    force = {"OF3D_K12": "1"} | ({"OF3D_K12_ZC": str(zc)} if zc else {})
    kernels = []
    new = _run(img, 1, 2, 5, 3, mode, old=False, force=force, kernels=kernels)
    assert "k_grad_xyz_c" in kernels, kernels
    ref = _run(img, 1, 2, 5, 3, mode, old=True)
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("case", range(3))
@pytest.mark.parametrize("fp32", [False, True])
def test_wz_solve_eight_wave_blocks(case, fp32):
    """K5c with 8-wave, 128-plane blocks (OF3D_K5C_NW=8; the default for volumes with >= 128
    output planes) forced on small volumes: bit-identical to the older kernels."""
    shape, (s, t, w), ndim = CASES[case]
    img = np.random.default_rng(600 + case).integers(0, 4096, size=shape).astype(np.uint16)
    mode = _lib.OF3D_FP32 if fp32 else 0
    new = _run(img, s, t, w, ndim, mode, old=False, force={"OF3D_K5C_NW": "8"})
    ref = _run(img, s, t, w, ndim, mode, old=True)
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("case", range(3))
@pytest.mark.parametrize("fp32", [False, True])
def test_wxy_plain_and_tiled_layouts(case, fp32):
    """The K34 -> K5c hand-off in plain planes (OF3D_WXY_TILE=0) and z-tiled (OF3D_WXY_TILE=1; the
    default for fp64 workspaces of >= 128 planes with nx a multiple of 32) against the older
    kernels: bit-identical.  nx is rounded up to a multiple of 32 here (288, 160, 544)."""
    shape, (s, t, w), ndim = CASES[case]
    shape = shape[:-1] + (((shape[-1] + 31) // 32) * 32,)  # nx a multiple of 32: the tiled layout
    img = np.random.default_rng(660 + case).integers(0, 4096, size=shape).astype(np.uint16)
    mode = _lib.OF3D_FP32 if fp32 else 0
    tiled = _run(img, s, t, w, ndim, mode, old=False, force={"OF3D_WXY_TILE": "1"})
    plain = _run(img, s, t, w, ndim, mode, old=False, force={"OF3D_WXY_TILE": "0"})
    ref = _run(img, s, t, w, ndim, mode, old=True)
    for a, b, c in zip(tiled, plain, ref):
        assert a.dtype == c.dtype and np.array_equal(a.view(np.uint8), c.view(np.uint8))
        assert np.array_equal(b.view(np.uint8), c.view(np.uint8))


W_RADII = [
    ((7, 10, 90, 200), (2, 1, 3), 3),     # rw 9
    ((13, 12, 100, 268), (1, 2, 6), 3),   # rw 18 (fp32 K5c: nx % 4 == 0)
    ((7, 1, 300, 140), (2, 1, 3), 2),     # 2D, rw 9
    ((7, 1, 240, 300), (1, 1, 6), 2),     # 2D, rw 18
]


@pytest.mark.parametrize("case", range(len(W_RADII)))
@pytest.mark.parametrize("fp32", [False, True])
def test_fused_w_kernels_wsig3_wsig6(case, fp32):
    """wSig 3 and 6 (W radii 9, 18) run the fused K34 / K5c instances (of3d_plan_kernels
    says so) and agree bit for bit with the separate-pass kernels."""
    shape, (s, t, w), ndim = W_RADII[case]
    img = np.random.default_rng(700 + case).integers(0, 4096, size=shape).astype(np.uint16)
    if ndim == 2:
        img = img[:, 0]
    mode = _lib.OF3D_FP32 if fp32 else 0
    used = []
    new = _run(img, s, t, w, ndim, mode, old=False, kernels=used)
    assert any(k.startswith("k_prod_wyx") for k in used), used
    if ndim == 3:
        assert any(k.startswith("k_wz_solve_c") for k in used), used
    old_used = []
    ref = _run(img, s, t, w, ndim, mode, old=True, kernels=old_used)
    assert not any(k.startswith("k_prod_wyx") for k in old_used), old_used
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("case", range(len(CASES)))
def test_packed_fp32_products_w(case):
    """The packed-fp32 K34 (k_prod_wyx_pk: float2 column pairs in W y, row pairs in W x,
    v_pk_mul/add_f32) forced (OF3D_K34_UQ=3) against the older fp32 kernels: bit-identical."""
    shape, (s, t, w), ndim = CASES[case]
    img = np.random.default_rng(800 + case).integers(0, 4096, size=shape).astype(np.uint16)
    if ndim == 2:
        img = img[:, 0]
    used = []
    new = _run(img, s, t, w, ndim, _lib.OF3D_FP32, old=False, force={"OF3D_K34_UQ": "3"}, kernels=used)
    assert "k_prod_wyx_pk" in used, used
    ref = _run(img, s, t, w, ndim, _lib.OF3D_FP32, old=True)
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("case", range(len(W_RADII)))
def test_packed_fp32_products_w_radii(case):
    shape, (s, t, w), ndim = W_RADII[case]
    img = np.random.default_rng(900 + case).integers(0, 4096, size=shape).astype(np.uint16)
    if ndim == 2:
        img = img[:, 0]
    used = []
    new = _run(img, s, t, w, ndim, _lib.OF3D_FP32, old=False, force={"OF3D_K34_UQ": "3"}, kernels=used)
    assert "k_prod_wyx_pk" in used, used
    ref = _run(img, s, t, w, ndim, _lib.OF3D_FP32, old=True)
    for a, b in zip(new, ref):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))
