"""GPU parity: the HIP path (through the C-ABI libof3d.so) against the
reference's golden vectors and the CPU oracle.

Tolerances:
  * 2D vx, vy, rel and 3D vx, vy, vz: bit-identical (NaN positions included).
  * 3D rel (float32) vs the reference's complex64-LAPACK rel:
      |d| <= 1e-6 * |lambda_max| per voxel.
  * 3D rel computed in fp64 (OF3D_REL_F64) vs fp64 eigvalsh of the same
    tensor: |d| <= 1e-10 * |lambda_max| per voxel.
"""
import numpy as np
import pytest

from conftest import bits_equal, golden_cases, load_golden
from opticalflow3d_dev_amd import calc_flow2D, calc_flow3D
from opticalflow3d_dev_amd.calc_flow import _flow3d
from oracle import cpu_ref

pytestmark = pytest.mark.gpu

REL_TOL_REF = 1e-6
REL_TOL_FP64 = 1e-10


def assert_rel_close(rel, ref, lmax, tol):
    err = np.abs(rel.astype(np.float64) - ref.astype(np.float64))
    bound = tol * np.abs(lmax) + 1e-300
    bad = err > bound
    assert not bad.any(), f"{bad.sum()} voxels: max err/lmax {np.max(err / (np.abs(lmax) + 1e-300)):.3e}"


@pytest.mark.parametrize("name", golden_cases("c3d"))
def test_golden_3d(name):
    g = load_golden(name)
    vx, vy, vz, rel = calc_flow3D(g["images"], g["sig"], g["tsig"], g["wsig"])
    assert bits_equal(vx, g["vx"]) and bits_equal(vy, g["vy"]) and bits_equal(vz, g["vz"])
    assert rel.dtype == np.float32 and rel.shape == g["rel"].shape
    assert_rel_close(rel, g["rel"], g["lmax64"], REL_TOL_REF)


@pytest.mark.parametrize("name", golden_cases("c3d"))
def test_golden_3d_rel_fp64(name):
    g = load_golden(name)
    *_, rel64 = _flow3d(g["images"], g["sig"], g["tsig"], g["wsig"], rel_fp64=True)
    assert rel64.dtype == np.float64
    assert_rel_close(rel64, g["lmin64"], g["lmax64"], REL_TOL_FP64)


@pytest.mark.parametrize("name", golden_cases("c2d"))
def test_golden_2d(name):
    g = load_golden(name)
    vx, vy, rel = calc_flow2D(g["images"], g["sig"], g["tsig"], g["wsig"])
    for a, k in ((vx, "vx"), (vy, "vy"), (rel, "rel")):
        assert bits_equal(a, g[k]), k


SEEDED_3D = [
    ((7, 16, 40, 70), (1, 1, 3), np.uint16),
    ((13, 20, 64, 64), (2, 2, 5), np.uint16),
    ((9, 9, 33, 65), (1.2, 1.2, 2.2), np.uint16),
    ((7, 5, 70, 130), (1, 1, 2), np.uint8),
    ((7, 6, 30, 40), (1, 1, 2), np.int16),
    ((7, 6, 30, 40), (1, 1, 2), np.int32),
    ((7, 6, 30, 40), (1, 1, 2), np.uint32),
    ((7, 6, 30, 40), (1, 1, 2), np.float64),
    ((7, 6, 30, 40), (1, 1, 2), np.int64),      # host cast to float64, as the reference does
    ((7, 6, 30, 40), (1, 1, 2), ">u2"),         # big-endian (TIFF 'MM') input
    # fused products + W y + W x (K34) geometry: several column blocks, row chunks
    # not a multiple of the tile, columns shorter than the register ring, rw 12/15/21
    ((7, 4, 37, 600), (1, 1, 5), np.uint16),
    ((7, 3, 300, 50), (1, 1, 4), np.uint16),
    ((7, 3, 5, 20), (1, 1, 7), np.uint16),
    ((7, 2, 70, 1100), (1, 1, 7), np.uint16),
]


def _rand(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        return rng.uniform(-50, 4000, size=shape).astype(dt)
    hi = 255 if dt.itemsize == 1 else 4096
    lo = -2000 if dt.kind == "i" else 0
    return rng.integers(lo, hi, size=shape).astype(dt)


@pytest.mark.parametrize("case", range(len(SEEDED_3D)))
def test_seeded_3d_vs_oracle(case):
    shape, (s, t, w), dt = SEEDED_3D[case]
    img = _rand(shape, dt, 100 + case)
    vx, vy, vz, rel = calc_flow3D(img, s, t, w)
    st = cpu_ref.structure_tensor3d(img, s, t, w, backend="scipy")
    ox, oy, oz = cpu_ref.solve3d(st)
    assert bits_equal(vx, ox) and bits_equal(vy, oy) and bits_equal(vz, oz)
    lmin, lmax = cpu_ref.eig_fp64_3d(st)
    assert_rel_close(rel, lmin, lmax, REL_TOL_REF)


SEEDED_2D = [
    ((7, 256, 256), (1, 1, 5), np.uint16),
    ((13, 100, 37), (2, 2, 5), np.uint16),
    ((9, 64, 200), (1.5, 1.3, 3.7), np.float32),
    ((7, 1, 50), (1, 1, 2), np.uint16),
    ((7, 50, 1), (1, 1, 2), np.uint16),
    ((7, 333, 531), (1, 1, 7), np.uint16),
    ((7, 3, 900), (1, 1, 5), np.uint16),
]


@pytest.mark.parametrize("case", range(len(SEEDED_2D)))
def test_seeded_2d_vs_oracle(case):
    shape, (s, t, w), dt = SEEDED_2D[case]
    img = _rand(shape, dt, 200 + case)
    out = calc_flow2D(img, s, t, w)
    ref = cpu_ref.calc_flow2D(img, s, t, w, backend="scipy")
    for a, b in zip(out, ref):
        assert bits_equal(a, b)


def test_flat_volume_known_answer():
    img = np.full((7, 5, 9, 11), 1234, np.uint16)
    vx, vy, vz, rel = calc_flow3D(img, 1, 1, 2)
    assert np.all(vx == 0) and np.all(vy == 0) and np.all(vz == 0) and np.all(rel == 0)
    assert np.all(np.signbit(vx))  # -0.0 exactly like the reference (-R * 0)


def test_translation_known_answer_signs():
    """Known motion (FigS1 idea): sign and rough magnitude only (the LK estimate is biased)."""
    img = cpu_ref.synthetic_stack_np((7, 24, 48, 48), seed=5, motion=(0.3, -0.2, 0.1))
    vx, vy, vz, rel = calc_flow3D(img, 2, 1, 4)
    c = (slice(8, 16), slice(12, 36), slice(12, 36))
    assert 0.02 < np.median(vx[c]) < 0.6
    assert -0.5 < np.median(vy[c]) < -0.03
    assert 0.01 < np.median(vz[c]) < 0.4


def test_deterministic():
    img = _rand((7, 8, 40, 40), np.uint16, 7)
    a = calc_flow3D(img, 1, 1, 3)
    b = calc_flow3D(img, 1, 1, 3)
    for x, y in zip(a, b):
        assert bits_equal(x, y)


@pytest.mark.parametrize("name", golden_cases("c3d"))
def test_golden_3d_fused_gradients(name, monkeypatch):
    """K12 (the fused y/x/z gradient kernel) forced on: still bit-identical to the reference."""
    monkeypatch.setenv("OF3D_K12", "1")
    g = load_golden(name)
    vx, vy, vz, rel = calc_flow3D(g["images"], g["sig"], g["tsig"], g["wsig"])
    assert bits_equal(vx, g["vx"]) and bits_equal(vy, g["vy"]) and bits_equal(vz, g["vz"])
    assert_rel_close(rel, g["rel"], g["lmax64"], REL_TOL_REF)


@pytest.mark.parametrize("case", range(len(SEEDED_3D)))
def test_seeded_3d_fused_gradients(case, monkeypatch):
    monkeypatch.setenv("OF3D_K12", "1")
    test_seeded_3d_vs_oracle(case)


@pytest.fixture
def general_path(monkeypatch):
    """OF3D_GENERAL=1: every plan runs the general-radius kernels (k_corr_gen passes); the
    host entry's cached plans are dropped before and after."""
    from opticalflow3d_dev_amd import _lib

    _lib.cache_clear()
    monkeypatch.setenv("OF3D_GENERAL", "1")
    yield
    monkeypatch.delenv("OF3D_GENERAL")
    _lib.cache_clear()


@pytest.mark.parametrize("name", golden_cases("c3d"))
def test_golden_3d_general_path(name, general_path):
    g = load_golden(name)
    vx, vy, vz, rel = calc_flow3D(g["images"], g["sig"], g["tsig"], g["wsig"])
    assert bits_equal(vx, g["vx"]) and bits_equal(vy, g["vy"]) and bits_equal(vz, g["vz"])
    assert_rel_close(rel, g["rel"], g["lmax64"], REL_TOL_REF)


@pytest.mark.parametrize("name", golden_cases("c2d"))
def test_golden_2d_general_path(name, general_path):
    g = load_golden(name)
    vx, vy, rel = calc_flow2D(g["images"], g["sig"], g["tsig"], g["wsig"])
    for a, k in ((vx, "vx"), (vy, "vy"), (rel, "rel")):
        assert bits_equal(a, g[k]), k


@pytest.mark.parametrize("case", [0, 1, 3, 8, 10])
def test_seeded_3d_general_path(case, general_path):
    test_seeded_3d_vs_oracle(case)


def test_zslabs_general_path(general_path):
    """z-slab plans on the general path: plane ranges and clamping as the tiled pipeline."""
    from opticalflow3d_dev_amd.shard import flow3d_zslabs_host

    g = load_golden("c3d_big_xyzsig9")
    for world in (2, 3):
        vx, vy, vz, rel = flow3d_zslabs_host(g["images"], g["sig"], g["tsig"], g["wsig"], world)
        assert bits_equal(vx, g["vx"]) and bits_equal(vy, g["vy"]) and bits_equal(vz, g["vz"])


@pytest.mark.parametrize("psd", [False, True])
def test_rel3d_device_formula_near_degenerate(psd):
    """The device eigenvalue (of3d_rel3d: the eigmin3 instance the flow kernels store) on
    tools/eig_poly.py's sets — generic, near-degenerate, exact pairs, near-degenerate smallest
    pair, near-isotropic, rank 1 — against fp64 eigvalsh: fp64 rel <= 1e-10 lambda_max (the
    deflation branch), float32 rel <= 1e-6 lambda_max."""
    import os
    import sys

    import torch

    from conftest import REPO
    from opticalflow3d_dev_amd import _lib

    sys.path.insert(0, os.path.join(REPO, "tools"))
    import eig_poly

    args, ref = eig_poly.test_set(n=120000, seed=5, psd=psd)
    lmax = np.abs(ref).max(axis=1)
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(np.ascontiguousarray(np.stack(args))).to(dev)
    lib = _lib.load()
    s = torch.cuda.current_stream(dev).cuda_stream
    for f64, tol in ((1, REL_TOL_FP64), (0, REL_TOL_REF)):
        out = torch.empty(len(lmax), dtype=torch.float64 if f64 else torch.float32, device=dev)
        _lib.check(lib.of3d_rel3d(t.data_ptr(), len(lmax), out.data_ptr(), f64, s))
        torch.cuda.synchronize(dev)
        err = np.abs(out.cpu().numpy().astype(np.float64) - ref[:, 0]) / lmax
        assert err.max() <= tol, (f64, err.max())
        if f64:
            assert err.max() <= 1e-12, err.max()
    # fp64 rel on tensors of magnitude 1e-100 / 1e100 too (the deflation on the scaled matrix:
    # no under- or overflow; float32 rel cannot hold such values)
    args, ref = eig_poly.test_set(n=60000, seed=13, psd=psd, extreme=True)
    lmax = np.abs(ref).max(axis=1)
    t = torch.from_numpy(np.ascontiguousarray(np.stack(args))).to(dev)
    out = torch.empty(len(lmax), dtype=torch.float64, device=dev)
    _lib.check(lib.of3d_rel3d(t.data_ptr(), len(lmax), out.data_ptr(), 1, s))
    torch.cuda.synchronize(dev)
    got = out.cpu().numpy()
    assert np.isfinite(got).all()
    assert (np.abs(got - ref[:, 0]) / lmax).max() <= 1e-12
