"""The z-slab (configs[3]) and fp32 (configs[4]) paths checked directly
against the reference's golden vectors and the oracle — not against the
unsharded / fp64 HIP path (calc_flow.py:175-360).

Tolerances:
  * z-slabs: vx, vy, vz bit-identical to the golden vectors / oracle, rel
    within 1e-6 * lambda_max of the reference's complex64 rel.
  * fp32 path: max|dv| <= 1e-4 * max|v_ref| against the reference's fp64
    vx/vy/vz; rel within 1e-4 * max|rel_ref| (float32 tensor, fp64 solve).
"""
import numpy as np
import pytest

from conftest import assert_flow3d_matches_oracle, assert_rel_within, bits_equal, golden_cases, load_golden, oracle3d
from opticalflow3d_dev_amd import _lib, calc_flow2D_fp32, calc_flow3D_fp32
from opticalflow3d_dev_amd.shard import flow3d_zslabs_host
from oracle import cpu_ref

pytestmark = pytest.mark.gpu

ZSLAB_GOLDEN = ["c3d_rand_c2params", "c3d_rand_c3params", "c3d_nz1", "c3d_nz2", "c3d_nz3", "c3d_nz4",
                "c3d_default_params", "c3d_smooth_translate", "c3d_frac_sigmas", "c3d_big_wsig17",
                "c3d_pub_s3t1w4_nz4", "c3d_wsig3", "c3d_wsig6"]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name", ZSLAB_GOLDEN)
def test_zslabs_vs_golden(name, world):
    """Slabs of `world` virtual ranks (thinner than the halo for most cases,
    empty ones for Nz < world) against the reference's own outputs."""
    g = load_golden(name)
    vx, vy, vz, rel = flow3d_zslabs_host(g["images"], g["sig"], g["tsig"], g["wsig"], world)
    assert bits_equal(vx, g["vx"]) and bits_equal(vy, g["vy"]) and bits_equal(vz, g["vz"])
    assert_rel_within(rel, g["lmin64"], g["lmax64"], 1e-6)
    err = np.abs(rel.astype(np.float64) - g["rel"].astype(np.float64))
    assert np.all(err <= 1e-6 * np.abs(g["lmax64"]) + 1e-300)


@pytest.mark.parametrize("world", [2, 4])
def test_zslabs_seeded_vs_oracle(world):
    img = np.random.default_rng(40 + world).integers(0, 4096, size=(13, 40, 64, 64)).astype(np.uint16)
    out = flow3d_zslabs_host(img, 2, 2, 5, world)
    assert_flow3d_matches_oracle(out, img, 2, 2, 5)


def test_zslab_gloo_two_ranks_vs_oracle():
    """Two real processes on the product slab path (FlowStream(zslab=...)), each holding only
    its own planes and exchanging halos over gloo: the union of the slabs equals the oracle
    bit for bit."""
    from test_gpu_shard import run_stream_slabs

    img = np.random.default_rng(9).integers(0, 4096, size=(13, 36, 24, 28)).astype(np.uint16)
    sig = (2, 2, 5)
    vx, vy, vz, lmin, lmax = oracle3d(img, *sig)
    covered = 0
    for rank, z0, z1, outs in run_stream_slabs(2, img, sig, 0):
        covered += z1 - z0
        shp = (z1 - z0, 24, 28)
        for got, want in zip(outs[:3], (vx, vy, vz)):
            assert bits_equal(got.reshape(shp), want[z0:z1])
        assert_rel_within(outs[3].reshape(shp), lmin[z0:z1], lmax[z0:z1], 1e-6)
    assert covered == 36


FP32_TOL = 1e-4


def _assert_fp32_close(got, want_v, want_rel):
    for name, a, b in zip(("vx", "vy", "vz"), want_v, got[:len(want_v)]):
        assert b.dtype == np.float32 and b.shape == a.shape
        err = np.abs(b.astype(np.float64) - a).max()
        assert err <= FP32_TOL * np.abs(a).max(), (name, err, np.abs(a).max())
    rel = got[len(want_v)].astype(np.float64)
    want_rel = np.asarray(want_rel, np.float64)
    assert np.abs(rel - want_rel).max() <= FP32_TOL * np.abs(want_rel).max()


def _smooth(shape, seed):
    return cpu_ref.synthetic_stack_np(shape, seed=seed)


@pytest.mark.parametrize("name", ["c3d_smooth_translate", "c3d_float32_nt11", "c3d_rand_c2params",
                                  "c3d_rand_c3params", "c3d_default_params", "c3d_flat", "c3d_big_xyzsig9",
                                  "c3d_big_wsig17", "c3d_pub_s3t1w4_nz4", "c3d_wsig3", "c3d_wsig6"])
def test_fp32_3d_vs_golden(name):
    g = load_golden(name)
    got = calc_flow3D_fp32(g["images"], g["sig"], g["tsig"], g["wsig"])
    _assert_fp32_close(got, (g["vx"], g["vy"], g["vz"]), g["rel"])


@pytest.mark.parametrize("name", ["c2d_smooth_translate", "c2d_c1params", "c2d_c2params", "c2d_float32",
                                  "c2d_big_sigmas"])
def test_fp32_2d_vs_golden(name):
    g = load_golden(name)
    got = calc_flow2D_fp32(g["images"], g["sig"], g["tsig"], g["wsig"])
    _assert_fp32_close(got, (g["vx"], g["vy"]), g["rel"])


@pytest.mark.parametrize("shape,sig", [((13, 24, 48, 56), (2, 2, 5)), ((19, 16, 40, 44), (2, 3, 7))])
def test_fp32_3d_vs_oracle(shape, sig):
    img = _smooth(shape, 31)
    vx, vy, vz, lmin, lmax = oracle3d(img, *sig)
    got = calc_flow3D_fp32(img, *sig)
    _assert_fp32_close(got, (vx, vy, vz), lmin)


@pytest.mark.parametrize("world,axis", [(2, 0), (3, 0), (2, 1), (3, 1)])
def test_fp32_slab_ranks_vs_oracle(world, axis):
    """configs[4]'s fp32 path split over ranks (FlowStream(zslab=..., precision="fp32"),
    gloo): every rank's part within 1e-4 * max|v| of the oracle's fp64 flow, and equal bit
    for bit to the same part of the one-process fp32 result (slabs never change a bit)."""
    from test_gpu_shard import run_stream_slabs

    img = _smooth((13, 18, 40, 36), 5)
    sig = (2, 2, 5)
    vx, vy, vz, lmin, lmax = oracle3d(img, *sig)
    one = calc_flow3D_fp32(img, *sig)
    covered = 0
    for rank, a0, a1, outs in run_stream_slabs(world, img, sig, axis, precision="fp32"):
        covered += a1 - a0
        cut = (lambda a: a[a0:a1]) if axis == 0 else (lambda a: a[:, a0:a1])
        shp = cut(vx).shape
        got = [o.reshape(shp) for o in outs]
        _assert_fp32_close(got, (cut(vx), cut(vy), cut(vz)), cut(lmin))
        for a, b in zip(one, got):
            assert bits_equal(cut(a), b)
    assert covered == (18, 40)[axis]
