"""The device's smallest-eigenvalue formula (csrc/of3d_dev.hpp eigmin3 / eigmin3_deflate),
restated in numpy by tools/eig_poly.py, against fp64 eigvalsh — CPU only.

3D rel is LAPACK cgeev in complex64 in the reference (calc_flow.py:352-357) and double
pageeig in MATLAB (M/calc_flow3D.m:235-236).  The fp64-rel instances (OF3D_REL_F64, MATLAB
mode) must meet SURVEY §8(c)'s 1e-10 lambda_max against fp64 eigvalsh everywhere, including
near-degenerate smallest pairs, where the trigonometric form alone loses ~sqrt(eps).  The
device itself is checked on the same sets through of3d_rel3d (tests/test_gpu_parity.py)."""
import os
import sys

import numpy as np
import pytest

from conftest import REPO, golden_cases, load_golden
from oracle import cpu_ref

sys.path.insert(0, os.path.join(REPO, "tools"))
import eig_poly  # noqa: E402

TOL_FP64 = 1e-10


@pytest.fixture(scope="module")
def coef():
    return eig_poly.coefficients()


@pytest.mark.parametrize("psd", [False, True])
def test_refined_formula_meets_fp64_tolerance(coef, psd):
    args, ref = eig_poly.test_set(n=120000, seed=3, psd=psd)
    lmax = np.abs(ref).max(axis=1)
    err = np.abs(eig_poly.eigmin3(*args, m=coef, refine=True) - ref[:, 0]) / lmax
    assert err.max() <= 1e-12, err.max()
    # the float32-rel instances keep the plain form: far inside their 1e-6 lambda_max
    err32 = np.abs(eig_poly.eigmin3(*args, m=coef) - ref[:, 0]) / lmax
    assert err32.max() <= 1e-7, err32.max()
    # ... which alone would miss the fp64 tolerance on these sets (why the refinement exists)
    assert err32.max() > TOL_FP64


def test_refined_formula_extreme_magnitudes(coef):
    """Tensors of magnitude 1e-100 and 1e100 (every hard set): the deflation works on the
    scaled matrix, so nothing under- or overflows — still 1e-12 lambda_max, no NaN."""
    args, ref = eig_poly.test_set(n=60000, seed=11, extreme=True)
    lmax = np.abs(ref).max(axis=1)
    got = eig_poly.eigmin3(*args, m=coef, refine=True)
    assert np.isfinite(got).all()
    err = np.abs(got - ref[:, 0]) / lmax
    assert err.max() <= 1e-12, err.max()


def test_polynomial_matches_acos(coef):
    u = np.linspace(0, 1, 100001)
    assert np.abs(eig_poly.horner(coef, 2 * u - 1) - np.cos(2 / 3 * np.arccos(u))).max() < 5e-15


@pytest.mark.parametrize("name", [c for c in golden_cases("c3d") if c in (
    "c3d_ramp_xyz_rank1", "c3d_ramp_xy_planar", "c3d_wave_planar", "c3d_iso_smoothed_noise")])
def test_near_degenerate_fixtures(coef, name):
    """The round-4 fixtures' tensors (the oracle's, bitwise the device's): the refined formula
    within 1e-10 lambda_max of the fixture's eigvalsh; the planar ramp / wave are the cases where
    the plain form is not."""
    g = load_golden(name)
    st = cpu_ref.structure_tensor3d(g["images"], g["sig"], g["tsig"], g["wsig"], backend="scipy")
    T = cpu_ref.tensor_stack3d(st)
    args = (T[..., 0, 0], T[..., 1, 1], T[..., 2, 2], T[..., 0, 1], T[..., 0, 2], T[..., 1, 2])
    lmax = np.abs(g["lmax64"])
    err = np.abs(eig_poly.eigmin3(*args, m=coef, refine=True) - g["lmin64"]) / lmax
    assert err.max() <= TOL_FP64 * 1e-2, err.max()
    if name in ("c3d_ramp_xy_planar", "c3d_wave_planar"):
        plain = np.abs(eig_poly.eigmin3(*args, m=coef) - g["lmin64"]) / lmax
        assert plain.max() > TOL_FP64
