"""Oracle pinning (CPU): the NumPy restatement in oracle/cpu_ref.py against the
golden vectors generated from the reference's own calc_flow2D/calc_flow3D
(tests/golden/make_golden.py), and the restated correlate1d against scipy."""
import numpy as np
import pytest
from scipy.ndimage import correlate1d

from conftest import bits_equal, golden_cases, golden_manifest, load_golden
from oracle import cpu_ref


@pytest.mark.parametrize("name", golden_cases("c3d"))
def test_oracle_3d_bitwise(name):
    g = load_golden(name)
    vx, vy, vz, rel = cpu_ref.calc_flow3D(g["images"], g["sig"], g["tsig"], g["wsig"])
    for a, k in ((vx, "vx"), (vy, "vy"), (vz, "vz"), (rel, "rel")):
        assert bits_equal(a, g[k]), k


@pytest.mark.parametrize("name", golden_cases("c2d"))
def test_oracle_2d_bitwise(name):
    g = load_golden(name)
    vx, vy, rel = cpu_ref.calc_flow2D(g["images"], g["sig"], g["tsig"], g["wsig"])
    for a, k in ((vx, "vx"), (vy, "vy"), (rel, "rel")):
        assert bits_equal(a, g[k]), k


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_taps_match_fixture(name):
    g = load_golden(name)
    t = cpu_ref.make_taps(g["sig"], g["tsig"], g["wsig"])
    for k, v in t.items():
        assert bits_equal(v, g["taps"][k]), k


@pytest.mark.parametrize("r", [1, 2, 3, 6, 9, 15, 21])
@pytest.mark.parametrize("axis", [0, 1, 2])
def test_restated_correlate_matches_scipy(r, axis):
    rng = np.random.default_rng(r * 10 + axis)
    a = rng.normal(size=(9, 11, 13)) * 100
    x = np.arange(-r, r + 1)
    sym = np.exp(-x * x / 2 / (r / 3) ** 2)
    anti = sym * x
    for w in (sym, anti):
        ref = correlate1d(a, w, axis=axis, mode="nearest")
        assert bits_equal(cpu_ref.correlate1d_restated(a, w, axis), ref)


def test_oracle_error_messages():
    for name, e in golden_manifest()["_errors"].items():
        fn = cpu_ref.calc_flow3D if e["dims"] == 3 else cpu_ref.calc_flow2D
        with pytest.raises(SystemExit) as ex:
            fn(np.zeros(e["shape"], np.uint16), 1, e["tSig"], 2)
        assert str(ex.value.code) == e["message"], name


def test_rel_fp64_range_consistent():
    """The fp64 eigen range stored in the fixtures brackets the float32 rel."""
    for name in golden_cases("c3d"):
        g = load_golden(name)
        lmax = np.abs(g["lmax64"])
        err = np.abs(g["rel"].astype(np.float64) - g["lmin64"])
        assert np.all(err <= 1e-6 * lmax + 1e-30), name
