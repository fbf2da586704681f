import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libof3d.so on the device)")


def _gpu_count():
    """Devices the HIP library sees; 0 without a GPU.  On a machine WITH a GPU (/dev/kfd) a
    library that does not load (missing, stale sources, wrong arch) is an error, never a skip:
    the GPU tests must run through libof3d.so or fail."""
    try:
        from opticalflow3d_dev_amd import _lib
        return _lib.load().of3d_device_count()
    except Exception as e:
        if os.path.exists("/dev/kfd"):
            raise pytest.UsageError(f"GPU present but libof3d.so does not load: {e}") from e
        return 0


def pytest_collection_modifyitems(config, items):
    if any("gpu" in item.keywords for item in items):
        if _gpu_count() == 0:
            skip = pytest.mark.skip(reason="no HIP device visible")
            for item in items:
                if "gpu" in item.keywords:
                    item.add_marker(skip)


def golden_cases(prefix=""):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    out = {k: d[k] for k in d.files}
    s, t, w = (float(v) for v in out["params"])
    norm = lambda v: int(v) if v == int(v) else v
    out["sig"], out["tsig"], out["wsig"] = norm(s), norm(t), norm(w)
    out["taps"] = {k[5:]: out[k] for k in out if k.startswith("taps_")}
    return out


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def oracle3d(images, s, t, w):
    """The oracle's vx, vy, vz and the fp64 eigenvalue range of its tensor
    (the CPU restatement, scipy backend — tests only)."""
    from oracle import cpu_ref

    st = cpu_ref.structure_tensor3d(images, s, t, w, backend="scipy")
    vx, vy, vz = cpu_ref.solve3d(st)
    lmin, lmax = cpu_ref.eig_fp64_3d(st)
    return vx, vy, vz, lmin, lmax


def assert_rel_within(rel, lmin, lmax, tol):
    """|rel - lambda_min| <= tol * |lambda_max| per voxel."""
    err = np.abs(np.asarray(rel, np.float64) - lmin)
    bad = err > tol * np.abs(lmax) + 1e-300
    assert not bad.any(), f"{bad.sum()} voxels: max err/lmax {np.max(err / (np.abs(lmax) + 1e-300)):.3e}"


def assert_flow3d_matches_oracle(out, images, s, t, w, rel_tol=1e-6):
    """vx, vy, vz bit-identical to the oracle, rel within rel_tol * lambda_max."""
    vx, vy, vz, lmin, lmax = oracle3d(images, s, t, w)
    for got, want, name in zip(out[:3], (vx, vy, vz), ("vx", "vy", "vz")):
        assert bits_equal(np.asarray(got, np.float64).reshape(want.shape), want), name
    assert_rel_within(np.asarray(out[3]).reshape(lmin.shape), lmin, lmax, rel_tol)
