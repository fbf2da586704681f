"""§8f rank 4: downstream statistics on device outputs vs the notebook's
numpy cells (oracle.cpu_ref.analysis_reference): threshold, masked
velocities and magnitude bitwise (NaN positions included); theta/phi within
a few ulp (device atan/atan2 vs the host libm)."""
import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import calc_flow2D, calc_flow3D
from opticalflow3d_dev_amd.analysis import flow_statistics
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _ulps(a, b):
    ok = np.isnan(a) == np.isnan(b)
    a, b = a[~np.isnan(a)], b[~np.isnan(b)]
    return ok.all(), (np.abs(a - b) / np.maximum(np.spacing(np.abs(b)), 1e-300)).max() if a.size else 0.0


@pytest.mark.parametrize("pct", [90, 50, 99.5])
def test_stats_3d_match_notebook(pct):
    img = np.random.default_rng(3).integers(0, 4096, size=(7, 8, 30, 34)).astype(np.uint16)
    vx, vy, vz, rel = calc_flow3D(img, 1, 1, 2)
    vx[0, 0, :3] = 0.0  # exact zeros become NaN too
    ref = cpu_ref.analysis_reference(vx.copy(), vy.copy(), vz.copy(), rel, pct, 0.065, 0.2, 0.75)
    got = flow_statistics(vx, vy, vz, rel, pct, 0.065, 0.2, 0.75)
    assert got["threshold"] == ref["threshold"] and got["threshold"].dtype == ref["threshold"].dtype
    for k in ("vx", "vy", "vz", "magnitude"):
        assert bits_equal(got[k], ref[k]), k
    for k in ("theta", "phi"):
        same_nan, u = _ulps(got[k], ref[k])
        assert same_nan and u <= 4, (k, u)


def test_stats_2d_and_resident_tensors():
    import torch

    img = np.random.default_rng(4).integers(0, 4096, size=(7, 40, 44)).astype(np.uint16)
    vx, vy, rel = calc_flow2D(img, 1, 1, 2)
    ref = cpu_ref.analysis_reference(vx.copy(), vy.copy(), None, rel, 90)
    dev = [torch.from_numpy(a).cuda() for a in (vx, vy, rel)]
    got = flow_statistics(dev[0], dev[1], None, dev[2], 90)
    assert got["vx"].is_cuda and "phi" not in got
    assert got["threshold"] == ref["threshold"]
    for k in ("vx", "vy", "magnitude"):
        assert bits_equal(got[k].cpu().numpy(), ref[k]), k
