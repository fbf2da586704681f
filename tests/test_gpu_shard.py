"""z-slab decomposition on the device (virtual ranks on one GPU): concatenated
slabs are bit-identical to the unsharded calc_flow3D, including slabs thinner
than the stencil halo; the C-ABI's input range equals shard.halo_planes."""
import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import _lib, calc_flow3D, make_taps, radii
from opticalflow3d_dev_amd.shard import flow3d_zslabs_host, halo_planes, zslab_bounds

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_zslabs_bitwise_equal_full(world):
    img = np.random.default_rng(world).integers(0, 4096, size=(13, 24, 40, 36)).astype(np.uint16)
    full = calc_flow3D(img, 2, 2, 5)
    got = flow3d_zslabs_host(img, 2, 2, 5, world)
    for a, b in zip(full, got):
        assert bits_equal(a, b.astype(a.dtype))


def test_plan_input_range_matches_python():
    s, t, w = 2, 2, 5
    rd, rs, rt, rw = radii(s, t, w)
    plan = _lib.Plan(3, 64, 16, 16, make_taps(s, t, w))
    for world in (2, 3, 8):
        for r in range(world):
            z0, z1 = zslab_bounds(64, r, world)
            assert plan.input_range(z0, z1) == halo_planes(64, z0, z1, rd, rw)
    plan.close()
