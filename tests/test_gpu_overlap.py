"""Overlap mode (of3d_plan_set_overlap): the output planes in z chunks, the gradient stages
of chunk c+1 on the caller's stream beside K34 + K5 of chunk c on the plan's second
stream.  Every output bit-identical to the serial pipeline and (vx, vy, vz) to the oracle
(oracle/cpu_ref.py, pinned to the reference's calc_flow3D, calc_flow.py:175-360), for
whole volumes and for z sub-ranges (the z-slab path), chunk sizes that divide the range
and ones that leave a ragged last chunk, and chunks thinner than the W-z halo."""
import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import _lib, make_taps, radii
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _run_plan(img, s, t, w, chunk, z0=0, z1=None, mode=0, timing_stage=None):
    import torch

    dev = torch.device("cuda", 0)
    nt, nz, ny, nx = img.shape
    z1 = nz if z1 is None else z1
    rt = radii(s, t, w)[2]
    c = nt // 2
    d_in = torch.from_numpy(np.ascontiguousarray(img[c - rt:c + rt + 1]).view(np.int16)).to(dev)
    fp32 = bool(mode & _lib.OF3D_FP32)
    vt = torch.float32 if fp32 else torch.float64
    n = (z1 - z0) * ny * nx
    outs = [torch.full((n,), float("nan"), dtype=vt, device=dev) for _ in range(3)]
    rel = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
    plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=0, mode=mode, timing=4 if timing_stage else 0)
    try:
        plan.set_overlap(chunk)
        if timing_stage:
            plan.set_timing_stages([timing_stage])
        plan.execute([d_in[i].data_ptr() for i in range(2 * rt + 1)], _lib.OF3D_U16, 0, z0, z1,
                     outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), rel.data_ptr())
        torch.cuda.synchronize(dev)
        times = plan.stage_times() if timing_stage else None
    finally:
        plan.close()
    shape = (z1 - z0, ny, nx)
    return [o.cpu().numpy().reshape(shape) for o in outs] + [rel.cpu().numpy().reshape(shape)], times


@pytest.mark.parametrize("chunk", [8, 13, 24])
def test_overlap_whole_volume_bitwise(chunk):
    s, t, w = 2, 2, 5
    img = np.random.default_rng(40 + chunk).integers(0, 4096, size=(13, 48, 40, 56)).astype(np.uint16)
    serial, _ = _run_plan(img, s, t, w, 0)
    over, _ = _run_plan(img, s, t, w, chunk)
    for a, b in zip(serial, over):
        assert bits_equal(a, b)
    st = cpu_ref.structure_tensor3d(img, s, t, w, backend="scipy")
    for a, b in zip(over[:3], cpu_ref.solve3d(st)):
        assert bits_equal(a, b)


@pytest.mark.parametrize("z0,z1,chunk", [(10, 38, 8), (0, 20, 6), (30, 48, 5)])
def test_overlap_subrange_bitwise(z0, z1, chunk):
    s, t, w = 2, 3, 7  # c3 parameters: rw 21 > chunk
    img = np.random.default_rng(z0 + z1).integers(0, 4096, size=(19, 48, 36, 44)).astype(np.uint16)
    full, _ = _run_plan(img, s, t, w, 0)
    over, _ = _run_plan(img, s, t, w, chunk, z0, z1)
    for a, b in zip(full, over):
        assert bits_equal(a[z0:z1], b)


def test_overlap_fp32_equals_serial():
    s, t, w = 2, 2, 5
    img = np.random.default_rng(5).integers(0, 4096, size=(13, 40, 32, 64)).astype(np.uint16)
    serial, _ = _run_plan(img, s, t, w, 0, mode=_lib.OF3D_FP32)
    over, _ = _run_plan(img, s, t, w, 10, mode=_lib.OF3D_FP32)
    for a, b in zip(serial, over):
        assert bits_equal(a, b)


def test_overlap_one_stage_timing():
    s, t, w = 2, 2, 5
    img = np.random.default_rng(6).integers(0, 4096, size=(13, 40, 32, 64)).astype(np.uint16)
    out, times = _run_plan(img, s, t, w, 10, timing_stage="prod_wy")
    assert set(times) == {"prod_wy"} and times["prod_wy"] > 0


@pytest.mark.parametrize("chunk", [8, 13])
def test_overlap_with_k12_forced(monkeypatch, chunk):
    """Overlap mode on the fused gradient kernel (K12 forced below its size heuristic: dt0
    lives in Y4 there, the plane ranges of the two streams must still be disjoint): bitwise
    equal to the serial pipeline and to the oracle."""
    monkeypatch.setenv("OF3D_K12", "1")
    s, t, w = 2, 2, 5
    img = np.random.default_rng(70 + chunk).integers(0, 4096, size=(13, 48, 40, 56)).astype(np.uint16)
    serial, _ = _run_plan(img, s, t, w, 0)
    over, _ = _run_plan(img, s, t, w, chunk)
    for a, b in zip(serial, over):
        assert bits_equal(a, b)
    st = cpu_ref.structure_tensor3d(img, s, t, w, backend="scipy")
    for a, b in zip(over[:3], cpu_ref.solve3d(st)):
        assert bits_equal(a, b)


def test_overlap_and_row_range_exclude_each_other():
    """of3d_plan_set_overlap fails on a plan with an output row range, and set_rows on a
    chunked plan (the combination is not implemented)."""
    plan = _lib.Plan(3, 24, 40, 48, make_taps(2, 2, 5), device=0)
    try:
        plan.set_rows(5, 30)
        with pytest.raises(RuntimeError, match="row range"):
            plan.set_overlap(8)
        plan.set_rows(0, 40)
        plan.set_overlap(8)
        with pytest.raises(RuntimeError):
            plan.set_rows(5, 30)
    finally:
        plan.close()


@pytest.mark.parametrize("chunk", [8, 13])
def test_overlap_z_tiled_bitwise(chunk, monkeypatch):
    """Overlap mode with the z-tiled W-xy hand-off forced (OF3D_WXY_TILE=1, nx 64): every chunk's
    K34 writes its planes 32 elements per plane into the tiles (csrc/of3d_host.hip k34 lambda) and
    K5c reads them back — bit-identical to the serial pipeline in plain planes."""
    s, t, w = 2, 2, 5
    img = np.random.default_rng(70 + chunk).integers(0, 4096, size=(13, 48, 40, 64)).astype(np.uint16)
    monkeypatch.setenv("OF3D_WXY_TILE", "0")
    serial, _ = _run_plan(img, s, t, w, 0)
    monkeypatch.setenv("OF3D_WXY_TILE", "1")
    over, _ = _run_plan(img, s, t, w, chunk)
    sub, _ = _run_plan(img, s, t, w, chunk, z0=10, z1=38)
    for a, b, c in zip(serial, over, sub):
        assert bits_equal(a, b)
        assert bits_equal(a[10:38], c)
