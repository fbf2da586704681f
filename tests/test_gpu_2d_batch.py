"""2D plans over a batch of output frames (of3d_plan_create(ndim=2, nz=B)): plane b of the plan is
output frame b, and the 2rt+1 frame pointers are the series shifted by 0 .. 2rt frames (plane b of
frame j = series frame b + j, the window of output b).  Every output frame against the oracle
(oracle/cpu_ref.py calc_flow2D, pinned to the reference's calc_flow.py:18-173) and against the
one-frame host entry, bitwise (vx, vy, rel); fp32 within 1e-4 of the fp64 oracle; a sub-range of
the batch; the general-radius path (OF3D_GENERAL=1)."""
import os

import numpy as np
import pytest

from opticalflow3d_dev_amd import _lib, calc_flow2D, make_taps, radii
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _batch(series, s, t, w, zo0=None, zo1=None, mode=0):
    import torch

    rt = radii(s, t, w)[2]
    nwin = 2 * rt + 1
    nt, ny, nx = series.shape
    nout = nt - nwin + 1
    zo0 = 0 if zo0 is None else zo0
    zo1 = nout if zo1 is None else zo1
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(np.ascontiguousarray(series).view(np.int16)).to(dev)
    fp32 = bool(mode & _lib.OF3D_FP32)
    vt = torch.float32 if fp32 else torch.float64
    n = (zo1 - zo0) * ny * nx
    vx, vy, rel = (torch.empty(n, dtype=vt, device=dev) for _ in range(3))
    plan = _lib.Plan(2, nout, ny, nx, make_taps(s, t, w), device=0, mode=mode)
    try:
        plan.execute([d_in[j].data_ptr() for j in range(nwin)], _lib.OF3D_U16, 0, zo0, zo1, vx.data_ptr(),
                     vy.data_ptr(), 0, rel.data_ptr())
        torch.cuda.synchronize(dev)
        kernels = plan.kernels()
    finally:
        plan.close()
    return [o.view(zo1 - zo0, ny, nx).cpu().numpy() for o in (vx, vy, rel)], kernels, nwin


def _same(a, b):
    return a.dtype == b.dtype and np.array_equal(a.view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.parametrize("sig", [(1, 1, 5), (2, 1, 4), (3, 2, 3)])
def test_batch_plan_vs_oracle_and_host_entry(sig):
    s, t, w = sig
    series = np.random.default_rng(1200 + s).integers(0, 4096, size=(16, 72, 96)).astype(np.uint16)
    outs, kernels, nwin = _batch(series, s, t, w)
    assert "k_solve2d" in kernels, kernels
    for j in range(series.shape[0] - nwin + 1):
        want = cpu_ref.calc_flow2D(series[j:j + nwin], s, t, w, backend="scipy")
        host = calc_flow2D(series[j:j + nwin], s, t, w)
        for o, a, b, name in zip(outs, want, host, ("vx", "vy", "rel")):
            assert _same(o[j], a), (sig, j, name)
            assert _same(o[j], b), (sig, j, name)


def test_batch_plan_sub_range():
    s, t, w = 1, 1, 5
    series = np.random.default_rng(1300).integers(0, 4096, size=(16, 64, 80)).astype(np.uint16)
    full, _, nwin = _batch(series, s, t, w)
    part, _, _ = _batch(series, s, t, w, zo0=3, zo1=7)
    for a, b in zip(full, part):
        assert _same(b, a[3:7])


def test_batch_plan_fp32():
    s, t, w = 1, 1, 5
    series = np.random.default_rng(1400).integers(0, 4096, size=(14, 64, 80)).astype(np.uint16)
    outs, _, nwin = _batch(series, s, t, w, mode=_lib.OF3D_FP32)
    for j in range(series.shape[0] - nwin + 1):
        want = cpu_ref.calc_flow2D(series[j:j + nwin], s, t, w, backend="scipy")
        for o, a in zip(outs[:2], want[:2]):
            fin = np.isfinite(a)
            assert np.array_equal(fin, np.isfinite(o[j]))
            assert np.max(np.abs(o[j][fin] - a[fin])) <= 1e-4 * max(np.max(np.abs(a[fin])), 1e-30)


def test_batch_plan_general_path():
    s, t, w = 1, 1, 5
    series = np.random.default_rng(1500).integers(0, 4096, size=(12, 48, 64)).astype(np.uint16)
    ref, _, nwin = _batch(series, s, t, w)
    os.environ["OF3D_GENERAL"] = "1"
    try:
        gen, kernels, _ = _batch(series, s, t, w)
    finally:
        del os.environ["OF3D_GENERAL"]
    assert "general" in kernels, kernels
    for a, b in zip(ref, gen):
        assert _same(b, a)


def test_c1_full_series_batch_plan_vs_oracle():
    """configs[0] exactly as bench.py --config c1 times it: a 16-frame 256 x 256 series (the bench's
    synthetic family and seed), xySig 1, tSig 1, wSig 5 — one 2D plan of 10 planes over the series
    shifted by 0 .. 6 frames, so plane b is output frame b — then every one of the 10 output frames
    bitwise (vx, vy, rel) against the oracle's calc_flow2D of its own 7-frame window."""
    import torch

    import bench

    s, t, w = 1, 1, 5
    nt, ny, nx = 16, 256, 256
    dev = torch.device("cuda", 0)
    series = bench.synthetic_slab(nt, 1, ny, nx, 0, 1, 20260206 + 1, dev).view(nt, ny, nx).cpu().numpy()
    series = series.view(np.uint16)
    outs, kernels, nwin = _batch(series, s, t, w)
    assert nwin == 7 and outs[0].shape == (nt - nwin + 1, ny, nx)
    assert "k_solve2d" in kernels, kernels
    for j in range(nt - nwin + 1):
        want = cpu_ref.calc_flow2D(series[j:j + nwin], s, t, w, backend="scipy")
        for o, a, name in zip(outs, want, ("vx", "vy", "rel")):
            assert _same(o[j], a), (j, name)
