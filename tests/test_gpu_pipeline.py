"""Frame pipelining (of3d_plan_execute_next): a call's W-z/solve kernel also forms the NEXT
output frame's temporal derivative (calc_flow.py:276-277), and the next call for exactly those
frames skips its own K0 launch.  Every output must equal of3d_plan_execute's bit for bit (the
same K0 arithmetic), whatever the call sequence: a series, a break in the series (other
frames next), the last frame (no lookahead), z-slab sub-ranges, fp32 plans, and the
streaming driver's lookahead ring (stream.FlowStream) against the host entry point."""
import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import _lib, calc_flow3D, make_taps, radii

pytestmark = pytest.mark.gpu


def _windows(stack, rt):
    nt = stack.shape[0]
    return [stack[k:k + 2 * rt + 1] for k in range(nt - 2 * rt)]


def _run(plan, dev_frames, z0, z1, nvox_shape, vt, calls, rt_dtype=None):
    """calls: list of (window index, next window index or None, pipelined) -> outputs per call."""
    import torch

    res = []
    for w, nw, pipe in calls:
        n = int(np.prod(nvox_shape))
        outs = [torch.full((n,), float("nan"), dtype=vt, device="cuda") for _ in range(3)]
        outs.append(torch.full((n,), float("nan"), dtype=rt_dtype or torch.float32, device="cuda"))
        ptrs = [f.data_ptr() for f in dev_frames[w]]
        nxt = [f.data_ptr() for f in dev_frames[nw]] if nw is not None else None
        plan.execute(ptrs, _lib.OF3D_U16, 0 if z0 is None else z0[0], z1[0], z1[1],
                     *[o.data_ptr() for o in outs], next_ptrs=nxt, pipelined=pipe)
        torch.cuda.synchronize()
        res.append([o.cpu().numpy().reshape(nvox_shape) for o in outs])
    return res


def _series(shape, s, t, w, seed):
    import torch

    rt = radii(s, t, w)[2]
    stack = np.random.default_rng(seed).integers(0, 4096, size=shape).astype(np.uint16)
    frames = [torch.from_numpy(stack[i].view(np.int16)).to("cuda") for i in range(shape[0])]
    wins = [[frames[k + i] for i in range(2 * rt + 1)] for k in range(shape[0] - 2 * rt)]
    return stack, wins, rt


@pytest.mark.parametrize("sig,mode", [((2, 2, 5), 0), ((2, 3, 7), 0), ((2, 2, 5), _lib.OF3D_FP32),
                                      ((2, 3, 7), _lib.OF3D_REL_F64)])
def test_series_pipelined_equals_plain(sig, mode):
    import torch

    s, t, w = sig
    rt = radii(s, t, w)[2]
    nt = 2 * rt + 1 + 3
    stack, wins, rt = _series((nt, 24, 40, 48), s, t, w, 3)
    nz = 24
    vt = torch.float32 if mode & _lib.OF3D_FP32 else torch.float64
    reld = torch.float64 if mode & _lib.OF3D_REL_F64 else torch.float32
    plan = _lib.Plan(3, nz, 40, 48, make_taps(s, t, w), device=0, mode=mode)
    plain_plan = _lib.Plan(3, nz, 40, 48, make_taps(s, t, w), device=0, mode=mode)
    try:
        calls = [(k, k + 1 if k + 1 < len(wins) else None, True) for k in range(len(wins))]
        got = _run(plan, wins, None, (0, nz), (nz, 40, 48), vt, calls, reld)
        assert "k_wz_solve_c_next" in plan.kernels(), plan.kernels()
        want = _run(plain_plan, wins, None, (0, nz), (nz, 40, 48), vt, [(k, None, False) for k in range(len(wins))],
                    reld)
        for k, (g, wv) in enumerate(zip(got, want)):
            for a, b in zip(g, wv):
                assert bits_equal(a, b), k
        if mode == 0:  # and the host entry point (calc_flow3D), rel included
            for k in (0, len(wins) - 1):
                for a, b in zip(got[k], calc_flow3D(stack[k:k + 2 * rt + 1], s, t, w)):
                    assert bits_equal(a, b)
    finally:
        plan.close()
        plain_plan.close()


@pytest.mark.parametrize("env", [{"OF3D_K34": "0"}, {"OF3D_K34": "0", "OF3D_K12": "1"}])
def test_pipelining_off_with_k34_fallback(env, monkeypatch):
    """Without the fused W kernel (K3 + K4: W-xy in Y, where the next dt0 would go) the plan
    does not fuse the next frame's K0 into K5c, and the series stays exact."""
    import torch

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s, t, w = 2, 2, 5
    stack, wins, rt = _series((13 + 3, 16, 32, 40), s, t, w, 6)
    plan = _lib.Plan(3, 16, 32, 40, make_taps(s, t, w), device=0)
    try:
        got = _run(plan, wins, None, (0, 16), (16, 32, 40), torch.float64,
                   [(k, k + 1 if k + 1 < len(wins) else None, True) for k in range(len(wins))])
        for k, g in enumerate(got):
            for a, b in zip(g, calc_flow3D(stack[k:k + 2 * rt + 1], s, t, w)):
                assert bits_equal(a, b), k
        assert "k_wz_solve_c_next" not in plan.kernels(), plan.kernels()
    finally:
        plan.close()


def test_break_in_series_recomputes():
    """execute_next(A, next=B) then a call for other frames (C): the pending dt0 (for B) must
    not be used; then B after C: recomputed too."""
    import torch

    s, t, w = 2, 2, 5
    stack, wins, rt = _series((13 + 4, 16, 32, 40), s, t, w, 5)
    plan = _lib.Plan(3, 16, 32, 40, make_taps(s, t, w), device=0)
    try:
        got = _run(plan, wins, None, (0, 16), (16, 32, 40), torch.float64,
                   [(0, 1, True), (3, None, True), (1, 2, True), (2, None, True), (4, 0, True), (0, None, False)])
        for (k, _, _), g in zip([(0, 1, 1), (3, 0, 0), (1, 0, 0), (2, 0, 0), (4, 0, 0), (0, 0, 0)], got):
            for a, b in zip(g, calc_flow3D(stack[k:k + 2 * rt + 1], s, t, w)):
                assert bits_equal(a, b), k
    finally:
        plan.close()


def test_zslab_subrange_pipelined():
    """A z-slab plan (outputs [z0, z1), frames holding the halo planes): pipelined series equal
    to the same planes of the whole-volume result."""
    import torch

    s, t, w = 2, 2, 5
    rd, rs, rt, rw = radii(s, t, w)
    nz, ny, nx = 40, 24, 32
    stack = np.random.default_rng(8).integers(0, 4096, size=(13 + 2, nz, ny, nx)).astype(np.uint16)
    z0, z1 = 12, 26
    zi0, zi1 = max(z0 - rd - rw, 0), min(z1 + rd + rw, nz)
    frames = [torch.from_numpy(np.ascontiguousarray(stack[i, zi0:zi1]).view(np.int16)).to("cuda")
              for i in range(stack.shape[0])]
    wins = [[frames[k + i] for i in range(2 * rt + 1)] for k in range(3)]
    plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=0, max_out_planes=z1 - z0)
    try:
        got = _run(plan, wins, (zi0,), (z0, z1), (z1 - z0, ny, nx), torch.float64,
                   [(0, 1, True), (1, 2, True), (2, None, True)])
        for k, g in enumerate(got):
            full = calc_flow3D(stack[k:k + 2 * rt + 1], s, t, w)
            for a, b in zip(g, full):
                assert bits_equal(a, b[z0:z1]), k
    finally:
        plan.close()


@pytest.mark.parametrize("lookahead", [True, False])
def test_flowstream_lookahead_ring(lookahead):
    """The streaming driver with one frame of lookahead (push the next window's newest frame
    before submit): every output equals calc_flow3D of its window, rel included."""
    from opticalflow3d_dev_amd.stream import FlowStream

    s, t, w = 1, 2, 5  # (rw, rt) = (15, 6): the fused instance
    nwin = 13
    stack = np.random.default_rng(9).integers(0, 3000, size=(nwin + 7, 6, 20, 24)).astype(np.uint16)
    fs = FlowStream(3, stack.shape[1:], np.uint16, s, t, w, depth=2, lookahead=lookahead)
    try:
        pend, k = [], 0
        for i in range(stack.shape[0]):
            fs.push(stack[i])
            while len(fs.order) >= fs.nwin + fs.L or (i == stack.shape[0] - 1 and fs.ready):
                pend.append((k, fs.submit()))
                k += 1
                if len(pend) == fs.depth:
                    kk, p = pend.pop(0)
                    for a, b in zip(p.result(), calc_flow3D(stack[kk:kk + nwin], s, t, w)):
                        assert bits_equal(a, b), kk
                    p.release()
        for kk, p in pend:
            for a, b in zip(p.result(), calc_flow3D(stack[kk:kk + nwin], s, t, w)):
                assert bits_equal(a, b), kk
            p.release()
        assert k == stack.shape[0] - nwin + 1
        if lookahead:
            assert "k_wz_solve_c_next" in fs.plan.kernels()
    finally:
        fs.close()


@pytest.mark.parametrize("producer_aligned", [True, False])
def test_pipelined_dt0_across_gradient_flows(producer_aligned, monkeypatch):
    """The fused gradient kernel (K12) is chosen per call by the frames' alignment (16-byte
    planes): the dt0 a pipelined call formed lives where ITS flow puts it (Y4 with K12, Y0
    without), so a consumer on the other flow must not take it (of3d_host.hip: pipe_k12) —
    a producer whose window is 16-byte aligned and whose next window sits 8 bytes off (K12 ->
    K1c + K2c), and the reverse: both calls bit-identical to the host entry point."""
    import torch

    monkeypatch.setenv("OF3D_K12", "1")  # K12 wherever the alignment allows, at this size
    s, t, w = 2, 2, 5
    rt = radii(s, t, w)[2]
    nwin = 2 * rt + 1
    shape = (24, 40, 48)
    n = int(np.prod(shape))
    stack = np.random.default_rng(77).integers(0, 4096, size=(nwin + 1,) + shape).astype(np.uint16)

    def frames(k, aligned):
        out = []
        for i in range(nwin):
            buf = torch.empty(n + 8, dtype=torch.int16, device="cuda")
            v = buf[:n] if aligned else buf[4:4 + n]  # 8 bytes off: 8-byte but not 16-byte aligned
            v.copy_(torch.from_numpy(stack[k + i].reshape(-1).view(np.int16)))
            out.append(v)
        return out

    w0, w1 = frames(0, producer_aligned), frames(1, not producer_aligned)
    assert (w0[rt].data_ptr() % 16 == 0) == producer_aligned and (w1[rt].data_ptr() % 16 == 0) != producer_aligned
    plan = _lib.Plan(3, *shape, make_taps(s, t, w), device=0)
    try:
        got = _run(plan, [w0, w1], None, (0, shape[0]), shape, torch.float64, [(0, 1, True), (1, None, True)])
        ks = plan.kernels()
        assert "k_wz_solve_c_next" in ks and "k_grad_xyz_c" in ks and "k_grad_xy_c" in ks, ks
    finally:
        plan.close()
    for k in range(2):
        for a, b in zip(got[k], calc_flow3D(stack[k:k + nwin], s, t, w)):
            assert bits_equal(a, b), (producer_aligned, k)
