"""K0 batching (of3d_plan_execute_ahead): one pass over 2rt+M frames forms the temporal
derivatives (calc_flow.py:276-277) of M consecutive windows of a series, and the later calls
for exactly those windows skip their K0.  Every output must equal of3d_plan_execute's bit for
bit, whatever the call sequence: a series with 0..3 frames of lookahead, windows out of order,
a plain call in between (drops the batch), the series' end, fp32 / REL_F64 plans, and the
streaming driver (FlowStream(k0_batch=M)) against the host entry point."""
import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import _lib, calc_flow3D, make_taps, radii

pytestmark = pytest.mark.gpu

NZ, NY, NX = 24, 40, 48  # nx a multiple of 8: the fused gradient kernel's 16-byte rows


@pytest.fixture(autouse=True)
def _k12(monkeypatch):
    # batching rides on the fused gradient kernel's workspace layout; force it at test sizes
    monkeypatch.setenv("OF3D_K12", "1")


def _series(nt, s, t, w, seed, shape=(NZ, NY, NX)):
    import torch

    stack = np.random.default_rng(seed).integers(0, 4096, size=(nt,) + shape).astype(np.uint16)
    frames = [torch.from_numpy(stack[i].view(np.int16)).to("cuda") for i in range(nt)]
    return stack, frames


def _call(plan, frames, k, nwin, n_ahead, vt, reld, plain=False):
    """Window k (frames k .. k+nwin-1) with n_ahead frames of lookahead (None: plain execute)."""
    import torch

    n = NZ * NY * NX
    outs = [torch.full((n,), float("nan"), dtype=vt, device="cuda") for _ in range(3)]
    outs.append(torch.full((n,), float("nan"), dtype=reld, device="cuda"))
    ptrs = [f.data_ptr() for f in frames[k:k + nwin]]
    ahead = None if plain else [f.data_ptr() for f in frames[k + nwin:k + nwin + n_ahead]]
    plan.execute(ptrs, _lib.OF3D_U16, 0, 0, NZ, *[o.data_ptr() for o in outs], ahead_ptrs=ahead)
    torch.cuda.synchronize()
    return [o.cpu().numpy().reshape(NZ, NY, NX) for o in outs]


@pytest.mark.parametrize("sig,mode,m", [((2, 2, 5), 0, 4), ((2, 3, 7), 0, 4), ((2, 3, 7), 0, 2), ((2, 3, 7), 0, 5),
                                        ((2, 2, 5), _lib.OF3D_FP32, 5),
                                        ((2, 2, 5), _lib.OF3D_FP32, 4), ((2, 3, 7), _lib.OF3D_REL_F64, 3)])
def test_series_batched_equals_plain(sig, mode, m):
    import torch

    s, t, w = sig
    nwin = 2 * radii(s, t, w)[2] + 1
    nt = nwin + 7  # 8 windows: two batches of 4 (or 4 of 2), the last ones short of lookahead
    stack, frames = _series(nt, s, t, w, 11)
    vt = torch.float32 if mode & _lib.OF3D_FP32 else torch.float64
    reld = torch.float64 if mode & _lib.OF3D_REL_F64 else torch.float32
    plan = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0, mode=mode)
    ref = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0, mode=mode)
    try:
        for k in range(nt - nwin + 1):
            got = _call(plan, frames, k, nwin, min(m - 1, nt - nwin - k), vt, reld)
            want = _call(ref, frames, k, nwin, 0, vt, reld, plain=True)
            for a, b in zip(got, want):
                assert bits_equal(a, b), k
            if mode == 0 and k in (0, 5):
                for a, b in zip(got, calc_flow3D(stack[k:k + nwin], s, t, w)):
                    assert bits_equal(a, b), k
        assert "k_tderiv_multi" in plan.kernels(), plan.kernels()
    finally:
        plan.close()
        ref.close()


@pytest.mark.parametrize("env", [{"OF3D_K34": "0"}, {"OF3D_ZCHUNK": "8"}, {"OF3D_GENERAL": "1"}])
def test_batching_off_paths(env, monkeypatch):
    """Plans whose workspace or schedule cannot hold the batch (K3 + K4 instead of the fused W
    kernel: W-xy lands on the slots; overlap chunks; the general-radius path) ignore the
    lookahead and stay exact."""
    import torch

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s, t, w = 2, 2, 5
    nwin = 2 * radii(s, t, w)[2] + 1
    stack, frames = _series(nwin + 4, s, t, w, 16)
    plan = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0)
    try:
        for k in range(5):
            got = _call(plan, frames, k, nwin, min(3, 4 - k), torch.float64, torch.float32)
            for a, b in zip(got, calc_flow3D(stack[k:k + nwin], s, t, w)):
                assert bits_equal(a, b), (env, k)
        assert "k_tderiv_multi" not in plan.kernels(), plan.kernels()
    finally:
        plan.close()


def test_out_of_order_and_plain_calls():
    """Batched windows used out of order, a plain call dropping the batch, a window whose
    frames are not the batch's (other pointers), the same window twice: all exact."""
    import torch

    s, t, w = 2, 2, 5
    nwin = 2 * radii(s, t, w)[2] + 1
    nt = nwin + 8
    stack, frames = _series(nt, s, t, w, 12)
    plan = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0)
    seq = [(0, 3, False), (2, 0, False), (1, 0, False), (1, 0, False), (4, 3, False), (5, 0, True), (6, 0, False),
           (3, 1, False), (8, 0, False), (7, 1, False), (8, 0, False)]
    try:
        for k, na, plain in seq:
            got = _call(plan, frames, k, nwin, na, torch.float64, torch.float32, plain=plain)
            for a, b in zip(got, calc_flow3D(stack[k:k + nwin], s, t, w)):
                assert bits_equal(a, b), (k, na, plain)
    finally:
        plan.close()


def test_copied_window_not_matched():
    """The same frame CONTENTS at other addresses are another window: recomputed, and equal."""
    import torch

    s, t, w = 2, 2, 5
    nwin = 2 * radii(s, t, w)[2] + 1
    stack, frames = _series(nwin + 3, s, t, w, 13)
    copies = [f.clone() for f in frames]
    plan = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0)
    try:
        _call(plan, frames, 0, nwin, 3, torch.float64, torch.float32)
        got = _call(plan, copies, 1, nwin, 0, torch.float64, torch.float32)
        for a, b in zip(got, calc_flow3D(stack[1:1 + nwin], s, t, w)):
            assert bits_equal(a, b)
    finally:
        plan.close()


@pytest.mark.parametrize("m", [2, 4, 5])
def test_flowstream_k0_batch(m):
    """The streaming driver with K0 batching: every output equals calc_flow3D of its window."""
    from opticalflow3d_dev_amd.stream import FlowStream

    s, t, w = 2, 2, 5
    nwin = 13
    stack = np.random.default_rng(14).integers(0, 3000, size=(nwin + 9, NZ, NY, NX)).astype(np.uint16)
    fs = FlowStream(3, stack.shape[1:], np.uint16, s, t, w, depth=2, k0_batch=m)
    try:
        assert fs.lookahead == m - 1
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
        assert "k_tderiv_multi" in fs.plan.kernels(), fs.plan.kernels()
    finally:
        fs.close()


def test_process_flow_k0_batched(tmp_path, capsys):
    """process_flow (calc_flow.py:362-625) through the batched K0: a OneTif series with 8
    output frames, the driver pushing 3 frames of lookahead; every output TIFF equals the host
    entry point's calc_flow3D of its window bit for bit (rel included)."""
    from opticalflow3d_dev_amd import process_flow
    from opticalflow3d_dev_amd import tiff as tf

    s, t, w = 2, 1, 3
    nwin = 2 * radii(s, t, w)[2] + 1
    stack = np.random.default_rng(15).integers(0, 4096, size=(nwin + 7, NZ, NY, NX)).astype(np.uint16)
    tf.imwrite(tmp_path / "b.tif", stack, imagej=True)
    process_flow(str(tmp_path), "b", "OneTif", 3, s, t, w)
    out = tmp_path / "OpticalFlow3D" / "b"
    h = nwin // 2
    for k in range(stack.shape[0] - nwin + 1):
        got = [tf.imread(out / f"b_{n}_t{k + h:04d}.tiff") for n in ("vx", "vy", "vz", "rel")]
        for a, b in zip(got, calc_flow3D(stack[k:k + nwin], s, t, w)):
            assert bits_equal(a, b), k
    assert capsys.readouterr().out.count("saved.  Duration") == stack.shape[0] - nwin + 1


@pytest.mark.parametrize("room,want", [(None, (3, 5, 4)), ("one_set_batch2", (1, 2, 1)), ("one_set_plain", (1, 0, 0))])
def test_flowstream_fits_device_memory(room, want, monkeypatch):
    """With little device memory left the stream keeps fewer output sets in flight, then less
    lookahead (K0 batching 5 -> 2 -> none), and stays exact."""
    import torch

    from opticalflow3d_dev_amd.stream import FlowStream

    s, t, w = 2, 2, 5
    nwin = 13
    vox = NZ * NY * NX
    slot, oset = vox * 2, vox * (3 * 8 + 4)
    if room is not None:
        extra = {"one_set_batch2": 1, "one_set_plain": 0}[room]
        fake = (1 << 30) + slot * (nwin + 1 + extra) + oset + 1024
        real = torch.cuda.mem_get_info
        monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (fake, real(dev)[1]))
    stack = np.random.default_rng(17).integers(0, 3000, size=(nwin + 5, NZ, NY, NX)).astype(np.uint16)
    fs = FlowStream(3, stack.shape[1:], np.uint16, s, t, w, depth=3)
    try:
        assert (fs.depth, fs.batch, fs.L) == want
        k = 0
        for i in range(stack.shape[0]):
            fs.push(stack[i])
            while len(fs.order) >= fs.nwin + fs.L or (i == stack.shape[0] - 1 and fs.ready):
                p = fs.submit()
                for a, b in zip(p.result(), calc_flow3D(stack[k:k + nwin], s, t, w)):
                    assert bits_equal(a, b), k
                p.release()
                k += 1
        assert k == stack.shape[0] - nwin + 1
    finally:
        fs.close()


@pytest.mark.parametrize("z0,z1", [(0, 14), (10, 24), (6, 18)])
def test_zslab_subrange_batched(z0, z1):
    """A z-slab plan (outputs [z0, z1), frames holding only the halo planes, frame_z0 = zi0) as
    the slab bench runs it: a series through the batched K0 equals the same planes of the
    whole-volume result."""
    import torch

    s, t, w = 2, 2, 5
    rd, rs, rt, rw = radii(s, t, w)
    nwin = 2 * rt + 1
    stack = np.random.default_rng(18).integers(0, 4096, size=(nwin + 5, NZ, NY, NX)).astype(np.uint16)
    zi0, zi1 = max(z0 - rd - rw, 0), min(z1 + rd + rw, NZ)
    frames = [torch.from_numpy(np.ascontiguousarray(stack[i, zi0:zi1]).view(np.int16)).to("cuda")
              for i in range(stack.shape[0])]
    plan = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0, max_out_planes=z1 - z0)
    try:
        n = (z1 - z0) * NY * NX
        for k in range(stack.shape[0] - nwin + 1):
            outs = [torch.full((n,), float("nan"), dtype=torch.float64, device="cuda") for _ in range(3)]
            outs.append(torch.full((n,), float("nan"), dtype=torch.float32, device="cuda"))
            ptrs = [f.data_ptr() for f in frames[k:k + nwin]]
            ahead = [f.data_ptr() for f in frames[k + nwin:k + nwin + 3]]
            plan.execute(ptrs, _lib.OF3D_U16, zi0, z0, z1, *[o.data_ptr() for o in outs], ahead_ptrs=ahead)
            torch.cuda.synchronize()
            full = calc_flow3D(stack[k:k + nwin], s, t, w)
            for a, b in zip(outs, full):
                assert bits_equal(a.cpu().numpy().reshape(z1 - z0, NY, NX), b[z0:z1]), (k, z0, z1)
        assert "k_tderiv_multi" in plan.kernels(), plan.kernels()
    finally:
        plan.close()


@pytest.mark.parametrize("tsig", [10.5, 1.5])
def test_flowstream_unbatchable_radius(tsig):
    """Temporal radii without a batched K0 (rt 32 = tSig 10.5: a 65-frame window, the plan's
    whole frame table; rt 5 = tSig 1.5: no k_tderiv_multi instance): the stream holds no
    lookahead and runs the plain K0, every output equal to calc_flow3D of its window."""
    from opticalflow3d_dev_amd.stream import FlowStream

    s, w = 1, 2
    shape = (6, 20, 24)
    rt = radii(s, tsig, w)[2]
    nwin = 2 * rt + 1
    stack = np.random.default_rng(19).integers(0, 3000, size=(nwin + 2,) + shape).astype(np.uint16)
    fs = FlowStream(3, shape, np.uint16, s, tsig, w, depth=1)
    try:
        assert fs.batch == 0 and fs.L == 0, (fs.batch, fs.L)
        k = 0
        for i in range(stack.shape[0]):
            fs.push(stack[i])
            while len(fs.order) >= fs.nwin + fs.L or (i == stack.shape[0] - 1 and fs.ready):
                p = fs.submit()
                for a, b in zip(p.result(), calc_flow3D(stack[k:k + nwin], s, tsig, w)):
                    assert bits_equal(a, b), k
                p.release()
                k += 1
        assert k == 3
        assert "k_tderiv_multi" not in fs.plan.kernels()
    finally:
        fs.close()


def test_execute_ahead_clamps_past_frame_table():
    """of3d_plan_execute_ahead with more lookahead than the 65-frame table holds: clamped, not
    an error (rt 30: a 61-frame window leaves 4 frames of lookahead), and exact."""
    import torch

    s, t, w = 1, 10, 2
    rt = radii(s, t, w)[2]
    nwin = 2 * rt + 1
    stack, frames = _series(nwin + 6, s, t, w, 20, shape=(NZ, NY, NX))
    plan = _lib.Plan(3, NZ, NY, NX, make_taps(s, t, w), device=0)
    try:
        got = _call(plan, frames, 0, nwin, 6, torch.float64, torch.float32)
        for a, b in zip(got, calc_flow3D(stack[:nwin], s, t, w)):
            assert bits_equal(a, b)
    finally:
        plan.close()
