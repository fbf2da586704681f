"""fp32 path (OF3D_FP32, configs[4]): float32 filter passes and structure
tensor, fp64 solve.  Checked against the bit-exact fp64 path on smooth
synthetic stacks with the SURVEY §8(c) tolerance max|dv| <= 1e-4 max|v_ref|
(parity of this mode is against our own fp64 path, which is itself bitwise
pinned to the reference's golden vectors)."""
import numpy as np
import pytest

from opticalflow3d_dev_amd import calc_flow2D, calc_flow2D_fp32, calc_flow3D, calc_flow3D_fp32
from opticalflow3d_dev_amd.stream import FlowStream

pytestmark = pytest.mark.gpu


def smooth_stack(nt, shape, seed, vel=(0.3, -0.2, -0.1)):
    rng = np.random.default_rng(seed)
    axes = np.meshgrid(*[np.arange(n, dtype=np.float64) for n in shape], indexing="ij")
    out = np.empty((nt,) + tuple(shape), np.uint16)
    k = rng.uniform(2 * np.pi / 24, 2 * np.pi / 8, size=(3, len(shape)))
    ph = rng.uniform(0, 2 * np.pi, size=(3, len(shape)))
    v = vel[::-1][-len(shape):]  # axis order z, y, x
    for t in range(nt):
        s = np.zeros(shape)
        for q in range(3):
            term = np.ones(shape)
            for a, ax in enumerate(axes):
                term = term * np.sin(k[q, a] * (ax - v[a] * t) + ph[q, a])
            s += term
        out[t] = np.clip(1000 + 300 * s + rng.integers(-2, 3, size=shape), 0, 65535).astype(np.uint16)
    return out


@pytest.mark.parametrize("shape,sig", [((16, 40, 48), (2, 2, 5)), ((12, 32, 36), (1, 1, 3)), ((20, 24, 30), (2, 3, 7))])
def test_fp32_3d_close_to_fp64(shape, sig):
    s, t, w = sig
    img = smooth_stack(6 * t + 1, shape, 11)
    ref = calc_flow3D(img, s, t, w)
    got = calc_flow3D_fp32(img, s, t, w)
    for name, a, b in zip(("vx", "vy", "vz"), ref[:3], got[:3]):
        assert b.dtype == np.float32 and b.shape == a.shape
        err = np.abs(b.astype(np.float64) - a).max()
        assert err <= 1e-4 * np.abs(a).max(), (name, err, np.abs(a).max())
    rel_ref, rel = ref[3].astype(np.float64), got[3].astype(np.float64)
    assert np.abs(rel - rel_ref).max() <= 1e-4 * np.abs(rel_ref).max()


def test_fp32_2d_close_to_fp64():
    img = smooth_stack(7, (64, 72), 3)
    ref = calc_flow2D(img, 1, 1, 5)
    got = calc_flow2D_fp32(img, 1, 1, 5)
    for a, b in zip(ref, got):
        assert b.dtype == np.float32
        assert np.abs(b.astype(np.float64) - a).max() <= 1e-4 * np.abs(a).max()


def test_fp32_stream_matches_oneshot():
    """The ring-buffer driver in fp32 gives the same float32 bits as the one-shot call."""
    img = smooth_stack(9, (10, 24, 28), 5)
    fs = FlowStream(3, img.shape[1:], np.uint16, 1, 1, 3, precision="fp32")
    try:
        for t in range(9):
            fs.push(img[t])
            if fs.ready:
                p = fs.submit()
                k = t - 6
                want = calc_flow3D_fp32(img[k:k + 7], 1, 1, 3)
                for a, b in zip(p.result(), want):
                    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
                p.release()
    finally:
        fs.close()
