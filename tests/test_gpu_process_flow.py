"""process_flow end to end on the device (calc_flow.py:362-625): OneTif ImageJ
hyperstack and SequenceT series in, per-frame TIFFs + parameters CSV out;
pixel values equal the oracle's calc_flow3D/2D of the same window."""
import re

import numpy as np
import pytest

from conftest import assert_flow3d_matches_oracle, assert_rel_within, bits_equal, oracle3d
from opticalflow3d_dev_amd import process_flow
from opticalflow3d_dev_amd import tiff as tf
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _stack(shape, seed):
    return np.random.default_rng(seed).integers(0, 4096, size=shape).astype(np.uint16)


def test_onetif_3d(tmp_path, capsys):
    stack = _stack((9, 5, 20, 24), 1)  # Nt=9 -> 3 output frames at tSig=1
    tf.imwrite(tmp_path / "cells.tif", stack, imagej=True)
    process_flow(str(tmp_path), "cells", "OneTif", 3, 1, 1, 2)
    out = tmp_path / "OpticalFlow3D" / "cells"
    assert (out / "cells_parameters.csv").read_text() == "xyzSig,tiSig,wSig,Nx,Ny,Nz,Nt\n1,1,2,24,20,5,9\n"
    files = sorted(p.name for p in out.glob("*.tiff"))
    assert files == sorted(f"cells_{n}_t{t:04d}.tiff" for n in ("vx", "vy", "vz", "rel") for t in (3, 4, 5))
    for hh in range(3):
        got = [tf.imread(out / f"cells_{name}_t{hh + 3:04d}.tiff") for name in ("vx", "vy", "vz", "rel")]
        assert got[3].dtype == np.float32 and got[3].shape == (5, 20, 24)
        assert_flow3d_matches_oracle(got, stack[hh:hh + 7], 1, 1, 2)
    text = capsys.readouterr().out
    assert "Note: regardless of input filenames, the first image = frame 0." in text
    assert len(re.findall(r"No data will be saved for frame", text)) == 6
    assert len(re.findall(r"Frame \d+ saved\.  Duration: ", text)) == 3


def test_sequencet_2d(tmp_path):
    stack = _stack((8, 30, 26), 2)
    for t in range(8):
        tf.imwrite(tmp_path / f"img_t{t}_ch0.tif", stack[t])
    tf.imwrite(tmp_path / "other.tif", stack[0])
    process_flow(str(tmp_path), "img_t.*_ch0", "SequenceT", 2, 1, 1, 3)
    out = tmp_path / "OpticalFlow2D" / "img_t_ch0"
    assert (out / "img_t_ch0_parameters.csv").read_text() == "xyzSig,tiSig,wSig,Nx,Ny,Nz,Nt\n1,1,3,26,30,1,8\n"
    for hh in range(2):
        ref = cpu_ref.calc_flow2D(stack[hh:hh + 7], 1, 1, 3, backend="scipy")
        for name, r in zip(("vx", "vy", "rel"), ref):
            assert bits_equal(tf.imread(out / f"img_t_ch0_{name}_t{hh + 3:04d}.tiff"), r)


def test_sequencet_3d_natural_order(tmp_path):
    stack = _stack((7, 3, 12, 14), 3)
    for t in range(7):
        tf.imwrite(tmp_path / f"v_t{t * 5}.tif", stack[t])  # t0, t5, t10, ... natural order != ASCII order
    process_flow(str(tmp_path), "v_t.*", "SequenceT", 3, 1, 1, 2)
    out = tmp_path / "OpticalFlow3D" / "v_t"
    got = [tf.imread(out / f"v_t_{name}_t0003.tiff") for name in ("vx", "vy", "vz", "rel")]
    assert_flow3d_matches_oracle(got, stack, 1, 1, 2)


def test_stdout_order(tmp_path, capsys):
    stack = _stack((10, 4, 16, 18), 4)
    tf.imwrite(tmp_path / "s.tif", stack, imagej=True)
    process_flow(str(tmp_path), "s", "OneTif", 3, 1, 1, 2)
    lines = [l.split(" - ", 1)[1] for l in capsys.readouterr().out.splitlines() if " - " in l]
    want = [f"No data will be saved for frame {h} to avoid edge effects" for h in range(3)]
    for f in range(3, 7):
        want += [f"Processing frame {f}...", f"Frame {f} saved."]
    want += [f"No data will be saved for frame {h} to avoid edge effects" for h in range(7, 10)]
    assert [l.split("  Duration")[0] for l in lines] == want


@pytest.mark.parametrize("ndim,dtype,d2h", [(3, np.uint16, "dma"), (3, np.float32, "kernel"), (2, np.uint8, "dma"),
                                            (2, ">u2", "runtime")])
def test_flowstream_ring_wraps(ndim, dtype, d2h):
    """Many frames through the device ring (wraps it several times, every
    buffer set reused) — each output equals calc_flow3D/2D of its window."""
    from opticalflow3d_dev_amd.stream import FlowStream

    tsig = 2 if ndim == 3 else 1
    nwin = 6 * tsig + 1
    shape = (nwin + 9,) + ((6, 14, 22) if ndim == 3 else (40, 36))
    stack = np.random.default_rng(5).integers(0, 250, size=shape).astype(dtype)
    fs = FlowStream(ndim, shape[1:], np.dtype(dtype).newbyteorder("="), 1, tsig, 2, d2h=d2h)
    try:
        pend = []
        for t in range(shape[0]):
            fs.push(stack[t])
            if fs.ready:
                pend.append((t - nwin + 1, fs.submit()))
                if len(pend) == fs.depth:  # keep every buffer set in flight
                    k, p = pend.pop(0)
                    _check_stream(p, stack[k:k + nwin], ndim, tsig)
        for k, p in pend:
            _check_stream(p, stack[k:k + nwin], ndim, tsig)
    finally:
        fs.close()


def _check_stream(p, win, ndim, tsig):
    """One ring output against the oracle of its window, and bit for bit (rel included)
    against the host entry point calc_flow3D / calc_flow2D of the same window."""
    from opticalflow3d_dev_amd import calc_flow2D, calc_flow3D

    got = p.result()
    win = np.asarray(win).astype(np.asarray(win).dtype.newbyteorder("="))
    direct = (calc_flow3D if ndim == 3 else calc_flow2D)(win, 1, tsig, 2)
    for g, d in zip(got, direct):
        assert bits_equal(g, d)
    if ndim == 3:
        assert_flow3d_matches_oracle(got, win, 1, tsig, 2)
    else:
        for g, r in zip(got, cpu_ref.calc_flow2D(win, 1, tsig, 2, backend="scipy")):
            assert bits_equal(g, r)
    p.release()


@pytest.mark.parametrize("nbytes,off", [(1, 0), (4097, 0), (1 << 20, 0), ((1 << 20) + 13, 3), (33 << 20, 0)])
def test_copy_async_device_to_pinned(nbytes, off):
    import torch
    from opticalflow3d_dev_amd import _lib

    src = torch.randint(0, 256, (nbytes + off,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros(nbytes + off + 7, dtype=torch.uint8).pin_memory()
    s = torch.cuda.current_stream()
    _lib.copy_async(dst.data_ptr() + off, src.data_ptr() + off, nbytes, 16, s.cuda_stream)
    s.synchronize()
    assert torch.equal(dst[off:off + nbytes], src[off:].cpu())
    assert int(dst[:off].sum()) == 0 and int(dst[off + nbytes:].sum()) == 0


def test_dma_copy_roundtrip():
    import torch
    from opticalflow3d_dev_amd import _lib

    a = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, device="cuda")
    b = torch.randint(0, 256, (4099,), dtype=torch.uint8, device="cuda")
    ha = torch.zeros(a.numel(), dtype=torch.uint8).pin_memory()
    hb = torch.zeros(b.numel(), dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    _lib.dma_copy([ha.data_ptr(), hb.data_ptr()], [a.data_ptr(), b.data_ptr()], [a.numel(), b.numel()])
    assert torch.equal(ha, a.cpu()) and torch.equal(hb, b.cpu())
    d = torch.zeros_like(a)
    _lib.dma_copy([d.data_ptr()], [ha.data_ptr()], [a.numel()])  # host -> device too
    assert torch.equal(d, a)
    with pytest.raises(RuntimeError):
        pageable = np.zeros(16, np.uint8)
        _lib.dma_copy([pageable.ctypes.data], [a.data_ptr()], [16])


def test_matlab_output_mode(tmp_path):
    """matlab_output=True: LZW BigTIFF float64 files (M/TIFFwrite.m), read back
    with libtiff; vx bit-identical to the default mode, rel = the fp64 eigenvalue."""
    import importlib

    cf = importlib.import_module("opticalflow3d_dev_amd.calc_flow")  # the module (the package's calc_flow is a function)

    stack = _stack((8, 4, 18, 20), 6)
    tf.imwrite(tmp_path / "m.tif", stack, imagej=True)
    process_flow(str(tmp_path), "m", "OneTif", 3, 1, 1, 2, matlab_output=True)
    out = tmp_path / "OpticalFlow3D" / "m"
    ref = cf._flow3d(stack[0:7], 1, 1, 2, rel_fp64=True)
    raw = (out / "m_vx_t0003.tiff").read_bytes()
    assert raw[:4] == b"II+\x00"  # BigTIFF
    got = []
    for name, r in zip(("vx", "vy", "vz", "rel"), ref):
        got.append(tf.imread_libtiff(out / f"m_{name}_t0003.tiff"))
        assert got[-1].dtype == np.float64 and bits_equal(got[-1], r)
    vx, vy, vz, lmin, lmax = oracle3d(stack[0:7], 1, 1, 2)
    for g, want in zip(got[:3], (vx, vy, vz)):
        assert bits_equal(g, want)
    assert_rel_within(got[3], lmin, lmax, 1e-10)  # fp64 rel vs fp64 eigvalsh


FP32_TOL = 1e-4


def assert_fp32_flow_close(got, images, s, t, w):
    """fp32 outputs within 1e-4 * max|v| of the oracle's fp64 flow (rel: of max|lambda_max|)."""
    from conftest import oracle3d

    vx, vy, vz, lmin, lmax = oracle3d(images, s, t, w)
    for g, want in zip(got[:3], (vx, vy, vz)):
        assert g.dtype == np.float32 and g.shape == want.shape
        assert np.abs(g.astype(np.float64) - want).max() <= FP32_TOL * np.abs(want).max()
    assert np.abs(got[3].astype(np.float64) - lmin).max() <= FP32_TOL * np.abs(lmax).max()


@pytest.mark.parametrize("fileType", ["OneTif", "SequenceT"])
def test_process_flow_fp32_vs_oracle(tmp_path, fileType):
    """configs[4]'s product entry, process_flow(..., precision="fp32") (calc_flow.py:507-534's
    loop on the fp32 path): float32 TIFFs whose pixels are within 1e-4 of the oracle's fp64
    flow of each window."""
    from opticalflow3d_dev_amd.calc_flow import calc_flow3D_fp32

    stack = cpu_ref.synthetic_stack_np((9, 10, 24, 28), seed=21)
    if fileType == "OneTif":
        tf.imwrite(tmp_path / "f.tif", stack, imagej=True)
        name = "f"
    else:
        for t in range(9):
            tf.imwrite(tmp_path / f"f_t{t}.tif", stack[t])
        name = "f_t.*"
    process_flow(str(tmp_path), name, fileType, 3, 1, 1, 2, precision="fp32")
    save = name.replace(".*", "")
    out = tmp_path / "OpticalFlow3D" / save
    for hh in range(3):
        got = [tf.imread(out / f"{save}_{n}_t{hh + 3:04d}.tiff") for n in ("vx", "vy", "vz", "rel")]
        assert all(g.dtype == np.float32 for g in got)
        assert_fp32_flow_close(got, stack[hh:hh + 7], 1, 1, 2)
        for g, d in zip(got, calc_flow3D_fp32(stack[hh:hh + 7], 1, 1, 2)):
            assert bits_equal(g, d)  # the ring path = the one-shot fp32 entry, bit for bit


@pytest.mark.parametrize("name", ["c3d_ramp_xy_planar", "c3d_wave_planar", "c3d_ramp_xyz_rank1"])
def test_matlab_output_near_degenerate(tmp_path, name):
    """MATLAB mode end to end (M/calc_flow3D.m:235-236's double pageeig) on the near-degenerate
    golden inputs — where the trigonometric eigenvalue alone misses 1e-10 lambda_max: the rel
    file is within 1e-10 lambda_max of the fixture's fp64 eigvalsh, vx bit-identical to the
    reference's."""
    from conftest import load_golden

    g = load_golden(name)
    stack = g["images"]
    tf.imwrite(tmp_path / "d.tif", stack, imagej=True)
    process_flow(str(tmp_path), "d", "OneTif", 3, g["sig"], g["tsig"], g["wsig"], matlab_output=True)
    out = tmp_path / "OpticalFlow3D" / "d"
    c = stack.shape[0] // 2
    rel = tf.imread_libtiff(out / f"d_rel_t{c:04d}.tiff")
    vx = tf.imread_libtiff(out / f"d_vx_t{c:04d}.tiff")
    assert rel.dtype == np.float64 and bits_equal(vx, g["vx"])
    assert_rel_within(rel, g["lmin64"], g["lmax64"], 1e-10)
