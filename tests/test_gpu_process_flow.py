"""process_flow end to end on the device (calc_flow.py:362-625): OneTif ImageJ
hyperstack and SequenceT series in, per-frame TIFFs + parameters CSV out;
pixel values equal the oracle's calc_flow3D/2D of the same window."""
import re

import numpy as np
import pytest

from conftest import bits_equal
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
        ref = cpu_ref.calc_flow3D(stack[hh:hh + 7], 1, 1, 2, backend="scipy")
        for name, r in zip(("vx", "vy", "vz", "rel"), ref):
            got = tf.imread(out / f"cells_{name}_t{hh + 3:04d}.tiff")
            if name == "rel":
                assert got.dtype == np.float32 and got.shape == r.shape
            else:
                assert bits_equal(got, r)
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
    ref = cpu_ref.calc_flow3D(stack, 1, 1, 2, backend="scipy")
    assert bits_equal(tf.imread(out / "v_t_vx_t0003.tiff"), ref[0])
