"""Host-side logic (CPU only, no device calls): taps, argument checks, TIFF
I/O, natural sort, parameters CSV, process_flow's file discovery errors."""
import os

import numpy as np
import pytest

from conftest import bits_equal, golden_cases, golden_manifest, load_golden
from opticalflow3d_dev_amd import calc_flow2D, calc_flow3D, make_taps, process_flow, radii
from opticalflow3d_dev_amd import tiff as tf
from opticalflow3d_dev_amd.calc_flow import _write_parameters


@pytest.mark.parametrize("name", golden_cases())
def test_product_taps_match_reference_bits(name):
    g = load_golden(name)
    t = make_taps(g["sig"], g["tsig"], g["wsig"])
    for k, v in t.items():
        assert bits_equal(v, g["taps"][k]), k
    rd, rs, rt, rw = radii(g["sig"], g["tsig"], g["wsig"])
    assert (len(t["gauss"]), len(t["smooth"]), len(t["tderiv"]), len(t["window"])) == \
        (2 * rd + 1, 2 * rs + 1, 2 * rt + 1, 2 * rw + 1)


def test_product_error_messages_match_reference():
    """SystemExit text identical to the reference (checks run before any device call)."""
    for name, e in golden_manifest()["_errors"].items():
        fn = calc_flow3D if e["dims"] == 3 else calc_flow2D
        with pytest.raises(SystemExit) as ex:
            fn(np.zeros(e["shape"], np.uint16), 1, e["tSig"], 2)
        assert str(ex.value.code) == e["message"], name


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int16, np.float32, np.float64])
@pytest.mark.parametrize("shape", [(5, 7), (3, 4, 6), (2, 3, 4, 5)])
def test_tiff_roundtrip(tmp_path, dtype, shape):
    a = (np.random.default_rng(0).uniform(0, 100, size=shape)).astype(dtype)
    p = tmp_path / "x.tiff"
    tf.imwrite(p, a, photometric="minisblack")
    b = tf.imread(p)
    assert b.shape == a.shape and b.dtype == a.dtype and np.array_equal(a, b)
    t = tf.TiffFile(p)
    assert len(t.pages) == (int(np.prod(shape[:-2])) if len(shape) > 2 else 1)
    assert t.pages[0].shape == shape[-2:]
    m = tf.memmap(p)
    assert np.array_equal(np.asarray(m), a)


def _raw_ifds(path):
    """Every IFD of a little-endian classic TIFF as {tag: (type, count, values)} — a parser of
    its own (TIFF 6.0 §2), independent of tiff.TiffFile."""
    import struct
    b = open(path, "rb").read()
    assert b[:4] == b"II*\0"
    size = {1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 16: 8}
    fmt = {1: "B", 2: "c", 3: "H", 4: "I", 16: "Q"}
    out, off = [], struct.unpack_from("<I", b, 4)[0]
    while off:
        n = struct.unpack_from("<H", b, off)[0]
        tags = {}
        for i in range(n):
            code, typ, cnt = struct.unpack_from("<HHI", b, off + 2 + 12 * i)
            nb = size[typ] * cnt
            at = off + 2 + 12 * i + 8 if nb <= 4 else struct.unpack_from("<I", b, off + 2 + 12 * i + 8)[0]
            raw = b[at:at + nb]
            tags[code] = (typ, cnt, raw if typ == 2 else struct.unpack("<%d%s" % (cnt, fmt[typ]), raw))
        out.append(tags)
        off = struct.unpack_from("<I", b, off + 2 + 12 * n)[0]
    return b, out


@pytest.mark.parametrize("dtype,bits,fmt", [(np.float32, 32, 3), (np.float64, 64, 3), (np.uint16, 16, 1)])
def test_tiff_layout_pinned_by_spec(tmp_path, dtype, bits, fmt):
    """The output files' tag set, pinned by specification (byte identity against tifffile
    2025.3.13 is unverifiable here: tifffile is absent).  tifffile.imwrite(path, arr,
    photometric='minisblack') of a (Z, Y, X) array — calc_flow.py:526-529 — writes one
    uncompressed single-strip page per plane, tags in ascending order, the shaped-series JSON
    description '{"shape": [Z, Y, X]}' on page 0 only, SampleFormat 3 for floats, data in
    page order (contiguous, so readers memory-map it)."""
    import json
    a = np.random.default_rng(2).uniform(0, 9, size=(3, 5, 7)).astype(dtype)
    p = tmp_path / "vx.tiff"
    tf.imwrite(p, a, photometric="minisblack")
    raw, ifds = _raw_ifds(p)
    assert len(ifds) == 3
    want = {254, 256, 257, 258, 259, 262, 273, 277, 278, 279, 305, 339}
    plane = 5 * 7 * a.itemsize
    for i, t in enumerate(ifds):
        assert set(t) == want | ({270} if i == 0 else set())
        assert t[254][2] == (0,) and t[256][2] == (7,) and t[257][2] == (5,)
        assert t[258][2] == (bits,) and t[259][2] == (1,) and t[262][2] == (1,)  # none, minisblack
        assert t[277][2] == (1,) and t[278][2] == (5,) and t[279][2] == (plane,) and t[339][2] == (fmt,)
        assert t[273][2][0] == ifds[0][273][2][0] + i * plane  # contiguous, page order
        assert t[273][2][0] % 2 == 0
    desc = ifds[0][270][2].rstrip(b"\0").decode()
    assert json.loads(desc) == {"shape": [3, 5, 7]} and desc == json.dumps({"shape": [3, 5, 7]})
    o = ifds[0][273][2][0]
    assert np.array_equal(np.frombuffer(raw[o:o + 3 * plane], dtype=dtype).reshape(a.shape), a)


def test_tiff_bigtiff_roundtrip(tmp_path):
    a = np.arange(2 * 3 * 4, dtype=np.float64).reshape(2, 3, 4)
    p = tmp_path / "big.tiff"
    tf.imwrite(p, a, bigtiff=True)
    assert tf.TiffFile(p).bigtiff
    assert np.array_equal(tf.imread(p), a)


def test_tiff_float32_readable_by_pillow(tmp_path):
    from PIL import Image
    a = np.random.default_rng(1).normal(size=(3, 6, 5)).astype(np.float32)
    p = tmp_path / "rel.tiff"
    tf.imwrite(p, a)
    im = Image.open(p)
    for i in range(3):
        im.seek(i)
        assert np.array_equal(np.asarray(im, dtype=np.float32), a[i])


def test_imagej_hyperstack_memmap(tmp_path):
    a = np.random.default_rng(2).integers(0, 4000, size=(7, 3, 5, 6)).astype(np.uint16)
    p = tmp_path / "stack.tif"
    tf.imwrite(p, a, imagej=True)
    t = tf.TiffFile(p)
    ij = t.imagej_metadata
    assert ij["frames"] == 7 and ij["slices"] == 3 and ij["images"] == 21
    m = tf.memmap(p)
    assert m.shape == (7, 3, 5, 6) and np.array_equal(np.asarray(m), a)


def test_imagej_single_ifd_contiguous(tmp_path):
    """ImageJ > 4 GB layout: one IFD, planes contiguous after it (M/TIFFvolume.m:48-52)."""
    a = np.random.default_rng(3).integers(0, 4000, size=(7, 2, 4, 5)).astype(np.uint16)
    p = tmp_path / "one_ifd.tif"
    tf.imwrite(p, a[0, 0], description=tf.imagej_description(a.shape))
    # append the remaining planes contiguously after the first page's data
    t = tf.TiffFile(p)
    off = t.pages[0].offsets[0]
    with open(p, "r+b") as f:
        f.seek(off)
        f.write(a.tobytes())
    assert np.array_equal(np.asarray(tf.memmap(p)), a)


def test_natsorted():
    names = ["im_t10.tif", "im_t2.tif", "im_t1.tif", "im_t100.tif", "im_t20.tif"]
    assert tf.natsorted(names) == ["im_t1.tif", "im_t2.tif", "im_t10.tif", "im_t20.tif", "im_t100.tif"]


def test_parameters_csv(tmp_path):
    p = tmp_path / "x_parameters.csv"
    _write_parameters(p, 3, 1, 4, 512, 256, 64, 13)
    assert p.read_text() == "xyzSig,tiSig,wSig,Nx,Ny,Nz,Nt\n3,1,4,512,256,64,13\n"
    _write_parameters(p, 1.5, 1, 2.5, 8, 8, 1, 7)
    assert p.read_text() == "xyzSig,tiSig,wSig,Nx,Ny,Nz,Nt\n1.5,1,2.5,8,8,1,7\n"


def test_process_flow_errors(tmp_path):
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path / "nope"), "x")
    assert str(e.value.code) == "ERROR: image path '%s' does not exist" % (tmp_path / "nope")
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path), "x")
    assert str(e.value.code) == "ERROR: No image files found. imName: x imDir: " + str(tmp_path)
    for i in range(3):
        tf.imwrite(tmp_path / f"s_t{i}.tif", np.zeros((4, 4), np.uint16))
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path), "s_t.*", "SequenceT", 2)
    assert str(e.value.code) == ("ERROR: Image sequence found for file name s_t.* only contains 3 files. "
                                 "Minimum 6*tsig+1 (7) files required.")
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path), "s_t.*", "OneTif", 2)
    assert str(e.value.code) == "ERROR: Type is OneTif but more than one file was found for imName: s_t.*"
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path), "s_t.*", "Other", 2)
    assert str(e.value.code) == "ERROR: fileType must be either OneTif or SequenceT."
    tf.imwrite(tmp_path / "plain.tif", np.zeros((2, 4, 4), np.uint16))
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path), "plain", "OneTif", 3)
    assert str(e.value.code) == "ERROR: fileType is OneTif, but no ImageJ metadata was detected"
    with pytest.raises(SystemExit) as e:
        process_flow(str(tmp_path), "plain", "OneTif", 4)
    assert str(e.value.code) == "ERROR: Number of spatial dimensions must be either 2 or 3."


@pytest.mark.parametrize("shape,dtype", [((3, 17, 29), np.float64), ((40, 33), np.float64), ((2, 300, 70), np.float32)])
def test_matlab_lzw_writer_roundtrip(tmp_path, shape, dtype):
    """MATLAB-mode writer (M/TIFFwrite.m layout through the system libtiff):
    BigTIFF, LZW (tag 259 = 5), IEEE samples; pixels round-trip exactly."""
    import struct

    a = np.random.default_rng(1).standard_normal(shape).astype(dtype)
    a.flat[0] = -0.0
    p = tmp_path / "x.tiff"
    tf.imwrite_matlab(p, a)
    raw = p.read_bytes()
    assert raw[:4] == b"II+\x00"
    ifd = struct.unpack_from("<Q", raw, 8)[0]
    n = struct.unpack_from("<Q", raw, ifd)[0]
    tags = {struct.unpack_from("<H", raw, ifd + 8 + 20 * i)[0]: struct.unpack_from("<Q", raw, ifd + 8 + 20 * i + 12)[0]
            for i in range(n)}
    assert tags[259] == 5 and tags[339] == 3 and tags[258] == 8 * a.itemsize and tags[262] == 1
    b = tf.imread_libtiff(p)
    assert b.dtype == a.dtype and b.shape == a.shape
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_percentile_threshold_matches_numpy(dtype):
    """analysis.percentile_threshold (order statistics + numpy's lerp) equals
    np.percentile bit for bit (torch CPU tensors here; CUDA on the box)."""
    import torch

    from opticalflow3d_dev_amd.analysis import percentile_threshold

    rng = np.random.default_rng(7)
    for n in (1, 2, 5, 1000, 65537):
        a = rng.standard_normal(n).astype(dtype)
        for p in (0, 10, 33.3333, 50, 63.7, 90, 99.9, 100):
            r = np.percentile(a, p)
            g = percentile_threshold(torch.from_numpy(a), p)
            assert r.dtype == g.dtype and r.tobytes() == np.asarray(g).tobytes(), (n, p)


def test_eigenvalue_polynomial_pinned_to_its_generator():
    """The device eigenvalue's cos((2/3) acos u) polynomial (csrc/of3d_dev.hpp,
    cos_two_thirds_acos) carries exactly the coefficients tools/eig_poly.py fits, its error is
    at fp64 rounding level, and the eigenvalue formula built on it matches the acos form it
    replaced against eigvalsh (both limited by the r ~ 1 square-root conditioning)."""
    import re
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import eig_poly

    src = open(os.path.join(root, "opticalflow3d_dev_amd", "csrc", "of3d_dev.hpp")).read()
    body = src[src.index("double cos_two_thirds_acos(double u)"):]
    body = body[:body.index("\n}\n")]
    lits = [float(x) for x in re.findall(r"fma_sk\((?:c|-?[0-9.e+-]+), t, (-?[0-9.e+-]+)\)", body)]
    first = float(re.search(r"fma_sk\((-?[0-9.e+-]+), t,", body).group(1))
    dev = [first] + lits  # highest degree first, as Horner runs
    m = eig_poly.coefficients()
    assert len(dev) == eig_poly.DEG + 1
    # the generator's doubles, lowest degree first (a refit on another numpy / LAPACK may move
    # the last bits, so not bit-for-bit)
    assert np.allclose(np.array(dev[::-1]), m, rtol=1e-9, atol=1e-17)
    u = np.linspace(0, 1, 100001)
    assert np.abs(eig_poly.horner(m, 2 * u - 1) - np.cos(2 / 3 * np.arccos(u))).max() < 3e-15
    rng = np.random.default_rng(3)
    n = 20000
    q, _ = np.linalg.qr(rng.standard_normal((n, 3, 3)))
    lam = rng.standard_normal((n, 3))
    lam[: n // 2, 1] = lam[: n // 2, 0] * (1 + 1e-9 * rng.standard_normal(n // 2))
    a = np.einsum("nij,nj,nkj->nik", q, lam, q)
    args = (a[:, 0, 0], a[:, 1, 1], a[:, 2, 2], a[:, 0, 1], a[:, 0, 2], a[:, 1, 2])
    ref = np.linalg.eigvalsh(a)
    lmax = np.abs(ref).max(axis=1)
    err_poly = np.abs(eig_poly.eigmin3(*args, m=m) - ref[:, 0]) / lmax
    err_acos = np.abs(eig_poly.eigmin3(*args) - ref[:, 0]) / lmax
    assert err_poly.max() <= max(2 * err_acos.max(), 1e-12)
    assert err_poly.max() < 1e-7
