"""The C-ABI from plain C (examples/of3d_cli.c): compiled with gcc against include/of3d.h and
linked to libof3d.so only — no Python, no torch in the caller.  CPU: it builds, links and
reports the library; GPU: calc_flow3D through it is bit-identical to the Python host entry and
to the oracle (vx/vy/vz; rel within the SURVEY §8(c) tolerances)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, assert_rel_within, bits_equal, oracle3d

LIBDIR = os.path.join(REPO, "opticalflow3d_dev_amd")


@pytest.fixture(scope="module")
def cli(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("cli") / "of3d_cli")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-std=c11", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "examples", "of3d_cli.c"), "-L", LIBDIR, "-lof3d",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def test_cli_builds_and_links(cli):
    out = subprocess.run([cli, "--version"], check=True, capture_output=True, text=True).stdout
    assert out.startswith("of3d 10000,") and "src_hash" in out


def test_cli_usage_error(cli):
    r = subprocess.run([cli], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def test_cli_rejects_bad_taps_header_and_pipes(cli, tmp_path):
    """Malformed inputs fail with status 2 before any pointer arithmetic or device call: a
    negative / fractional tap radius, a taps file whose size does not match its radii, an input
    that cannot be sized (a FIFO), bad dimensions."""
    img = tmp_path / "img.u16"
    np.zeros((7, 2, 8, 8), np.uint16).tofile(img)
    for hdr in ([-5, 1, 1, 3], [2.5, 1, 1, 3], [2, 1, 40, 3], [1e9, 1, 1, 3]):
        tp = tmp_path / "bad.f64"
        np.array(hdr + [0.0] * 64, np.float64).tofile(tp)
        r = subprocess.run([cli, str(img), "7", "2", "8", "8", str(tp), str(tmp_path / "o_")],
                           capture_output=True, text=True)
        assert r.returncode == 2 and "bad tap radius" in r.stderr, (hdr, r.stderr)
    tp = tmp_path / "short.f64"
    np.array([1, 1, 1, 1] + [0.0] * 3, np.float64).tofile(tp)
    r = subprocess.run([cli, str(img), "7", "2", "8", "8", str(tp), str(tmp_path / "o_")], capture_output=True, text=True)
    assert r.returncode == 2 and "does not match" in r.stderr
    # the image through a pipe (/dev/stdin): ftell cannot size it -> refused, no overrun
    good = tmp_path / "good.f64"
    _taps_file(good, 1, 1, 1)
    r = subprocess.run([cli, "/dev/stdin", "7", "2", "8", "8", str(good), str(tmp_path / "o_")],
                       input=np.zeros(7 * 2 * 8 * 8, np.uint16).tobytes(), capture_output=True)
    assert r.returncode == 2 and b"bad input files" in r.stderr
    r = subprocess.run([cli, str(img), "7", "0", "8", "8", str(tp), str(tmp_path / "o_")], capture_output=True, text=True)
    assert r.returncode == 2 and "bad dimensions" in r.stderr
    # a frame count that does not match the file, including one whose byte count nt * nz * ny * nx
    # * 2 would overflow int64 and wrap: the size is compared as a quotient
    for nt in ("6", "8", str(2 ** 62 + 7), str(2 ** 63 - 1)):
        r = subprocess.run([cli, str(img), nt, "2", "8", "8", str(good), str(tmp_path / "o_")],
                           capture_output=True, text=True)
        assert r.returncode == 2 and "bad input files" in r.stderr, (nt, r.stderr)


def _taps_file(path, s, t, w):
    from opticalflow3d_dev_amd import make_taps, radii

    rd, rs, rt, rw = radii(s, t, w)
    tp = make_taps(s, t, w)
    parts = [np.array([rd, rs, rt, rw], np.float64)] + [np.asarray(tp[k], np.float64) for k in
                                                         ("gauss", "deriv", "smooth", "tderiv", "window")]
    np.concatenate(parts).tofile(path)


@pytest.mark.gpu
@pytest.mark.parametrize("rel64", [False, True])
def test_cli_flow3d_matches_host_and_oracle(cli, tmp_path, rel64):
    from opticalflow3d_dev_amd import calc_flow3D

    s, t, w = 2, 2, 5
    img = np.random.default_rng(41).integers(0, 4096, size=(13, 12, 40, 48)).astype(np.uint16)
    img.tofile(tmp_path / "in.u16")
    _taps_file(tmp_path / "taps.f64", s, t, w)
    args = [cli, str(tmp_path / "in.u16"), *map(str, img.shape), str(tmp_path / "taps.f64"), str(tmp_path / "o_")]
    subprocess.run(args + (["rel64"] if rel64 else []), check=True, capture_output=True, timeout=120)
    shape = img.shape[1:]
    got = [np.fromfile(tmp_path / f"o_{n}.f64").reshape(shape) for n in ("vx", "vy", "vz")]
    rel = np.fromfile(tmp_path / ("o_rel.f64" if rel64 else "o_rel.f32"),
                      dtype=np.float64 if rel64 else np.float32).reshape(shape)
    host = calc_flow3D(img, s, t, w)
    vx, vy, vz, lmin, lmax = oracle3d(img, s, t, w)
    for g, h, o in zip(got, host[:3], (vx, vy, vz)):
        assert bits_equal(g, h) and bits_equal(g, o)
    if rel64:
        assert_rel_within(rel, lmin, lmax, 1e-10)
    else:
        assert bits_equal(rel, host[3])
