"""The C-ABI library loads and exports every symbol include/of3d.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from conftest import REPO
from opticalflow3d_dev_amd import _lib


def declared_functions():
    src = open(os.path.join(REPO, "include", "of3d.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(of3d_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_set():
    assert declared_functions() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_version_and_errors():
    lib = _lib.load()
    assert lib.of3d_version() == 10000
    assert isinstance(lib.of3d_last_error(), bytes)
    assert lib.of3d_stage_name(0) == b"grad_xy"
    assert lib.of3d_stage_name(99) == b""
    assert lib.of3d_device_count() >= 0


def test_null_plan_is_an_error_not_a_crash():
    lib = _lib.load()
    assert lib.of3d_plan_destroy(None) == 0
    assert lib.of3d_plan_set_timing(None, 1) != 0
    assert "null" in _lib.last_error()
    a, b = ctypes.c_int64(), ctypes.c_int64()
    assert lib.of3d_plan_input_range(None, 0, 1, ctypes.byref(a), ctypes.byref(b)) != 0


def test_build_provenance_matches_tree():
    """of3d_build_info: the library was built from exactly the sources in the tree, with no
    EXTRA (experiment) flags — the loader refuses anything else (OF3D_ALLOW_STALE aside)."""
    info = _lib.build_info()
    assert info["src_hash"] == info["tree_hash"] == _lib.source_hash()
    assert info["extra"] == "" and info["arch"] == "gfx950"
    assert "-ffp-contract=off" in info["flags"]
