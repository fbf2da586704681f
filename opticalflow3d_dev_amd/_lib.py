"""ctypes binding of libof3d.so (include/of3d.h).

The shared library is built in-tree (``opticalflow3d_dev_amd/libof3d.so``,
``make -C opticalflow3d_dev_amd/csrc``).  There is no CPU fallback: if the
library is missing or no GPU is visible, calls raise loudly.
"""

from __future__ import annotations

import ctypes
import json
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OF3D_LIB", os.path.join(_HERE, "libof3d.so"))

OF3D_U8, OF3D_U16, OF3D_I16, OF3D_U32, OF3D_I32, OF3D_F32, OF3D_F64 = 1, 2, 3, 4, 5, 6, 7
OF3D_FP64_EXACT = 0
OF3D_REL_F64 = 0x100
OF3D_FP32 = 0x200

DTYPE_CODES = {
    np.dtype(np.uint8): OF3D_U8,
    np.dtype(np.uint16): OF3D_U16,
    np.dtype(np.int16): OF3D_I16,
    np.dtype(np.uint32): OF3D_U32,
    np.dtype(np.int32): OF3D_I32,
    np.dtype(np.float32): OF3D_F32,
    np.dtype(np.float64): OF3D_F64,
}

# Every symbol include/of3d.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "of3d_version", "of3d_last_error", "of3d_device_count", "of3d_flow3d", "of3d_flow2d",
    "of3d_plan_create", "of3d_plan_destroy", "of3d_plan_workspace_bytes", "of3d_plan_input_range",
    "of3d_plan_execute", "of3d_plan_stage_times", "of3d_stage_name", "of3d_plan_set_timing",
    "of3d_copy_async", "of3d_dma_copy", "of3d_plan_set_timing_mask", "of3d_flow_stats",
    "of3d_plan_set_overlap", "of3d_cache_clear", "of3d_plan_set_rows",
    "of3d_plan_kernels", "of3d_build_info", "of3d_plan_execute_next", "of3d_plan_execute_ahead",
    "of3d_rel3d", "of3d_plan_geometry",
)

CSRC = os.path.join(_HERE, "csrc")
INCLUDE_H = os.path.join(os.path.dirname(_HERE), "include", "of3d.h")


def source_hash() -> str | None:
    """sha256 (16 hex digits) of the library's sources, concatenated in csrc/Makefile's
    HASH_FILES order (sorted *.hip / *.hpp, Makefile, include/of3d.h); None when the
    sources are not beside the package."""
    import glob
    import hashlib

    files = sorted(os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(
        os.path.join(CSRC, "*.hpp")))
    paths = [os.path.join(CSRC, f) for f in files] + [os.path.join(CSRC, "Makefile"), INCLUDE_H]
    if not files or not all(os.path.exists(p) for p in paths):
        return None
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_info() -> dict:
    """of3d_build_info() of the loaded library, plus the hash of the sources beside it."""
    import json

    info = json.loads(load().of3d_build_info().decode())
    info["tree_hash"] = source_hash()
    info["lib"] = os.path.relpath(LIB_PATH, os.path.dirname(_HERE))
    return info


def _check_provenance(lib):
    """Refuse a library built from other sources than the tree's, or with EXTRA flags (an
    A/B experiment build): OF3D_ALLOW_STALE=1 loads it anyway, with a warning."""
    import json
    import warnings

    info = json.loads(lib.of3d_build_info().decode())
    tree = source_hash()
    problems = []
    if tree is not None and info.get("src_hash") != tree:
        problems.append(f"built from sources {info.get('src_hash')}, tree has {tree} (rebuild: make -C "
                        "opticalflow3d_dev_amd/csrc)")
    if info.get("extra"):
        problems.append(f"built with EXTRA flags {info['extra']!r} (experiment build)")
    if problems:
        msg = f"opticalflow3d_dev_amd: {LIB_PATH}: " + "; ".join(problems)
        if os.environ.get("OF3D_ALLOW_STALE") == "1":
            warnings.warn(msg + " [loaded: OF3D_ALLOW_STALE=1]")
        else:
            raise ImportError(msg)


class Taps(ctypes.Structure):
    _fields_ = [
        ("gauss", ctypes.POINTER(ctypes.c_double)),
        ("deriv", ctypes.POINTER(ctypes.c_double)),
        ("rd", ctypes.c_int),
        ("smooth", ctypes.POINTER(ctypes.c_double)),
        ("rs", ctypes.c_int),
        ("tderiv", ctypes.POINTER(ctypes.c_double)),
        ("rt", ctypes.c_int),
        ("window", ctypes.POINTER(ctypes.c_double)),
        ("rw", ctypes.c_int),
    ]


class Perf(ctypes.Structure):
    _fields_ = [("ms_h2d", ctypes.c_double), ("ms_kernels", ctypes.c_double),
                ("ms_d2h", ctypes.c_double), ("ms_total", ctypes.c_double)]


_lib = None
_lock = threading.Lock()


def load():
    """Load libof3d.so once; raise if it is absent (no silent fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"opticalflow3d_dev_amd: HIP library not built ({LIB_PATH} missing); "
                "run `make -C opticalflow3d_dev_amd/csrc` or __graft_entry__.build()")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7.
        # Loaded first, it satisfies our NEEDED entry by soname; loaded after
        # /opt/rocm's copy, it would start a second runtime that sees no GPUs.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(LIB_PATH)
        if not hasattr(lib, "of3d_build_info"):
            raise ImportError(f"opticalflow3d_dev_amd: {LIB_PATH} predates build provenance; rebuild it")
        lib.of3d_build_info.restype = ctypes.c_char_p
        _check_provenance(lib)
        P = ctypes.c_void_p
        D = ctypes.POINTER(ctypes.c_double)
        F = ctypes.POINTER(ctypes.c_float)
        i64 = ctypes.c_int64
        lib.of3d_version.restype = ctypes.c_int
        lib.of3d_last_error.restype = ctypes.c_char_p
        lib.of3d_device_count.restype = ctypes.c_int
        lib.of3d_cache_clear.restype = ctypes.c_int
        lib.of3d_flow3d.argtypes = [P, ctypes.c_int, i64, i64, i64, i64, ctypes.POINTER(Taps), ctypes.c_int,
                                    ctypes.c_int, D, D, D, P, ctypes.POINTER(Perf)]
        lib.of3d_flow3d.restype = ctypes.c_int
        lib.of3d_flow2d.argtypes = [P, ctypes.c_int, i64, i64, i64, ctypes.POINTER(Taps), ctypes.c_int,
                                    ctypes.c_int, D, D, D, ctypes.POINTER(Perf)]
        lib.of3d_flow2d.restype = ctypes.c_int
        lib.of3d_plan_create.argtypes = [ctypes.POINTER(P), ctypes.c_int, i64, i64, i64, ctypes.POINTER(Taps),
                                         ctypes.c_int, ctypes.c_int, i64]
        lib.of3d_plan_create.restype = ctypes.c_int
        lib.of3d_plan_destroy.argtypes = [P]
        lib.of3d_plan_destroy.restype = ctypes.c_int
        lib.of3d_plan_workspace_bytes.argtypes = [P]
        lib.of3d_plan_workspace_bytes.restype = ctypes.c_size_t
        lib.of3d_plan_input_range.argtypes = [P, i64, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]
        lib.of3d_plan_input_range.restype = ctypes.c_int
        lib.of3d_plan_execute.argtypes = [P, ctypes.POINTER(P), ctypes.c_int, i64, i64, i64, P, P, P, P, P]
        lib.of3d_plan_execute.restype = ctypes.c_int
        lib.of3d_plan_execute_next.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.c_int, i64, i64, i64,
                                               P, P, P, P, P]
        lib.of3d_plan_execute_next.restype = ctypes.c_int
        lib.of3d_plan_execute_ahead.argtypes = [P, ctypes.POINTER(P), ctypes.c_int, ctypes.c_int, i64, i64, i64,
                                                P, P, P, P, P]
        lib.of3d_plan_execute_ahead.restype = ctypes.c_int
        lib.of3d_plan_stage_times.argtypes = [P, D, ctypes.c_int]
        lib.of3d_plan_stage_times.restype = ctypes.c_int
        lib.of3d_stage_name.argtypes = [ctypes.c_int]
        lib.of3d_stage_name.restype = ctypes.c_char_p
        lib.of3d_plan_set_timing.argtypes = [P, ctypes.c_int]
        lib.of3d_plan_set_timing.restype = ctypes.c_int
        lib.of3d_plan_set_timing_mask.argtypes = [P, ctypes.c_uint]
        lib.of3d_plan_set_timing_mask.restype = ctypes.c_int
        lib.of3d_plan_set_overlap.argtypes = [P, i64]
        lib.of3d_plan_set_overlap.restype = ctypes.c_int
        lib.of3d_plan_set_rows.argtypes = [P, i64, i64]
        lib.of3d_plan_set_rows.restype = ctypes.c_int
        lib.of3d_plan_kernels.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t]
        lib.of3d_plan_kernels.restype = ctypes.c_int
        lib.of3d_plan_geometry.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t]
        lib.of3d_plan_geometry.restype = ctypes.c_int
        d = ctypes.c_double
        lib.of3d_flow_stats.argtypes = [P, P, P, P, ctypes.c_int, ctypes.c_int, i64, d, d, d, d, P, P, P, P, P, P, P]
        lib.of3d_flow_stats.restype = ctypes.c_int
        lib.of3d_rel3d.argtypes = [P, i64, P, ctypes.c_int, P]
        lib.of3d_rel3d.restype = ctypes.c_int
        lib.of3d_copy_async.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int, P]
        lib.of3d_copy_async.restype = ctypes.c_int
        lib.of3d_dma_copy.argtypes = [ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.c_int]
        lib.of3d_dma_copy.restype = ctypes.c_int
        _lib = lib
        return lib


def cache_clear():
    """of3d_cache_clear: release the device workspaces cached by calc_flow3D / calc_flow2D."""
    check(load().of3d_cache_clear())


def last_error() -> str:
    return load().of3d_last_error().decode(errors="replace")


def check(rc: int) -> int:
    if rc < 0:
        raise RuntimeError("of3d: " + last_error())
    return rc


def copy_async(dst_ptr, src_ptr, nbytes, max_blocks=0, stream=0):
    """of3d_copy_async: kernel copy with at most max_blocks workgroups (pinned host <-> device)."""
    check(load().of3d_copy_async(dst_ptr, src_ptr, nbytes, max_blocks, stream))


def dma_copy(dst_ptrs, src_ptrs, nbytes):
    """of3d_dma_copy: blocking SDMA copies (pinned host / device buffers); ctypes drops the GIL."""
    n = len(dst_ptrs)
    check(load().of3d_dma_copy((ctypes.c_void_p * n)(*dst_ptrs), (ctypes.c_void_p * n)(*src_ptrs),
                               (ctypes.c_size_t * n)(*nbytes), n))


def device_index() -> int:
    """GPU used by the host entry points: $OF3D_DEVICE, else $LOCAL_RANK, else 0."""
    for k in ("OF3D_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(k)
        if v is not None and v != "":
            return int(v)
    return 0


class TapSet:
    """Keeps the tap arrays alive and exposes the of3d_taps struct."""

    def __init__(self, taps: dict):
        self.arrays = {k: np.ascontiguousarray(v, dtype=np.float64) for k, v in taps.items()}
        r = lambda k: len(self.arrays[k]) // 2
        ptr = lambda k: self.arrays[k].ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        self.struct = Taps(ptr("gauss"), ptr("deriv"), r("gauss"), ptr("smooth"), r("smooth"),
                           ptr("tderiv"), r("tderiv"), ptr("window"), r("window"))
        self.rd, self.rs, self.rt, self.rw = r("gauss"), r("smooth"), r("tderiv"), r("window")


class Plan:
    """Device-resident plan (of3d_plan_*): inputs/outputs are device pointers."""

    def __init__(self, ndim, nz, ny, nx, taps: dict, device=0, max_out_planes=0, timing=0, mode=0):
        self.lib = load()
        self.taps = TapSet(taps)
        self.ndim, self.nz, self.ny, self.nx, self.device = ndim, nz, ny, nx, device
        h = ctypes.c_void_p()
        check(self.lib.of3d_plan_create(ctypes.byref(h), ndim, nz, ny, nx, ctypes.byref(self.taps.struct),
                                        mode, device, max_out_planes))
        self.handle = h
        if timing:
            check(self.lib.of3d_plan_set_timing(h, int(timing)))

    @property
    def workspace_bytes(self):
        return self.lib.of3d_plan_workspace_bytes(self.handle)

    def input_range(self, z_out0, z_out1):
        a, b = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.of3d_plan_input_range(self.handle, z_out0, z_out1, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def execute(self, frame_ptrs, dtype_code, frame_z0, z_out0, z_out1, vx, vy, vz, rel, stream=0,
                next_ptrs=None, pipelined=False, ahead_ptrs=None):
        """of3d_plan_execute; pipelined=True: of3d_plan_execute_next (uses the dt0 the previous
        pipelined call formed for these frames; with next_ptrs also forms the next frame's);
        ahead_ptrs (a list, possibly empty): of3d_plan_execute_ahead with the frames after the
        window (K0 batching: one pass forms this and the next windows' dt0)."""
        if ahead_ptrs is not None:
            allp = list(frame_ptrs) + list(ahead_ptrs)
            arr = (ctypes.c_void_p * len(allp))(*allp)
            check(self.lib.of3d_plan_execute_ahead(self.handle, arr, len(ahead_ptrs), dtype_code, frame_z0, z_out0,
                                                   z_out1, vx, vy, vz, rel, stream or None))
            return
        arr = (ctypes.c_void_p * len(frame_ptrs))(*frame_ptrs)
        if not pipelined and next_ptrs is None:
            check(self.lib.of3d_plan_execute(self.handle, arr, dtype_code, frame_z0, z_out0, z_out1,
                                             vx, vy, vz, rel, stream or None))
            return
        nxt = (ctypes.c_void_p * len(next_ptrs))(*next_ptrs) if next_ptrs is not None else None
        check(self.lib.of3d_plan_execute_next(self.handle, arr, nxt, dtype_code, frame_z0, z_out0, z_out1,
                                              vx, vy, vz, rel, stream or None))

    def stage_times(self):
        buf = (ctypes.c_double * 8)()
        n = check(self.lib.of3d_plan_stage_times(self.handle, buf, 8))
        return {self.lib.of3d_stage_name(i).decode(): buf[i] for i in range(n) if buf[i] >= 0}

    STAGES = ("grad_xy", "grad_z", "prod_wy", "wx", "wz_solve")

    def set_overlap(self, chunk_planes):
        """of3d_plan_set_overlap: z chunks of chunk_planes output planes, gradient stages of the next
        chunk beside the W-xy / W-z / solve stages of this one (0: serial)."""
        check(self.lib.of3d_plan_set_overlap(self.handle, int(chunk_planes)))

    def set_rows(self, y0, y1):
        """of3d_plan_set_rows: outputs only rows [y0, y1), compact; raises where unsupported."""
        check(self.lib.of3d_plan_set_rows(self.handle, int(y0), int(y1)))

    def kernels(self):
        """of3d_plan_kernels: the kernel families this plan has launched so far."""
        n = check(self.lib.of3d_plan_kernels(self.handle, None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        check(self.lib.of3d_plan_kernels(self.handle, buf, n + 1))
        return [k for k in buf.value.decode().split(",") if k]

    def geometry(self):
        """of3d_plan_geometry: the plan's kernel shapes (W-xy layout, K34, K5c) and the last
        execution's K12 march / batched-K0 windows, as a dict."""
        n = check(self.lib.of3d_plan_geometry(self.handle, None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        check(self.lib.of3d_plan_geometry(self.handle, buf, n + 1))
        return json.loads(buf.value.decode())

    def set_timing_stages(self, names=None):
        """Time only these stages (None: all); fewer events, less perturbation."""
        mask = 0
        for n in (names or self.STAGES):
            mask |= 1 << self.STAGES.index(n)
        check(self.lib.of3d_plan_set_timing_mask(self.handle, mask))

    def close(self):
        if getattr(self, "handle", None):
            self.lib.of3d_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
