"""ORACLE — test infrastructure, never product code.

CPU restatement of the reference hot path (ScientistRachel/OpticalFlow3D_dev,
``src/Python/calc_flow.py``), written from scratch in NumPy.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (``opticalflow3d_dev_amd``) never imports it.

Pinning: every function below is checked against golden vectors produced by
importing the reference ``calc_flow2D`` / ``calc_flow3D`` in the build
container (``tests/golden/make_golden.py``; see ``tests/test_oracle.py``).
Agreement is bitwise for 2D (vx, vy, rel) and 3D (vx, vy, vz); 3D ``rel`` uses
the same LAPACK ``cgeev`` (complex64) call the reference makes.

Two backends for the separable 1-D correlation:

* ``"restated"`` — a from-scratch statement of scipy's ``NI_Correlate1D``
  summation order (scipy 1.15, ``scipy/ndimage/src/ni_filters.c``): for a
  symmetric tap vector ``w`` of radius ``r``
  ``o[i] = c[i]*w[r]; for j=-r..-1: o[i] += (c[i+j] + c[i-j]) * w[r+j]``,
  antisymmetric: ``-`` instead of ``+``; indices clamped (``mode='nearest'``).
* ``"scipy"`` — ``scipy.ndimage.correlate1d`` itself (the primitive the
  reference calls, ``calc_flow.py:8``); used for the timed CPU baseline
  because it is the reference's own speed.
"""

from __future__ import annotations

import math
import sys

import numpy as np

DBL_EPSILON = np.finfo(float).eps  # 2.220446049250313e-16, calc_flow.py:155,338


# --------------------------------------------------------------------------
# T1 — taps.  calc_flow.py:230-267 (3D), :72-101 (2D).  Evaluated with the
# same expression trees, left to right.
# --------------------------------------------------------------------------
def make_taps(xyzSig, tSig, wSig):
    """Return dict of the five distinct tap vectors used by calc_flow2D/3D.

    gauss  : fderiv == fx (calc_flow.py:233,253)   radius rd = ceil(3*sig)
    deriv  : fderiv*gderiv (calc_flow.py:239)       radius rd (antisymmetric)
    smooth : fsmooth (calc_flow.py:234)             radius rs = ceil(3*sig/4)
    tderiv : ft*gt (calc_flow.py:260)               radius rt (antisymmetric)
    window : gw (calc_flow.py:264)                  radius rw
    """
    x = np.arange(-math.ceil(3 * xyzSig), math.ceil(3 * xyzSig) + 1)
    sig2 = xyzSig / 4
    y = np.arange(-math.ceil(3 * sig2), math.ceil(3 * sig2) + 1)
    fderiv = np.exp(-x * x / 2 / xyzSig / xyzSig) / math.sqrt(2 * math.pi) / xyzSig
    fsmooth = np.exp(-y * y / 2 / sig2 / sig2) / math.sqrt(2 * math.pi) / sig2
    gderiv = x / xyzSig / xyzSig
    t = np.arange(-math.ceil(3 * tSig), math.ceil(3 * tSig) + 1)
    fx = np.exp(-x * x / 2 / xyzSig / xyzSig) / math.sqrt(2 * math.pi) / xyzSig
    ft = np.exp(-t * t / 2 / tSig / tSig) / math.sqrt(2 * math.pi) / tSig
    gt = t / tSig / tSig
    wr = np.arange(-math.ceil(3 * wSig), math.ceil(3 * wSig) + 1)
    gw = np.exp(-wr * wr / 2 / wSig / wSig) / math.sqrt(2 * math.pi) / wSig
    return {
        "gauss": np.asarray(fx * 1, dtype=np.float64),       # fx*gx, gx = 1
        "deriv": np.asarray(fderiv * gderiv, dtype=np.float64),
        "smooth": np.asarray(fsmooth * 1, dtype=np.float64),  # fsmooth*gsmooth
        "tderiv": np.asarray(ft * gt, dtype=np.float64),
        "window": np.asarray(gw, dtype=np.float64),
    }


def _symmetry(w):
    """scipy NI_Correlate1D symmetry test: +1 symmetric, -1 anti, 0 general."""
    n = len(w)
    if not (n & 1):
        return 0
    r = n // 2
    if all(abs(w[r + k] - w[r - k]) <= DBL_EPSILON for k in range(1, r + 1)):
        return 1
    if all(abs(w[r + k] + w[r - k]) <= DBL_EPSILON for k in range(1, r + 1)):
        return -1
    return 0


def correlate1d_restated(a, w, axis):
    """From-scratch scipy.ndimage.correlate1d(a, w, axis, mode='nearest')."""
    a = np.asarray(a, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    r = len(w) // 2
    L = a.shape[axis]
    sym = _symmetry(w)
    base = np.arange(L)

    def shifted(off):
        return np.take(a, np.clip(base + off, 0, L - 1), axis=axis)

    if sym == 0:  # general branch: o = c[+r']*w[last]; for j=-r..r'-1: o += c[j]*w[j]
        r2 = len(w) - r - 1
        out = shifted(r2) * w[r + r2]
        for j in range(-r, r2):
            out = out + shifted(j) * w[r + j]
        return out
    out = a * w[r]
    for j in range(-r, 0):
        if sym > 0:
            out = out + (shifted(j) + shifted(-j)) * w[r + j]
        else:
            out = out + (shifted(j) - shifted(-j)) * w[r + j]
    return out


def _correlate(backend):
    if backend == "restated":
        return correlate1d_restated
    if backend == "scipy":
        from scipy.ndimage import correlate1d

        return lambda a, w, axis: correlate1d(a, w, axis=axis, mode="nearest")
    raise ValueError(backend)


# --------------------------------------------------------------------------
# T9 — argument checks (calc_flow.py:54-64, :212-222) — messages verbatim.
# --------------------------------------------------------------------------
MSG_NDIM_3D = "ERROR: Input image must be a 3D matrix with dimensions N_T, N_Z, N_Y, N_X"
MSG_NDIM_2D = "ERROR: Input image must be a 3D matrix with dimensions N_T, N_Y, N_X"
MSG_EDGE = "ERROR: Input images will lead to edge effects. N_T must be >= 6*tSig+1"
MSG_ODD = ("ERROR: Input images must have an odd number of timepoints. "
           "Only the central time point is analyzed")


def _check(images, ndim, tSig, msg_ndim):
    if not (len(images.shape) == ndim):
        sys.exit(msg_ndim)
    Nt = images.shape[0]
    if Nt < 6 * tSig + 1:
        sys.exit(MSG_EDGE)
    if not (Nt % 2):
        sys.exit(MSG_ODD)
    return math.ceil(Nt / 2) - 1


# --------------------------------------------------------------------------
# 3D — calc_flow.py:175-360
# --------------------------------------------------------------------------
def structure_tensor3d(images, xyzSig=3, tSig=1, wSig=4, backend="restated", taps=None):
    """Steps T2-T5: returns the nine windowed products (fp64 volumes)."""
    c = _check(images, 4, tSig, MSG_NDIM_3D)
    cor = _correlate(backend)
    tp = make_taps(xyzSig, tSig, wSig) if taps is None else taps
    G, D, S, T, W = tp["gauss"], tp["deriv"], tp["smooth"], tp["tderiv"], tp["window"]
    imgs = np.asarray(images)
    # T2 (calc_flow.py:276-277): temporal derivative, only the centre frame is
    # kept, so only the centre output line of the time correlation is formed.
    rt = len(T) // 2
    Nt = imgs.shape[0]
    dt0 = None
    frame = lambda k: imgs[min(max(k, 0), Nt - 1)].astype(np.float64)
    dt0 = frame(c) * T[rt]
    for j in range(-rt, 0):
        dt0 = dt0 + (frame(c + j) - frame(c - j)) * T[rt + j]
    I = imgs[c].astype(np.float64)
    # T4 (calc_flow.py:279-288): y (axis 1) -> x (axis 2) -> z (axis 0)
    dt = cor(cor(cor(dt0, G, 1), G, 2), G, 0)
    dy = cor(cor(cor(I, D, 1), S, 2), S, 0)
    dx = cor(cor(cor(I, S, 1), D, 2), S, 0)
    dz = cor(cor(cor(I, S, 1), S, 2), D, 0)
    # T5 (calc_flow.py:300-313)
    wf = lambda p: cor(cor(cor(p, W, 1), W, 2), W, 0)
    return {
        "tx": wf(dx * dt), "ty": wf(dy * dt), "tz": wf(dz * dt),
        "xy": wf(dx * dy), "xz": wf(dx * dz), "x2": wf(dx * dx),
        "yz": wf(dy * dz), "y2": wf(dy * dy), "z2": wf(dz * dz),
    }


def solve3d(st):
    """T6 (calc_flow.py:337-340): closed-form 3x3 solve, same expression trees."""
    x2, y2, z2 = st["x2"], st["y2"], st["z2"]
    xy, xz, yz = st["xy"], st["xz"], st["yz"]
    tx, ty, tz = st["tx"], st["ty"], st["tz"]
    det = (x2 * y2 * z2) + (2 * xy * xz * yz) - (y2 * xz**2) - (z2 * xy**2) - (x2 * yz**2)
    R = (det + DBL_EPSILON) ** -1
    vx = -R * ((y2 * z2 - yz * yz) * tx + (xz * yz - xy * z2) * ty + (xy * yz - xz * y2) * tz)
    vy = -R * ((yz * xz - xy * z2) * tx + (x2 * z2 - xz * xz) * ty + (xz * xy - x2 * yz) * tz)
    vz = -R * ((xy * yz - y2 * xz) * tx + (xy * xz - x2 * yz) * ty + (x2 * y2 - xy * xy) * tz)
    return vx, vy, vz


def tensor_stack3d(st):
    """(Nz,Ny,Nx,3,3) symmetric tensor, as calc_flow.py:352-354 builds it."""
    w = np.array([[st["x2"], st["xy"], st["xz"]],
                  [st["xy"], st["y2"], st["yz"]],
                  [st["xz"], st["yz"], st["z2"]]])
    return np.moveaxis(w, [0, 1], [-1, -2])


def rel3d_reference(st):
    """T7 (calc_flow.py:352-357): min real eigenvalue via LAPACK cgeev, complex64."""
    w = tensor_stack3d(st).astype(np.complex64)
    ev = np.linalg.eigvals(w)
    return np.ascontiguousarray(np.real(np.amin(ev, axis=-1)))


def eig_fp64_3d(st):
    """fp64 eigvalsh of the same tensor: (lambda_min, lambda_max) per voxel."""
    ev = np.linalg.eigvalsh(tensor_stack3d(st))
    return ev[..., 0], ev[..., -1]


def calc_flow3D(images, xyzSig=3, tSig=1, wSig=4, backend="restated"):
    """Restated calc_flow.py:175-360 -> (vx, vy, vz, rel[float32])."""
    st = structure_tensor3d(images, xyzSig, tSig, wSig, backend)
    vx, vy, vz = solve3d(st)
    return vx, vy, vz, rel3d_reference(st)


# --------------------------------------------------------------------------
# 2D — calc_flow.py:18-173
# --------------------------------------------------------------------------
def structure_tensor2d(images, xySig=3, tSig=1, wSig=4, backend="restated", taps=None):
    c = _check(images, 3, tSig, MSG_NDIM_2D)
    cor = _correlate(backend)
    tp = make_taps(xySig, tSig, wSig) if taps is None else taps
    G, D, S, T, W = tp["gauss"], tp["deriv"], tp["smooth"], tp["tderiv"], tp["window"]
    imgs = np.asarray(images)
    Nt = imgs.shape[0]
    rt = len(T) // 2
    frame = lambda k: imgs[min(max(k, 0), Nt - 1)].astype(np.float64)
    dt0 = frame(c) * T[rt]
    for j in range(-rt, 0):
        dt0 = dt0 + (frame(c + j) - frame(c - j)) * T[rt + j]
    I = imgs[c].astype(np.float64)
    # calc_flow.py:116-122: y (axis 0) -> x (axis 1)
    dt = cor(cor(dt0, G, 0), G, 1)
    dy = cor(cor(I, D, 0), S, 1)
    dx = cor(cor(I, S, 0), D, 1)
    wf = lambda p: cor(cor(p, W, 0), W, 1)
    return {"tx": wf(dx * dt), "ty": wf(dy * dt), "xy": wf(dx * dy),
            "x2": wf(dx * dx), "y2": wf(dy * dy)}


def solve2d(st):
    """T8 (calc_flow.py:154-168)."""
    x2, y2, xy, tx, ty = st["x2"], st["y2"], st["xy"], st["tx"], st["ty"]
    det = (x2 * y2) - (xy * xy)
    vx = ((det + DBL_EPSILON) ** -1) * ((y2 * -tx) + (-xy * -ty))
    vy = ((det + DBL_EPSILON) ** -1) * ((-xy * -tx) + (x2 * -ty))
    tr = x2 + y2
    with np.errstate(invalid="ignore"):
        L1 = (tr + np.sqrt(tr**2 - 4 * det)) / 2
        L2 = (tr - np.sqrt(tr**2 - 4 * det)) / 2
    rel = np.real(np.minimum(L1, L2))
    return vx, vy, rel


def calc_flow2D(images, xySig=3, tSig=1, wSig=4, backend="restated"):
    """Restated calc_flow.py:18-173 -> (vx, vy, rel[float64])."""
    return solve2d(structure_tensor2d(images, xySig, tSig, wSig, backend))


# --------------------------------------------------------------------------
# Synthetic inputs — deterministic, regenerated on the box.
# --------------------------------------------------------------------------
def synthetic_stack(shape, seed=20260206, motion=(0.3, -0.2, -0.1)):
    """uint16 stack (Nt,[Nz,]Ny,Nx): translated sum of sinusoids + hash noise."""
    return synthetic_stack_np(shape, seed, motion)


def synthetic_stack_np(shape, seed=20260206, motion=(0.3, -0.2, -0.1)):
    rng = np.random.default_rng(seed)
    nd = len(shape) - 1
    Nt = shape[0]
    sp = shape[1:]
    k = rng.uniform(2 * np.pi / 24, 2 * np.pi / 6, size=(4, nd)) * rng.choice([-1, 1], size=(4, nd))
    ph = rng.uniform(0, 2 * np.pi, size=4)
    grids = np.meshgrid(*[np.arange(n, dtype=np.float64) for n in sp], indexing="ij")
    # motion is (vx, vy, vz); axes are ([z,] y, x)
    mv = {1: motion[0], 2: motion[1], 3: motion[2]}
    out = np.empty(shape, dtype=np.uint16)
    for t in range(Nt):
        s = np.zeros(sp)
        for q in range(4):
            arg = ph[q]
            for a in range(nd):
                axis_vel = mv[nd - a]  # last axis is x
                arg = arg + k[q, a] * (grids[a] - axis_vel * t)
            s += np.sin(arg)
        noise = rng.integers(-8, 9, size=sp)
        out[t] = np.clip(1000 + 300 * s + noise, 0, 65535).astype(np.uint16)
    return out


def analysis_reference(vx, vy, vz, rel, relPer=90, xyscale=1.0, zscale=1.0, tscale=1.0):
    """The reference's post-processing, restated from
    src/Python/example_analysis_script.ipynb cells 4-6 (reliability percentile
    mask, masked velocities in physical units, magnitude, theta, phi), on host
    arrays.  vz None for 2D (then no phi and a 2-term magnitude)."""
    relThresh = np.percentile(rel, relPer)                      # cell 4
    relMask = rel > relThresh
    out = {"threshold": relThresh}
    vx = vx * relMask                                           # cell 5
    vx[vx == 0] = np.nan
    vx = vx * xyscale / tscale
    vy = vy * relMask
    vy[vy == 0] = np.nan
    vy = vy * xyscale / tscale
    out["vx"], out["vy"] = vx, vy
    if vz is not None:
        vz = vz * relMask
        vz[vz == 0] = np.nan
        vz = vz * zscale / tscale
        out["vz"] = vz
        out["magnitude"] = np.sqrt(np.power(vx, 2) + np.power(vy, 2) + np.power(vz, 2))   # cell 6
        out["phi"] = np.arctan(vz / np.sqrt(np.power(vx, 2) + np.power(vy, 2)))
    else:
        out["magnitude"] = np.sqrt(np.power(vx, 2) + np.power(vy, 2))
    out["theta"] = np.arctan2(vy, vx)
    return out
