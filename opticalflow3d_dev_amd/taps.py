"""Filter taps of the LK pipeline (host side, NumPy).

The taps are computed exactly as the reference builds them
(``src/Python/calc_flow.py:230-267`` for 3D, ``:72-101`` for 2D): same NumPy
expression trees, so the coefficients handed to the device are the
reference's own bits.  The device then evaluates every 1-D pass in scipy's
symmetric summation order.
"""

from __future__ import annotations

import math

import numpy as np


def radii(xyzSig, tSig, wSig):
    """(rd, rs, rt, rw): derivative/Gaussian, smoothing, temporal, window radii."""
    return (math.ceil(3 * xyzSig), math.ceil(3 * (xyzSig / 4)), math.ceil(3 * tSig), math.ceil(3 * wSig))


def make_taps(xyzSig=3, tSig=1, wSig=4) -> dict:
    """The five distinct tap vectors (full length 2r+1, centre at index r).

    gauss  = fderiv == fx   (calc_flow.py:233, :253)   used by dt's y/x/z passes
    deriv  = fderiv*gderiv  (calc_flow.py:239)          derivative direction
    smooth = fsmooth        (calc_flow.py:234)          cross directions
    tderiv = ft*gt          (calc_flow.py:260)          temporal derivative
    window = gw             (calc_flow.py:264)          Lucas–Kanade window W
    """
    x = np.arange(-math.ceil(3 * xyzSig), math.ceil(3 * xyzSig) + 1)
    xyzSig2 = xyzSig / 4
    y = np.arange(-math.ceil(3 * xyzSig2), math.ceil(3 * xyzSig2) + 1)
    fderiv = np.exp(-x * x / 2 / xyzSig / xyzSig) / math.sqrt(2 * math.pi) / xyzSig
    fsmooth = np.exp(-y * y / 2 / xyzSig2 / xyzSig2) / math.sqrt(2 * math.pi) / xyzSig2
    gderiv = x / xyzSig / xyzSig
    t = np.arange(-math.ceil(3 * tSig), math.ceil(3 * tSig) + 1)
    fx = np.exp(-x * x / 2 / xyzSig / xyzSig) / math.sqrt(2 * math.pi) / xyzSig
    ft = np.exp(-t * t / 2 / tSig / tSig) / math.sqrt(2 * math.pi) / tSig
    gt = t / tSig / tSig
    wRange = np.arange(-math.ceil(3 * wSig), math.ceil(3 * wSig) + 1)
    gw = np.exp(-wRange * wRange / 2 / wSig / wSig) / math.sqrt(2 * math.pi) / wSig
    as64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
    return {
        "gauss": as64(fx * 1),
        "deriv": as64(fderiv * gderiv),
        "smooth": as64(fsmooth * 1),
        "tderiv": as64(ft * gt),
        "window": as64(gw),
    }
