"""opticalflow3d_dev_amd — MI355X-native Lucas–Kanade optical flow.

Drop-in for the hot path of ScientistRachel/OpticalFlow3D_dev
(src/Python/calc_flow.py): ``calc_flow3D``, ``calc_flow2D``, ``process_flow``
(alias ``calc_flow``).  The arithmetic runs as HIP kernels for gfx950 in
``libof3d.so`` (C-ABI: include/of3d.h).
"""

from .calc_flow import calc_flow, calc_flow2D, calc_flow2D_fp32, calc_flow3D, calc_flow3D_fp32, process_flow  # noqa: F401
from .taps import make_taps, radii  # noqa: F401

__all__ = ["calc_flow", "calc_flow2D", "calc_flow3D", "process_flow", "calc_flow2D_fp32", "calc_flow3D_fp32",
           "make_taps", "radii"]
