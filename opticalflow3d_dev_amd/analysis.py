"""Downstream statistics on the flow outputs.

The reference post-processes the saved TIFFs in
``src/Python/example_analysis_script.ipynb``: cell 4 thresholds the
reliability at a percentile (``np.percentile(rel, relPer)``, ``rel >
thresh``), cell 5 masks vx/vy/vz, turns exact zeros into NaN and scales to
physical units, cell 6 forms the magnitude and the angles theta (in the xy
plane) and phi (against the z axis).  Here that runs on outputs still
resident in HBM (FlowStream / plans): the percentile from two order
statistics selected on the GPU, the rest in one fused HIP pass
(``of3d_flow_stats``).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def percentile_threshold(rel, percentile):
    """``np.percentile(rel, percentile)`` (method 'linear') of a tensor, any device.

    The two order statistics around the virtual index come from
    torch.kthvalue on the tensor's device; the interpolation repeats
    numpy's (``a + (b-a)*g``, or ``b - (b-a)*(1-g)`` for g >= 0.5, in the
    array's dtype), so the value equals numpy's.  NaN in -> NaN out."""
    import torch

    flat = rel.reshape(-1)
    n = flat.numel()
    if n == 0:
        raise ValueError("percentile of an empty array")
    dt = np.dtype(str(flat.dtype).replace("torch.", ""))
    if bool(torch.isnan(flat).any()):
        return dt.type(np.nan)
    # numpy's arithmetic, in the array's dtype (numpy/lib/_function_base_impl.py: percentile ->
    # _quantile, method 'linear': virtual index (n-1)*q, gamma, _lerp)
    q = np.asanyarray(np.true_divide(percentile, dt.type(100)))
    vi = (n - 1) * q
    if vi >= n - 1:
        lo = hi = n - 1
    elif vi < 0:
        lo = hi = 0
    else:
        lo = int(np.floor(vi))
        hi = lo + 1
    gamma = np.asanyarray(vi - lo, dtype=dt)
    a = dt.type(flat.kthvalue(lo + 1).values.item())
    b = dt.type(flat.kthvalue(hi + 1).values.item()) if hi != lo else a
    diff = np.subtract(b, a)
    res = np.add(a, diff * gamma) if gamma < 0.5 else np.subtract(b, diff * (1 - gamma))
    return dt.type(res)


def flow_statistics(vx, vy, vz, rel, rel_percentile=90, xyscale=1.0, zscale=1.0, tscale=1.0, device=None):
    """Masked physical velocities, magnitude and angles of one output frame.

    vx, vy, vz, rel: numpy arrays or torch tensors (CUDA tensors stay on
    their device); vz None for 2D.  Returns a dict: threshold, vx, vy, [vz,]
    magnitude, theta, [phi] — torch tensors on the GPU (numpy arrays when the
    inputs were numpy).  Matches example_analysis_script.ipynb cells 4-6:
    bitwise for the threshold, the mask, the velocities and the magnitude;
    theta/phi to the last bits of atan2/atan (device libm vs the host's)."""
    import torch

    host = isinstance(vx, np.ndarray)
    dev = torch.device("cuda", _lib.device_index() if device is None else device)
    to = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev) if host else a.contiguous()
    tx, ty, tr = to(vx), to(vy), to(rel)
    tz = to(vz) if vz is not None else None
    if tx.dtype not in (torch.float64, torch.float32) or tr.dtype not in (torch.float32, torch.float64):
        raise TypeError("vx/vy/vz must be float64 or float32, rel float32 or float64")
    shape = tuple(tx.shape)
    n = tx.numel()
    thresh = percentile_threshold(tr, rel_percentile)
    out = {k: torch.empty(shape, dtype=torch.float64, device=tx.device)
           for k in (("vx", "vy", "vz", "magnitude", "theta", "phi") if tz is not None
                     else ("vx", "vy", "magnitude", "theta"))}
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    stream = torch.cuda.current_stream(tx.device).cuda_stream
    _lib.check(_lib.load().of3d_flow_stats(
        ptr(tx), ptr(ty), ptr(tz), ptr(tr), int(tx.dtype == torch.float32), int(tr.dtype == torch.float64), n,
        float(thresh), float(xyscale), float(zscale), float(tscale), ptr(out["vx"]), ptr(out["vy"]),
        ptr(out.get("vz")), ptr(out["magnitude"]), ptr(out["theta"]), ptr(out.get("phi")), stream))
    if host:
        torch.cuda.synchronize(tx.device)
        out = {k: v.cpu().numpy() for k, v in out.items()}
    out["threshold"] = thresh
    return out
