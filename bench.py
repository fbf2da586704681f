#!/usr/bin/env python3
"""Benchmark: Mvoxels/s per output frame of the LK optical-flow hot path on MI355X.

Metric (BASELINE.json): "Mvoxels/s per frame-pair (and HBM GB/s fraction) at
1/2/4/8 MI355X".  One step = one pass of the hot path (calc_flow3D,
src/Python/calc_flow.py:175-360) over one output frame: the 2*rt+1 input
frames are resident in HBM when the timed region starts; the step runs the
five-kernel pipeline through the C-ABI (of3d_plan_execute) and leaves
vx, vy, vz (fp64) and rel (fp32) in HBM.

Default workload = BASELINE.json configs[2] (c3), the largest single-GPU
config: 3D 512x512x128, 19 frames, xyzSig=2 tSig=3 wSig=7, fp64, run as a time
series (K0 batching over 5 windows; the line also carries configs[2] as stated,
one 19-frame window with K0 every step, as single_window_ms).  --config c2
selects configs[1]; c4/c5 are configs[3]/[4].
N > 1 (torch.distributed.run, one rank per GPU): the north star's z-shard —
ONE volume per output frame split over the ranks as z-slabs, the newest frame's
rd + rw halo exchanged over RCCL P2P beside the previous step's compute — on the
volume BASELINE names for N GPUs (c4 at N = 2 and 4, c5 at N = 8); value = the
volume's voxels / max-over-ranks step time ("scaling": "strong").  Beside it:
"replicas" (every rank computes the whole volume alone first: the one-GPU
frame t1 of the split's efficiency) and "row_slabs" (the other axis).  Every
line carries "parity_sample": one output crop checked against the oracle
outside the timed region (on N > 1 across the cut between rank 0 and rank 1),
and "build": the library's source hash (of3d_build_info).

Roofline: the dominant kernel's average duration from HIP events recorded on
the launch stream over the timed region (of3d_plan_set_timing ring), with its
algorithmic bytes and fp64 VALU op count; HBM traffic
from the committed rocprofv3 PMC summary (profiles/) when present.
cpu_baseline: the oracle (oracle/cpu_ref.py, scipy correlate1d + LAPACK cgeev
as the reference uses) on one thread, rank 0 at N=1 only.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    # name: (Nt, Nz, Ny, Nx, xyzSig, tSig, wSig, description)
    # configs[0]: the reference's 2D example (calc_flow2D, calc_flow.py:18-173) as a series of 16
    # frames (10 output frames); Nz = 1 marks the 2D path
    "c1": (16, 1, 256, 256, 1, 1, 5, "configs[0]: 2D 256x256 x16 frames (SequenceT series, 10 output frames), "
                                     "xySig=1 tSig=1 wSig=5, fp64 calc_flow2D on the GPU"),
    "c2": (13, 64, 256, 256, 2, 2, 5, "configs[1]: 3D OneTif 256x256x64 x13 frames (tSig=2), xyzSig=2 wSig=5, fp64"),
    "c3": (19, 128, 512, 512, 2, 3, 7, "configs[2]: 3D 512x512x128 x19 frames (tSig=3), xyzSig=2 wSig=7, fp64"),
    # configs[3]: one frame z-sharded over the ranks (strong scaling), halo exchange over RCCL
    "c4": (13, 256, 1024, 1024, 2, 2, 5, "configs[3]: 3D 1024x1024x256 x13 frames, z-slabs over the GPUs with "
                                         "RCCL halo exchange (sigmas as c2, SURVEY §8d), fp64"),
    "c5": (13, 512, 2048, 2048, 2, 2, 5, "configs[4]: 3D 2048x2048x512 x13 frames, fp32 path (OF3D_FP32), z-slabs "
                                         "over the GPUs with RCCL halo exchange (sigmas as c2, SURVEY §8d)"),
}
ZSLAB_CONFIGS = ("c4", "c5")
FP32_CONFIGS = ("c5",)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TOPS = 39.3     # 78.6 TFLOP/s fp64 vector counts an FMA as 2; add/mul issue at half
FP32_VALU_PEAK_TOPS = 78.6     # 157.3 TFLOP/s fp32 vector, same convention


def synthetic_frames(nt, nz, ny, nx, seed):
    """uint16 stack: translated separable sinusoids + bounded noise."""
    rng = np.random.default_rng(seed)
    z = np.arange(nz, dtype=np.float64)[:, None, None]
    y = np.arange(ny, dtype=np.float64)[None, :, None]
    x = np.arange(nx, dtype=np.float64)[None, None, :]
    k = rng.uniform(2 * np.pi / 24, 2 * np.pi / 6, size=(3, 3))
    ph = rng.uniform(0, 2 * np.pi, size=(3, 3))
    vel = (0.3, -0.2, -0.1)  # (vx, vy, vz) voxels/frame
    out = np.empty((nt, nz, ny, nx), np.uint16)
    for t in range(nt):
        s = np.zeros((nz, ny, nx))
        for q in range(3):
            s = s + (np.sin(k[q, 0] * (x - vel[0] * t) + ph[q, 0]) * np.sin(k[q, 1] * (y - vel[1] * t) + ph[q, 1])
                     * np.sin(k[q, 2] * (z - vel[2] * t) + ph[q, 2]))
        noise = rng.integers(-8, 9, size=(nz, ny, nx))
        out[t] = np.clip(1000 + 300 * s + noise, 0, 65535).astype(np.uint16)
    return out


def synthetic_slab(nt, nz, ny, nx, z0, z1, seed, device, out=None, zchunk=32, rows=None):
    """Planes [z0, z1) (rows [y0, y1) of them with rows=(y0, y1)) of a device-generated
    uint16 stack of the same family as synthetic_frames (for the large configs: each rank
    generates only its own part, and the values do not depend on the decomposition).
    Returned as int16 bits (values stay below 32768); generated zchunk planes at a time so
    the fp64 temporaries stay small next to a c5 workspace."""
    import torch

    rng = np.random.default_rng(seed)
    k = rng.uniform(2 * np.pi / 24, 2 * np.pi / 6, size=(3, 3))
    ph = rng.uniform(0, 2 * np.pi, size=(3, 3))
    vel = (0.3, -0.2, -0.1)
    f64 = dict(dtype=torch.float64, device=device)
    ya, yb = rows if rows is not None else (0, ny)
    if out is None:
        out = torch.empty((nt, z1 - z0, yb - ya, nx), dtype=torch.int16, device=device)
    y = torch.arange(ya, yb, **f64)[None, :, None]
    x = torch.arange(nx, **f64)[None, None, :]
    for c0 in range(z0, z1, zchunk):
        c1 = min(c0 + zchunk, z1)
        z = torch.arange(c0, c1, **f64)[:, None, None]
        lin = ((torch.arange(c0, c1, device=device)[:, None, None] * ny
                + torch.arange(ya, yb, device=device)[None, :, None]) * nx
               + torch.arange(nx, device=device)[None, None, :])
        for t in range(nt):
            sv = torch.zeros((c1 - c0, yb - ya, nx), **f64)
            for q in range(3):
                sv += (torch.sin(k[q, 0] * (x - vel[0] * t) + ph[q, 0])
                       * torch.sin(k[q, 1] * (y - vel[1] * t) + ph[q, 1])
                       * torch.sin(k[q, 2] * (z - vel[2] * t) + ph[q, 2]))
            idx = lin + t * nz * ny * nx
            noise = ((idx ^ (idx >> 7)) * 747796405 + 2891336453) % 17 - 8
            out[t, c0 - z0:c1 - z0] = torch.clamp(1000 + 300 * sv + noise, 0, 32767).to(torch.int16)
    return out


def stage_model_2d(nt_win, rd, rs, rt, rw, plane):
    """2D (calc_flow2D, calc_flow.py:18-173) per-launch algorithmic bytes / ops of each stage:
    grad_xy = K0 + the y and x passes (dt: y(G) x(G); dy: y(D) x(S); dx: y(S) x(D)), products +
    W y + W x of the five products, the 2x2 solve + rel (~30 ops: det, two products, the
    discriminant's sqrt, two roots)."""
    C = lambda r: 1 + 3 * r
    return {
        "grad_xy": {"bytes": (nt_win * 2 + 3 * 8) * plane, "ops": (C(rt) + 4 * C(rd) + 2 * C(rs)) * plane},
        "grad_z": {"bytes": 0, "ops": 0},
        "prod_wy_wx": {"bytes": (3 * 8 + 5 * 8) * plane, "ops": (5 + 10 * C(rw)) * plane},
        "wz_solve": {"bytes": (5 * 8 + 3 * 8) * plane, "ops": 30 * plane},
    }


def run_2d(args, world, rank, dev):
    """configs[0]: the 2D path (calc_flow2D, calc_flow.py:18-173) over a resident series of 16
    frames (256 x 256, xySig 1, tSig 1, wSig 5: 7-frame windows, 10 output frames).  One step =
    the series' 10 output frames in one pass: a 2D plan of 10 planes, each plane an output frame
    (the frames handed to the plan are the series shifted by 0 .. 6 frames, so plane b of frame j is
    series frame b + j: window b), the plan's four launches (K0, the y / x gradient passes, K34 over
    the five products, the 2x2 solve) each over the 10 frames.  Beside it: `single_frame`, the same
    series one output frame per execute (10 launches of each kernel).  N > 1: every rank its own
    series (replicas, weak scaling).  cpu_baseline: the oracle's calc_flow2D over the same 10
    windows, 1 thread."""
    import torch
    import torch.distributed as dist

    from opticalflow3d_dev_amd import _lib, make_taps, radii

    nt, _, ny, nx, s, t, w, desc = CONFIGS["c1"]
    rd, rs, rt, rw = radii(s, t, w)
    nwin = 2 * rt + 1
    nout = nt - nwin + 1
    d_in = synthetic_slab(nt, 1, ny, nx, 0, 1, 20260206 + 1 + 100 * rank, dev).view(nt, ny, nx)
    plane = ny * nx
    d_vx = torch.empty(nout * plane, dtype=torch.float64, device=dev)
    d_vy = torch.empty_like(d_vx)
    d_rel = torch.empty_like(d_vx)
    plan = _lib.Plan(2, nout, ny, nx, make_taps(s, t, w), device=dev.index, timing=max(args.steps, 1))
    stream = torch.cuda.current_stream(dev).cuda_stream
    ptrs = [d_in[i].data_ptr() for i in range(nt)]

    def step():  # the series' nout output frames: plane b of frame j = series frame b + j
        plan.execute(ptrs[:nwin], _lib.OF3D_U16, 0, 0, nout, d_vx.data_ptr(), d_vy.data_ptr(), 0, d_rel.data_ptr(),
                     stream)

    elapsed, profile, dom, dom_ms = timed_region(step, plan, args, world, dev)
    if world > 1:
        (elapsed,) = max_over_ranks([elapsed], dev)
    kernels = set(plan.kernels())
    geometry = plan.geometry()
    plan.close()
    # the same series one output frame per execute (a 1-plane plan, window j)
    plan1 = _lib.Plan(2, 1, ny, nx, make_taps(s, t, w), device=dev.index)
    s_vx, s_vy, s_rel = (torch.empty(plane, dtype=torch.float64, device=dev) for _ in range(3))
    last = {"i": 0}

    def step1():
        j = last["i"] % nout
        last["i"] += 1
        plan1.execute(ptrs[j:j + nwin], _lib.OF3D_U16, 0, 0, 1, s_vx.data_ptr(), s_vy.data_ptr(), 0, s_rel.data_ptr(),
                      stream)

    el1 = timed_steps(step1, nout * args.steps, nout * args.warmup, world, dev)
    plan1.close()
    if rank != 0:
        return
    from oracle import cpu_ref

    host = d_in.cpu().numpy().view(np.uint16)
    same = []
    for j in range(nout):  # every output frame of the last timed step vs the oracle, bitwise
        want = cpu_ref.calc_flow2D(host[j:j + nwin], s, t, w, backend="scipy")
        got = [o.view(nout, ny, nx)[j].cpu().numpy() for o in (d_vx, d_vy, d_rel)]
        same += [np.array_equal(a.view(np.uint64), np.ascontiguousarray(b).view(np.uint64)) for a, b in zip(got, want)]
    parity = {"ok": all(same), "crop_out": f"all {nout} output frames of the last step",
              "vx_vy_rel": "bitwise" if all(same) else "MISMATCH", "checker": "oracle/cpu_ref.py (scipy backend)"}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from threadpoolctl import threadpool_limits

        with threadpool_limits(limits=1):
            reps, t0 = 0, time.perf_counter()
            while True:  # whole passes over the series' 10 output frames, ~min(budget, 10 s)
                for k in range(nout):
                    cpu_ref.calc_flow2D(host[k:k + nwin], s, t, w, backend="scipy")
                reps += 1
                dt = time.perf_counter() - t0
                if dt >= min(args.cpu_budget, 10.0):
                    break
        cpu = {"value": round(reps * nout * plane / dt / 1e6, 4), "unit": "Mvoxels/s", "cores": 1, "kind": "port",
               "sample": f"{reps} passes over the series' {nout} output frames ({ny}x{nx}, {nwin}-frame windows): "
                         f"oracle/cpu_ref.py calc_flow2D (scipy.ndimage.correlate1d), 1 thread, {dt:.2f} s",
               "seconds": round(dt, 3), "host_cpus": os.cpu_count(),
               **calibrated(reps * nout * plane / dt / 1e6, "c1")}
    plane_b = plane
    plane = nout * plane  # per launch: the batch's planes
    C = lambda r: 1 + 3 * r
    frame_ops = (C(rt) + 4 * C(rd) + 2 * C(rs) + 5 + 10 * C(rw) + 30) * plane
    roof = roofline(profile, dom, dom_ms, stage_model_2d(nwin, rd, rs, rt, rw, plane), "c1",
                    (nwin * 2 + 3 * 8) * plane, frame_ops, nwin, 8, used=kernels)
    roof["frame"]["bytes_per_voxel"] = nwin * 2 + 3 * 8  # vx, vy, rel: fp64 (2D rel is fp64)
    ms = elapsed / args.steps * 1e3
    ms1 = el1 / (nout * args.steps) * 1e3
    line = {
        "metric": "Mvoxels/s per frame-pair (and HBM GB/s fraction) at 1/2/4/8 MI355X",
        "value": round(world * plane * args.steps / elapsed / 1e6, 3), "unit": "Mvoxels/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": desc, "nt": nt, "nt_window": nwin, "ny": ny, "nx": nx, "xySig": s, "tSig": t, "wSig": w,
                   "parallelism": f"series replicas x{world}" if world > 1 else "single GPU",
                   "inputs": f"a series of {nt} uint16 frames resident in HBM; one step = its {nout} output "
                             f"frames as one batch (a 2D plan of {nout} planes)",
                   "frames_per_step": nout, "kernels": sorted(kernels), "geometry": geometry},
        "roofline": roof, "cpu_baseline": cpu, "parity_sample": parity, "build": build_stamp(),
        "single_frame": {"ms_per_frame": round(ms1, 5), "value": round(world * plane_b / (ms1 * 1e-3) / 1e6, 3),
                         "unit": "Mvoxels/s", "what": "the same series one output frame per execute (a 1-plane plan)"},
    }
    print(json.dumps(line), flush=True)


def stage_model(nt_win, rd, rs, rt, rw, nb, ng, no, plane, sv=8):
    """Algorithmic HBM bytes and VALU ops per launch of each stage.

    Bytes are the compulsory reads + writes of the stage's own inputs/outputs
    (each element once; sv = bytes per workspace/output value: 8 fp64, 4 fp32);
    ops count every add and multiply of the scipy-order passes (C(r) = 1 + 3r
    per symmetric/antisymmetric output)."""
    C = lambda r: 1 + 3 * r
    return {
        "grad_xy": {"bytes": (nt_win * 2 + 4 * sv) * nb * plane,
                    "ops": (C(rt) + C(rd) * 2 + C(rs) + C(rd) * 2 + C(rs) * 2) * nb * plane},
        "grad_z": {"bytes": (4 * sv + 4 * sv) * ng * plane, "ops": (C(rd) * 2 + C(rs) * 2) * ng * plane},
        "prod_wy": {"bytes": (4 * sv + 9 * sv) * ng * plane, "ops": (9 + 9 * C(rw)) * ng * plane},
        # fused products + W y + W x (k_prod_wyx): the W-y result never leaves the CU
        "prod_wy_wx": {"bytes": (4 * sv + 9 * sv) * ng * plane, "ops": (9 + 18 * C(rw)) * ng * plane},
        "wx": {"bytes": (9 * sv + 9 * sv) * ng * plane, "ops": 9 * C(rw) * ng * plane},
        "wz_solve": {"bytes": (9 * sv + 3 * sv + 4) * no * plane, "ops": (9 * C(rw) + 65 + 50) * no * plane},
        # the next frame's temporal derivative (K0) when it runs inside the solve kernel
        # (frame pipelining, k_wz_solve_c_next): its frames in, dt0 out
        "tderiv_next": {"bytes": (nt_win * 2 + sv) * nb * plane, "ops": C(rt) * nb * plane},
    }


STAGE_KERNELS = {"grad_xy": ("k_tderiv", "k_grad_xy_", "k_grad_xy<"), "grad_z": ("k_grad_z", "k_grad_xyz"),
                 "prod_wy": ("k_prod_wy",),
                 "prod_wy_wx": ("k_prod_wyx",), "wx": ("k_wx",), "wz_solve": ("k_wz_solve",)}


def fused_names(profile):
    """The plan reports no "wx" stage when K34 (products + W y + W x) is one kernel:
    its time is under "prod_wy"; name it for what it is."""
    if profile and "wx" not in profile and "prod_wy" in profile:
        profile = dict(profile)
        profile["prod_wy_wx"] = profile.pop("prod_wy")
    return profile


# kernel families a plan reports (of3d_plan_kernels; kKernelNames in csrc/of3d_host.hip)
PLAN_FAMILIES = {"k_tderiv_c", "k_tderiv", "k_grad_xy_c", "k_grad_xy", "k_grad_xyz_c", "k_grad_z_c", "k_grad_z",
                 "k_prod_wyx", "k_prod_wyx_ws", "k_prod_wy", "k_wx", "k_wz_solve_c", "k_wz_solve_c2",
                 "k_wz_solve_dma", "k_wz_solve", "k_solve2d", "k_prod_wyx_pk", "k_wz_solve_c_next",
                 "k_tderiv_multi"}


def kernel_family(name):
    """Plan family of a profiled kernel name: the solve kernel with a non-zero temporal radius
    template argument (RT0, the 7th) carries the next frame's K0 (k_wz_solve_c_next)."""
    base = name.split("<")[0]
    if base == "k_wz_solve_c" and "<" in name:
        args = [a.strip() for a in name.split("<", 1)[1].rstrip(">").split(",")]
        if len(args) > 6 and args[6] != "0":
            return "k_wz_solve_c_next"
    return base


def load_pmc_traffic(stage, cfg, used=None):
    """HBM bytes per launch of the stage's kernels from the committed rocprofv3 PMC summary
    (profiles/pmc_<cfg>.json: FETCH_SIZE x2 + WRITE_SIZE, calibrated in profiles/pmc_calibration.json).
    used: the families the measured plan launched (plan.kernels()); a known family it did not
    launch (a K34 autotune candidate of another family) is not counted."""
    path = os.path.join(REPO, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        ks = d.get("kernels", {})
        # one value per kernel of the stage; of several template instances of one kernel (plan-time
        # autotune candidates) the one dispatched most often is the one the plan uses
        best = {}
        for k, e in ks.items():
            for pre in STAGE_KERNELS[stage]:
                if k.startswith(pre):
                    base = kernel_family(k)
                    if used and base in PLAN_FAMILIES and base not in used:
                        continue
                    rank = (e.get("dispatches", 0), -e.get("profiled_ms", 0.0))
                    if base not in best or rank > best[base][0]:
                        best[base] = (rank, e)
        best = {b: e for b, (_, e) in best.items()}
        if used and "k_wz_solve_c_next" in used:
            best.pop("k_wz_solve_c", None)  # the plain solve ran only on the series' first frame
        vals = [e.get("hbm_bytes_per_launch") for e in best.values()]
        if not vals or any(v is None for v in vals):
            return None
        return round(sum(vals))
    except (OSError, ValueError, KeyError):
        return None


def cpu_sample_planes(nz, ny, nx, budget_s):
    """z-planes of the bounded CPU sample: the whole frame if it fits the budget, else a z-subvolume."""
    est = nz * ny * nx / 0.5e6  # ~0.5 Mvox/s on one core (measured 0.54 at c2)
    return nz if est <= budget_s else max(1, int(nz * budget_s / est))


def load_cpu_calibration(cfg):
    """t_reference / t_oracle on the same input, one thread, measured in the build container
    (tools/calibrate_cpu.py -> profiles/cpu_calibration.json; the reference itself does not
    travel to the GPU box)."""
    path = os.path.join(REPO, "profiles", "cpu_calibration.json")
    try:
        with open(path) as f:
            cases = json.load(f)["cases"]
    except (OSError, ValueError, KeyError):
        return None
    for name, c in cases.items():
        if name.split("_")[0] == cfg:
            return dict(c, case=name)
    return None


def cpu_baseline(frames, s, t, w, budget_s, nz_total=None, cfg=None):
    """Time the oracle (scipy correlate1d + LAPACK cgeev, the reference's primitives) on 1 thread;
    reference_equiv = that rate / the committed reference-vs-oracle time ratio."""
    from threadpoolctl import threadpool_limits

    from oracle import cpu_ref

    nt, nz, ny, nx = frames.shape
    nz = nz_total or nz
    with threadpool_limits(limits=1):
        sub_nz = min(cpu_sample_planes(nz, ny, nx, budget_s), frames.shape[1])
        sample = frames[:, :sub_nz]
        t0 = time.perf_counter()
        cpu_ref.calc_flow3D(sample, s, t, w, backend="scipy")
        dt = time.perf_counter() - t0
    vox = sub_nz * ny * nx
    what = "full frame" if sub_nz == nz else f"z-subvolume {sub_nz} of {nz} planes"
    return {"value": round(vox / dt / 1e6, 4), "unit": "Mvoxels/s", "cores": 1, "kind": "port",
            "sample": f"{what} ({sub_nz}x{ny}x{nx} voxels, {nt} frames): oracle/cpu_ref.py calc_flow3D with "
                      f"scipy.ndimage.correlate1d + numpy.linalg.eigvals(complex64), 1 thread, {dt:.2f} s",
            "seconds": round(dt, 3), "host_cpus": os.cpu_count(),
            **calibrated(vox / dt / 1e6, cfg)}


def calibrated(oracle_mvox_s, cfg):
    cal = load_cpu_calibration(cfg) if cfg else None
    if not cal:
        return {}
    return {"reference_equiv_value": round(oracle_mvox_s / cal["ratio"], 4),
            "calibration": {"case": cal["case"], "t_reference_over_t_oracle": cal["ratio"],
                            "reference_s": cal["reference_s"], "oracle_s": cal["oracle_s"],
                            "source": "profiles/cpu_calibration.json (tools/calibrate_cpu.py, build container, "
                                      "1 thread, same input)"}}


def max_over_ranks(values, dev):
    """Element-wise MAX over ranks (device tensor for RCCL, host tensor for gloo)."""
    import torch
    import torch.distributed as dist

    where = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor(values, dtype=torch.float64, device=where)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def timed_region(step, plan, args, world, dev, align=None):
    """warmup -> stage profile (K steps with all five stages timed, outside the timed
    region: every HIP event is a barrier packet between kernels, so timing all stages
    inflates the frame by ~8 %) -> the timed region: K steps bracketed by barrier +
    synchronize, with HIP events only around the dominant stage (the roofline kernel).
    align: called (untimed) before the profile pass and the timed region — K0 batching puts
    both on a batch boundary, so K steps hold ceil(K / M) batched K0 launches.
    Returns (elapsed_s, stage profile ms, dominant stage, its ms inside the timed region)."""
    import torch
    import torch.distributed as dist

    for _ in range(args.warmup):
        step()
    if align:
        align()
    torch.cuda.synchronize(dev)
    profile, dom, dom_ms = {}, None, None
    if plan is not None:
        try:
            plan.stage_times()  # drop warmup records
        except RuntimeError:
            pass
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        profile = fused_names(plan.stage_times())
        dom = max(profile, key=profile.get)
        plan.set_timing_stages(["prod_wy" if dom == "prod_wy_wx" else dom])
    if align:
        align()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if plan is not None:
        t = plan.stage_times()
        dom_ms = t["prod_wy" if dom == "prod_wy_wx" else dom]
    return elapsed, profile, dom, dom_ms


def frame_ops_per_voxel(rd, rs, rt, rw):
    """SURVEY §8(d) algorithmic fp64 add/mul count per output voxel (gather form, no FMA):
    C(rt) + 3 C(rd) + 3 [C(rd) + 2 C(rs)] + 9 + 27 C(rw) + 65 + 50 (solve + eigenvalue)."""
    C = lambda r: 1 + 3 * r
    return C(rt) + 3 * C(rd) + 3 * (C(rd) + 2 * C(rs)) + 9 + 27 * C(rw) + 65 + 50


def roofline(profile, dom, dom_ms, model, cfg, frame_bytes, frame_ops, nwin, sv=8, used=None):
    """roofline object of the bench line.

    The exact fp64 path is VALU-bound by construction (28-37 algorithmic
    flop/B against a ridge of ~4.9 flop/B; no FMA allowed by the bit-exact contract), so
    the binding roof is the fp64 (fp32 in OF3D_FP32) add/mul issue rate: achieved = the
    dominant kernel's algorithmic ops per launch (its §8(d) share, stage_model) / its
    HIP-event average over the timed region, against the no-FMA VALU peak.  Beside it:
    the HBM fraction by §8(d)'s algorithmic bytes for the whole frame (nt*2 + 3*sv + 4
    B/voxel) over the frame's device time, the dominant kernel's PMC traffic, and the
    per-stage profile."""
    peak_v = FP64_VALU_PEAK_TOPS if sv == 8 else FP32_VALU_PEAK_TOPS
    model = dict(model)
    if dom == "wz_solve" and used and "k_wz_solve_c_next" in used:
        model["wz_solve"] = {k: model["wz_solve"][k] + model["tderiv_next"][k] for k in ("bytes", "ops")}
    ach = model[dom]["ops"] / (dom_ms * 1e-3) / 1e12
    frame_ms = sum(profile.values())
    k_gbs = model[dom]["bytes"] / (dom_ms * 1e-3) / 1e9
    f_gbs = frame_bytes / (frame_ms * 1e-3) / 1e9
    f_tops = frame_ops / (frame_ms * 1e-3) / 1e12
    return {
        "bound": "valu", "kernel": dom, "achieved": round(ach, 3), "peak": peak_v,
        "unit": "Top/s (%s add/mul lane-ops, no FMA)" % ("fp64" if sv == 8 else "fp32"),
        "frac": round(ach / peak_v, 4), "traffic": load_pmc_traffic(dom, cfg, used),
        "algorithmic_ops_per_launch": model[dom]["ops"], "avg_launch_ms": round(dom_ms, 5),
        "kernel_hbm": {"workspace_bytes_per_launch": model[dom]["bytes"], "achieved_GBs": round(k_gbs, 2),
                       "frac": round(k_gbs / HBM_PEAK_GBS, 4)},
        "stage_ms": {k: round(v, 5) for k, v in profile.items()},
        "stage_ms_note": "separate profile pass with events at every stage boundary (adds ~5 us per event)",
        "frame": {"bytes_per_voxel": nwin * 2 + 3 * sv + 4, "algorithmic_bytes": frame_bytes,
                  "algorithmic_ops": frame_ops, "device_ms": round(frame_ms, 4),
                  "hbm_GBs": round(f_gbs, 2), "hbm_frac": round(f_gbs / HBM_PEAK_GBS, 4),
                  "valu_tops": round(f_tops, 3), "valu_frac": round(f_tops / peak_v, 4)},
    }


class SlabBench:
    """One rank's share of ONE volume per output frame, split over the ranks (strong scaling),
    as process_flow's slab path runs a time series of it (stream.FlowStream(zslab=...)): the
    rank holds its own part (z-planes: axis 0, or rows: axis 1) plus the rd + rw halo of
    2*rt+2 resident frames; a step = the newest frame's halo exchange with the neighbours
    (shard.exchange_frame_halo: RCCL P2P on its own stream, beside the previous step's
    compute) + the rank's compute.  vrank=(r, P): rank r of a P-way split on this one GPU,
    no exchange (the per-rank compute of the scaling model)."""

    def __init__(self, dims, sig, axis, rank, world, dev, fp32=False, timing=0, vrank=None, seed=20260206,
                 pipeline=True, k0_batch=0):
        import torch

        from opticalflow3d_dev_amd import _lib, make_taps, radii
        from opticalflow3d_dev_amd.shard import check_slab_split, halo_planes, zslab_bounds

        nz, ny, nx = dims
        s, t, w = sig
        self.dims, self.axis, self.rank, self.world, self.dev = dims, axis, rank, world, dev
        self.sig, self.seed = (s, t, w), seed
        self.rd, self.rs, self.rt, self.rw = radii(s, t, w)
        self.nwin = 2 * self.rt + 1
        self.fp32 = fp32
        self.vrank = vrank
        prank, pworld = vrank if vrank else (rank, world)
        self.n_ax = nz if axis == 0 else ny
        check_slab_split(self.n_ax, pworld)
        self.a0, self.a1 = zslab_bounds(self.n_ax, prank, pworld)
        self.ai0, self.ai1 = (halo_planes(self.n_ax, self.a0, self.a1, self.rd, self.rw) if pworld > 1
                              else (0, self.n_ax))
        mode = _lib.OF3D_FP32 if fp32 else 0
        taps = make_taps(s, t, w)
        self.rows_direct = False
        if axis == 0:
            self.plan = _lib.Plan(3, nz, ny, nx, taps, device=dev.index, max_out_planes=self.a1 - self.a0,
                                  timing=timing, mode=mode)
            self.blk_shape = (self.ai1 - self.ai0, ny, nx)
        else:
            self.plan = _lib.Plan(3, nz, self.ai1 - self.ai0, nx, taps, device=dev.index, timing=timing, mode=mode)
            self.blk_shape = (nz, self.ai1 - self.ai0, nx)
            self.rows_direct = os.environ.get("OF3D_BENCH_ROWS", "1") == "1"
            if self.rows_direct:
                try:  # the W kernels write only the own rows (halo rows only in K0 / gradients / W y)
                    self.plan.set_rows(self.a0 - self.ai0, self.a1 - self.ai0)
                except RuntimeError:
                    self.rows_direct = False
        # 2 rt + 2 slots (+ 1 with frame pipelining, + M - 1 with K0 batching): the step's
        # exchange goes to the slot the frame before last read
        self.batch = min(k0_batch, 5) if k0_batch >= 2 else 0
        self.L = self.batch - 1 if self.batch else (1 if pipeline else 0)
        nslot = self.nwin + 1 + self.L
        self.ring = torch.empty((nslot,) + self.blk_shape, dtype=torch.int16, device=dev)
        for f in range(nslot):
            if axis == 0:
                synthetic_slab(1, nz, ny, nx, self.ai0, self.ai1, seed + f, dev, out=self.ring[f:f + 1])
            else:
                synthetic_slab(1, nz, ny, nx, 0, nz, seed + f, dev, out=self.ring[f:f + 1], rows=(self.ai0, self.ai1))
        self.own = (self.a1 - self.a0) * (ny * nx if axis == 0 else nz * nx)
        n_out = self.own if (axis == 0 or self.rows_direct) else int(np.prod(self.blk_shape))
        vt = torch.float32 if fp32 else torch.float64
        self.n_out = n_out
        self.outs = [torch.empty(max(n_out, 1), dtype=vt, device=dev) for _ in range(3)]
        self.rel = torch.empty(max(n_out, 1), dtype=torch.float32, device=dev)
        self.comp = torch.cuda.current_stream(dev)
        self.xs = torch.cuda.Stream(device=dev)
        # the ring was generated on the compute stream: the first exchanges (on xs, before any
        # compute event exists for their slots) must not send or overwrite planes still being
        # generated — the 4-rank gloo rehearsal caught halo planes received before the
        # sender's generation finished (a slot exchanged only once before the parity window)
        self.xs.wait_stream(self.comp)
        self.done = {}  # slot -> event of the last compute that read it
        self.xev = {}   # slot -> event of its frame's halo exchange (not yet waited for)
        self.order = list(range(self.nwin + self.L))  # the window (+ the lookahead frames)
        self.k = 0  # steps computed (K0 batching: step k % M == 0 forms M windows' dt0)
        self.last_window = None  # ring slots of the last computed window (slot f holds seed + f)

    def _xchg_view(self, slot):
        v = self.ring[slot]
        return v if self.axis == 0 else v.transpose(0, 1)

    def exchange(self, slot):
        from opticalflow3d_dev_amd.shard import exchange_frame_halo

        exchange_frame_halo(self._xchg_view(slot), self.ai0, self.a0, self.a1, self.n_ax, self.rd + self.rw,
                            self.rank, self.world)

    def step(self, exchange=True, compute=True):
        """A new frame into the free slot (its halo exchanged on the side stream), and the
        rank's compute of the current window on the compute stream.  Without pipelining the
        new frame is the window's newest (the compute waits for its exchange); with it, the
        new frame is the NEXT window's newest (exchanged one step ahead, beside this compute)
        and this compute forms the next window's dt0 (of3d_plan_execute_next); with K0
        batching the M-1 frames after the window are resident and every M-th step's K0 forms
        M windows' dt0 (of3d_plan_execute_ahead)."""
        import torch

        from opticalflow3d_dev_amd import _lib

        new = next(sl for sl in range(len(self.ring)) if sl not in self.order)  # the free slot
        if exchange and self.world > 1 and not self.vrank:
            with torch.cuda.stream(self.xs):
                if new in self.done:
                    self.xs.wait_event(self.done[new])
                self.exchange(new)
                ev = torch.cuda.Event()
                ev.record(self.xs)
            self.xev[new] = ev
        if not self.L:
            self.order.pop(0)
            self.order.append(new)
        for sl in self.order:  # the exchanges this compute reads
            if sl in self.xev:
                self.comp.wait_event(self.xev.pop(sl))
        if compute:
            window = self.order[:self.nwin]
            self.last_window = list(window)
            ptrs = [self.ring[sl].data_ptr() for sl in window]
            nxt = [self.ring[sl].data_ptr() for sl in self.order[1:]] if self.L and not self.batch else None
            ahead = [self.ring[sl].data_ptr() for sl in self.order[self.nwin:]] if self.batch else None
            pipe = bool(self.L) and not self.batch
            o = [t.data_ptr() for t in self.outs] + [self.rel.data_ptr()]
            if self.axis == 0:
                self.plan.execute(ptrs, _lib.OF3D_U16, self.ai0, self.a0, self.a1, *o, self.comp.cuda_stream,
                                  next_ptrs=nxt, pipelined=pipe, ahead_ptrs=ahead)
            else:
                self.plan.execute(ptrs, _lib.OF3D_U16, 0, 0, self.dims[0], *o, self.comp.cuda_stream,
                                  next_ptrs=nxt, pipelined=pipe, ahead_ptrs=ahead)
            ev = torch.cuda.Event()
            ev.record(self.comp)
            for sl in self.order:
                self.done[sl] = ev
            self.k += 1
        if self.L:
            self.order.pop(0)
            self.order.append(new)

    def finite(self):
        return bool(self.outs[0][:self.n_out].isfinite().all().item()) if self.n_out else True

    def describe(self):
        split = "z-slabs" if self.axis == 0 else "row slabs"
        return "%s: %s %d..%d (with halo %d..%d) of %d" % (split, "planes" if self.axis == 0 else "rows", self.a0,
                                                           self.a1, self.ai0, self.ai1, self.n_ax)

    def close(self):
        import torch

        torch.cuda.synchronize(self.dev)
        self.plan.close()


def timed_steps(step, steps, warmup, world, dev):
    """warmup, then `steps` steps between barrier + synchronize; max over ranks (s)."""
    import torch
    import torch.distributed as dist

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    return max_over_ranks([el], dev)[0] if world > 1 else el


def gather_owned_crop(crop, rank, world, dev):
    """Every rank's (5, ...) crop — 4 outputs + an ownership mask of its own voxels — merged on
    rank 0 (all_gather over the process group: device tensors on RCCL, host tensors on gloo):
    each voxel's value from its owner (bits kept) and the count of owners per voxel (1
    everywhere when the slabs tile the crop).  Rank 0 gets the merged crop, the others None."""
    import torch
    import torch.distributed as dist

    where = dev if dist.get_backend() == "nccl" else "cpu"
    mine = crop.to(where)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank != 0:
        return None
    out = torch.zeros_like(mine)
    for q in parts:  # select, not sum: keeps the owner's bits (-0.0 included)
        own = q[4] > 0
        out[:4] = torch.where(own, q[:4], out[:4])
        out[4] += q[4]
    return out


def ring_check(sb, lo, hi):
    """Diagnostics of a failed slab parity sample (rank 0's own ring): for each frame of the last
    window, the planes (rows) of the crop's input box that rank 0 holds, compared with their
    regeneration from the synthetic family — which input frames, if any, differ."""
    import torch

    nz, ny, nx = sb.dims
    out = {}
    a0, a1 = (lo[0], hi[0]) if sb.axis == 0 else (lo[1], hi[1])
    b0, b1 = max(a0, sb.ai0), min(a1, sb.ai1)
    if b1 <= b0:
        return {"note": "rank 0 holds none of the box"}
    for pos, sl in enumerate(sb.last_window):
        if sb.axis == 0:
            have = sb.ring[sl][b0 - sb.ai0:b1 - sb.ai0, lo[1]:hi[1], lo[2]:hi[2]]
            want = synthetic_slab(1, nz, ny, nx, b0, b1, sb.seed + sl, sb.dev, rows=(lo[1], hi[1]))[0][:, :, lo[2]:hi[2]]
        else:
            have = sb.ring[sl][lo[0]:hi[0], b0 - sb.ai0:b1 - sb.ai0, lo[2]:hi[2]]
            want = synthetic_slab(1, nz, ny, nx, lo[0], hi[0], sb.seed + sl, sb.dev, rows=(b0, b1))[0][:, :, lo[2]:hi[2]]
        bad = (have != want)
        if bool(bad.any()):
            idx = bad.nonzero()
            planes = sorted(set(int(v) for v in idx[:, 0].tolist()))
            rec = {"n": int(bad.sum()), "planes_abs": [b0 + v for v in planes][:24]}
            # whose frame is it?  the seed (ring slot) whose regeneration matches the first bad plane
            q = planes[0]
            for other in range(len(sb.ring)):
                if sb.axis == 0:
                    w2 = synthetic_slab(1, nz, ny, nx, b0 + q, b0 + q + 1, sb.seed + other, sb.dev,
                                        rows=(lo[1], hi[1]))[0][:, :, lo[2]:hi[2]]
                    if bool(torch.equal(have[q:q + 1], w2)):
                        rec["first_bad_plane_is_slot"] = other
                        break
            out[f"pos{pos}_slot{sl}"] = rec
    return out or {"note": "rank 0's input planes of the box equal their regeneration", "window": sb.last_window}


def slab_parity(sb, fp32):
    """parity_sample of a slab run (every rank calls it; rank 0 returns the result, the others
    None): one 16^3 output crop straddling the cut between rank 0 and rank 1 on the split axis
    (the volume centre on one GPU), its planes / rows gathered from their owner ranks, checked on
    rank 0 against the oracle of the crop's input box — regenerated from the synthetic family
    the ranks generated their parts from (synthetic_slab: values are a function of the global
    coordinates and the frame's seed), for the frames of the last computed window."""
    import torch
    import torch.distributed as dist

    from opticalflow3d_dev_amd.shard import zslab_bounds

    nz, ny, nx = sb.dims
    dims = (nz, ny, nx)
    world = 1 if sb.vrank else sb.world
    n_ax = dims[sb.axis]
    cut = zslab_bounds(n_ax, 0, world)[1] if world > 1 else n_ax // 2
    box = list(parity_box(dims, sb.axis, cut))
    z0, z1, y0, y1, x0, x1 = box
    # this rank's own outputs inside the box: 4 outputs + an ownership mask, as float64
    crop = torch.zeros((5, z1 - z0, y1 - y0, x1 - x0), dtype=torch.float64, device=sb.dev)
    b0, b1 = (z0, z1) if sb.axis == 0 else (y0, y1)
    o0, o1 = max(b0, sb.a0), min(b1, sb.a1)
    if o1 > o0 and sb.n_out:
        for k, o in enumerate(sb.outs + [sb.rel]):
            if sb.axis == 0:
                v = o[:sb.n_out].view(sb.a1 - sb.a0, ny, nx)[o0 - sb.a0:o1 - sb.a0, y0:y1, x0:x1]
                crop[k, o0 - z0:o1 - z0] = v.double()
            else:
                r0 = sb.a0 if sb.rows_direct else sb.ai0
                rows = (sb.a1 - sb.a0) if sb.rows_direct else (sb.ai1 - sb.ai0)
                v = o[:sb.n_out].view(nz, rows, nx)[z0:z1, o0 - r0:o1 - r0, x0:x1]
                crop[k, :, o0 - y0:o1 - y0] = v.double()
        if sb.axis == 0:
            crop[4, o0 - z0:o1 - z0] = 1
        else:
            crop[4, :, o0 - y0:o1 - y0] = 1
    if world > 1:
        crop = gather_owned_crop(crop, sb.rank, world, sb.dev)
        if crop is None:
            return None
    if not bool((crop[4] == 1).all()):
        return {"ok": False, "error": "crop voxels not owned exactly once", "crop_out": box}
    got = [crop[k].cpu().numpy() for k in range(4)]
    # the window's input box (crop + the rd + rw halo), regenerated on rank 0
    h = sb.rd + sb.rw
    lo = [max(a - h, 0) for a in (z0, y0, x0)]
    hi = [min(b + h, n) for b, n in zip((z1, y1, x1), dims)]
    sub = np.stack([synthetic_slab(1, nz, ny, nx, lo[0], hi[0], sb.seed + sl, sb.dev, rows=(lo[1], hi[1]))[0]
                    [:, :, lo[2]:hi[2]].cpu().numpy().view(np.uint16) for sl in sb.last_window])
    r = parity_check(sub, lo, box, got, *sb.sig, fp32=fp32)
    if not r["ok"] and os.environ.get("OF3D_BENCH_RING_CHECK", "1") == "1":
        r["ring_check"] = ring_check(sb, lo, hi)
    r["window_slots"] = list(sb.last_window)
    r["where"] = ("across the cut between rank 0 and rank 1 (%s %d)" % ("plane" if sb.axis == 0 else "row", cut)
                  if world > 1 else "volume centre")
    return r


def default_config(world):
    """The BASELINE.json config named for `world` GPUs: configs[2] (c3) on one GPU, configs[3]
    (c4, "z-slab split across 2 and 4 MI355X") below 8, configs[4] (c5, "8 MI355X") at 8+."""
    return "c3" if world == 1 else ("c4" if world < 8 else "c5")


def parity_box(dims, axis, cut, size=16, dx=44):
    """The slab parity crop (z0, z1, y0, y1, x0, x1): `size` voxels per side centred on `cut`
    along the split axis (the first rank cut; the volume centre on one GPU) and near the volume
    centre (x offset dx) on the other axes, clipped into the volume."""
    ctr = [dims[0] // 2, dims[1] // 2, dims[2] // 2 + dx]
    ctr[axis] = cut
    box = []
    for c, n in zip(ctr, dims):
        a = min(max(c - size // 2, 0), max(n - size, 0))
        box += [a, min(a + size, n)]
    return tuple(box)


def device_used_gb(dev):
    """Device memory in use on `dev` right now (every allocator: torch's and the plans'
    hipMalloc), from hipMemGetInfo, GB."""
    import torch

    free, total = torch.cuda.mem_get_info(dev)
    return round((total - free) / 1e9, 2), round(total / 1e9, 2)


def slab_on_every_rank(world, dev, *a, **kw):
    """SlabBench(*a, **kw) on every rank, or on none: the ranks agree (a MAX over ranks) before
    any of them starts timed steps, so a rank that cannot allocate its part (device memory)
    does not leave the others waiting in a collective; raises on every rank then."""
    import torch

    sb, err = None, ""
    try:
        sb = SlabBench(*a, **kw)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"[:200]
    bad = max_over_ranks([0.0 if sb is not None else 1.0], dev)[0] if world > 1 else (0.0 if sb else 1.0)
    if bad:
        if sb is not None:
            sb.close()
        del sb
        torch.cuda.empty_cache()
        raise RuntimeError("slab setup failed on a rank" + (": " + err if err else ""))
    return sb


def strong_split(cfg, axis, world, rank, dev, steps, warmup, t1_ms, pipeline=True, k0_batch=0, fp32=False,
                 parity=True):
    """A volume's frame split over the N ranks (strong scaling) — the path configs[3]/[4] and
    process_flow(parallel="zslab"/"yslab") run: per-rank compute alone, the halo exchange alone
    (RCCL P2P of the newest frame's rd + rw planes / rows), and the pipelined step (exchange
    beside the previous step's compute), with a parity sample across the rank-0/1 cut.
    efficiency = the one-GPU frame time t1 (None: not measured) / (N * step)."""
    nt, nz, ny, nx, s, t, w, _ = CONFIGS[cfg]
    sb = slab_on_every_rank(world, dev, (nz, ny, nx), (s, t, w), axis, rank, world, dev, fp32=fp32,
                            seed=20260206 + 50, pipeline=pipeline, k0_batch=k0_batch)
    used = device_used_gb(dev)[0]
    if world > 1:
        used = max_over_ranks([used], dev)[0]
    try:
        comp = timed_steps(lambda: sb.step(exchange=False), steps, warmup, world, dev)
        xchg = timed_steps(lambda: sb.step(compute=False), steps, warmup, world, dev)
        both = timed_steps(sb.step, steps, warmup, world, dev)
        finite = sb.finite()
        desc = sb.describe()
        par = slab_parity(sb, fp32) if parity else None
    finally:
        sb.close()
    ms = both / steps * 1e3
    return {"split": "z-slabs" if axis == 0 else "row slabs", "halo": sb.rd + sb.rw, "rank0_part": desc,
            "ms_per_step": round(ms, 5), "value": round(nz * ny * nx / (ms * 1e-3) / 1e6, 3), "unit": "Mvoxels/s",
            "compute_ms_max_rank": round(comp / steps * 1e3, 5), "exchange_ms": round(xchg / steps * 1e3, 5),
            "efficiency_vs_one_gpu_frame": round(t1_ms / (world * ms), 4) if t1_ms else None,
            "device_used_GB_max_rank": used, "outputs_finite_rank0": finite, "parity_sample": par}


def replica_frame(cfg, world, rank, dev, steps, warmup, fp32, pipeline, k0_batch):
    """Every rank computes the WHOLE volume of cfg on its own GPU at once (one-GPU frames,
    replicas): the one-GPU frame time t1 the split's efficiency is measured against, on this
    node in this job (max over ranks), and the weak-scaling throughput of N replicas."""
    import torch

    nt, nz, ny, nx, s, t, w, _ = CONFIGS[cfg]
    sb = slab_on_every_rank(world, dev, (nz, ny, nx), (s, t, w), 0, rank, world, dev, fp32=fp32, vrank=(0, 1),
                            seed=20260206 + 60 + rank, pipeline=pipeline, k0_batch=k0_batch)
    try:
        used, total = device_used_gb(dev)
        el = timed_steps(sb.step, steps, warmup, world, dev)
    finally:
        sb.close()
        del sb
        torch.cuda.empty_cache()
    ms = el / steps * 1e3
    if world > 1:
        used = max_over_ranks([used], dev)[0]
    return {"ms_per_step": round(ms, 5), "value": round(world * nz * ny * nx / (ms * 1e-3) / 1e6, 3),
            "unit": "Mvoxels/s", "scaling": "weak", "device_used_GB": used, "device_total_GB": total,
            "what": f"{world} one-GPU frames at once (every rank its own whole volume), max over ranks"}


def run_slab(args, world, rank, local_rank, dev):
    """configs[3] / configs[4], and every N > 1 line: ONE volume per output frame, split over the
    ranks (strong scaling) — SlabBench, as process_flow(parallel="zslab") runs it.  The split
    axis defaults to z (the north star's "volumes shard along z"); --split y / auto.  N > 1
    also measures, beside the headline split: the one-GPU frame of the same volume on every
    rank at once ("replicas": t1 for the efficiency) and the other axis's split ("row_slabs").
    OF3D_BENCH_VRANK="r/P": time rank r of a P-way split on this one GPU (no exchange) — the
    per-rank compute the scaling model in DESIGN.md uses."""
    import torch

    from opticalflow3d_dev_amd import radii
    from opticalflow3d_dev_amd.shard import slab_axis

    cfg = args.config
    nt, nz, ny, nx, s, t, w, desc = CONFIGS[cfg]
    rd, rs, rt, rw = radii(s, t, w)
    nwin = 2 * rt + 1
    fp32 = cfg in FP32_CONFIGS or args.precision == "fp32"
    sv = 4 if fp32 else 8
    vr = os.environ.get("OF3D_BENCH_VRANK")
    prank, pworld = (int(v) for v in vr.split("/")) if vr else (rank, world)
    axis = {"z": 0, "y": 1}.get(args.split, None)
    if axis is None:
        axis = slab_axis(nz, ny, pworld, rd, rw)
    kb = 0 if args.no_pipeline else args.k0_batch
    replicas = None
    if world > 1 and not vr and not args.no_replicas:
        try:  # the one-GPU frame first (it holds the whole volume: freed before the split)
            replicas = replica_frame(cfg, world, rank, dev, args.steps, args.warmup, fp32, not args.no_pipeline, kb)
        except Exception as e:  # noqa: BLE001
            replicas = {"error": f"{type(e).__name__}: {e}"[:300]}
            torch.cuda.empty_cache()
    seed = 20260206 + (5 if fp32 else 4)
    # the replicas' whole-volume plan, ring and outputs must be gone before the split allocates
    # (c5 at N = 8: ~266 GB of 288 per GPU for the replica, then the slab plans)
    base_used, total_gb = device_used_gb(dev)
    # (one GPU per rank under RCCL; gloo rehearsals share a device between ranks)
    if replicas is not None and os.environ.get("OF3D_BENCH_BACKEND", "nccl") == "nccl" and base_used > 8.0:
        raise RuntimeError(f"replica buffers not freed before the split: {base_used} GB still in use")
    sb = SlabBench((nz, ny, nx), (s, t, w), axis, rank, world, dev, fp32=fp32, timing=max(args.steps, 1),
                   vrank=(prank, pworld) if vr else None, seed=seed, pipeline=not args.no_pipeline, k0_batch=kb)
    split_used = device_used_gb(dev)[0]
    plan = sb.plan

    def align():
        while sb.k % sb.batch:
            sb.step()

    elapsed, profile, dom, dom_ms = timed_region(sb.step, plan, args, world, dev, align=align if sb.batch else None)
    finite = sb.finite()
    if world > 1:
        elapsed, bad, split_used = max_over_ranks([elapsed, 0.0 if finite else 1.0, split_used], dev)
        finite = bad == 0.0
    parity = None if args.no_parity_sample or vr else slab_parity(sb, fp32)
    split_detail = None
    if world > 1 and not vr:  # compute alone / exchange alone on the same ranks and ring
        comp = timed_steps(lambda: sb.step(exchange=False), args.steps, args.warmup, world, dev)
        xchg = timed_steps(lambda: sb.step(compute=False), args.steps, args.warmup, world, dev)
        split_detail = {"compute_ms_max_rank": round(comp / args.steps * 1e3, 5),
                        "exchange_ms": round(xchg / args.steps * 1e3, 5),
                        "pipelined_step_ms": round(elapsed / args.steps * 1e3, 5),
                        "exchange": f"RCCL P2P ({'nccl' if os.environ.get('OF3D_BENCH_BACKEND', 'nccl') == 'nccl' else 'gloo rehearsal'}) "
                                    f"of the newest frame's {rd + rw} halo {'planes' if axis == 0 else 'rows'} per "
                                    "neighbour, on its own stream beside the previous step's compute"}
    kernels = set(plan.kernels())
    geometry = plan.geometry()
    own, ai0, ai1, a0, a1, describe = sb.own, sb.ai0, sb.ai1, sb.a0, sb.a1, sb.describe()
    rows_direct = sb.rows_direct
    sb.close()
    del sb
    torch.cuda.empty_cache()
    other = None
    if world > 1 and not vr and not args.no_strong and world <= (nz, ny)[1 - axis]:
        try:  # the other axis's split of the same volume (row slabs beside the z-slab headline)
            t1 = replicas.get("ms_per_step") if replicas else None
            other = strong_split(cfg, 1 - axis, world, rank, dev, args.steps, args.warmup, t1,
                                 pipeline=not args.no_pipeline, k0_batch=kb, fp32=fp32,
                                 parity=not args.no_parity_sample)
        except Exception as e:  # noqa: BLE001
            other = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0:
        vox = nz * ny * nx
        if axis == 0:
            nb, no, ng = ai1 - ai0, a1 - a0, min(a1 + rw, nz) - max(a0 - rw, 0)
            plane = ny * nx
        else:
            nb = no = ng = nz
            plane = (ai1 - ai0) * nx
        roof = roofline(profile, dom, dom_ms, stage_model(nwin, rd, rs, rt, rw, nb, ng, no, plane, sv), cfg,
                        (nwin * 2 + 3 * sv + 4) * own, frame_ops_per_voxel(rd, rs, rt, rw) * own, nwin, sv,
                        used=kernels)
        roof["frame"]["note"] = "this rank's share: " + describe
        if world > 1 or vr:
            # the committed PMC profile measured a whole-volume launch: its bytes do not describe
            # this rank's slab launch (fewer planes + the halo), and no slab PMC pass exists
            whole = roof["traffic"]
            roof["traffic"] = None
            roof["traffic_note"] = (f"not measured for slab launches (profiles/pmc_{cfg}.json is the whole-volume "
                                    f"launch: {whole} B); kernel_hbm.workspace_bytes_per_launch is this slab's")
        cpu = None
        if world == 1 and not vr and not args.no_cpu_baseline:
            sub = cpu_sample_planes(nz, ny, nx, args.cpu_budget)
            host = synthetic_slab(nwin, nz, ny, nx, 0, sub, seed, dev).cpu().numpy().view(np.uint16)
            cpu = cpu_baseline(host, s, t, w, args.cpu_budget, nz_total=nz, cfg=cfg)
        split = ("z-slabs" if axis == 0 else "row slabs")
        ms = elapsed / args.steps * 1e3
        if split_detail is not None and replicas and "ms_per_step" in replicas:
            split_detail["efficiency_vs_one_gpu_frame"] = round(replicas["ms_per_step"] / (world * ms), 4)
        nres = nwin + 1 + (kb - 1 if kb >= 2 else (0 if args.no_pipeline else 1))
        line = {
            "metric": "Mvoxels/s per frame-pair (and HBM GB/s fraction) at 1/2/4/8 MI355X",
            "value": round((own if vr else vox) * args.steps / elapsed / 1e6, 3), "unit": "Mvoxels/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 5), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32" if fp32 else "f64", "data": "synthetic",
            "config": {"workload": desc, "nt": nt, "nz": nz, "ny": ny, "nx": nx, "xyzSig": s, "tSig": t,
                       "wSig": w,
                       "parallelism": (f"virtual rank {prank} of {pworld} ({split}, compute only)" if vr else
                                       f"{split} x{world}, halo {rd + rw}" if world > 1 else "single GPU (whole frame)"),
                       "inputs": f"own part (+ halo) of a ring of {nres} uint16 frames resident in HBM; per step the "
                                 "newest frame's halo exchange (RCCL P2P, own stream) + compute",
                       "outputs_finite": finite, "geometry": geometry,
                       "row_outputs": "own rows only (of3d_plan_set_rows)" if (axis == 1 and rows_direct) else None,
                       "series": (f"K0 batching: {kb} windows per K0 pass (of3d_plan_execute_ahead)") if kb >= 2 else
                                 ("frame pipelining (of3d_plan_execute_next)" if not args.no_pipeline else "plain")},
            "roofline": roof, "cpu_baseline": cpu, "parity_sample": parity, "build": build_stamp(),
            "memory": {"device_total_GB": total_gb, "before_split_GB": base_used,
                       "split_GB_max_rank": split_used,
                       "replicas_GB_max_rank": (replicas or {}).get("device_used_GB")},
        }
        if split_detail is not None:
            line["split"] = split_detail
        if replicas is not None:
            line["replicas"] = replicas
        if other is not None:
            line["row_slabs" if axis == 0 else "z_slabs"] = other
        print(json.dumps(line), flush=True)


def build_stamp():
    """The loaded library's provenance (of3d_build_info: source hash, flags; the tree's hash)."""
    from opticalflow3d_dev_amd import _lib

    i = _lib.build_info()
    return {"src_hash": i["src_hash"], "tree_hash": i["tree_hash"], "extra": i["extra"], "lib": i["lib"]}


def parity_check(sub, lo, box, got, s, t, w, fp32=False):
    """Outputs `got` (vx, vy, vz, rel host arrays of the box) against the oracle
    (oracle/cpu_ref.py, the CPU restatement pinned to the reference) run on `sub`, the
    window's uint16 input over the box + the rd + rw halo (origin `lo`) — outside any timed
    region, the checker only.  Output voxels further than rd + rw from every face where the
    crop cuts the volume are exact (tests/test_gpu_bench_geometry.py): vx/vy/vz must match bit
    for bit (fp32 runs: within 1e-4 max|v|), rel within 1e-6 lambda_max (fp32: 1e-4)."""
    from oracle import cpu_ref

    z0, z1, y0, y1, x0, x1 = box
    st = cpu_ref.structure_tensor3d(np.ascontiguousarray(sub), s, t, w, backend="scipy")
    want = cpu_ref.solve3d(st)
    lmin, lmax = cpu_ref.eig_fp64_3d(st)
    sl = (slice(z0 - lo[0], z1 - lo[0]), slice(y0 - lo[1], y1 - lo[1]), slice(x0 - lo[2], x1 - lo[2]))
    if fp32:
        dv = max(float(np.abs(np.asarray(g, np.float64) - v[sl]).max() / np.abs(v[sl]).max())
                 for g, v in zip(got, want))
        ok_v = dv <= 1e-4
    else:
        ok_v = all(np.array_equal(np.ascontiguousarray(g, np.float64).view(np.uint64),
                                  np.ascontiguousarray(v[sl]).view(np.uint64)) for g, v in zip(got, want))
    rel_err = float(np.max(np.abs(np.asarray(got[3], np.float64) - lmin[sl]) / (np.abs(lmax[sl]) + 1e-300)))
    ok = bool(ok_v and rel_err <= (1e-4 if fp32 else 1e-6))
    r = {"ok": ok, "crop_out": list(box), "vxyz": ("within 1e-4 max|v|" if fp32 else "bitwise") if ok_v else
         "MISMATCH", "rel_max_err_over_lmax": rel_err, "checker": "oracle/cpu_ref.py (scipy backend)"}
    if not ok_v:  # where and how far (crop-relative z planes of the differing voxels)
        diff = [np.asarray(g, np.float64) != v[sl] for g, v in zip(got[:3], want)]
        bad = diff[0] | diff[1] | diff[2]
        r["n_mismatch"] = int(bad.sum())
        r["mismatch_planes"] = sorted(set(int(z) for z in np.nonzero(bad)[0]))
        r["max_abs_diff_over_max"] = max(float(np.abs(np.asarray(g, np.float64) - v[sl]).max() /
                                             (np.abs(v[sl]).max() + 1e-300)) for g, v in zip(got[:3], want))
    return r


def parity_sample(d_in, outs, box, s, t, w, fp32=False):
    """The single-GPU headline's parity sample: one crop of the resident outputs against the
    oracle of the same device input (parity_check)."""
    from opticalflow3d_dev_amd import radii

    rd, _, _, rw = radii(s, t, w)
    h = rd + rw
    nt, nz, ny, nx = d_in.shape
    z0, z1, y0, y1, x0, x1 = box
    lo = [max(a - h, 0) for a in (z0, y0, x0)]
    hi = [min(b + h, n) for b, n in zip((z1, y1, x1), (nz, ny, nx))]
    sub = d_in[:, lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]].cpu().numpy().view(np.uint16)
    got = [o.view(nz, ny, nx)[z0:z1, y0:y1, x0:x1].cpu().numpy() for o in outs]
    return parity_check(sub, lo, box, got, s, t, w, fp32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: c3 = configs[2] on one GPU (the single-GPU headline); at N > 1 the volume "
                         "the BASELINE config names for N GPUs, z-sharded over the ranks: c4 = configs[3] "
                         "(2 and 4 GPUs), c5 = configs[4] (8 GPUs); c2 = configs[1]; c1 = configs[0] (2D)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--overlap", type=int, default=int(os.environ.get("OF3D_BENCH_OVERLAP", "-1")),
                    help="z chunk (output planes) of the plan's overlap mode; 0 = serial; -1 = the plan's default")
    ap.add_argument("--cpu-budget", type=float, default=25.0, help="seconds of CPU work for cpu_baseline")
    ap.add_argument("--split", default="z", choices=("auto", "z", "y"),
                    help="c4/c5 and N > 1: split axis of the volume over the ranks (z: the north star's "
                         "z-shard, the default; auto: the axis with less halo work, process_flow's choice)")
    ap.add_argument("--no-strong", action="store_true", help="N > 1: skip the other axis's split (sub-object)")
    ap.add_argument("--no-replicas", action="store_true",
                    help="N > 1: skip the one-GPU frame of the same volume on every rank (t1 of the efficiency)")
    ap.add_argument("--no-single-window", action="store_true",
                    help="c2/c3: skip the single-window measurement (2rt+1 resident frames, K0 every step)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="neither K0 batching nor frame pipelining: every step launches its own K0 "
                         "(of3d_plan_execute)")
    ap.add_argument("--k0-batch", type=int, default=int(os.environ.get("OF3D_BENCH_K0_BATCH", "5")),
                    help="K0 batching (of3d_plan_execute_ahead, the default series mode): M = 2..5 consecutive "
                         "windows of a series of 2rt+M resident frames, one K0 pass every M steps; 0 = frame "
                         "pipelining (of3d_plan_execute_next) instead")
    ap.add_argument("--no-parity-sample", action="store_true", help="skip the oracle check of one output crop")
    ap.add_argument("--precision", default="fp64", choices=("fp64", "fp32"),
                    help="fp64 = bit-exact path (the metric's); fp32 = OF3D_FP32 (configs[4]'s path; c5 forces it)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    explicit = args.config is not None
    if not explicit:  # the BASELINE config for this GPU count
        args.config = default_config(world)
    nt, nz, ny, nx, s, t, w, desc = CONFIGS[args.config]

    import torch
    import torch.distributed as dist

    from opticalflow3d_dev_amd import _lib, make_taps, radii

    # OF3D_BENCH_BACKEND=gloo rehearses the N>1 logic with several ranks on fewer GPUs
    # (ranks share devices round-robin); the driver's runs use RCCL ("nccl"), one GPU per rank.
    backend = os.environ.get("OF3D_BENCH_BACKEND", "nccl")
    gpu = local_rank % max(torch.cuda.device_count(), 1) if backend == "gloo" else local_rank
    os.environ["OF3D_DEVICE"] = str(gpu)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if args.config == "c1":
        run_2d(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.config in ZSLAB_CONFIGS or (world > 1 and not explicit):
        run_slab(args, world, rank, local_rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    rd, rs, rt, rw = radii(s, t, w)
    nwin = 2 * rt + 1
    # the 2*rt+1 frames around the centre, generated on the device (synthetic_slab: the
    # SURVEY §8d family; every rank its own seed, i.e. its own output frame)
    kb = max(0, min(args.k0_batch, 5))
    kb = kb if kb >= 2 and not args.no_pipeline else 0
    nres = nwin + (kb - 1 if kb else 0)  # resident frames: the window (+ the batch's lookahead)
    d_in = synthetic_slab(nres, nz, ny, nx, 0, nz, 20260206 + int(args.config[1:]) + 100 * rank, dev)
    vox = nz * ny * nx
    fp32 = args.precision == "fp32"
    sv = 4 if fp32 else 8
    d_vx = torch.empty(vox, dtype=torch.float32 if fp32 else torch.float64, device=dev)
    d_vy = torch.empty_like(d_vx)
    d_vz = torch.empty_like(d_vx)
    d_rel = torch.empty(vox, dtype=torch.float32, device=dev)

    plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=dev.index, timing=max(args.steps, 1),
                     mode=_lib.OF3D_FP32 if fp32 else 0)
    if args.overlap >= 0:
        plan.set_overlap(args.overlap)
    aptrs = [d_in[i].data_ptr() for i in range(nres)]
    fptrs = aptrs[:nwin]
    stream = torch.cuda.current_stream(dev).cuda_stream

    pipe = not args.no_pipeline and not kb
    last = {"j": 0, "i": 0}

    def step():
        if kb:
            # K0 batching (of3d_plan_execute_ahead): step i is window j = i mod M of a series of
            # 2rt+M resident frames; the j = 0 step forms the M windows' temporal derivatives in one
            # pass, the next M-1 steps use theirs (every M timed steps run one batched K0)
            j = last["i"] % kb
            last["i"] += 1
            last["j"] = j
            plan.execute(aptrs[j:j + nwin], _lib.OF3D_U16, 0, 0, nz, d_vx.data_ptr(), d_vy.data_ptr(),
                         d_vz.data_ptr(), d_rel.data_ptr(), stream, ahead_ptrs=aptrs[j + nwin:])
            return
        # frame pipelining (of3d_plan_execute_next): this step's W-z/solve kernel also forms the
        # next step's temporal derivative (the next frame of a series; here the same resident
        # frames), so every timed step runs K12 + K34 + K5c-with-the-next-K0
        plan.execute(fptrs, _lib.OF3D_U16, 0, 0, nz, d_vx.data_ptr(), d_vy.data_ptr(), d_vz.data_ptr(),
                     d_rel.data_ptr(), stream, next_ptrs=fptrs if pipe else None, pipelined=pipe)

    def align():
        while last["i"] % kb:
            step()

    elapsed, profile, dom, dom_ms = timed_region(step, plan, args, world, dev, align=align if kb else None)
    if world > 1:
        (elapsed,) = max_over_ranks([elapsed], dev)

    # sanity: finite outputs
    finite = bool(torch.isfinite(d_vx).all().item())
    kernels = set(plan.kernels())
    geometry = plan.geometry()
    ms_step = elapsed / args.steps * 1e3
    parity = None
    if rank == 0 and not args.no_parity_sample:
        # one 16^3 output crop across the kernels' seams (K5c / K12 z chunk 64, K34 row chunk
        # 256 at c3) against the oracle, outside the timed region
        zc, yc, xc = min(64, nz // 2), min(256, ny // 2), nx // 2 + 44
        box = (zc - 8, zc + 8, yc - 8, yc + 8, min(xc, nx - 16), min(xc, nx - 16) + 16)
        jl = last["j"]  # the window of the last step (its outputs are in d_v*)
        parity = parity_sample(d_in[jl:jl + nwin], (d_vx, d_vy, d_vz, d_rel), box, s, t, w, fp32)
    single = None
    if kb and not args.no_single_window:
        # configs[2] as stated: ONE window of 2rt+1 resident frames, every step a plain
        # of3d_plan_execute (K0 every step), the same warmup / steps between barrier + sync
        def step1():
            plan.execute(fptrs, _lib.OF3D_U16, 0, 0, nz, d_vx.data_ptr(), d_vy.data_ptr(), d_vz.data_ptr(),
                         d_rel.data_ptr(), stream)

        el1 = timed_steps(step1, args.steps, args.warmup, world, dev)
        single = {"ms_per_step": round(el1 / args.steps * 1e3, 5),
                  "value": round(world * vox * args.steps / el1 / 1e6, 3), "unit": "Mvoxels/s",
                  "resident_frames": nwin,
                  "what": f"one {nwin}-frame window resident (configs[{int(args.config[1:]) - 1}] as stated), a plain "
                          "of3d_plan_execute per step: K0 + K12 + K34 + K5c every step"}
    plan.close()

    # N > 1: the same frame split over the ranks (strong scaling, halo exchange over RCCL):
    # z-slabs (the north star's axis) and the axis with less halo work (row slabs here)
    strong = None
    if world > 1 and not args.no_strong:
        from opticalflow3d_dev_amd.shard import slab_axis

        axes = [0] + ([1] if slab_axis(nz, ny, world, rd, rw) == 1 else [])
        strong = {}
        for ax in axes:
            if world > (nz, ny)[ax]:
                continue
            try:  # the replica line stands on its own: a failed split is reported in it, not fatal
                r = strong_split(args.config, ax, world, rank, dev, args.steps, args.warmup, ms_step,
                                 pipeline=not args.no_pipeline, k0_batch=kb, fp32=fp32,
                                 parity=not args.no_parity_sample)
            except Exception as e:  # noqa: BLE001
                r = {"error": f"{type(e).__name__}: {e}"[:300]}
            strong["zslab" if ax == 0 else "yslab"] = r

    if rank == 0:
        value = world * vox * args.steps / elapsed / 1e6
        roof = roofline(profile, dom, dom_ms, stage_model(nwin, rd, rs, rt, rw, nz, nz, nz, ny * nx, sv),
                        args.config if not fp32 else args.config + "_fp32", (nwin * 2 + 3 * sv + 4) * vox,
                        frame_ops_per_voxel(rd, rs, rt, rw) * vox, nwin, sv, used=kernels)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sub = min(cpu_sample_planes(nz, ny, nx, args.cpu_budget), nz)
            host = d_in[:nwin, :sub].cpu().numpy().view(np.uint16)
            cpu = cpu_baseline(host, s, t, w, args.cpu_budget, nz_total=nz, cfg=args.config)
        line = {
            "metric": "Mvoxels/s per frame-pair (and HBM GB/s fraction) at 1/2/4/8 MI355X",
            "value": round(value, 3), "unit": "Mvoxels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32" if fp32 else "f64", "data": "synthetic",
            "config": {"workload": desc, "nt": nres, "nt_window": nwin, "nz": nz, "ny": ny, "nx": nx, "xyzSig": s,
                       "tSig": t, "wSig": w, "parallelism": f"frame replicas x{world}" if world > 1 else "single GPU",
                       "inputs": (f"a time series of {nres} uint16 frames resident in HBM: {kb} consecutive "
                                  f"{nwin}-frame windows (output frames), step i computes window i mod {kb}"
                                  if kb else f"one {nwin}-frame window of uint16 frames resident in HBM"),
                       "outputs_finite": finite, "geometry": geometry,
                       "frame_pipelining": ("each step's W-z/solve kernel also forms the next step's temporal "
                                            "derivative (of3d_plan_execute_next); stage grad_xy is then empty")
                       if pipe else None,
                       "k0_batch": (f"{kb} consecutive windows of a series of {nres} resident frames; one "
                                    f"batched K0 pass (of3d_plan_execute_ahead) every {kb} steps"
                                    + ("; the timed region starts on a batch" if args.steps % kb == 0 else
                                       f"; the timed region starts on a batch: {-(-args.steps // kb)} passes in "
                                       f"{args.steps} steps"))
                       if kb else None},
            "roofline": roof, "cpu_baseline": cpu,
            "parity_sample": parity, "build": build_stamp(),
        }
        if single is not None:
            line["single_window_ms"] = single["ms_per_step"]
            line["single_window_value"] = single["value"]
            line["single_window"] = single
        if strong is not None:
            line["strong"] = dict(strong, note="the same frame split over the ranks (halo exchange over "
                                               "RCCL P2P beside compute); value = frame voxels / step time")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
