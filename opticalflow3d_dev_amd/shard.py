"""Multi-GPU decomposition of the LK hot path.

Two ways the path shards, both one process per GPU (process_flow picks one per run):

1. Frame replicas — output frames are independent (the reference's own note,
   calc_flow.py:512: "this could become a parfor loop").  Rank r takes output
   frames r, r+P, ...; no collective on the data path.

2. Slabs of one large frame — rank p owns output planes [z0_p, z1_p) (or rows, the
   same way).  Every stage clamps at the GLOBAL volume edge (scipy mode='nearest' on
   the whole volume), so a slab computed from input planes [z0-H, z1+H) ∩ [0, Nz) with
   H = rd + rw (gradient z-pass radius + window z-pass radius) is bit-identical to the
   same planes of the unsharded result.  The plan reports the exact input range
   (of3d_plan_input_range).  Each rank reads only its own planes of every frame; the
   halo planes come from the neighbours: ``exchange_frame_halo`` (one frame per output
   frame, stream.FlowStream(zslab=...)) sends/receives them with torch.distributed
   point-to-point (RCCL over xGMI for CUDA tensors, gloo staged through host memory) —
   the only collective on this path.  Every rank must own at least one plane (row):
   ``check_slab_split`` refuses thinner splits (process_flow then splits frames).
"""

from __future__ import annotations

import numpy as np

from . import _lib
from .taps import make_taps, radii


def init_distributed(backend=None):
    """One process per GPU under torchrun (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* in the
    environment): selects GPU LOCAL_RANK and initialises torch.distributed — RCCL ("nccl")
    by default, $OF3D_DIST_BACKEND or `backend` to override (gloo: tests / rehearsals).
    Returns (rank, world).  process_flow then splits its work over the ranks."""
    import os

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world == 1 or dist.is_initialized():
        return (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    backend = backend or os.environ.get("OF3D_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ngpu = torch.cuda.device_count()
    gpu = local % max(ngpu, 1)
    os.environ["OF3D_DEVICE"] = str(gpu)
    if ngpu:
        torch.cuda.set_device(gpu)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    else:
        dist.init_process_group(backend)
    return rank, world


# measured share of each stage in a c3 frame (profiles/r02c_c3_k12_bench.log): K0 tderiv,
# K12 gradients, K34 products + W y + W x, K5c W z + solve
STAGE_SHARE = {"tderiv": 0.08, "grad": 0.16, "prod_wyx": 0.49, "wz_solve": 0.27}


def slab_work(n_split: int, n_other_split: int, world: int, rd: int, rw: int, axis: int) -> float:
    """Predicted work of the busiest slab rank relative to 1/world of the frame, from the
    stage shares: z-slabs (axis 0) recompute K0 / gradients on rd + rw and the products
    on rw halo planes per cut side (K5c only on own planes); row slabs (axis 1) run the
    whole pipeline on the rank's rows + rd + rw halo rows per cut side."""
    own = -(-n_split // world)
    cuts = 2 if world > 2 else (1 if world == 2 else 0)
    if axis == 0:
        extra = (STAGE_SHARE["tderiv"] + STAGE_SHARE["grad"]) * (rd + rw) + STAGE_SHARE["prod_wyx"] * rw
        return 1.0 + cuts * extra / own
    return 1.0 + cuts * (rd + rw) / own


def slab_axis(nz: int, ny: int, world: int, rd: int, rw: int) -> int:
    """The split axis with less predicted halo work: 0 (z-slabs) or 1 (row slabs)."""
    return 0 if slab_work(nz, ny, world, rd, rw, 0) <= slab_work(ny, nz, world, rd, rw, 1) else 1


def frame_assignment(n_frames: int, rank: int, world: int) -> list:
    """Output frames of rank `rank` under round-robin replicas."""
    return list(range(rank, n_frames, world))


def frame_blocks(n_frames: int, rank: int, world: int) -> tuple:
    """Contiguous output frames [a, b) of rank `rank` (balanced): a rank streaming its block
    through a frame ring uploads b - a + 2 rt frames instead of (b - a) (2 rt + 1)."""
    return zslab_bounds(n_frames, rank, world)


def halo_transfers(nz: int, rank: int, world: int, halo: int) -> tuple:
    """One frame's halo traffic of rank `rank`: ([(peer, s0, s1)] planes it sends,
    [(peer, g0, g1)] planes it receives); global plane indices.  Slabs thinner than the
    halo exchange with several ranks; empty slabs neither send nor receive."""
    z0, z1 = zslab_bounds(nz, rank, world)
    if z1 <= z0:
        return [], []
    zi0, zi1 = max(z0 - halo, 0), min(z1 + halo, nz)
    sends, recvs = [], []
    for r in range(world):
        rz0, rz1 = zslab_bounds(nz, r, world)
        if r == rank or rz1 <= rz0:
            continue
        s0, s1 = max(max(rz0 - halo, 0), z0), min(min(rz1 + halo, nz), z1)
        if s1 > s0:
            sends.append((r, s0, s1))
        g0, g1 = max(zi0, rz0), min(zi1, rz1)
        if g1 > g0:
            recvs.append((r, g0, g1))
    return sends, recvs


def exchange_frame_halo(block, zi0: int, z0: int, z1: int, nz: int, halo: int, rank: int, world: int, group=None):
    """Halo exchange of ONE frame of a z-slab time series (the per-step traffic of
    FlowStream(zslab=...)): ``block`` (zi1 - zi0, ny, nx) holds this rank's planes
    [z0, z1) at offset z0 - zi0; the neighbours' planes are received straight into it and
    this rank's boundary planes sent from it (whole planes are contiguous: no staging on
    RCCL).  CUDA tensors over RCCL run on the current stream (the caller's upload stream,
    so the exchange overlaps compute on another stream); gloo stages through host memory.
    Every rank calls it for the same frames in the same order.  ``block`` may be a strided
    view whose first axis is the split axis (row slabs: rows first); non-contiguous pieces
    travel through contiguous temporaries."""
    import torch
    import torch.distributed as dist

    if world == 1 or block is None:
        return
    sends, recvs = halo_transfers(nz, rank, world, halo)
    if not sends and not recvs:
        return
    stage = block.is_cuda and dist.get_backend(group) == "gloo"
    ops, back = [], []
    for peer, a, b in sends:
        t = block[a - zi0:b - zi0]
        t = t.cpu() if stage else t.contiguous()
        ops.append(dist.P2POp(dist.isend, _bytes(t), peer, group))
    for peer, a, b in recvs:
        t = block[a - zi0:b - zi0]
        if stage or not t.is_contiguous():  # host staging (gloo) / strided rows (row slabs)
            buf = torch.empty(t.shape, dtype=t.dtype, device="cpu" if stage else t.device)
            back.append((t, buf))
            t = buf
        ops.append(dist.P2POp(dist.irecv, _bytes(t), peer, group))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    for t, buf in back:
        t.copy_(buf)


def check_slab_split(n_axis: int, world: int) -> None:
    """Slab splits give every rank at least one plane (row) of the split axis: a rank with an
    empty slab would take no part in the halo exchange's P2P batches (RCCL needs every rank
    of the communicator in its first batch) and hold a zero-size plan."""
    if world > n_axis:
        raise ValueError(f"slab split of {n_axis} planes over {world} ranks leaves empty slabs "
                         "(at most one rank per plane; split frames instead)")


def zslab_bounds(nz: int, rank: int, world: int) -> tuple:
    """Balanced contiguous output planes [z0, z1) of rank `rank` (may be empty when world > nz)."""
    base, extra = divmod(nz, world)
    z0 = rank * base + min(rank, extra)
    z1 = z0 + base + (1 if rank < extra else 0)
    return z0, z1


def halo_planes(nz: int, z0: int, z1: int, rd: int, rw: int) -> tuple:
    """Input planes [zi0, zi1) a slab producing outputs [z0, z1) must hold (matches of3d_plan_input_range)."""
    if z1 <= z0:
        return z0, z0
    h = rd + rw
    return max(z0 - h, 0), min(z1 + h, nz)


def _bytes(t):
    """Byte view of a contiguous tensor: NCCL/RCCL has no 16-bit integer type, so the
    frames (uint16 bits in int16 tensors) travel as uint8."""
    import torch

    return t.reshape(-1).view(torch.uint8)


def flow3d_zslabs_host(images, xyzSig, tSig, wSig, world, device=0):
    """Reference-shaped helper: run calc_flow3D as `world` z-slabs on one device
    (virtual ranks) through device plans, concatenating the slabs.  Used to
    prove slab decomposition is bit-identical to the unsharded path."""
    import torch

    a = np.ascontiguousarray(images)
    nt, nz, ny, nx = a.shape
    rd, rs, rt, rw = radii(xyzSig, tSig, wSig)
    c = nt // 2
    win = a[c - rt:c + rt + 1]
    code = _lib.DTYPE_CODES[a.dtype]
    dev = torch.device("cuda", device)
    outs = [np.empty((nz, ny, nx)) for _ in range(3)] + [np.empty((nz, ny, nx), np.float32)]
    for rank in range(world):
        z0, z1 = zslab_bounds(nz, rank, world)
        if z1 <= z0:
            continue
        plan = _lib.Plan(3, nz, ny, nx, make_taps(xyzSig, tSig, wSig), device=device, max_out_planes=z1 - z0)
        try:
            zi0, zi1 = plan.input_range(z0, z1)
            assert (zi0, zi1) == halo_planes(nz, z0, z1, rd, rw)
            part = np.ascontiguousarray(win[:, zi0:zi1])
            t_in = torch.from_numpy(part.view(np.int16) if a.dtype == np.uint16 else part).to(dev)
            n = (z1 - z0) * ny * nx
            vx, vy, vz = (torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3))
            rel = torch.empty(n, dtype=torch.float32, device=dev)
            plan.execute([t_in[i].data_ptr() for i in range(t_in.shape[0])], code, zi0, z0, z1, vx.data_ptr(),
                         vy.data_ptr(), vz.data_ptr(), rel.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
            for o, t in zip(outs, (vx, vy, vz, rel)):
                o[z0:z1] = t.cpu().numpy().reshape(z1 - z0, ny, nx)
        finally:
            plan.close()
    return tuple(outs)
