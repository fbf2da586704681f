"""Multi-GPU decomposition logic on CPU: slab partitioning, halo ranges, and the
neighbour halo exchange over torch.distributed (gloo, world_size 2-4)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from opticalflow3d_dev_amd.shard import (check_slab_split, exchange_frame_halo, frame_assignment, halo_planes,
                                         halo_transfers, zslab_bounds)


@pytest.mark.parametrize("nz,world", [(64, 1), (64, 2), (64, 3), (7, 8), (256, 4), (5, 5), (1, 2)])
def test_zslab_bounds_partition(nz, world):
    b = [zslab_bounds(nz, r, world) for r in range(world)]
    assert b[0][0] == 0 and b[-1][1] == nz
    for (a0, a1), (c0, c1) in zip(b, b[1:]):
        assert a1 == c0 and a1 >= a0
    sizes = [z1 - z0 for z0, z1 in b]
    assert max(sizes) - min(sizes) <= 1


def test_frame_assignment_covers_all():
    got = sorted(sum((frame_assignment(10, r, 4) for r in range(4)), []))
    assert got == list(range(10))


def test_halo_planes():
    assert halo_planes(64, 0, 32, 6, 15) == (0, 53)
    assert halo_planes(64, 32, 64, 6, 15) == (11, 64)
    assert halo_planes(64, 10, 20, 6, 15) == (0, 41)
    assert halo_planes(8, 3, 3, 6, 15) == (3, 3)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame_halo_worker(rank, world, port, nz, halo, axis, q):
    """A time series of frames through exchange_frame_halo, as FlowStream(zslab=...) runs it:
    each rank's block holds only its own planes (rows) of every frame, then receives the
    halo; afterwards it equals the global frame over the rank's input range."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        for frame in range(3):
            full = (torch.arange(nz * 4 * 5, dtype=torch.int16) + 1000 * frame).reshape(nz, 4, 5)
            if axis == 1:  # rows first, the block a strided view (row slabs)
                full = full.reshape(4, nz, 5).transpose(0, 1)
            z0, z1 = zslab_bounds(nz, rank, world)
            zi0, zi1 = max(z0 - halo, 0), min(z1 + halo, nz)
            if axis == 0:
                block = torch.full((zi1 - zi0, 4, 5), -1, dtype=torch.int16)
            else:
                block = torch.full((4, zi1 - zi0, 5), -1, dtype=torch.int16).transpose(0, 1)
            block[z0 - zi0:z1 - zi0] = full[z0:z1]
            exchange_frame_halo(block, zi0, z0, z1, nz, halo, rank, world)
            ok = ok and bool(torch.equal(block, full[zi0:zi1]))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz,halo,axis", [(2, 16, 3, 0), (3, 10, 4, 0), (4, 6, 3, 0), (2, 5, 21, 0),
                                                (3, 9, 27, 0), (2, 16, 3, 1), (3, 11, 5, 1), (4, 4, 2, 1)])
def test_exchange_frame_halo_gloo(world, nz, halo, axis):
    """The product halo exchange (shard.exchange_frame_halo): z-slabs (contiguous planes) and
    row slabs (strided rows through temporaries), slabs thinner than the halo included."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frame_halo_worker, args=(r, world, port, nz, halo, axis, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def test_slab_split_refuses_empty_slabs():
    check_slab_split(8, 8)
    check_slab_split(512, 8)
    with pytest.raises(ValueError, match="empty slabs"):
        check_slab_split(3, 4)


@pytest.mark.parametrize("nz,world,halo", [(64, 2, 27), (64, 8, 27), (9, 3, 27), (256, 4, 21)])
def test_halo_transfers_symmetric(nz, world, halo):
    """Every planned send has the matching receive on the peer (same planes)."""
    sends = {r: halo_transfers(nz, r, world, halo)[0] for r in range(world)}
    recvs = {r: halo_transfers(nz, r, world, halo)[1] for r in range(world)}
    got = sorted((r, p, a, b) for r in range(world) for p, a, b in sends[r])
    want = sorted((p, r, a, b) for r in range(world) for p, a, b in recvs[r])
    assert got == want


def _crop_worker(rank, world, port, axis, q):
    """bench.gather_owned_crop as slab_parity runs it: every rank fills the crop voxels of its
    own planes (rows) of a known field; rank 0's merge must equal the field with every voxel
    owned exactly once."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dims = (40, 36, 30)
        n_ax = dims[axis]
        cut = zslab_bounds(n_ax, 0, world)[1]
        box = bench.parity_box(dims, axis, cut)
        z0, z1, y0, y1, x0, x1 = box
        field = torch.arange(40 * 36 * 30, dtype=torch.float64).reshape(dims)
        field[::3] = -0.0  # owners' -0.0 bits survive the merge
        want = field[z0:z1, y0:y1, x0:x1]
        a0, a1 = zslab_bounds(n_ax, rank, world)
        crop = torch.zeros((5,) + tuple(want.shape), dtype=torch.float64)
        b0, b1 = box[2 * axis], box[2 * axis + 1]
        o0, o1 = max(b0, a0), min(b1, a1)
        if o1 > o0:
            sl = [slice(None)] * 3
            sl[axis] = slice(o0 - b0, o1 - b0)
            for k in range(4):
                crop[(k, *sl)] = want[tuple(sl)] * (k + 1)
            crop[(4, *sl)] = 1
        out = bench.gather_owned_crop(crop, rank, world, "cpu")
        if rank == 0:
            ok = bool((out[4] == 1).all()) and all(
                torch.equal(out[k].view(torch.int64), (want * (k + 1)).view(torch.int64)) for k in range(4))
        else:
            ok = out is None
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,axis", [(2, 0), (2, 1), (4, 0), (3, 1)])
def test_bench_parity_crop_gather_gloo(world, axis):
    """The N > 1 bench line's parity crop: straddles the rank-0/1 cut and is reassembled on
    rank 0 from its owners (gloo, CPU)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_crop_worker, args=(r, world, port, axis, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res
