"""Multi-GPU decomposition logic on CPU: slab partitioning, halo ranges, and the
neighbour halo exchange over torch.distributed (gloo, world_size 2-4)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from opticalflow3d_dev_amd.shard import exchange_halos, frame_assignment, halo_planes, zslab_bounds, fill_halos


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


def _worker(rank, world, port, nz, halo, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(3 * nz * 4 * 5, dtype=torch.int32).reshape(3, nz, 4, 5)
        z0, z1 = zslab_bounds(nz, rank, world)
        local = full[:, z0:z1].contiguous()
        got, zi0 = exchange_halos(local, z0, z1, nz, halo, rank, world)
        zi1 = min(z1 + halo, nz)
        ok = zi0 == max(z0 - halo, 0) and torch.equal(got, full[:, zi0:zi1])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz,halo", [(2, 16, 3), (3, 10, 4), (4, 6, 3), (2, 5, 21)])
def test_exchange_halos_gloo(world, nz, halo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nz, halo, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def _fill_worker(rank, world, port, nz, rd, rw, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(3 * nz * 4 * 5, dtype=torch.int16).reshape(3, nz, 4, 5)
        z0, z1 = zslab_bounds(nz, rank, world)
        zi0, zi1 = halo_planes(nz, z0, z1, rd, rw)
        block = torch.full((3, zi1 - zi0, 4, 5), -1, dtype=torch.int16)
        block[:, z0 - zi0:z1 - zi0] = full[:, z0:z1]
        fill_halos(block, zi0, z0, z1, nz, rd + rw, rank, world)
        q.put((rank, bool(torch.equal(block, full[:, zi0:zi1]))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz,rd,rw", [(2, 16, 1, 2), (3, 20, 2, 3), (4, 9, 1, 3), (4, 3, 1, 1), (2, 64, 6, 15)])
def test_fill_halos_gloo(world, nz, rd, rw):
    """In-place halo fill used by ZSlabFlow (bench.py c4): every rank's block
    equals the global stack over [zi0, zi1), including empty slabs (world > nz)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fill_worker, args=(r, world, port, nz, rd, rw, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res
