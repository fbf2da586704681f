"""z-slab decomposition on the device (virtual ranks on one GPU): concatenated
slabs are bit-identical to the unsharded calc_flow3D, including slabs thinner
than the stencil halo; the C-ABI's input range equals shard.halo_planes."""
import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import _lib, calc_flow3D, make_taps, radii
from opticalflow3d_dev_amd.shard import flow3d_zslabs_host, halo_planes, zslab_bounds

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_zslabs_bitwise_equal_full(world):
    img = np.random.default_rng(world).integers(0, 4096, size=(13, 24, 40, 36)).astype(np.uint16)
    full = calc_flow3D(img, 2, 2, 5)
    got = flow3d_zslabs_host(img, 2, 2, 5, world)
    for a, b in zip(full, got):
        assert bits_equal(a, b.astype(a.dtype))


def test_plan_input_range_matches_python():
    s, t, w = 2, 2, 5
    rd, rs, rt, rw = radii(s, t, w)
    plan = _lib.Plan(3, 64, 16, 16, make_taps(s, t, w))
    for world in (2, 3, 8):
        for r in range(world):
            z0, z1 = zslab_bounds(64, r, world)
            assert plan.input_range(z0, z1) == halo_planes(64, z0, z1, rd, rw)
    plan.close()


def _zslab_worker(rank, world, port, q):
    import os

    import torch
    import torch.distributed as dist

    from opticalflow3d_dev_amd.shard import ZSlabFlow

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        img = np.random.default_rng(7).integers(0, 4096, size=(13, 30, 20, 24)).astype(np.uint16)
        dev = torch.device("cuda", 0)
        zf = ZSlabFlow(30, 20, 24, 2, 2, 5, rank, world, device=0)
        own = zf.allocate(torch.int16, dev)
        own.copy_(torch.from_numpy(img[:, zf.z0:zf.z1].view(np.int16)))
        n = (zf.z1 - zf.z0) * 20 * 24
        outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
        rel = torch.empty(n, dtype=torch.float32, device=dev)
        zf.run(_lib.OF3D_U16, *outs, rel, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        q.put((rank, zf.z0, zf.z1, [t.cpu().numpy() for t in outs + [rel]]))
        zf.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_zslab_ranks_with_halo_exchange(world):
    """ZSlabFlow as bench.py's c4 path runs it: each rank holds only its own
    planes, fetches halos from its neighbours (gloo here, staged through host
    memory; RCCL on a multi-GPU node), and its slab equals the same planes of
    the unsharded frame bit for bit."""
    import multiprocessing as mp
    import socket

    img = np.random.default_rng(7).integers(0, 4096, size=(13, 30, 20, 24)).astype(np.uint16)
    full = calc_flow3D(img, 2, 2, 5)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_zslab_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    covered = 0
    for rank, z0, z1, outs in res:
        covered += z1 - z0
        for a, b in zip(full, outs):
            assert bits_equal(a[z0:z1], b.reshape(z1 - z0, 20, 24))
    assert covered == 30


@pytest.mark.parametrize("rows", [(0, 60), (7, 41), (0, 1), (59, 60), (13, 14)])
@pytest.mark.parametrize("fp32", [False, True])
def test_plan_output_rows(rows, fp32):
    """of3d_plan_set_rows: the fused W kernels write only rows [y0, y1) (compact), bit-identical
    to the same rows of the whole-plane outputs (row slabs keep their own rows this way)."""
    import torch

    ya, yb = rows
    img = np.random.default_rng(11).integers(0, 4096, size=(13, 20, 60, 40)).astype(np.uint16)
    s, t, w = 2, 2, 5
    rt = radii(s, t, w)[2]
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(np.ascontiguousarray(img[6 - rt:6 + rt + 1]).view(np.int16)).to(dev)
    mode = _lib.OF3D_FP32 if fp32 else 0
    vt = torch.float32 if fp32 else torch.float64

    def run(r0, r1):
        plan = _lib.Plan(3, 20, 60, 40, make_taps(s, t, w), device=0, mode=mode)
        try:
            if (r0, r1) != (0, 60):
                plan.set_rows(r0, r1)
            n = 20 * (r1 - r0) * 40
            outs = [torch.empty(n, dtype=vt, device=dev) for _ in range(3)] + [torch.empty(n, dtype=torch.float32,
                                                                                          device=dev)]
            plan.execute([d_in[i].data_ptr() for i in range(2 * rt + 1)], _lib.OF3D_U16, 0, 0, 20,
                         *[o.data_ptr() for o in outs])
            torch.cuda.synchronize(dev)
            return [o.cpu().numpy().reshape(20, r1 - r0, 40) for o in outs]
        finally:
            plan.close()

    full = run(0, 60)
    part = run(ya, yb)
    for a, b in zip(full, part):
        assert np.array_equal(a[:, ya:yb].view(np.uint8), b.view(np.uint8))
