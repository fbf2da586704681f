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


def stream_slab_worker(rank, world, port, q, img, sig, axis, precision="fp64"):
    """One rank of a slab split on the product path: FlowStream(zslab=(rank, world, group,
    axis)) holds only the rank's planes (axis 0) or rows (axis 1) of every frame, fetches the
    halo with shard.exchange_frame_halo (gloo here, all ranks on the one GPU; RCCL on a
    node), and returns the rank's part of vx, vy, vz, rel."""
    import os

    import torch.distributed as dist

    from opticalflow3d_dev_amd.shard import zslab_bounds
    from opticalflow3d_dev_amd.stream import FlowStream

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nt, nz, ny, nx = img.shape
        a0, a1 = zslab_bounds((nz, ny)[axis], rank, world)
        fs = FlowStream(3, (nz, ny, nx), img.dtype, *sig, device=0, depth=1, precision=precision,
                        zslab=(rank, world, None, axis))
        try:
            rt = fs.rt
            c = nt // 2
            for k in range(c - rt, c + rt + 1):
                fs.push(img[k, a0:a1] if axis == 0 else img[k, :, a0:a1])
            pend = fs.submit()
            outs = [o.copy() for o in pend.result()]
            pend.release()
        finally:
            fs.close()
        q.put((rank, a0, a1, outs))
    finally:
        dist.destroy_process_group()


def run_stream_slabs(world, img, sig, axis, precision="fp64"):
    """stream_slab_worker on `world` spawned processes; [(rank, a0, a1, outs)] by rank."""
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=stream_slab_worker, args=(r, world, port, q, img, sig, axis, precision))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,axis", [(2, 0), (3, 0), (2, 1), (3, 1)])
def test_slab_ranks_with_halo_exchange(world, axis):
    """The product slab path (FlowStream(zslab=...) + exchange_frame_halo, as process_flow and
    bench.py's slab configs run it): each rank's part equals the same planes / rows of the
    unsharded frame bit for bit."""
    img = np.random.default_rng(7).integers(0, 4096, size=(13, 30, 20, 24)).astype(np.uint16)
    full = calc_flow3D(img, 2, 2, 5)
    covered = 0
    for rank, a0, a1, outs in run_stream_slabs(world, img, (2, 2, 5), axis):
        covered += a1 - a0
        for a, b in zip(full, outs):
            want = a[a0:a1] if axis == 0 else a[:, a0:a1]
            assert bits_equal(want, b.reshape(want.shape)), (rank, axis)
    assert covered == (30, 20)[axis]


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


@pytest.mark.parametrize("rows", [(7, 41), (59, 60), (0, 60)])
@pytest.mark.parametrize("fp32", [False, True])
def test_plan_output_rows_z_tiled(rows, fp32, monkeypatch):
    """of3d_plan_set_rows with the z-tiled W-xy hand-off forced (OF3D_WXY_TILE=1; nx a multiple of
    32): the rows K34 writes and K5c reads in the tiled layout, bit-identical to the plain-plane
    whole-plane outputs."""
    import torch

    ya, yb = rows
    nz, ny, nx = 20, 60, 64
    img = np.random.default_rng(12).integers(0, 4096, size=(13, nz, ny, nx)).astype(np.uint16)
    s, t, w = 2, 2, 5
    rt = radii(s, t, w)[2]
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(np.ascontiguousarray(img[6 - rt:6 + rt + 1]).view(np.int16)).to(dev)
    mode = _lib.OF3D_FP32 if fp32 else 0
    vt = torch.float32 if fp32 else torch.float64

    def run(r0, r1, tile):
        monkeypatch.setenv("OF3D_WXY_TILE", tile)
        plan = _lib.Plan(3, nz, ny, nx, make_taps(s, t, w), device=0, mode=mode)
        try:
            if (r0, r1) != (0, ny):
                plan.set_rows(r0, r1)
            n = nz * (r1 - r0) * nx
            outs = [torch.empty(n, dtype=vt, device=dev) for _ in range(3)] + [torch.empty(n, dtype=torch.float32,
                                                                                          device=dev)]
            plan.execute([d_in[i].data_ptr() for i in range(2 * rt + 1)], _lib.OF3D_U16, 0, 0, nz,
                         *[o.data_ptr() for o in outs])
            torch.cuda.synchronize(dev)
            return [o.cpu().numpy().reshape(nz, r1 - r0, nx) for o in outs]
        finally:
            plan.close()

    full = run(0, ny, "0")
    part = run(ya, yb, "1")
    for a, b in zip(full, part):
        assert np.array_equal(a[:, ya:yb].view(np.uint8), b.view(np.uint8))
