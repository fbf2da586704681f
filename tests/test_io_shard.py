"""Host-side pieces of the multi-GPU process_flow (CPU, no device): TIFF slab writes are
byte-identical to a whole-volume write, compressed / tiled inputs decode through libtiff,
page ranges read only their planes, and the per-frame halo plan + exchange (gloo,
world 2-4) deliver exactly the planes each z-slab needs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from opticalflow3d_dev_amd import tiff as tf
from opticalflow3d_dev_amd.shard import exchange_frame_halo, frame_blocks, halo_planes, halo_transfers, zslab_bounds


@pytest.mark.parametrize("shape,dtype", [((7, 20, 24), np.float64), ((5, 9, 33), np.float32), ((1, 8, 8), np.float64),
                                         ((13, 4, 6), np.float32)])
@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_write_planes_equals_imwrite(tmp_path, shape, dtype, world):
    v = np.random.default_rng(1).standard_normal(shape).astype(dtype)
    tf.imwrite(tmp_path / "full.tiff", v, photometric="minisblack")
    order = list(range(world))[::-1]  # slabs land in any order
    for r in order:
        z0, z1 = zslab_bounds(shape[0], r, world)
        tf.write_planes(tmp_path / "part.tiff", v.shape, v.dtype, z0, v[z0:z1])
    assert (tmp_path / "full.tiff").read_bytes() == (tmp_path / "part.tiff").read_bytes()
    assert np.array_equal(tf.imread(tmp_path / "part.tiff"), v)


def test_write_planes_over_stale_file(tmp_path):
    p = tmp_path / "x.tiff"
    p.write_bytes(b"\xff" * 100000)  # a longer file from an earlier run
    v = np.arange(2 * 5 * 6, dtype=np.float64).reshape(2, 5, 6)
    tf.write_planes(p, v.shape, v.dtype, 0, v)
    tf.imwrite(tmp_path / "y.tiff", v)
    assert p.read_bytes() == (tmp_path / "y.tiff").read_bytes()


@pytest.mark.parametrize("compression", [5, 8])
def test_compressed_onetif_reads(tmp_path, compression):
    a = np.random.default_rng(2).integers(0, 4096, (6, 5, 37, 45)).astype(np.uint16)
    tf.imwrite_libtiff(tmp_path / "c.tif", a.reshape(-1, 37, 45), compression=compression, bigtiff=False,
                       description=tf.imagej_description(a.shape))
    t = tf.TiffFile(tmp_path / "c.tif")
    assert t.imagej_metadata["frames"] == 6 and t.imagej_metadata["slices"] == 5
    assert np.array_equal(t.asarray(), a)
    with pytest.raises(ValueError):
        tf.memmap(tmp_path / "c.tif")  # process_flow falls back to page-range decodes
    # frame i plane z = page i * Nz + z: a frame's planes / a slab's planes, decoded alone
    for i, z0, z1 in ((0, 0, 5), (3, 1, 4), (5, 4, 5)):
        assert np.array_equal(t.read_planes(i * 5 + z0, i * 5 + z1), a[i, z0:z1])
    assert np.array_equal(tf.imread_libtiff(tmp_path / "c.tif", pages=(29, 30)), a[5, 4:5])
    with pytest.raises(ValueError):
        tf.imread_libtiff(tmp_path / "c.tif", pages=(28, 31))


def test_tiled_and_page_ranges(tmp_path):
    a = np.random.default_rng(3).integers(0, 60000, (4, 50, 70)).astype(np.uint16)
    tf.imwrite_libtiff(tmp_path / "t.tif", a, compression=8, bigtiff=False, tile=(16, 32))
    assert np.array_equal(tf.imread(tmp_path / "t.tif"), a)
    assert np.array_equal(tf.TiffFile(tmp_path / "t.tif").read_planes(1, 3), a[1:3])
    tf.imwrite(tmp_path / "u.tif", a)
    assert np.array_equal(tf.TiffFile(tmp_path / "u.tif").read_planes(2, 4), a[2:4])


@pytest.mark.parametrize("nz,world,halo", [(64, 2, 21), (64, 4, 21), (30, 8, 5), (7, 8, 3), (100, 3, 40), (1, 2, 4)])
def test_halo_transfers_consistent(nz, world, halo):
    plans = [halo_transfers(nz, r, world, halo) for r in range(world)]
    sent = {(r, p, a, b) for r in range(world) for p, a, b in plans[r][0]}
    got = {(p, r, a, b) for r in range(world) for p, a, b in plans[r][1]}
    assert sent == got  # every send has its matching receive
    for r in range(world):
        z0, z1 = zslab_bounds(nz, r, world)
        if z1 <= z0:
            continue
        zi0, zi1 = max(z0 - halo, 0), min(z1 + halo, nz)
        cover = set(range(z0, z1))
        for _, a, b in plans[r][1]:
            cover |= set(range(a, b))
        assert cover == set(range(zi0, zi1))


def test_frame_blocks_cover():
    for n, w in ((10, 4), (3, 8), (1, 1), (17, 5)):
        got = []
        for r in range(w):
            a, b = frame_blocks(n, r, w)
            got += list(range(a, b))
        assert got == list(range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _xchg_worker(rank, world, port, nz, halo, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(nz * 3 * 4, dtype=torch.int16).reshape(nz, 3, 4)
        ok = True
        for frame in range(3):  # a few frames, as a time series pushes them
            f = full + frame
            z0, z1 = zslab_bounds(nz, rank, world)
            zi0, zi1 = halo_planes(nz, z0, z1, halo, 0)
            blk = torch.full((zi1 - zi0, 3, 4), -1, dtype=torch.int16)
            blk[z0 - zi0:z1 - zi0] = f[z0:z1]
            exchange_frame_halo(blk, zi0, z0, z1, nz, halo, rank, world)
            ok = ok and torch.equal(blk, f[zi0:zi1])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz,halo", [(2, 40, 9), (3, 20, 9), (4, 10, 6)])
def test_exchange_frame_halo_gloo(world, nz, halo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_xchg_worker, args=(r, world, port, nz, halo, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(res.values()) and len(res) == world


@pytest.mark.parametrize("world", [1, 2, 3, 7])
def test_write_rows_equals_imwrite(tmp_path, world):
    v = np.random.default_rng(4).standard_normal((5, 19, 23))
    tf.imwrite(tmp_path / "full.tiff", v, photometric="minisblack")
    for r in range(world)[::-1]:
        y0, y1 = zslab_bounds(19, r, world)
        tf.write_rows(tmp_path / "part.tiff", v.shape, v.dtype, y0, v[:, y0:y1])
    assert (tmp_path / "full.tiff").read_bytes() == (tmp_path / "part.tiff").read_bytes()


def test_read_rows(tmp_path):
    a = np.random.default_rng(5).integers(0, 60000, (4, 30, 21)).astype(np.uint16)
    tf.imwrite(tmp_path / "u.tif", a)
    assert np.array_equal(tf.TiffFile(tmp_path / "u.tif").read_rows(7, 19), a[:, 7:19])
    tf.imwrite_libtiff(tmp_path / "c.tif", a, compression=5, bigtiff=False)
    assert np.array_equal(tf.TiffFile(tmp_path / "c.tif").read_rows(0, 5), a[:, 0:5])


@pytest.mark.parametrize("layout", ["strips4", "strips7", "tiles"])
def test_read_rows_decodes_only_their_strips(tmp_path, layout):
    """Row slabs of compressed pages (process_flow's row-slab ranks): every row window equals
    the full decode, for windows inside one strip / tile row, across several, at both edges."""
    a = np.random.default_rng(6).integers(0, 60000, (3, 45, 40)).astype(np.uint16)
    kw = dict(tile=(16, 32)) if layout == "tiles" else dict(rows_per_strip=int(layout[6:]))
    tf.imwrite_libtiff(tmp_path / "c.tif", a, compression=8, bigtiff=False, **kw)
    t = tf.TiffFile(tmp_path / "c.tif")
    assert np.array_equal(t.asarray(), a)
    for y0, y1 in ((0, 45), (0, 1), (3, 4), (4, 8), (5, 30), (17, 33), (44, 45), (31, 45)):
        assert np.array_equal(t.read_rows(y0, y1), a[:, y0:y1]), (y0, y1)
        assert np.array_equal(t.read_rows(y0, y1, pages=(1, 3)), a[1:3, y0:y1]), (y0, y1)


def test_page_ranges_jump_to_their_ifd(tmp_path):
    """read_planes on compressed pages opens libtiff at the first page's IFD offset (no walk over
    the earlier directories): every page range of a long page series decodes exactly."""
    a = np.random.default_rng(7).integers(0, 4096, (40, 9, 13)).astype(np.uint16)
    tf.imwrite_libtiff(tmp_path / "c.tif", a, compression=5, bigtiff=True)
    t = tf.TiffFile(tmp_path / "c.tif")
    assert len(t.ifd_offsets) == 40
    for z0, z1 in ((0, 1), (39, 40), (12, 20), (0, 40), (25, 26)):
        assert np.array_equal(t.read_planes(z0, z1), a[z0:z1])


def test_slab_axis_prefers_rows_for_flat_volumes():
    from opticalflow3d_dev_amd.shard import slab_axis, slab_work

    assert slab_axis(256, 1024, 4, 6, 15) == 1      # configs[3]
    assert slab_axis(512, 2048, 8, 6, 15) == 1      # configs[4]
    assert slab_axis(2048, 64, 4, 6, 15) == 0       # tall volume: z-slabs
    assert slab_work(1024, 256, 4, 6, 15, 1) < 1.2  # c4 row slabs: < 20 % halo work at P = 4
