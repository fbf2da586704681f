"""process_flow over several processes (torch.distributed, gloo here on one GPU; RCCL on a
node): frame blocks and z-slab ranks write the same files, byte for byte, as one process,
and their pixels equal the oracle's (calc_flow.py:507-534, :512 "this could become a parfor
loop").  Also: LZW-compressed input stacks (tifffile decodes them for the reference)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import assert_flow3d_matches_oracle
from opticalflow3d_dev_amd import process_flow
from opticalflow3d_dev_amd import tiff as tf

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pf_worker(rank, world, port, args, kwargs, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OF3D_DIST_BACKEND="gloo")
    from opticalflow3d_dev_amd.shard import init_distributed

    try:
        init_distributed()
        os.environ["OF3D_DEVICE"] = "0"  # every rank on the one GPU of this box
        process_flow(*args, **kwargs)
        q.put((rank, "ok"))
    except BaseException as e:  # reported to the parent
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_ranks(world, args, kwargs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_pf_worker, args=(r, world, port, args, kwargs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def _tree(d):
    return {os.path.relpath(os.path.join(r, f), d): open(os.path.join(r, f), "rb").read()
            for r, _, fs in os.walk(d) for f in fs if f.endswith((".tiff", ".csv"))}


@pytest.mark.parametrize("world,parallel,shape", [(2, "frames", (9, 12, 20, 24)), (2, "zslab", (9, 12, 20, 24)),
                                                  (3, "zslab", (7, 10, 16, 20)), (2, "auto", (7, 10, 16, 20)),
                                                  (2, "yslab", (9, 6, 40, 24)), (3, "yslab", (7, 5, 31, 20)),
                                                  (4, "auto", (8, 4, 64, 30))])
def test_onetif_multi_rank_equals_single(tmp_path, world, parallel, shape):
    stack = np.random.default_rng(world).integers(0, 4096, size=shape).astype(np.uint16)
    single, multi = tmp_path / "single", tmp_path / "multi"
    for d in (single, multi):
        d.mkdir()
        tf.imwrite(d / "cells.tif", stack, imagej=True)
    process_flow(str(single), "cells", "OneTif", 3, 1, 1, 2)
    _run_ranks(world, (str(multi), "cells", "OneTif", 3, 1, 1, 2), {"parallel": parallel})
    a, b = _tree(single / "OpticalFlow3D"), _tree(multi / "OpticalFlow3D")
    assert sorted(a) == sorted(b) and len(a) == 1 + 4 * (shape[0] - 6)
    for k in a:
        assert a[k] == b[k], k
    out = multi / "OpticalFlow3D" / "cells"
    for hh in range(shape[0] - 6):
        got = [tf.imread(out / f"cells_{n}_t{hh + 3:04d}.tiff") for n in ("vx", "vy", "vz", "rel")]
        assert_flow3d_matches_oracle(got, stack[hh:hh + 7], 1, 1, 2)


@pytest.mark.parametrize("world,parallel", [(2, "zslab"), (3, "zslab"), (2, "yslab"), (3, "yslab"), (2, "frames")])
def test_fp32_multi_rank_equals_single_and_oracle(tmp_path, world, parallel):
    """configs[4]: process_flow(precision="fp32") split over ranks (slabs with the halo
    exchange, or frames) writes the same float32 files, byte for byte, as one process, and
    their pixels are within 1e-4 of the oracle's fp64 flow (calc_flow.py:507-534)."""
    from oracle import cpu_ref
    from test_gpu_process_flow import assert_fp32_flow_close

    stack = cpu_ref.synthetic_stack_np((8, 12, 30, 24), seed=30 + world)
    single, multi = tmp_path / "single", tmp_path / "multi"
    for d in (single, multi):
        d.mkdir()
        tf.imwrite(d / "c.tif", stack, imagej=True)
    process_flow(str(single), "c", "OneTif", 3, 1, 1, 2, precision="fp32")
    _run_ranks(world, (str(multi), "c", "OneTif", 3, 1, 1, 2), {"parallel": parallel, "precision": "fp32"})
    a, b = _tree(single / "OpticalFlow3D"), _tree(multi / "OpticalFlow3D")
    assert sorted(a) == sorted(b) and len(a) == 1 + 4 * 2
    for k in a:
        assert a[k] == b[k], k
    out = multi / "OpticalFlow3D" / "c"
    for hh in range(2):
        got = [tf.imread(out / f"c_{n}_t{hh + 3:04d}.tiff") for n in ("vx", "vy", "vz", "rel")]
        assert_fp32_flow_close(got, stack[hh:hh + 7], 1, 1, 2)


def test_slab_split_wider_than_volume_runs_frames(tmp_path):
    """parallel="zslab" with more ranks than planes: no empty slabs (shard.check_slab_split),
    the run falls back to frame blocks and writes the single-process files."""
    stack = np.random.default_rng(12).integers(0, 4096, size=(9, 2, 16, 20)).astype(np.uint16)
    single, multi = tmp_path / "single", tmp_path / "multi"
    for d in (single, multi):
        d.mkdir()
        tf.imwrite(d / "e.tif", stack, imagej=True)
    process_flow(str(single), "e", "OneTif", 3, 1, 1, 2)
    _run_ranks(3, (str(multi), "e", "OneTif", 3, 1, 1, 2), {"parallel": "zslab"})
    a, b = _tree(single / "OpticalFlow3D"), _tree(multi / "OpticalFlow3D")
    assert sorted(a) == sorted(b)
    for k in a:
        assert a[k] == b[k], k


def test_sequencet_zslab_three_ranks(tmp_path):
    stack = np.random.default_rng(5).integers(0, 4096, size=(8, 9, 14, 18)).astype(np.uint16)
    for t in range(8):
        tf.imwrite(tmp_path / f"v_t{t}.tif", stack[t])
    _run_ranks(3, (str(tmp_path), "v_t.*", "SequenceT", 3, 1, 1, 2), {"parallel": "zslab"})
    out = tmp_path / "OpticalFlow3D" / "v_t"
    for hh in range(2):
        got = [tf.imread(out / f"v_t_{n}_t{hh + 3:04d}.tiff") for n in ("vx", "vy", "vz", "rel")]
        assert_flow3d_matches_oracle(got, stack[hh:hh + 7], 1, 1, 2)


@pytest.mark.parametrize("world", [2, 3])
def test_yslab_row_ranges_wsig5(tmp_path, world):
    """Row slabs where the fused W kernels are in use (wSig 5: rw 15), so every rank's plan
    writes only its own rows (of3d_plan_set_rows): files equal one GPU's, pixels the oracle's."""
    stack = np.random.default_rng(10 + world).integers(0, 4096, size=(7, 3, 96, 40)).astype(np.uint16)
    single, multi = tmp_path / "single", tmp_path / "multi"
    for d in (single, multi):
        d.mkdir()
        tf.imwrite(d / "w.tif", stack, imagej=True)
    process_flow(str(single), "w", "OneTif", 3, 1, 1, 5)
    _run_ranks(world, (str(multi), "w", "OneTif", 3, 1, 1, 5), {"parallel": "yslab"})
    a, b = _tree(single / "OpticalFlow3D"), _tree(multi / "OpticalFlow3D")
    assert sorted(a) == sorted(b)
    for k in a:
        assert a[k] == b[k], k
    got = [tf.imread(multi / "OpticalFlow3D" / "w" / f"w_{n}_t0003.tiff") for n in ("vx", "vy", "vz", "rel")]
    assert_flow3d_matches_oracle(got, stack, 1, 1, 5)


def test_sequencet_yslab_two_ranks(tmp_path):
    stack = np.random.default_rng(8).integers(0, 4096, size=(7, 4, 36, 18)).astype(np.uint16)
    for t in range(7):
        tf.imwrite(tmp_path / f"r_t{t}.tif", stack[t])
    _run_ranks(2, (str(tmp_path), "r_t.*", "SequenceT", 3, 1, 1, 2), {"parallel": "yslab"})
    out = tmp_path / "OpticalFlow3D" / "r_t"
    got = [tf.imread(out / f"r_t_{n}_t0003.tiff") for n in ("vx", "vy", "vz", "rel")]
    assert_flow3d_matches_oracle(got, stack, 1, 1, 2)


@pytest.mark.parametrize("world,parallel", [(1, "auto"), (2, "zslab"), (2, "yslab")])
def test_lzw_onetif_multi_rank(tmp_path, world, parallel):
    """An LZW-compressed hyperstack split over ranks: every rank decodes only the pages of
    its planes (tiff.imread_libtiff page ranges; row slabs: only the strips holding its rows),
    results equal the oracle."""
    stack = np.random.default_rng(16).integers(0, 4096, size=(7, 6, 18, 22)).astype(np.uint16)
    tf.imwrite_libtiff(tmp_path / "q.tif", stack.reshape(-1, 18, 22), compression=5, bigtiff=False,
                       description=tf.imagej_description(stack.shape), rows_per_strip=4)
    if world == 1:
        process_flow(str(tmp_path), "q", "OneTif", 3, 1, 1, 2)
    else:
        _run_ranks(world, (str(tmp_path), "q", "OneTif", 3, 1, 1, 2), {"parallel": parallel})
    got = [tf.imread(tmp_path / "OpticalFlow3D" / "q" / f"q_{n}_t0003.tiff") for n in ("vx", "vy", "vz", "rel")]
    assert_flow3d_matches_oracle(got, stack, 1, 1, 2)


def test_lzw_onetif_input(tmp_path):
    """An LZW-compressed ImageJ hyperstack (not memory-mappable): decoded, same results."""
    stack = np.random.default_rng(6).integers(0, 4096, size=(8, 6, 18, 22)).astype(np.uint16)
    tf.imwrite_libtiff(tmp_path / "z.tif", stack.reshape(-1, 18, 22), compression=5, bigtiff=False,
                       description=tf.imagej_description(stack.shape))
    process_flow(str(tmp_path), "z", "OneTif", 3, 1, 1, 2)
    out = tmp_path / "OpticalFlow3D" / "z"
    for hh in range(2):
        got = [tf.imread(out / f"z_{n}_t{hh + 3:04d}.tiff") for n in ("vx", "vy", "vz", "rel")]
        assert_flow3d_matches_oracle(got, stack[hh:hh + 7], 1, 1, 2)
