"""Stream ordering of the slab halo exchange under RCCL's semantics, on one GPU.

The gloo tests stage every halo through synchronous .cpu() copies, so they cannot catch an
ordering bug of the RCCL path (FlowStream.push issues the H2D and shard.exchange_frame_halo on
the upload stream and the compute waits on that stream's event).  Two ranks cannot share one
GPU under RCCL, so the ranks here are threads of one process, each with its own FlowStream,
and torch.distributed's P2P calls are replaced by a model of ProcessGroupNCCL's documented
stream contract:
  * batch_isend_irecv: the rank's communication stream waits on the caller's current stream
    (the sends read what that stream wrote), then runs the transfers;
  * Work.wait(): the caller's current stream waits on the communication stream (the
    receiving rank's later work sees the halo; the sending rank's later writes to the sent
    planes wait for the peer's copy) — the host does not block.
The transfers start after a device-side delay (torch.cuda._sleep) on the communication
stream, so a consumer that did not wait for them reads stale planes.  Checked: every rank's
part equals the unsharded frame bit for bit, the exchange was issued on the rank's upload
stream, and (negative control) the same run with Work.wait() doing nothing differs.
Reference: calc_flow.py:512 (the per-frame loop the slabs split)."""
import threading

import numpy as np
import pytest

from conftest import bits_equal
from opticalflow3d_dev_amd import calc_flow3D, radii

pytestmark = pytest.mark.gpu


class _World:
    def __init__(self, world, delay):
        import torch

        self.world, self.delay = world, delay
        self.bar = threading.Barrier(world, timeout=60)
        self.lock = threading.Lock()
        self.sends, self.done = {}, {}
        self.comm = [torch.cuda.Stream(device=0) for _ in range(world)]
        self.issued = [[] for _ in range(world)]


class _Group:
    def __init__(self, w, rank):
        self.w, self.rank, self.seq = w, rank, 0


class _Op:
    def __init__(self, op, tensor, peer, group):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


class _Work:
    def __init__(self, events, wait):
        self.events, self.do_wait = events, wait

    def wait(self):
        import torch

        if self.do_wait:
            cur = torch.cuda.current_stream()
            for e in self.events:
                cur.wait_event(e)
        return True


def _install(monkeypatch, wait=True):
    import torch
    import torch.distributed as dist

    isend, irecv = dist.isend, dist.irecv

    def batch_isend_irecv(ops):
        g = ops[0].group
        w, r, seq = g.w, g.rank, g.seq
        g.seq += 1
        cur = torch.cuda.current_stream()
        w.issued[r].append(cur)
        comm = w.comm[r]
        comm.wait_stream(cur)
        ready = torch.cuda.Event()
        ready.record(comm)
        with w.lock:
            for op in ops:
                if op.op is isend:
                    w.sends[(r, op.peer, seq)] = (op.tensor, ready)
        w.bar.wait()
        with torch.cuda.stream(comm):
            for op in ops:
                if op.op is irecv:
                    src, ev = w.sends[(op.peer, r, seq)]
                    assert src.numel() == op.tensor.numel()
                    comm.wait_event(ev)
                    torch.cuda._sleep(w.delay)
                    op.tensor.copy_(src)
                    src.record_stream(comm)  # as ProcessGroupNCCL does for its inputs
                    op.tensor.record_stream(comm)
        done = torch.cuda.Event()
        done.record(comm)
        with w.lock:
            w.done[(r, seq)] = done
        w.bar.wait()
        evs = [done] + [w.done[(op.peer, seq)] for op in ops if op.op is isend]
        return [_Work(evs, wait)]

    monkeypatch.setattr(dist, "batch_isend_irecv", batch_isend_irecv)
    monkeypatch.setattr(dist, "P2POp", _Op)
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")


def _run(world, axis, img, sig, delay):
    import torch

    from opticalflow3d_dev_amd.shard import zslab_bounds
    from opticalflow3d_dev_amd.stream import FlowStream

    w = _World(world, delay)
    res, errs, h2d = {}, [], {}

    def rank_main(rank):
        try:
            nt, nz, ny, nx = img.shape
            a0, a1 = zslab_bounds((nz, ny)[axis], rank, world)
            fs = FlowStream(3, (nz, ny, nx), img.dtype, *sig, device=0, depth=2, zslab=(rank, world, _Group(w, rank),
                                                                                       axis))
            h2d[rank] = fs.h2d
            try:
                outs, k = [], 0
                for i in range(nt):
                    fs.push(img[i, a0:a1] if axis == 0 else img[i, :, a0:a1])
                    while len(fs.order) >= fs.nwin + fs.L or (i == nt - 1 and fs.ready):
                        pend = fs.submit()
                        outs.append((k, [o.copy() for o in pend.result()]))
                        pend.release()
                        k += 1
            finally:
                fs.close()
            res[rank] = (a0, a1, outs)
        except BaseException as e:
            errs.append(repr(e))
            w.bar.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    torch.cuda.synchronize()
    assert not errs, errs
    return w, res, h2d


def _matches(full_by_t, res, axis):
    ok = True
    for rank, (a0, a1, outs) in res.items():
        for k, parts in outs:
            for a, b in zip(full_by_t(k), parts):
                want = a[a0:a1] if axis == 0 else a[:, a0:a1]
                ok &= bits_equal(want, b.reshape(want.shape))
    return ok


@pytest.mark.parametrize("world,axis", [(2, 0), (3, 0), (2, 1)])
def test_halo_exchange_stream_order(world, axis, monkeypatch):
    sig = (2, 1, 5)  # rt 3: 7-frame windows, 6 of them in 12 frames
    img = np.random.default_rng(40 + world).integers(0, 4096, size=(12, 24, 20, 32)).astype(np.uint16)
    _install(monkeypatch)
    w, res, h2d = _run(world, axis, img, sig, delay=1_000_000)
    nwin = 2 * radii(*sig)[2] + 1
    assert nwin == 7 and len(res) == world and all(len(o) == img.shape[0] - nwin + 1 for _, _, o in res.values())
    cache = {}

    def full(k):  # window k: frames k .. k + nwin - 1
        if k not in cache:
            cache[k] = calc_flow3D(img[k:k + nwin], *sig)
        return cache[k]

    assert _matches(full, res, axis)
    for r in range(world):  # every exchange on the rank's upload stream (after its H2D)
        assert w.issued[r] and all(s == h2d[r] for s in w.issued[r]), r


def test_halo_exchange_negative_control(monkeypatch):
    """The same run with Work.wait() a no-op (the consumer does not wait for the transfer):
    the model's delayed transfers are then visibly late, so the test above can fail."""
    sig = (2, 1, 5)  # rt 3: 7-frame windows, 6 of them in 12 frames
    img = np.random.default_rng(45).integers(0, 4096, size=(12, 24, 20, 32)).astype(np.uint16)
    _install(monkeypatch, wait=False)
    _, res, _ = _run(2, 0, img, sig, delay=10_000_000)
    nwin = 2 * radii(*sig)[2] + 1
    assert all(len(o) == img.shape[0] - nwin + 1 for _, _, o in res.values())
    cache = {}

    def full(k):
        if k not in cache:
            cache[k] = calc_flow3D(img[k:k + nwin], *sig)
        return cache[k]

    assert not _matches(full, res, 0)
