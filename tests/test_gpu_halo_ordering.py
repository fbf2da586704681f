"""Stream ordering of the slab halo exchange under RCCL's semantics, on one GPU.

The gloo tests stage every halo through synchronous .cpu() copies, so they cannot catch an
ordering bug of the RCCL path (FlowStream.push issues the H2D and shard.exchange_frame_halo on
the upload stream and the compute waits on that stream's event; the N > 1 bench's SlabBench
exchanges on a side stream beside the previous step's compute).  Two ranks cannot share one
GPU under RCCL, so the ranks here are threads of one process, and torch.distributed's P2P
calls are replaced by a model of ProcessGroupNCCL's documented stream contract:
  * batch_isend_irecv: the rank's communication stream waits on the caller's current stream
    (the sends read what that stream wrote), then runs the transfers;
  * Work.wait(): the caller's current stream waits on the communication stream (the
    receiving rank's later work sees the halo; the sending rank's later writes to the sent
    planes wait for the peer's copy) — the host does not block.
A receive first fills its buffer with a garbage pattern (a receive buffer is undefined until
its work completes), then the transfer starts after a device-side delay (torch.cuda._sleep,
~4 ms: longer than a host step) on the communication stream, so a consumer that did not wait
for it reads garbage.  Each case runs in a child process with GPU_MAX_HW_QUEUES=16 (HIP's
default of 4 hardware queues multiplexes the 6-9 streams of the ranks, and streams sharing a
queue run in issue order — which would hide exactly the races looked for here).

Checked: every rank's part of every computed window equals the unsharded result bit for bit;
FlowStream's exchanges are issued on its upload stream; and the negative controls (Work.wait()
a no-op for FlowStream; SlabBench computes that forget their exchange events) differ, so the
model does expose a missing wait.  Reference: calc_flow.py:512 (the per-frame loop the slabs
split)."""
import multiprocessing as mp
import threading
import traceback

import numpy as np
import pytest

from conftest import bits_equal

pytestmark = pytest.mark.gpu

DELAY = 10_000_000  # torch.cuda._sleep cycles per transfer (~4 ms on MI355X)


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


_tls = threading.local()  # group=None (the default group, as SlabBench calls it): the thread's rank


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


def _install(wait=True):
    """Replace torch.distributed's P2P entry points (in this child process) by the model."""
    import torch
    import torch.distributed as dist

    isend, irecv = dist.isend, dist.irecv

    def batch_isend_irecv(ops):
        g = ops[0].group if ops[0].group is not None else _tls.group
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
                    op.tensor.fill_(0x7F)
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

    dist.batch_isend_irecv = batch_isend_irecv
    dist.P2POp = _Op
    dist.get_backend = lambda group=None: "nccl"


def _threads(world, w, body):
    errs = []

    def main(rank):
        try:
            body(rank)
        except BaseException:
            errs.append(traceback.format_exc()[-2000:])
            w.bar.abort()

    ts = [threading.Thread(target=main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs and not any(t.is_alive() for t in ts), errs


def _stream_case(world, axis, seed):
    """FlowStream(zslab=...) ranks over a 12-frame series: (windows, mismatching windows,
    exchanges issued on the upload stream)."""
    import torch

    from opticalflow3d_dev_amd import calc_flow3D, radii
    from opticalflow3d_dev_amd.shard import zslab_bounds
    from opticalflow3d_dev_amd.stream import FlowStream

    sig = (2, 1, 5)  # rt 3: 7-frame windows, 6 of them in 12 frames
    img = np.random.default_rng(seed).integers(0, 4096, size=(12, 24, 20, 32)).astype(np.uint16)
    nt, nz, ny, nx = img.shape
    w = _World(world, DELAY)
    res, h2d = {}, {}

    def body(rank):
        a0, a1 = zslab_bounds((nz, ny)[axis], rank, world)
        fs = FlowStream(3, (nz, ny, nx), img.dtype, *sig, device=0, depth=2, zslab=(rank, world, _Group(w, rank), axis))
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

    _threads(world, w, body)
    torch.cuda.synchronize()
    nwin = 2 * radii(*sig)[2] + 1
    windows, bad = 0, []
    for rank, (a0, a1, outs) in res.items():
        for k, parts in outs:
            windows += 1
            for a, b in zip(calc_flow3D(img[k:k + nwin], *sig), parts):
                want = a[a0:a1] if axis == 0 else a[:, a0:a1]
                if not bits_equal(want, b.reshape(want.shape)):
                    bad.append((rank, k))
    on_upload = all(w.issued[r] and all(s == h2d[r] for s in w.issued[r]) for r in range(world))
    return {"windows": windows, "expected": world * (nt - nwin + 1), "bad": bad, "on_upload": on_upload}


class _DropEvents(dict):
    """SlabBench.xev that forgets every exchange event: the compute never waits for the halo."""

    def __setitem__(self, k, v):
        pass


def _bench_case(world, axis, mode):
    """bench.SlabBench ranks through mixed steps: (computed windows, mismatching windows)."""
    import torch

    import bench

    dims, sig, seed = (48, 24, 32), (1, 1, 5), 777
    kw = dict(pipeline=mode != "plain", k0_batch=3 if mode == "k0_batch" else 0)
    plan_steps = ["both"] * 5 + ["comp"] * 2 + ["xchg"] * 2 + ["both"] * 4
    dev = torch.device("cuda", 0)

    def drive(sb):
        got = []
        for st in plan_steps:
            sb.step(exchange=st != "comp", compute=st != "xchg")
            if st != "xchg":
                with torch.cuda.stream(sb.comp):
                    got.append([o[:sb.n_out].clone() for o in sb.outs] + [sb.rel[:sb.n_out].clone()])
        torch.cuda.synchronize(dev)
        return [[t.cpu().numpy() for t in g] for g in got]

    # SlabBench computes on the stream current at its construction (the bench: the null stream,
    # which may order itself against other streams implicitly); a pool stream here, so the
    # only order between compute and exchange is the one SlabBench sets up
    with torch.cuda.stream(torch.cuda.Stream(device=dev)):
        ref_sb = bench.SlabBench(dims, sig, axis, 0, 1, dev, seed=seed, **kw)
        try:
            ref = drive(ref_sb)
        finally:
            ref_sb.close()
    w = _World(world, DELAY)
    res = {}

    def body(rank):
        _tls.group = _Group(w, rank)
        with torch.cuda.stream(torch.cuda.Stream(device=dev)):
            sb = bench.SlabBench(dims, sig, axis, rank, world, dev, seed=seed, **kw)
            if mode == "negative":
                sb.xev = _DropEvents()
            try:
                res[rank] = (sb.a0, sb.a1, drive(sb))
            finally:
                sb.close()

    _threads(world, w, body)
    nz, ny, nx = dims
    windows, bad = 0, []
    for rank, (a0, a1, got) in res.items():
        assert len(got) == len(ref)
        for i, (g, f) in enumerate(zip(got, ref)):
            windows += 1
            for a, b in zip(f, g):
                full = a.reshape(nz, ny, nx)
                want = full[a0:a1] if axis == 0 else full[:, a0:a1]
                if not bits_equal(want, b.reshape(want.shape)):
                    bad.append((rank, i))
    return {"windows": windows, "expected": world * len(ref), "bad": bad}


def _child(kind, params, q):
    try:
        _install(wait=params.pop("wait", True))
        q.put(("ok", (_stream_case if kind == "stream" else _bench_case)(**params)))
    except BaseException:
        q.put(("err", traceback.format_exc()[-3000:]))


def _spawn(kind, monkeypatch, **params):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "16")  # read by HIP in the child at its initialisation
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(kind, params, q))
    p.start()
    try:
        status, out = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert status == "ok", out
    assert out["windows"] == out["expected"] > 0, out
    return out


@pytest.mark.parametrize("world,axis", [(2, 0), (3, 0), (2, 1)])
def test_flowstream_halo_stream_order(world, axis, monkeypatch):
    out = _spawn("stream", monkeypatch, world=world, axis=axis, seed=40 + world)
    assert not out["bad"], out["bad"]
    assert out["on_upload"]  # every exchange on the rank's upload stream (after its H2D)


def test_flowstream_negative_control(monkeypatch):
    """Work.wait() a no-op (the consumer does not wait for the transfer): some window differs."""
    out = _spawn("stream", monkeypatch, world=2, axis=0, seed=45, wait=False)
    assert out["bad"], "the model did not expose a consumer that skips Work.wait()"


@pytest.mark.parametrize("world,axis,mode", [(2, 0, "pipeline"), (3, 0, "k0_batch"), (2, 1, "pipeline"),
                                             (2, 0, "plain")])
def test_slab_bench_stream_order(world, axis, mode, monkeypatch):
    """bench.SlabBench (the N > 1 line's strong split) under the model: every computed window's
    own part bitwise equal to a one-rank SlabBench over the same ring (the same synthetic
    frames by seed), through mixed steps (exchange + compute, compute alone, exchange alone)
    as strong_split runs them."""
    out = _spawn("bench", monkeypatch, world=world, axis=axis, mode=mode)
    assert not out["bad"], out["bad"]


def test_slab_bench_negative_control(monkeypatch):
    """SlabBench computes that forget their exchange events: some window differs."""
    out = _spawn("bench", monkeypatch, world=2, axis=0, mode="negative")
    assert out["bad"], "the model did not expose computes that skip the exchange wait"
