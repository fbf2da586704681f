"""Streaming driver for time series.

The reference's process_flow loads all NtChunk = 6*tSig+1 frames of every
window for every output frame (calc_flow.py:518, :571-574), computes, then
writes four TIFFs synchronously (:526-529).  Here:

* the input frames live in a device ring of 2*rt+1 slots: each output frame
  costs ONE host->device frame upload (the plan takes a table of frame
  pointers, so the ring is never shifted);
* uploads, compute and downloads run on their own HIP streams, ordered by
  events (upload of frame t+1 overlaps compute of frame t);
* outputs land in pinned host buffers and are handed to a writer thread, so
  TIFF writing overlaps the next frames' transfer and compute.

Results are the same kernels as calc_flow3D/calc_flow2D (bit-identical).
"""

from __future__ import annotations

import queue
import threading
import time

import numpy as np

from . import _lib
from .taps import make_taps, radii

K0_BATCH_RADII = (3, 6, 9)  # temporal radii with a batched K0 instance (csrc/kt_grad.hip k0m_fn)
MAX_FRAMES = 65  # frame pointers per plan call (kMaxT in csrc/of3d_host.hip)

# torch storage type holding each kernel-native input dtype (same width; the kernels read the bits)
_TORCH_VIEW = {
    np.dtype(np.uint8): "uint8",
    np.dtype(np.uint16): "int16",
    np.dtype(np.int16): "int16",
    np.dtype(np.uint32): "int32",
    np.dtype(np.int32): "int32",
    np.dtype(np.float32): "float32",
    np.dtype(np.float64): "float64",
}


class FlowStream:
    """Device-resident sliding window over a frame sequence.

    push(frame) uploads one frame (shape vol_shape); once 2*rt+1 frames are
    resident, submit() computes the flow of the window's centre frame (the oldest
    2*rt+1 resident frames; the oldest is then retired) and returns a Pending whose
    .result() gives host arrays (vx, vy, [vz,] rel); .release() hands the buffer set
    back (at most `depth` frames in flight).  With lookahead, push one frame more than
    the window before submit() to pipeline the next window's temporal derivative."""

    def __init__(self, ndim, vol_shape, dtype, xyzSig, tSig, wSig, device=None, depth=3, d2h="dma",
                 d2h_blocks=64, precision="fp64", rel_fp64=False, zslab=None, lookahead=None, k0_batch=None):
        """zslab=(rank, world, group[, axis]): this process holds one slab of every frame (3D
        only) — axis 0 (default): output planes shard.zslab_bounds(nz, rank, world); axis 1:
        rows zslab_bounds(ny, rank, world) of every plane.  push() then takes the rank's own
        part ((z1 - z0, ny, nx) or (nz, y1 - y0, nx)) and fetches the frame's rd + rw halo
        planes / rows from its neighbours (torch.distributed P2P: RCCL over xGMI, or gloo) on
        the upload stream — one frame's halo per output frame, overlapped with the previous
        frame's compute; results are the rank's part of vx, vy, vz, rel (no gather).
        Row slabs run the plan on the rank's rows + halo as a volume of its own (the y pass is
        the first pass of both filter chains, so rows further than rd + rw from a cut are
        exact: bit-identical), and keep the own rows.

        k0_batch=M (2..5; default 5 for whole-volume 3D streams unless `lookahead` is given):
        M-1 frames of lookahead resident before submit (push them BEFORE submitting the current
        window), and one K0 pass forms the temporal derivatives of M consecutive windows
        (of3d_plan_execute_ahead: 2rt+M frame reads for M windows); the ring then has 2*rt+1+M
        slots.  lookahead=True (with k0_batch unset or < 2): frame pipelining instead — one more
        frame resident, and the current window's W-z/solve kernel forms the next window's
        temporal derivative (of3d_plan_execute_next); 2*rt+3 slots.  Bit-identical either way."""
        import torch

        from .shard import check_slab_split, halo_planes, zslab_bounds

        self.torch = torch
        self.ndim = ndim
        self.device = _lib.device_index() if device is None else device
        self.dev = torch.device("cuda", self.device)
        dt = np.dtype(dtype)
        if dt not in _TORCH_VIEW:
            dt = np.dtype(np.float64)
        self.np_dtype = dt
        self.code = _lib.DTYPE_CODES[dt]
        tdt = getattr(torch, _TORCH_VIEW[dt])
        if ndim == 3:
            nz, ny, nx = vol_shape
        else:
            (ny, nx), nz = vol_shape, 1
        self.nz, self.ny, self.nx = nz, ny, nx
        self.rd, self.rs, self.rt, self.rw = radii(xyzSig, tSig, wSig)
        self.nwin = 2 * self.rt + 1
        self.batch = 0
        if k0_batch is None:  # default: K0 batching of 5 windows for whole-volume 3D streams
            k0_batch = 5 if lookahead is None else 0
        # batched K0 instances exist for rt 3, 6, 9 (tSig 1, 2, 3: csrc/kt_grad.hip k0m_fn) and
        # 2rt+M frames within the plan's 65-frame table; elsewhere the ring holds no lookahead
        if (k0_batch >= 2 and ndim == 3 and zslab is None and self.rt in K0_BATCH_RADII
                and self.nwin + min(int(k0_batch), 5) - 1 <= MAX_FRAMES):
            self.batch = min(int(k0_batch), 5)
            lookahead = False
        elif k0_batch >= 2 and lookahead is None:
            lookahead = False  # asked for batching: no frame pipelining in its place
        if lookahead is None:
            lookahead = ndim == 3 and zslab is None
        self.L = self.batch - 1 if self.batch else (1 if lookahead else 0)
        if zslab is not None and ndim != 3:
            raise ValueError("z-slabs need a 3D volume")
        self.rank, self.world, self.group = zslab[:3] if zslab is not None else (0, 1, None)
        self.axis = zslab[3] if zslab is not None and len(zslab) > 3 else 0
        if zslab is not None:
            check_slab_split((nz, ny)[self.axis], self.world)  # every rank owns planes (rows)
        plane = ny * nx
        taps = make_taps(xyzSig, tSig, wSig)
        if precision not in ("fp64", "fp32"):
            raise ValueError("precision must be 'fp64' (bit-exact) or 'fp32'")
        self.precision = precision
        mode = (_lib.OF3D_FP32 if precision == "fp32" else 0) | (_lib.OF3D_REL_F64 if rel_fp64 else 0)
        self.plan = None
        self.z0, self.z1, self.zi0, self.zi1 = 0, nz, 0, nz
        self.y0, self.y1, self.yi0, self.yi1 = 0, ny, 0, ny
        self.rows_direct = False
        if self.axis == 0:
            self.z0, self.z1 = zslab_bounds(nz, self.rank, self.world)
            if zslab is not None:
                self.zi0, self.zi1 = halo_planes(nz, self.z0, self.z1, self.rd, self.rw)
            self.shape = tuple(vol_shape) if zslab is None else (self.z1 - self.z0, ny, nx)  # pushed / returned
            self.nvox = (self.z1 - self.z0) * plane
            self.nblock = (self.zi1 - self.zi0) * plane
            self.own0 = (self.z0 - self.zi0) * plane  # own planes' offset in a ring slot
            if self.nvox > 0:
                self.plan = _lib.Plan(ndim, nz, ny, nx, taps, device=self.device, mode=mode,
                                      max_out_planes=self.z1 - self.z0 if zslab is not None else 0)
                if zslab is not None:
                    assert self.plan.input_range(self.z0, self.z1) == (self.zi0, self.zi1)
        else:
            self.y0, self.y1 = zslab_bounds(ny, self.rank, self.world)
            self.yi0, self.yi1 = halo_planes(ny, self.y0, self.y1, self.rd, self.rw)
            self.shape = (nz, self.y1 - self.y0, nx)
            self.nvox = nz * (self.y1 - self.y0) * nx
            self.nblock = nz * (self.yi1 - self.yi0) * nx
            self.own0 = 0
            self.rows_direct = False  # the plan writes only the own rows (of3d_plan_set_rows)
            if self.nvox > 0:
                self.plan = _lib.Plan(3, nz, self.yi1 - self.yi0, nx, taps, device=self.device, mode=mode)
                try:
                    self.plan.set_rows(self.y0 - self.yi0, self.y1 - self.yi0)
                    self.rows_direct = True
                except RuntimeError:  # kernels without row ranges: whole sub-volume, then a slice
                    pass
        depth = self._fit_device_memory(depth, tdt, ndim, precision, rel_fp64)
        # nwin + 1 (+ lookahead) slots: a new frame's upload (and halo exchange) goes to the slot
        # the frame before last read, so it overlaps the previous frame's compute
        nslot = self.nwin + 1 + self.L
        self.ring = torch.empty((nslot, max(self.nblock, 1)), dtype=tdt, device=self.dev)
        self.order = []  # ring slots of the resident frames, oldest first
        self.free = list(range(nslot))
        self.dstage = torch.empty(max(self.nvox, 1), dtype=tdt, device=self.dev) if self.axis == 1 else None
        self.stage = [torch.empty(max(self.nvox, 1), dtype=tdt).pin_memory() for _ in range(2)]
        self.stage_np = [t.numpy().view(dt)[:self.nvox].reshape(self.shape) for t in self.stage]
        self.stage_evt = [None, None]
        self.stage_i = 0
        # Downloads (d2h):
        #   "dma"     of3d_dma_copy on the SDMA engines from a download thread
        #             once the frame's kernels are done: no CU time, and the
        #             next frame's kernels run at full speed meanwhile;
        #   "kernel"  of3d_copy_async, d2h_blocks workgroups on a stream of its
        #             own priority (hence its own hardware queue);
        #   "runtime" torch copy_ — HIP's device->host path is a blit kernel
        #             over the whole GPU.
        # Kernel-driven PCIe writes (the last two) back up the memory pipeline
        # shared with the compute kernels and slow them several-fold.
        if d2h not in ("dma", "kernel", "runtime"):
            raise ValueError("d2h must be 'dma', 'kernel' or 'runtime'")
        self.d2h_mode = d2h
        self.h2d = torch.cuda.Stream(device=self.dev)
        self.comp = torch.cuda.Stream(device=self.dev)
        self.d2h = torch.cuda.Stream(device=self.dev, priority=-1)
        self.dl_q = None
        self.stats = {"dl_wait_s": 0.0, "dl_copy_s": 0.0, "dl_n": 0}
        self.trace = None  # list -> (time, event) records of the download thread
        if d2h == "dma":
            self.dl_q = queue.Queue()
            self.dl_thread = threading.Thread(target=self._download_loop, daemon=True)
            self.dl_thread.start()
        nout = 4 if ndim == 3 else 3
        v_t = torch.float32 if precision == "fp32" else torch.float64
        if precision == "fp32":
            rel_t = torch.float32
        else:
            rel_t = torch.float64 if (ndim == 2 or rel_fp64) else torch.float32
        self.depth = depth
        self.d2h_blocks = d2h_blocks
        nv = max(self.nvox, 1)
        mk = lambda pin, n=nv: [torch.empty(n, dtype=v_t, device=None if pin else self.dev,
                                            pin_memory=pin) for _ in range(nout - 1)] + \
                               [torch.empty(n, dtype=rel_t, device=None if pin else self.dev, pin_memory=pin)]
        self.dout = [mk(False) for _ in range(depth)]
        self.hout = [mk(True) for _ in range(depth)]
        # row slabs without row ranges: the plan writes all rows of its sub-volume here; the own
        # rows are copied out
        self.dfull = mk(False, max(self.nblock, 1)) if self.axis == 1 and not self.rows_direct else None
        self.host_free = [threading.Event() for _ in range(depth)]  # set: writer released the set
        for e in self.host_free:
            e.set()
        self.slot_evt = {}               # ring slot -> event of the last compute that read it
        self.k = 0

    def _fit_device_memory(self, depth, tdt, ndim, precision, rel_fp64, margin=1 << 30):
        """Output sets in flight and frames of lookahead that fit the device beside the plan's
        workspace (already allocated): fewer output sets first, then K0 batching M -> 2 -> none
        (frame pipelining: -> none); raises only when even one set and no lookahead do not fit.
        Returns the depth; self.batch / self.L are updated."""
        torch = self.torch
        free = torch.cuda.mem_get_info(self.dev)[0] - margin
        nout = 4 if ndim == 3 else 3
        v_sz = 4 if precision == "fp32" else 8
        rel_sz = 4 if precision == "fp32" else (8 if (ndim == 2 or rel_fp64) else 4)
        set_b = max(self.nvox, 1) * ((nout - 1) * v_sz + rel_sz)
        slot_b = max(self.nblock, 1) * torch.empty((), dtype=tdt).element_size()
        fixed = slot_b * (self.nwin + 1) + (max(self.nvox, 1) * slot_b // max(self.nblock, 1) if self.axis == 1 else 0)
        if self.axis == 1:  # row slabs without row ranges write a whole sub-volume set first
            fixed += max(self.nblock, 1) * ((nout - 1) * v_sz + rel_sz)
        need = lambda d, lk: fixed + lk * slot_b + d * set_b
        while depth > 1 and need(depth, self.L) > free:
            depth -= 1
        while self.L and need(depth, self.L) > free:
            if self.batch > 2:
                self.batch, self.L = 2, 1
            else:
                self.batch, self.L = 0, 0
        if need(depth, self.L) > free:
            raise MemoryError(f"FlowStream: {need(depth, self.L) / 2**30:.1f} GiB of frames and outputs do not fit "
                              f"the {free / 2**30:.1f} GiB left on device {self.device}")
        return depth

    def push(self, frame):
        torch = self.torch
        frame = np.asarray(frame)
        if frame.shape != self.shape:
            raise ValueError(f"frame shape {frame.shape} != stream shape {self.shape}")
        if not self.free:
            raise RuntimeError("FlowStream: every ring slot holds a frame of an unsubmitted window")
        slot = self.free.pop(0)  # the slot freed longest ago (its last reader is furthest done)
        st = self.stage[self.stage_i]
        if self.stage_evt[self.stage_i] is not None:
            self.stage_evt[self.stage_i].synchronize()  # pinned staging buffer free again
        # one host pass: (byte-swap / astype(float64) as _device_array) into pinned memory
        np.copyto(self.stage_np[self.stage_i], frame, casting="unsafe")
        with torch.cuda.stream(self.h2d):
            if slot in self.slot_evt:
                self.h2d.wait_event(self.slot_evt[slot])  # no compute still reads this slot
            if self.nvox and self.axis == 0:
                self.ring[slot, self.own0:self.own0 + self.nvox].copy_(st[:self.nvox], non_blocking=True)
            elif self.nvox:
                self.dstage.copy_(st, non_blocking=True)
                self._rows(self.ring[slot])[:, self.y0 - self.yi0:self.y1 - self.yi0].copy_(
                    self.dstage[:self.nvox].view(self.shape))
            if self.world > 1:  # this frame's halo planes from / to the z-neighbours
                self.exchange(slot)
            ev = torch.cuda.Event()
            ev.record(self.h2d)
        self.stage_evt[self.stage_i] = ev
        self.stage_i ^= 1
        self.order.append(slot)

    def _rows(self, flat):
        """A ring slot / output buffer of a row-slab stream as (nz, yi1 - yi0, nx)."""
        return flat[:self.nblock].view(self.nz, self.yi1 - self.yi0, self.nx)

    def exchange(self, slot):
        """Halo planes (rows) of the frame in ring slot `slot` (slab streams): issued on the
        current stream (the upload stream in push); every rank calls it for the same frame."""
        from .shard import exchange_frame_halo

        if not self.nblock:
            blk = None
        elif self.axis == 0:
            blk = self.ring[slot, :self.nblock].view(self.zi1 - self.zi0, self.ny, self.nx)
        else:
            blk = self._rows(self.ring[slot]).transpose(0, 1)  # rows first (strided)
        lo, hi, i0, n = ((self.z0, self.z1, self.zi0, self.nz) if self.axis == 0 else
                         (self.y0, self.y1, self.yi0, self.ny))
        exchange_frame_halo(blk, i0, lo, hi, n, self.rd + self.rw, self.rank, self.world, self.group)

    @property
    def ready(self):
        return len(self.order) >= self.nwin

    @property
    def lookahead(self):
        """Frames past the window to push before submit (frame pipelining: 1; K0 batching: M-1)."""
        return self.L

    def submit(self):
        torch = self.torch
        assert self.ready
        b = self.k % self.depth
        self.k += 1
        self.host_free[b].wait()  # previous user of this set has released its host buffers,
        self.host_free[b].clear()  # which also means its D2H (and so its compute) finished
        dout, hout = self.dout[b], self.hout[b]
        self.comp.wait_stream(self.h2d)
        window = self.order[:self.nwin]
        ptrs = [self.ring[s].data_ptr() for s in window]
        # lookahead: the next window (one frame on) is resident too -> its dt0 formed in this call
        nxt = [self.ring[s].data_ptr() for s in self.order[1:self.nwin + 1]] \
            if self.L and not self.batch and len(self.order) == self.nwin + 1 else None
        # K0 batching: the resident frames past the window (up to M-1; fewer at a series' end)
        ahead = [self.ring[s].data_ptr() for s in self.order[self.nwin:self.nwin + self.L]] if self.batch else None
        vz = dout[2].data_ptr() if self.ndim == 3 else 0
        if self.plan is not None and self.axis == 0:
            self.plan.execute(ptrs, self.code, self.zi0, self.z0, self.z1 if self.ndim == 3 else 1,
                              dout[0].data_ptr(), dout[1].data_ptr(), vz, dout[-1].data_ptr(), self.comp.cuda_stream,
                              next_ptrs=nxt, pipelined=bool(self.L) and not self.batch, ahead_ptrs=ahead)
        elif self.plan is not None and self.rows_direct:  # row slab: the plan writes the own rows
            self.plan.execute(ptrs, self.code, 0, 0, self.nz, dout[0].data_ptr(), dout[1].data_ptr(),
                              dout[2].data_ptr(), dout[-1].data_ptr(), self.comp.cuda_stream)
        elif self.plan is not None:  # row slab: whole sub-volume, then the own rows
            full = self.dfull
            self.plan.execute(ptrs, self.code, 0, 0, self.nz, full[0].data_ptr(), full[1].data_ptr(),
                              full[2].data_ptr(), full[3].data_ptr(), self.comp.cuda_stream)
            with torch.cuda.stream(self.comp):
                for d, f in zip(dout, full):
                    d[:self.nvox].view(self.shape).copy_(self._rows(f)[:, self.y0 - self.yi0:self.y1 - self.yi0])
        cev = torch.cuda.Event()
        cev.record(self.comp)
        for s in self.order[:self.nwin + self.L]:  # the window and (lookahead) the next frame
            self.slot_evt[s] = cev
        self.free.append(self.order.pop(0))  # the window's oldest frame is done with (after cev)
        pending = Pending(self, b)
        if self.d2h_mode == "dma":
            self.dl_q.put((cev, hout, dout, pending))
            return pending
        with torch.cuda.stream(self.d2h):
            self.d2h.wait_event(cev)
            for h, d in zip(hout, dout):
                if self.d2h_mode == "kernel":
                    _lib.copy_async(h.data_ptr(), d.data_ptr(), d.numel() * d.element_size(), self.d2h_blocks,
                                    self.d2h.cuda_stream)
                else:
                    h.copy_(d, non_blocking=True)
            pending.event = torch.cuda.Event()
            pending.event.record(self.d2h)
        return pending

    def _download_loop(self):
        while True:
            job = self.dl_q.get()
            if job is None:
                return
            cev, hout, dout, pending = job
            try:
                t0 = time.perf_counter()
                cev.synchronize()
                t1 = time.perf_counter()
                if self.nvox:
                    _lib.dma_copy([h.data_ptr() for h in hout], [d.data_ptr() for d in dout],
                                  [d.numel() * d.element_size() for d in dout])
                t2 = time.perf_counter()
                self.stats["dl_wait_s"] += t1 - t0
                self.stats["dl_copy_s"] += t2 - t1
                self.stats["dl_n"] += 1
                if self.trace is not None:
                    self.trace += [(t0, "dl_get"), (t1, "dl_cev"), (t2, "dl_done")]
            except BaseException as e:  # re-raised by Pending.result()
                pending.error = e
            pending.done.set()

    def close(self):
        if self.dl_q is not None:
            self.dl_q.put(None)
            self.dl_thread.join()
            self.dl_q = None
        self.torch.cuda.synchronize(self.dev)
        if self.plan is not None:
            self.plan.close()


class Pending:
    def __init__(self, fs, b):
        self.fs, self.b = fs, b
        self.event = None               # D2H on a stream: completion event
        self.done = threading.Event()   # D2H by the download thread
        self.error = None

    def result(self):
        """Host arrays: views of pinned buffers, valid until release()."""
        if self.event is not None:
            self.event.synchronize()
        else:
            self.done.wait()
            if self.error is not None:
                raise self.error
        shp, n = self.fs.shape, self.fs.nvox
        return [t.numpy()[:n].reshape(shp) for t in self.fs.hout[self.b]]

    def release(self):
        self.fs.host_free[self.b].set()


class Writer:
    """Background TIFF writer; jobs run in submission order."""

    def __init__(self, write_fn):
        self.q = queue.Queue(maxsize=4)
        self.write_fn = write_fn
        self.err = None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            job = self.q.get()
            if job is None:
                return
            try:
                self.write_fn(*job)
            except BaseException as e:  # surfaced on close()
                self.err = e
            finally:
                self.q.task_done()

    def put(self, *job):
        if self.err:
            raise self.err
        self.q.put(job)

    def close(self):
        self.q.put(None)
        self.t.join()
        if self.err:
            raise self.err
