"""Host API mirroring the reference module ``calc_flow`` (src/Python/calc_flow.py).

Same names, signatures, defaults, argument checks (``SystemExit`` with the
reference's messages), output dtypes and output files; the arithmetic runs on
the MI355X through ``libof3d.so`` (HIP kernels behind a C-ABI, include/of3d.h).

* ``calc_flow3D(images, xyzSig=3, tSig=1, wSig=4) -> (vx, vy, vz, rel)``
  — calc_flow.py:175-360.  vx/vy/vz float64, rel float32 (the reference's
  rel comes from complex64 LAPACK, calc_flow.py:355-357).
* ``calc_flow2D(images, xySig=3, tSig=1, wSig=4) -> (vx, vy, rel)``
  — calc_flow.py:18-173, all float64.
* ``process_flow(imDir, imName, fileType="SequenceT", spatialDimensions=3,
  xyzSig=3, tSig=1, wSig=4)`` — calc_flow.py:362-625 (alias ``calc_flow``).

There is no CPU fallback: without the HIP library or a GPU the calls raise.
"""

from __future__ import annotations

import ctypes
import math
import os
import re
import sys
from datetime import datetime
from pathlib import Path

import numpy as np

from . import _lib
from . import tiff as tf
from .taps import make_taps

MSG_NDIM_3D = "ERROR: Input image must be a 3D matrix with dimensions N_T, N_Z, N_Y, N_X"
MSG_NDIM_2D = "ERROR: Input image must be a 3D matrix with dimensions N_T, N_Y, N_X"
MSG_EDGE = "ERROR: Input images will lead to edge effects. N_T must be >= 6*tSig+1"
MSG_ODD = ("ERROR: Input images must have an odd number of timepoints. "
           "Only the central time point is analyzed")

_D = ctypes.POINTER(ctypes.c_double)
_F = ctypes.POINTER(ctypes.c_float)

last_perf = {}


def _check_args(images, ndim, tSig, msg_ndim):
    """T9: the reference's checks in its order (calc_flow.py:212-222 / :54-64)."""
    if not (len(images.shape) == ndim):
        sys.exit(msg_ndim)
    Nt = images.shape[0]
    if Nt < 6 * tSig + 1:
        sys.exit(MSG_EDGE)
    if not (Nt % 2):
        sys.exit(MSG_ODD)


def _device_array(images):
    """C-contiguous native-endian array of a dtype the kernels read directly.

    Other real dtypes are cast with astype(np.float64) — the same cast the
    reference applies to every input (calc_flow.py:225 / :67)."""
    a = np.asarray(images)
    dt = a.dtype.newbyteorder("=") if a.dtype.byteorder not in ("=", "|") else a.dtype
    if dt in _lib.DTYPE_CODES:
        a = np.ascontiguousarray(a, dtype=dt)
    else:
        a = np.ascontiguousarray(a.astype(np.float64))
    return a, _lib.DTYPE_CODES[a.dtype]


def _perf_dict(perf):
    return {"ms_h2d": perf.ms_h2d, "ms_kernels": perf.ms_kernels, "ms_d2h": perf.ms_d2h,
            "ms_total": perf.ms_total}


def calc_flow3D(images, xyzSig=3, tSig=1, wSig=4):
    """Three-dimensional LK optical flow of the centre frame of ``images``.

    images: (N_T, N_Z, N_Y, N_X), N_T odd and >= 6*tSig+1 (calc_flow.py:190-199).
    Returns vx, vy, vz (float64, pixels/frame) and rel (float32, smallest
    eigenvalue of A'wA)."""
    return _flow3d(images, xyzSig, tSig, wSig, rel_fp64=False)


def _flow3d(images, xyzSig, tSig, wSig, rel_fp64=False):
    """calc_flow3D; rel_fp64=True returns the fp64 eigenvalue (MATLAB-style rel)."""
    _check_args(images, 4, tSig, MSG_NDIM_3D)
    taps = _lib.TapSet(make_taps(xyzSig, tSig, wSig))
    a, code = _device_array(images)
    Nt, Nz, Ny, Nx = a.shape
    vx = np.empty((Nz, Ny, Nx), np.float64)
    vy = np.empty_like(vx)
    vz = np.empty_like(vx)
    rel = np.empty((Nz, Ny, Nx), np.float64 if rel_fp64 else np.float32)
    if vx.size == 0:
        return vx, vy, vz, rel
    lib = _lib.load()
    perf = _lib.Perf()
    _lib.check(lib.of3d_flow3d(a.ctypes.data, code, Nt, Nz, Ny, Nx, ctypes.byref(taps.struct),
                               _lib.OF3D_FP64_EXACT | (_lib.OF3D_REL_F64 if rel_fp64 else 0), _lib.device_index(),
                               vx.ctypes.data_as(_D), vy.ctypes.data_as(_D), vz.ctypes.data_as(_D), rel.ctypes.data,
                               ctypes.byref(perf)))
    last_perf.clear()
    last_perf.update(_perf_dict(perf))
    return vx, vy, vz, rel


def calc_flow2D(images, xySig=3, tSig=1, wSig=4):
    """Two-dimensional LK optical flow of the centre frame of ``images``.

    images: (N_T, N_Y, N_X) (calc_flow.py:33-35).  Returns vx, vy, rel, all
    float64; rel is NaN where the discriminant rounds negative (as NumPy)."""
    _check_args(images, 3, tSig, MSG_NDIM_2D)
    taps = _lib.TapSet(make_taps(xySig, tSig, wSig))
    a, code = _device_array(images)
    Nt, Ny, Nx = a.shape
    vx = np.empty((Ny, Nx), np.float64)
    vy = np.empty_like(vx)
    rel = np.empty_like(vx)
    if vx.size == 0:
        return vx, vy, rel
    lib = _lib.load()
    perf = _lib.Perf()
    _lib.check(lib.of3d_flow2d(a.ctypes.data, code, Nt, Ny, Nx, ctypes.byref(taps.struct),
                               _lib.OF3D_FP64_EXACT, _lib.device_index(), vx.ctypes.data_as(_D),
                               vy.ctypes.data_as(_D), rel.ctypes.data_as(_D), ctypes.byref(perf)))
    last_perf.clear()
    last_perf.update(_perf_dict(perf))
    return vx, vy, rel


def _flow_fp32(images, ndim, xyzSig, tSig, wSig):
    from .stream import FlowStream

    _check_args(images, ndim + 1, tSig, MSG_NDIM_3D if ndim == 3 else MSG_NDIM_2D)
    a = np.asarray(images)
    rt = math.ceil(3 * tSig)
    c = a.shape[0] // 2
    dt = a.dtype.newbyteorder("=") if a.dtype.byteorder not in ("=", "|") else a.dtype
    shape = a.shape[1:]
    if int(np.prod(shape)) == 0:
        out = np.empty(shape, np.float32)
        return tuple(out.copy() for _ in range(ndim + 1))
    fs = FlowStream(ndim, shape, dt, xyzSig, tSig, wSig, depth=1, precision="fp32")
    try:
        for k in range(c - rt, c + rt + 1):
            fs.push(a[k])
        pend = fs.submit()
        out = tuple(o.copy() for o in pend.result())
        pend.release()
    finally:
        fs.close()
    return out


def calc_flow3D_fp32(images, xyzSig=3, tSig=1, wSig=4):
    """calc_flow3D on the fp32 path (OF3D_FP32, configs[4]): filter passes and
    the structure tensor in float32 (scipy order), solve and eigenvalue in
    fp64 on that tensor; returns float32 vx, vy, vz, rel.  Not bit-exact:
    max|dv| <= 1e-4 max|v| against calc_flow3D on smooth data."""
    return _flow_fp32(images, 3, xyzSig, tSig, wSig)


def calc_flow2D_fp32(images, xySig=3, tSig=1, wSig=4):
    """calc_flow2D on the fp32 path; float32 vx, vy, rel."""
    return _flow_fp32(images, 2, xySig, tSig, wSig)


def _now():
    return str(datetime.now())


def _dist_context():
    """(rank, world) of an initialised torch.distributed job, else (0, 1)."""
    try:
        import torch.distributed as dist
    except ImportError:
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def process_flow(imDir, imName, fileType="SequenceT", spatialDimensions=3, xyzSig=3, tSig=1, wSig=4,
                 precision="fp64", matlab_output=False, parallel="auto"):
    """Parse a TIFF time lapse, run the flow per output frame, write TIFFs.

    Mirrors calc_flow.py:362-625: same checks and messages, the same
    ``OpticalFlow3D/<imNameSave>/`` (or ``OpticalFlow2D``) output folder,
    ``<imNameSave>_parameters.csv`` and ``<imNameSave>_{vx,vy,[vz,]rel}_t%04d.tiff``
    files, the same stdout lines.  Returns None.  Extensions: precision="fp32"
    (configs[4]) runs the float32 path and writes float32 TIFFs;
    matlab_output=True writes what the reference's MATLAB twin writes
    (M/TIFFwrite.m: LZW BigTIFF, float64; rel kept fp64 as pageeig does,
    M/calc_flow3D.m:235-236).

    Several GPUs (one process per GPU, torch.distributed initialised, e.g. by
    ``shard.init_distributed()`` under torchrun): the reference's own parallel axis
    (calc_flow.py:512, "this could become a parfor loop") — ``parallel="frames"``: each
    rank streams a contiguous block of output frames and writes their files;
    ``parallel="zslab"`` (3D): every rank reads only its z-planes of each frame, fetches
    the stencil halo planes from its z-neighbours (RCCL P2P) and writes its planes of
    every output file (shard, tiff.write_planes; no gather); ``"yslab"``: the same with
    rows of every plane (less halo work when Ny >> Nz: the y pass is the first pass of
    both filter chains).  ``"auto"``: frames when there are at least as many output
    frames as ranks, else the slab axis with less predicted halo work
    (shard.slab_axis).  A slab split that would leave a rank without planes (rows) runs
    as frames instead.  Files and pixel values are the same as on one GPU."""
    ### Check Inputs and Set Up Paths (calc_flow.py:413-442)
    imDir = Path(imDir)
    if not imDir.is_dir():
        sys.exit('ERROR: image path \'%s\' does not exist' % imDir)
    imNamePattern = re.compile(imName + '.tif')
    fileList = [f for f in os.listdir(imDir) if imNamePattern.fullmatch(f)]
    if len(fileList) == 0:
        sys.exit('ERROR: No image files found. imName: ' + imName + ' imDir: ' + str(imDir))
    if fileType == 'OneTif':
        if len(fileList) > 1:
            sys.exit('ERROR: Type is OneTif but more than one file was found for imName: ' + imName)
    elif fileType == 'SequenceT':
        if len(fileList) < 6 * tSig + 1:
            sys.exit('ERROR: Image sequence found for file name ' + imName + ' only contains '
                     + str(len(fileList)) + ' files. Minimum 6*tsig+1 (' + str(6 * tSig + 1) + ') files required.')
    else:
        sys.exit('ERROR: fileType must be either OneTif or SequenceT.')
    fileList = tf.natsorted(fileList)
    if spatialDimensions < 2 or spatialDimensions > 3:
        sys.exit('ERROR: Number of spatial dimensions must be either 2 or 3.')

    ### Metadata parsing and parameter saving (calc_flow.py:445-494)
    meta = tf.TiffFile(imDir / fileList[0])
    Ny = meta.pages[0].shape[0]
    Nx = meta.pages[0].shape[1]
    imj = meta.imagej_metadata
    if fileType == 'OneTif':
        if not imj:
            sys.exit('ERROR: fileType is OneTif, but no ImageJ metadata was detected')
        Nt = imj["frames"]
        if spatialDimensions == 3:
            Nz = imj["slices"]
        elif spatialDimensions == 2:
            Nz = 1
    elif fileType == 'SequenceT':
        Nz = len(meta.pages)
        Nt = len(fileList)
        if spatialDimensions == 2:
            if Nz != 1:
                sys.exit('ERROR: More than one z-slice detected for 2D processing')
        elif spatialDimensions == 3:
            if Nz <= 1:
                sys.exit('ERROR: 3D processing requested but Nz = ' + str(Nz))

    NtChunk = 6 * tSig + 1
    if not (NtChunk % 2):
        NtChunk = NtChunk + 1
    NtSlice = math.ceil(NtChunk / 2) - 1

    rank, world = _dist_context()
    savedir = imDir / ('OpticalFlow3D' if spatialDimensions == 3 else 'OpticalFlow2D')
    savedir.mkdir(exist_ok=True)
    imNameSave = imName.replace('.*', '')
    savedir = savedir / imNameSave
    savedir.mkdir(exist_ok=True)
    if rank == 0:
        _write_parameters(savedir / (imNameSave + '_parameters.csv'), xyzSig, tSig, wSig, Nx, Ny, Nz, Nt)

    ### Processing Loop (calc_flow.py:497-625)
    if rank == 0:
        print('Note: regardless of input filenames, the first image = frame 0.')
        print('If your file names start from 0, adjust indexing accordingly for reading the output files.')
        print(' ')
        for hh in range(0, NtSlice):
            print(_now() + ' - No data will be saved for frame ' + str(hh) + ' to avoid edge effects')

    prefix = str(savedir / imNameSave)
    names = ('vx', 'vy', 'vz', 'rel') if spatialDimensions == 3 else ('vx', 'vy', 'rel')
    flow = calc_flow3D if spatialDimensions == 3 else calc_flow2D

    allImages = None
    if fileType == 'OneTif':
        try:
            allImages = tf.memmap(imDir / (imName + '.tif'))
        except ValueError:  # compressed / tiled / scattered pages: each call decodes only its pages
            one = tf.TiffFile(imDir / (imName + '.tif'))
            npg = int(Nz) if spatialDimensions == 3 else 1  # frame i plane z = page i * Nz + z (ImageJ TZYX)
            load_frame = (lambda i: one.read_planes(i * npg, (i + 1) * npg)) if spatialDimensions == 3 else \
                (lambda i: one.read_planes(i, i + 1)[0])
            load_planes = lambda i, z0, z1: one.read_planes(i * npg + z0, i * npg + z1)
        if allImages is not None:
            load_frame = lambda i: allImages[i]
            load_planes = lambda i, z0, z1: np.asarray(allImages[i][z0:z1])
    else:
        load_frame = lambda i: tf.imread(imDir / fileList[i])
        load_planes = lambda i, z0, z1: tf.TiffFile(imDir / fileList[i]).read_planes(z0, z1)
    nOut = int(Nt) - NtChunk + 1
    rt = math.ceil(3 * tSig)
    if precision not in ("fp64", "fp32"):
        raise ValueError("precision must be 'fp64' or 'fp32'")
    if matlab_output and precision != "fp64":
        raise ValueError("matlab_output writes float64 files: use precision='fp64'")
    if parallel not in ("auto", "frames", "zslab", "yslab"):
        raise ValueError("parallel must be 'auto', 'frames', 'zslab' or 'yslab'")
    writer = tf.imwrite_matlab if matlab_output else None
    # multi-GPU split: slabs need the 3D ring path and uncompressed (slab-writable) outputs
    slab_ok = world > 1 and spatialDimensions == 3 and not matlab_output and NtChunk == 2 * rt + 1 and nOut > 0
    axis = None
    if slab_ok and parallel in ("zslab", "yslab"):
        axis = 0 if parallel == "zslab" else 1
    elif slab_ok and parallel == "auto" and nOut < world:
        from .shard import slab_axis
        from .taps import radii

        rd_, _, _, rw_ = radii(xyzSig, tSig, wSig)
        axis = slab_axis(int(Nz), int(Ny), world, rd_, rw_)
    if axis is not None and world > (int(Nz), int(Ny))[axis]:
        axis = None  # a slab per rank would leave ranks empty (shard.check_slab_split): split frames
    if axis is not None:
        if fileType == 'OneTif' and allImages is not None:
            load_rows = lambda i, y0, y1: np.asarray(allImages[i][:, y0:y1])
        elif fileType == 'OneTif':  # compressed / tiled: only the strips holding the rows
            load_rows = lambda i, y0, y1: one.read_rows(y0, y1, pages=(i * int(Nz), (i + 1) * int(Nz)))
        else:
            load_rows = lambda i, y0, y1: tf.TiffFile(imDir / fileList[i]).read_rows(y0, y1)
        _process_slab(load_planes if axis == 0 else load_rows, axis, (int(Nz), int(Ny), int(Nx)), nOut, NtChunk,
                      NtSlice, xyzSig, tSig, wSig, prefix, names, precision, rank, world)
    else:
        from .shard import frame_blocks

        h0, h1 = frame_blocks(nOut, rank, world) if nOut > 0 else (0, 0)
        if h1 > h0 and NtChunk == 2 * rt + 1:
            _process_stream(load_frame, (h0, h1), NtChunk, NtSlice, spatialDimensions, xyzSig, tSig, wSig, prefix,
                            names, precision, writer)
        else:  # window and temporal taps disagree (non-integer 6*tSig+1): one upload per window
            for hh in range(h0, h1):
                loopStart = datetime.now()
                print(_now() + ' - Processing frame ' + str(hh + NtSlice) + '...')
                images = np.stack([load_frame(hh + jj) for jj in range(NtChunk)])
                if matlab_output and spatialDimensions == 3:
                    out = _flow3d(images, xyzSig, tSig, wSig, rel_fp64=True)
                elif precision == "fp64":
                    out = flow(images, xyzSig, tSig, wSig)
                else:
                    out = _flow_fp32(images, spatialDimensions, xyzSig, tSig, wSig)
                _write_frame(prefix, names, hh + NtSlice, out, writer=writer)
                del out, images
                print(_now() + ' - Frame ' + str(hh + NtSlice) + ' saved.  Duration: ' + str(datetime.now() - loopStart))
    if world > 1:
        import torch.distributed as dist

        dist.barrier()  # every rank's files (or planes of them) are written
    if rank == 0:
        for hh in range(int(Nt) - NtSlice, int(Nt)):
            print(_now() + ' - No data will be saved for frame ' + str(hh) + ' to avoid edge effects')


calc_flow = process_flow


def _write_frame(prefix, names, frame, out, pool=None, writer=None):
    """The reference's per-frame outputs (calc_flow.py:526-529 / :579-581);
    with a thread pool the files are written concurrently."""
    tstr = str(frame).zfill(4)
    paths = [prefix + '_' + n + '_t' + tstr + '.tiff' for n in names]
    write = writer or (lambda path, arr: tf.imwrite(path, arr, photometric='minisblack'))
    if pool is None:
        for path, arr in zip(paths, out):
            write(path, arr)
    else:
        for f in [pool.submit(write, path, arr) for path, arr in zip(paths, out)]:
            f.result()


class _Shape:
    def __init__(self, shape):
        self.shape = shape


def _process_stream(load_frame, out_range, NtChunk, NtSlice, ndim, xyzSig, tSig, wSig, prefix, names,
                    precision="fp64", write_fn=None):
    """process_flow's loop on a device-resident frame ring (stream.py): one
    frame read + upload per output frame; compute, download and TIFF writing
    of consecutive frames overlap.  Files and stdout lines are the reference's
    (both lines of a frame are printed once its files are written).
    out_range = (h0, h1): the windows starting at frames h0 .. h1 - 1 (a rank's block)."""
    from concurrent.futures import ThreadPoolExecutor

    from .stream import FlowStream, Writer

    h0, h1 = out_range
    first = np.asarray(load_frame(h0))
    if len((NtChunk,) + first.shape) != ndim + 1:
        print(_now() + ' - Processing frame ' + str(NtSlice) + '...')
        _check_args(_Shape((NtChunk,) + first.shape), ndim + 1, tSig, MSG_NDIM_3D if ndim == 3 else MSG_NDIM_2D)
    dt = first.dtype.newbyteorder('=') if first.dtype.byteorder not in ('=', '|') else first.dtype
    fs = FlowStream(ndim, first.shape, dt, xyzSig, tSig, wSig, precision=precision,
                    rel_fp64=write_fn is not None and ndim == 3)

    def finish(frame, start, start_str, pending):
        print(start_str + ' - Processing frame ' + str(frame) + '...')
        try:
            _write_frame(prefix, names, frame, pending.result(), pool, write_fn)
        finally:
            pending.release()
        print(_now() + ' - Frame ' + str(frame) + ' saved.  Duration: ' + str(datetime.now() - start))

    pool = ThreadPoolExecutor(len(names))
    writer = Writer(finish)
    try:
        fs.push(first)
        pushed = h0 + 1  # next frame to upload
        for hh in range(h0, h1):
            start = datetime.now()
            start_str = str(start)
            # the window's frames, and (lookahead: frame pipelining / K0 batching) the next frames
            upto = min(hh + NtChunk + fs.lookahead, h1 + NtChunk - 1)
            while pushed < upto:
                fs.push(load_frame(pushed))
                pushed += 1
            writer.put(hh + NtSlice, start, start_str, fs.submit())
    finally:
        writer.close()
        pool.shutdown()
        fs.close()


def _process_slab(load_part, axis, vol, nOut, NtChunk, NtSlice, xyzSig, tSig, wSig, prefix, names, precision,
                  rank, world):
    """process_flow's loop on one slab rank (axis 0: z-planes, 1: rows): every frame's own part
    is read and uploaded, the halo comes from the neighbours (FlowStream(zslab=...), one
    frame's halo per output frame), and the rank writes its part of each output TIFF in place
    (tiff.write_planes / write_rows: the files end up byte-identical to single-GPU ones).
    Rank 0 prints the reference's per-frame lines once its own part is written."""
    from concurrent.futures import ThreadPoolExecutor

    from .shard import zslab_bounds
    from .stream import FlowStream, Writer

    Nz, Ny, Nx = vol
    a0, a1 = zslab_bounds(vol[axis], rank, world)
    first = np.asarray(load_part(0, a0, a1))
    dt = first.dtype.newbyteorder('=') if first.dtype.byteorder not in ('=', '|') else first.dtype
    fs = FlowStream(3, vol, dt, xyzSig, tSig, wSig, precision=precision, zslab=(rank, world, None, axis))
    write = tf.write_planes if axis == 0 else tf.write_rows

    def finish(frame, start, start_str, pending):
        try:
            out = pending.result()
            tstr = str(frame).zfill(4)
            for f in [pool.submit(write, prefix + '_' + n + '_t' + tstr + '.tiff', vol, a.dtype, a0, a)
                      for n, a in zip(names, out)]:
                f.result()
        finally:
            pending.release()
        if rank == 0:
            print(start_str + ' - Processing frame ' + str(frame) + '...')
            print(_now() + ' - Frame ' + str(frame) + ' saved.  Duration: ' + str(datetime.now() - start))

    pool = ThreadPoolExecutor(len(names))
    writer = Writer(finish)
    try:
        fs.push(first)
        for i in range(1, NtChunk - 1):
            fs.push(load_part(i, a0, a1))
        for hh in range(nOut):
            start = datetime.now()
            fs.push(load_part(hh + NtChunk - 1, a0, a1))
            writer.put(hh + NtSlice, start, str(start), fs.submit())
    finally:
        writer.close()
        pool.shutdown()
        fs.close()


def _fmt_csv(v):
    if isinstance(v, (bool, np.bool_)):
        return str(bool(v))
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    return repr(float(v))


def _write_parameters(path, xyzSig, tSig, wSig, Nx, Ny, Nz, Nt):
    """<imNameSave>_parameters.csv as pandas.DataFrame.to_csv(index=False) writes it
    (calc_flow.py:485-494; column name 'tiSig' sic)."""
    cols = ['xyzSig', 'tiSig', 'wSig', 'Nx', 'Ny', 'Nz', 'Nt']
    vals = [xyzSig, tSig, wSig, Nx, Ny, Nz, Nt]
    with open(path, 'w', newline='') as f:
        f.write(','.join(cols) + '\n')
        f.write(','.join(_fmt_csv(v) for v in vals) + '\n')
