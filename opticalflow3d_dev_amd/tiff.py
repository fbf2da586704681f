"""Minimal TIFF reader/writer for the process_flow driver.

The reference driver uses ``tifffile`` (calc_flow.py:12) for four things:
``TiffFile(...).pages[0].shape`` / ``len(pages)`` / ``imagej_metadata``
(calc_flow.py:445-465), ``memmap`` of an ImageJ hyperstack (:509),
``imread`` of one file per time point (:571-574) and
``imwrite(path, arr, photometric='minisblack')`` for the outputs (:526-529).
``tifffile`` is not installed in this image, so this module implements that
subset from the TIFF 6.0 / BigTIFF layout:

* reading: classic and BigTIFF, either byte order, uncompressed strips,
  uint8/16/32, int8/16/32, float32/64 samples, one sample per pixel; ImageJ
  hyperstacks whose image data is one contiguous block (ImageJ writes > 4 GB
  stacks with a single IFD and contiguous planes — the case the MATLAB twin
  handles in ``M/TIFFvolume.m:48-52,82-115``);
* writing: little-endian, uncompressed, one page per leading-axis slice with a
  tifffile-style shaped JSON description on the first page and
  SampleFormat/BitsPerSample from the array dtype; BigTIFF automatically once
  the file would pass ~4 GB (tifffile's threshold).
"""

from __future__ import annotations

import json
import os
import re
import struct

import numpy as np

_TYPES = {1: ("B", 1), 2: ("s", 1), 3: ("H", 2), 4: ("I", 4), 5: ("II", 8), 6: ("b", 1), 7: ("B", 1),
          8: ("h", 2), 9: ("i", 4), 10: ("ii", 8), 11: ("f", 4), 12: ("d", 8), 16: ("Q", 8), 17: ("q", 8),
          18: ("Q", 8)}


class Page:
    def __init__(self, tags, bo):
        self.tags = tags
        self.byteorder = bo
        self.width = int(tags[256][0])
        self.length = int(tags[257][0])
        bps = tags.get(258, (1,))
        self.bits = int(bps[0])
        self.spp = int(tags.get(277, (1,))[0])
        self.compression = int(tags.get(259, (1,))[0])
        fmt = int(tags.get(339, (1,))[0])
        kind = {1: "u", 2: "i", 3: "f"}.get(fmt)
        if kind is None:
            raise ValueError(f"unsupported SampleFormat {fmt}")
        self.dtype = np.dtype(f"{bo}{kind}{self.bits // 8}")
        self.offsets = [int(v) for v in tags.get(273, ())]
        self.counts = [int(v) for v in tags.get(279, ())]
        desc = tags.get(270)
        self.description = desc if isinstance(desc, str) else None

    @property
    def shape(self):
        if self.spp > 1:
            return (self.length, self.width, self.spp)
        return (self.length, self.width)

    @property
    def nbytes(self):
        return self.length * self.width * self.spp * self.dtype.itemsize

    def contiguous_offset(self):
        """Offset of the page data if its strips are one contiguous block."""
        if self.compression != 1 or not self.offsets:
            return None
        pos = self.offsets[0]
        for o, c in zip(self.offsets, self.counts):
            if o != pos:
                return None
            pos += c
        return self.offsets[0]


def _parse_imagej(desc):
    if not desc or not desc.startswith("ImageJ="):
        return None
    out = {}
    for line in desc.splitlines():
        if "=" not in line:
            continue
        k, v = line.split("=", 1)
        v = v.strip()
        for conv in (int, float):
            try:
                v = conv(v)
                break
            except ValueError:
                pass
        else:
            if v in ("true", "false"):
                v = v == "true"
        out[k.strip()] = v
    return out


class TiffFile:
    """Subset of tifffile.TiffFile: ``pages``, ``imagej_metadata``, ``asarray``, ``memmap``."""

    def __init__(self, path):
        self.path = os.fspath(path)
        with open(self.path, "rb") as f:
            head = f.read(16)
            if head[:2] == b"II":
                bo = "<"
            elif head[:2] == b"MM":
                bo = ">"
            else:
                raise ValueError(f"{self.path}: not a TIFF file")
            magic = struct.unpack(bo + "H", head[2:4])[0]
            if magic == 42:
                self.bigtiff = False
                first = struct.unpack(bo + "I", head[4:8])[0]
            elif magic == 43:
                self.bigtiff = True
                first = struct.unpack(bo + "Q", head[8:16])[0]
            else:
                raise ValueError(f"{self.path}: bad TIFF magic {magic}")
            self.byteorder = bo
            self.pages = []
            self.ifd_offsets = []  # file offset of each page's IFD (libtiff jumps straight to one)
            seen = set()
            off = first
            while off and off not in seen:
                seen.add(off)
                self.ifd_offsets.append(off)
                tags, off = self._read_ifd(f, off)
                self.pages.append(Page(tags, bo))
        self.imagej_metadata = _parse_imagej(self.pages[0].description) if self.pages else None
        self.shaped_metadata = None
        d = self.pages[0].description if self.pages else None
        if d and d.startswith("{"):
            try:
                self.shaped_metadata = json.loads(d)
            except ValueError:
                pass

    def _read_ifd(self, f, off):
        bo = self.byteorder
        f.seek(off)
        if self.bigtiff:
            n = struct.unpack(bo + "Q", f.read(8))[0]
            esz, vsz = 20, 8
        else:
            n = struct.unpack(bo + "H", f.read(2))[0]
            esz, vsz = 12, 4
        raw = f.read(n * esz)
        nxt_raw = f.read(vsz)
        nxt = struct.unpack(bo + ("Q" if self.bigtiff else "I"), nxt_raw)[0] if len(nxt_raw) == vsz else 0
        tags = {}
        for i in range(n):
            e = raw[i * esz:(i + 1) * esz]
            if self.bigtiff:
                code, typ, cnt = struct.unpack(bo + "HHQ", e[:12])
                val = e[12:20]
            else:
                code, typ, cnt = struct.unpack(bo + "HHI", e[:8])
                val = e[8:12]
            if typ not in _TYPES:
                continue
            fmt, size = _TYPES[typ]
            total = size * cnt
            if total > vsz:
                ptr = struct.unpack(bo + ("Q" if self.bigtiff else "I"), val)[0]
                pos = f.tell()
                f.seek(ptr)
                data = f.read(total)
                f.seek(pos)
            else:
                data = val[:total]
            if typ == 2:
                tags[code] = data.rstrip(b"\0").decode("latin-1")
            elif typ in (5, 10):
                tags[code] = struct.unpack(bo + fmt[0] * (2 * cnt), data)
            else:
                tags[code] = struct.unpack(bo + fmt * cnt, data)
        return tags, nxt

    # -- series shape (tifffile's "series[0]" for the layouts handled here)
    def series_shape(self):
        p0 = self.pages[0]
        ij = self.imagej_metadata
        if ij:
            images = int(ij.get("images", len(self.pages)))
            dims = []
            for k in ("frames", "slices", "channels"):
                v = int(ij.get(k, 1))
                if v > 1:
                    dims.append(v)
            shape = tuple(dims) + p0.shape
            if int(np.prod(dims or [1])) != images:
                shape = ((images,) if images > 1 else ()) + p0.shape
            return shape
        if self.shaped_metadata and "shape" in self.shaped_metadata:
            return tuple(int(v) for v in self.shaped_metadata["shape"])
        if len(self.pages) == 1:
            return p0.shape
        return (len(self.pages),) + p0.shape

    def _contiguous_block(self):
        """(offset, count) if all series images form one contiguous block."""
        p0 = self.pages[0]
        shape = self.series_shape()
        nimg = int(np.prod(shape)) // int(np.prod(p0.shape))
        off0 = p0.contiguous_offset()
        if off0 is None:
            return None
        if len(self.pages) >= nimg:
            pos = off0
            for p in self.pages[:nimg]:
                if p.contiguous_offset() != pos or p.shape != p0.shape or p.dtype != p0.dtype:
                    return None
                pos += p.nbytes
        elif not self.imagej_metadata:
            return None  # ImageJ >4 GB stacks: one IFD, planes contiguous after it
        return off0, nimg

    def memmap(self):
        blk = self._contiguous_block()
        if blk is None:
            raise ValueError(f"{self.path}: image data is not contiguous; cannot memory-map")
        return np.memmap(self.path, dtype=self.pages[0].dtype, mode="r", offset=blk[0], shape=self.series_shape())

    def _needs_codec(self):
        """Compressed or tiled pages: decoded through the system libtiff."""
        return any(p.compression != 1 or not p.offsets for p in self.pages)

    def read_planes(self, z0, z1):
        """Pages [z0, z1) of a plain page series (a SequenceT time point, or the planes of a
        OneTif hyperstack: frame i plane z is page i * Nz + z), as (z1 - z0, y, x): only those
        bytes are read when the pages are uncompressed, only those pages decoded otherwise."""
        p0 = self.pages[0]
        if self._needs_codec():
            arr = imread_libtiff(self.path, pages=(z0, z1), ifd_offset=self.ifd_offsets[z0])
            return np.ascontiguousarray(arr.reshape((z1 - z0,) + p0.shape), dtype=p0.dtype.newbyteorder("="))
        blk = self._contiguous_block()
        out = np.empty((z1 - z0,) + p0.shape, p0.dtype.newbyteorder("="))
        with open(self.path, "rb") as f:
            if blk is not None:
                f.seek(blk[0] + z0 * p0.nbytes)
                out[...] = np.frombuffer(f.read((z1 - z0) * p0.nbytes), dtype=p0.dtype).reshape(out.shape)
                return out
            for k, p in enumerate(self.pages[z0:z1]):
                chunks = []
                for o, c in zip(p.offsets, p.counts):
                    f.seek(o)
                    chunks.append(f.read(c))
                out[k] = np.frombuffer(b"".join(chunks), dtype=p.dtype)[: int(np.prod(p.shape))].reshape(p.shape)
        return out

    def read_rows(self, y0, y1, pages=None):
        """Rows [y0, y1) of every page (or of pages=(p0, p1): a OneTif frame's planes) of a
        plain page series, as (pages, y1 - y0, x)."""
        p0 = self.pages[0]
        a, b = pages if pages is not None else (0, len(self.pages))
        blk = self._contiguous_block()
        if blk is not None and not self._needs_codec():
            mm = np.memmap(self.path, dtype=p0.dtype, mode="r", offset=blk[0], shape=(len(self.pages),) + p0.shape)
            return np.ascontiguousarray(mm[a:b, y0:y1], dtype=p0.dtype.newbyteorder("="))
        if self._needs_codec():  # decode only the strips / tile rows that hold rows [y0, y1)
            arr = imread_libtiff(self.path, pages=(a, b), ifd_offset=self.ifd_offsets[a], rows=(y0, y1))
            return np.ascontiguousarray(arr, dtype=p0.dtype.newbyteorder("="))
        return np.ascontiguousarray(self.read_planes(a, b)[:, y0:y1])

    def asarray(self):
        blk = self._contiguous_block()
        shape = self.series_shape()
        p0 = self.pages[0]
        if self._needs_codec():  # LZW / deflate / tiled inputs (tifffile decodes them too)
            return np.ascontiguousarray(imread_libtiff(self.path).reshape(shape), dtype=p0.dtype.newbyteorder("="))
        if blk is not None:
            with open(self.path, "rb") as f:
                f.seek(blk[0])
                buf = f.read(int(np.prod(shape)) * p0.dtype.itemsize)
            return np.frombuffer(buf, dtype=p0.dtype).reshape(shape).astype(p0.dtype.newbyteorder("="))
        out = []
        with open(self.path, "rb") as f:
            for p in self.pages:
                if p.compression != 1:
                    raise ValueError(f"{self.path}: compressed TIFF (compression={p.compression}) not supported")
                chunks = []
                for o, c in zip(p.offsets, p.counts):
                    f.seek(o)
                    chunks.append(f.read(c))
                out.append(np.frombuffer(b"".join(chunks), dtype=p.dtype)[: int(np.prod(p.shape))].reshape(p.shape))
        arr = np.stack(out) if len(out) > 1 else out[0]
        return arr.reshape(shape).astype(p0.dtype.newbyteorder("="))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def imread(path):
    return TiffFile(path).asarray()


def memmap(path):
    return TiffFile(path).memmap()


_BIGTIFF_THRESHOLD = 2**32 - 2**25  # tifffile switches to BigTIFF past this size


def imwrite(path, data, photometric="minisblack", description=None, imagej=False, bigtiff=None):
    """Write ``data`` as an uncompressed little-endian TIFF, one page per 2-D plane.

    Layout (as tifffile lays out one series): header, first IFD with the
    description, then the image data of all pages as ONE contiguous block (so
    the file can be memory-mapped), then the IFDs of the remaining pages."""
    if photometric not in ("minisblack", None):
        raise ValueError("only photometric='minisblack' is supported")
    arr = np.asarray(data)
    if arr.dtype.kind == "b":
        arr = arr.astype(np.uint8)
    arr = np.ascontiguousarray(arr, dtype=arr.dtype.newbyteorder("<"))
    head, data_pos, tail = _layout(arr.shape, arr.dtype, description, imagej, bigtiff)
    flat = arr.reshape(-1)
    with open(path, "wb") as f:
        f.write(head)
        f.write(memoryview(flat).cast("B"))
        f.write(tail)


def write_planes(path, shape, dtype, z0, planes, description=None, imagej=False, bigtiff=None):
    """Write planes [z0, z0 + len(planes)) of a TIFF whose full content is ``imwrite(path,
    full_array)`` for a ``shape`` / ``dtype`` array (several processes each writing their
    own z-slab of one output volume; no gather, no coordination: every writer puts the
    same header and trailing IFDs in place and sizes the file, the planes are disjoint).
    Once every plane has been written, the file is byte-identical to imwrite's."""
    dt = np.dtype(dtype).newbyteorder("<")
    head, data_pos, tail = _layout(tuple(shape), dt, description, imagej, bigtiff)
    plane_bytes = int(shape[-1]) * int(shape[-2]) * dt.itemsize
    nbytes = int(np.prod(shape)) * dt.itemsize
    arr = np.ascontiguousarray(planes, dtype=dt)
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
    try:
        os.ftruncate(fd, data_pos + nbytes + len(tail))
        os.pwrite(fd, head, 0)
        os.pwrite(fd, tail, data_pos + nbytes)
        if arr.size:
            os.pwrite(fd, memoryview(arr.reshape(-1)).cast("B"), data_pos + int(z0) * plane_bytes)
    finally:
        os.close(fd)


def write_rows(path, shape, dtype, y0, rows, description=None, imagej=False, bigtiff=None):
    """write_planes for a row slab: rows [y0, y0 + rows.shape[-2]) of every plane of a
    ``shape`` / ``dtype`` volume (several processes, disjoint rows, no coordination)."""
    dt = np.dtype(dtype).newbyteorder("<")
    head, data_pos, tail = _layout(tuple(shape), dt, description, imagej, bigtiff)
    ny, nx = int(shape[-2]), int(shape[-1])
    plane_bytes = ny * nx * dt.itemsize
    nbytes = int(np.prod(shape)) * dt.itemsize
    arr = np.ascontiguousarray(rows, dtype=dt)
    arr = arr.reshape((-1,) + arr.shape[-2:])
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
    try:
        os.ftruncate(fd, data_pos + nbytes + len(tail))
        os.pwrite(fd, head, 0)
        os.pwrite(fd, tail, data_pos + nbytes)
        if arr.size:
            for z in range(arr.shape[0]):
                os.pwrite(fd, memoryview(arr[z].reshape(-1)).cast("B"), data_pos + z * plane_bytes + int(y0) * nx *
                          dt.itemsize)
    finally:
        os.close(fd)


def _layout(shape, dtype, description=None, imagej=False, bigtiff=None):
    """(header + first IFD bytes, data offset, trailing IFD bytes) of imwrite's file for an
    array of ``shape`` / little-endian ``dtype``."""
    dtype = np.dtype(dtype)
    if len(shape) < 2:
        shape = (1,) * (2 - len(shape)) + tuple(shape)
    ny, nx = shape[-2:]
    npages = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    fmt = {"u": 1, "i": 2, "f": 3}[dtype.kind]
    bits = dtype.itemsize * 8
    if description is None:
        description = imagej_description(shape) if imagej else json.dumps({"shape": list(shape)})
    desc = description.encode("latin-1") + b"\0"
    software = b"opticalflow3d_dev_amd\0"
    plane_bytes = ny * nx * dtype.itemsize
    if bigtiff is None:
        bigtiff = npages * (plane_bytes + 320) + len(desc) + 64 > _BIGTIFF_THRESHOLD
    ofmt, osz = ("Q", 8) if bigtiff else ("I", 4)
    cfmt, csz = ("Q", 8) if bigtiff else ("H", 2)
    esz = 20 if bigtiff else 12
    otyp = 16 if bigtiff else 4

    def entry(code, typ, count, value_bytes):
        head = struct.pack("<HHQ", code, typ, count) if bigtiff else struct.pack("<HHI", code, typ, count)
        return head + value_bytes.ljust(osz, b"\0")

    def ifd_block(i, pos, data_pos):
        """IFD of page i at byte `pos` (+ its out-of-line values); next-IFD field left 0."""
        ntags = 13 if i == 0 else 12
        extra_pos = pos + csz + ntags * esz + osz
        extras = b""
        desc_pos = extra_pos
        if i == 0:
            extras += desc + (b"\0" if len(desc) & 1 else b"")
        soft_pos = extra_pos + len(extras)
        extras += software + (b"\0" if len(software) & 1 else b"")
        u32 = lambda v: struct.pack("<I", v)
        u16 = lambda v: struct.pack("<H", v)
        off = lambda v: struct.pack("<" + ofmt, v)
        tags = [entry(254, 4, 1, u32(0)), entry(256, 4, 1, u32(nx)), entry(257, 4, 1, u32(ny)),
                entry(258, 3, 1, u16(bits)), entry(259, 3, 1, u16(1)), entry(262, 3, 1, u16(1))]
        if i == 0:
            tags.append(entry(270, 2, len(desc), off(desc_pos)))
        tags += [entry(273, otyp, 1, off(data_pos)), entry(277, 3, 1, u16(1)), entry(278, 4, 1, u32(ny)),
                 entry(279, otyp, 1, off(plane_bytes)), entry(305, 2, len(software), off(soft_pos)),
                 entry(339, 3, 1, u16(fmt))]
        assert len(tags) == ntags
        body = struct.pack("<" + cfmt, ntags) + b"".join(tags)
        return body, body + struct.pack("<" + ofmt, 0) + extras

    header = b"II" + (struct.pack("<HHHQ", 43, 8, 0, 16) if bigtiff else struct.pack("<HI", 42, 8))
    ifd0_pos = len(header)
    # size of IFD0 block does not depend on data_pos; place data after it, 16-B aligned
    _, blk0 = ifd_block(0, ifd0_pos, 0)
    data_pos = ifd0_pos + len(blk0)
    data_pos += (-data_pos) % 16
    nbytes = npages * plane_bytes
    body0, blk0 = ifd_block(0, ifd0_pos, data_pos)
    head = bytearray(header + blk0)
    head += b"\0" * (data_pos - len(head))
    # IFDs of pages 1.. assembled in memory (next-IFD links patched there), one write
    tail = bytearray()
    base = data_pos + nbytes
    prev = (head, ifd0_pos + len(body0))  # (buffer, offset of the next-IFD field in it)
    for i in range(1, npages):
        if (base + len(tail)) & 1:
            tail += b"\0"
        pos = base + len(tail)
        body, blk = ifd_block(i, pos, data_pos + i * plane_bytes)
        buf, at = prev
        buf[at:at + osz] = struct.pack("<" + ofmt, pos)
        prev = (tail, len(tail) + len(body))
        tail += blk
    return bytes(head), data_pos, bytes(tail)


def imagej_description(shape, frames=None, slices=None):
    """ImageJ hyperstack description for (T, Z, Y, X) / (T, Y, X) data."""
    if frames is None:
        if len(shape) == 4:
            frames, slices = shape[0], shape[1]
        elif len(shape) == 3:
            frames, slices = shape[0], 1
        else:
            frames, slices = 1, 1
    images = frames * slices
    lines = ["ImageJ=1.11a", f"images={images}"]
    if slices > 1:
        lines.append(f"slices={slices}")
    if frames > 1:
        lines.append(f"frames={frames}")
    lines += ["hyperstack=true", "mode=grayscale", "loop=false"]
    return "\n".join(lines) + "\n"


def natsorted(items):
    """Natural sort (natsort.natsorted default: unsigned integers compared numerically)."""
    def key(s):
        parts = re.split(r"(\d+)", s)
        return [(0, int(p)) if p.isdigit() else (1, p) for p in parts]
    return sorted(items, key=key)


# ---------------------------------------------------------------------------
# MATLAB-compatible output: the reference's MATLAB twin
# writes every output with M/TIFFwrite.m:19-38 — libtiff (MATLAB's Tiff class)
# in BigTIFF mode 'w8', one page per z-plane, 64-bit IEEE samples, LZW.  The
# same library writes them here, through ctypes on the system libtiff.
# ---------------------------------------------------------------------------
_TIFFTAG = dict(IMAGEWIDTH=256, IMAGELENGTH=257, BITSPERSAMPLE=258, COMPRESSION=259, PHOTOMETRIC=262,
                SAMPLESPERPIXEL=277, ROWSPERSTRIP=278, PLANARCONFIG=284, SAMPLEFORMAT=339, TILEWIDTH=322,
                TILELENGTH=323)
_libtiff_handle = None


def _libtiff():
    global _libtiff_handle
    if _libtiff_handle is None:
        import ctypes

        for name in ("libtiff.so.6", "libtiff.so.5", "libtiff.so"):
            try:
                lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        else:
            raise ImportError("MATLAB-compatible (LZW) TIFF I/O needs the system libtiff (libtiff.so.5/6)")
        P, U32 = ctypes.c_void_p, ctypes.c_uint32
        lib.TIFFOpen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        lib.TIFFOpen.restype = P
        lib.TIFFSetField.restype = ctypes.c_int  # variadic: callers pass typed arguments
        lib.TIFFGetField.restype = ctypes.c_int
        lib.TIFFDefaultStripSize.argtypes = [P, U32]
        lib.TIFFDefaultStripSize.restype = U32
        lib.TIFFWriteEncodedStrip.argtypes = [P, U32, P, ctypes.c_int64]
        lib.TIFFWriteEncodedStrip.restype = ctypes.c_int64
        lib.TIFFReadEncodedStrip.argtypes = [P, U32, P, ctypes.c_int64]
        lib.TIFFReadEncodedStrip.restype = ctypes.c_int64
        lib.TIFFNumberOfStrips.argtypes = [P]
        lib.TIFFNumberOfStrips.restype = U32
        lib.TIFFWriteDirectory.argtypes = [P]
        lib.TIFFWriteDirectory.restype = ctypes.c_int
        lib.TIFFReadDirectory.argtypes = [P]
        lib.TIFFReadDirectory.restype = ctypes.c_int
        lib.TIFFSetDirectory.argtypes = [P, ctypes.c_uint32]
        lib.TIFFSetDirectory.restype = ctypes.c_int
        lib.TIFFSetSubDirectory.argtypes = [P, ctypes.c_uint64]
        lib.TIFFSetSubDirectory.restype = ctypes.c_int
        lib.TIFFClose.argtypes = [P]
        lib.TIFFClose.restype = None
        lib.TIFFIsTiled.argtypes = [P]
        lib.TIFFIsTiled.restype = ctypes.c_int
        lib.TIFFComputeTile.argtypes = [P, U32, U32, U32, ctypes.c_uint16]
        lib.TIFFComputeTile.restype = U32
        lib.TIFFReadEncodedTile.argtypes = [P, U32, P, ctypes.c_int64]
        lib.TIFFReadEncodedTile.restype = ctypes.c_int64
        lib.TIFFWriteEncodedTile.argtypes = [P, U32, P, ctypes.c_int64]
        lib.TIFFWriteEncodedTile.restype = ctypes.c_int64
        _libtiff_handle = lib
    return _libtiff_handle


def imwrite_matlab(path, data):
    """Write ``data`` ((Nz,) Ny, Nx) as M/TIFFwrite.m does: BigTIFF, one page per
    plane, IEEE float samples of the array's width (64-bit for vx/vy/vz/rel in
    MATLAB mode), MinIsBlack, chunky, LZW, libtiff's default strip size.
    The encoding runs in libtiff with the GIL released (ctypes), so several
    files can be written from threads at once."""
    if np.asarray(data).dtype.kind != "f":
        raise ValueError("MATLAB-mode outputs are floating point")
    imwrite_libtiff(path, data, compression=5, bigtiff=True)


def imwrite_libtiff(path, data, compression=5, bigtiff=True, description=None, tile=None, rows_per_strip=None):
    """One page per plane through the system libtiff: ``compression`` (5 LZW, 8 deflate,
    1 none), optional ImageDescription, strips of libtiff's default size (or
    ``rows_per_strip`` rows) or ``tile`` (th, tw) tiles (multiples of 16).  Integer or float
    samples."""
    import ctypes

    lib = _libtiff()
    arr = np.asarray(data)
    arr = np.ascontiguousarray(arr, dtype=arr.dtype.newbyteorder("="))
    if arr.ndim == 2:
        arr = arr[None]
    if arr.ndim != 3:
        raise ValueError("expected a 2-D image or a (z, y, x) volume")
    nz, ny, nx = arr.shape
    fmt = {"u": 1, "i": 2, "f": 3}[arr.dtype.kind]
    tif = lib.TIFFOpen(os.fsencode(str(path)), b"w8" if bigtiff else b"w")
    if not tif:
        raise OSError("libtiff could not create " + str(path))
    U32, I = ctypes.c_uint32, ctypes.c_int
    T = _TIFFTAG
    try:
        for z in range(nz):
            for tag, val in ((T["IMAGELENGTH"], U32(ny)), (T["IMAGEWIDTH"], U32(nx)), (T["SAMPLESPERPIXEL"], I(1)),
                             (T["PLANARCONFIG"], I(1)), (T["BITSPERSAMPLE"], I(8 * arr.itemsize)),
                             (T["SAMPLEFORMAT"], I(fmt)), (T["PHOTOMETRIC"], I(1)),
                             (T["COMPRESSION"], I(compression))):
                if not lib.TIFFSetField(ctypes.c_void_p(tif), U32(tag), val):
                    raise OSError("libtiff rejected tag %d" % tag)
            if description is not None and z == 0:
                lib.TIFFSetField(ctypes.c_void_p(tif), U32(270), ctypes.c_char_p(description.encode("latin-1")))
            plane = arr[z]
            if tile is None:
                rps = int(rows_per_strip or lib.TIFFDefaultStripSize(tif, 0))
                lib.TIFFSetField(ctypes.c_void_p(tif), U32(T["ROWSPERSTRIP"]), U32(rps))
                row_bytes = nx * arr.itemsize
                for s, r0 in enumerate(range(0, ny, rps)):
                    chunk = plane[r0:r0 + rps]
                    if lib.TIFFWriteEncodedStrip(tif, s, chunk.ctypes.data, chunk.shape[0] * row_bytes) < 0:
                        raise OSError("libtiff failed writing " + str(path))
            else:
                th, tw = tile
                lib.TIFFSetField(ctypes.c_void_p(tif), U32(T["TILEWIDTH"]), U32(tw))
                lib.TIFFSetField(ctypes.c_void_p(tif), U32(T["TILELENGTH"]), U32(th))
                buf = np.zeros((th, tw), arr.dtype)
                for ty in range(0, ny, th):
                    for tx in range(0, nx, tw):
                        buf[...] = 0
                        blk = plane[ty:ty + th, tx:tx + tw]
                        buf[:blk.shape[0], :blk.shape[1]] = blk
                        if lib.TIFFWriteEncodedTile(tif, lib.TIFFComputeTile(tif, tx, ty, 0, 0), buf.ctypes.data,
                                                    buf.nbytes) < 0:
                            raise OSError("libtiff failed writing " + str(path))
            if not lib.TIFFWriteDirectory(tif):
                raise OSError("libtiff failed writing " + str(path))
    finally:
        lib.TIFFClose(tif)


def imread_libtiff(path, pages=None, ifd_offset=None, rows=None):
    """Read any single-sample TIFF libtiff can decode (e.g. the LZW BigTIFFs of
    imwrite_matlab / MATLAB's TIFFwrite) as a (pages, y, x) or (y, x) array.
    pages=(p0, p1): decode only pages [p0, p1) (always a (p1 - p0, y, x) array);
    ifd_offset: the file offset of page p0's IFD (TiffFile.ifd_offsets) — libtiff then
    jumps to it instead of walking the p0 directories before it; rows=(y0, y1): only
    those rows of each page, decoding only the strips / tile rows that hold them."""
    import ctypes

    lib = _libtiff()
    tif = lib.TIFFOpen(os.fsencode(str(path)), b"r")
    if not tif:
        raise OSError("libtiff could not open " + str(path))
    if pages is not None:
        p0, p1 = pages
        ok = p1 > p0 and (lib.TIFFSetSubDirectory(tif, ifd_offset) if ifd_offset is not None
                          else lib.TIFFSetDirectory(tif, p0))
        if not ok:
            lib.TIFFClose(tif)
            raise ValueError(f"{path}: no pages [{p0}, {p1})")
    T = _TIFFTAG
    get = lambda tag, ct: (lambda v: (lib.TIFFGetField(ctypes.c_void_p(tif), ctypes.c_uint32(tag), ctypes.byref(v)),
                                      v.value)[1])(ct())
    planes = []
    try:
        while True:
            w, h = get(T["IMAGEWIDTH"], ctypes.c_uint32), get(T["IMAGELENGTH"], ctypes.c_uint32)
            bits, fmt = get(T["BITSPERSAMPLE"], ctypes.c_uint16), get(T["SAMPLEFORMAT"], ctypes.c_uint16) or 1
            dt = np.dtype({1: "u", 2: "i", 3: "f"}[fmt] + str(bits // 8))
            y0, y1 = rows if rows is not None else (0, h)
            if lib.TIFFIsTiled(tif):
                tw, th = get(T["TILEWIDTH"], ctypes.c_uint32), get(T["TILELENGTH"], ctypes.c_uint32)
                r0 = (y0 // th) * th
                out = np.empty((min(-(-y1 // th) * th, h) - r0, w), dt)
                tile = np.empty((th, tw), dt)
                for ty in range(r0, y1, th):
                    for tx in range(0, w, tw):
                        n = lib.TIFFReadEncodedTile(tif, lib.TIFFComputeTile(tif, tx, ty, 0, 0), tile.ctypes.data,
                                                    tile.nbytes)
                        if n < 0:
                            raise OSError("libtiff failed decoding " + str(path))
                        out[ty - r0:ty - r0 + th, tx:tx + tw] = tile[:min(th, h - ty), :min(tw, w - tx)]
            else:
                rps = min(get(T["ROWSPERSTRIP"], ctypes.c_uint32) or h, h)
                r0 = (y0 // rps) * rps
                out = np.empty((min(-(-y1 // rps) * rps, h) - r0, w), dt)
                buf = out.reshape(-1).view(np.uint8)
                pos = 0
                for st in range(y0 // rps, -(-y1 // rps)):
                    n = lib.TIFFReadEncodedStrip(tif, st, buf[pos:].ctypes.data, buf.size - pos)
                    if n < 0:
                        raise OSError("libtiff failed decoding " + str(path))
                    pos += n
            planes.append(out[y0 - r0:y1 - r0])
            if (pages is not None and len(planes) == pages[1] - pages[0]) or not lib.TIFFReadDirectory(tif):
                break
    finally:
        lib.TIFFClose(tif)
    if pages is not None:
        if len(planes) != pages[1] - pages[0]:
            raise ValueError(f"{path}: fewer than {pages[1]} pages")
        return np.stack(planes)
    return planes[0] if len(planes) == 1 else np.stack(planes)
