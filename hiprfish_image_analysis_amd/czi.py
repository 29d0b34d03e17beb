"""Zeiss CZI (ZISRAW) reader for the acquisitions the measurement scripts load (row f3).

The reference reads every laser's spectral image with bioformats.load_image(filename)
(ecoli hiprfish_imaging_spectral_image_measurement.py:145, multispecies :184, reference :171):
a JVM (javabridge) running Bio-Formats' ZeissCZIReader, returning plane z=0, t=0 of series 0
with all C channels stacked as (H, W, C) and -- rescale=True -- integer samples divided by the
pixel type's maximum (uint8 255, uint16 65535) as float32.  This module reads the same plane
straight from the file with numpy, no JVM:

  file header segment "ZISRAWFILE"        -> position of the subblock directory
  directory segment   "ZISRAWDIRECTORY"   -> one DirectoryEntryDV per subblock: pixel type,
                                             compression, pyramid type and the dimension
                                             entries (X, Y, C, Z, T, S, M, ... start / size /
                                             stored size)
  subblock segments   "ZISRAWSUBBLOCK"    -> header padded to 256 bytes, metadata XML, pixel
                                             data (row-major, little endian), attachments

Subblocks of the first scene at z = 0, t = 0, pyramid level 0 (stored size == size) are placed
by their X / Y start (mosaic tiles stitched, later tiles over earlier ones in directory order)
and C index.  Supported: uncompressed Gray8 / Gray16 / Gray32Float / Gray32 subblocks -- what
ZEN 2.x writes for LSM 880 lambda-mode acquisitions.  JPEG-XR and zstd compressed subblocks
(later ZEN versions) raise with the compression named: no decoder for them is in this image.
Bio-Formats itself is absent here, so parity with load_image is unpinned; the layout follows
the published ZISRAW specification and is exercised on files written to it (tests/test_czi.py).
"""
from __future__ import annotations

import mmap
import struct

import numpy as np

PIXEL_TYPES = {0: ("Gray8", np.uint8, 255.0), 1: ("Gray16", np.dtype("<u2"), 65535.0),
               2: ("Gray32Float", np.dtype("<f4"), 1.0), 12: ("Gray32", np.dtype("<u4"), 4294967295.0)}
COMPRESSION = {0: "uncompressed", 1: "JpgFile", 2: "LZW", 4: "JpegXrFile", 5: "Zstd0", 6: "Zstd1"}
SEG_HEADER = struct.Struct("<16sqq")


class CziError(ValueError):
    pass


class DirectoryEntry:
    __slots__ = ("pixel_type", "file_position", "compression", "pyramid_type", "dims")

    def __init__(self, pixel_type, file_position, compression, pyramid_type, dims):
        self.pixel_type = pixel_type
        self.file_position = file_position
        self.compression = compression
        self.pyramid_type = pyramid_type
        self.dims = dims            # {name: (start, size, stored_size)}

    def start(self, d, default=0):
        return self.dims[d][0] if d in self.dims else default


def _parse_entry(buf, off):
    """DirectoryEntryDV at buf[off:] -> (entry, bytes used)"""
    if bytes(buf[off:off + 2]) != b"DV":
        raise CziError("directory entry schema %r is not DV" % bytes(buf[off:off + 2]))
    pixel_type, file_pos, _part, compression, pyramid = struct.unpack_from("<iqiiB", buf, off + 2)
    ndim, = struct.unpack_from("<i", buf, off + 28)
    dims = {}
    p = off + 32
    for _ in range(ndim):
        name, start, size, _coord, stored = struct.unpack_from("<4siifi", buf, p)
        dims[name.rstrip(b"\0").decode("ascii")] = (start, size, stored)
        p += 20
    return DirectoryEntry(pixel_type, file_pos, compression, pyramid, dims), p - off


def _segment(buf, pos, want):
    sid, alloc, used = SEG_HEADER.unpack_from(buf, pos)
    sid = sid.rstrip(b"\0").decode("ascii", "replace")
    if sid != want:
        raise CziError("expected segment %s at %d, found %r" % (want, pos, sid))
    return pos + SEG_HEADER.size


def read_directory(buf):
    """-> [DirectoryEntry] from the file header's directory position"""
    p = _segment(buf, 0, "ZISRAWFILE")
    major, = struct.unpack_from("<i", buf, p)
    if major != 1:
        raise CziError("ZISRAW major version %d" % major)
    dir_pos, = struct.unpack_from("<q", buf, p + 16 + 32 + 4)
    q = _segment(buf, dir_pos, "ZISRAWDIRECTORY")
    count, = struct.unpack_from("<i", buf, q)
    q += 128
    entries = []
    for _ in range(count):
        e, n = _parse_entry(buf, q)
        entries.append(e)
        q += n
    return entries


def _subblock_pixels(buf, e):
    p = _segment(buf, e.file_position, "ZISRAWSUBBLOCK")
    meta_size, _att_size, data_size = struct.unpack_from("<iiq", buf, p)
    _, esize = _parse_entry(buf, p + 16)
    head = max(256, 16 + esize)
    data_off = p + head + meta_size
    if e.compression != 0:
        raise CziError("subblock compression %s is not supported (no decoder in this build)"
                       % COMPRESSION.get(e.compression, e.compression))
    if e.pixel_type not in PIXEL_TYPES:
        raise CziError("pixel type %d is not a grey type this reader handles" % e.pixel_type)
    _, dt, _ = PIXEL_TYPES[e.pixel_type]
    ys, xs = e.dims["Y"][2], e.dims["X"][2]
    n = xs * ys
    if data_size < n * np.dtype(dt).itemsize:
        raise CziError("subblock data %d bytes, %d x %d pixels expected" % (data_size, ys, xs))
    return np.frombuffer(buf, dtype=dt, count=n, offset=data_off).reshape(ys, xs)


def load_image(path, rescale=True, z=0, t=0):
    """bioformats.load_image(path) for a CZI spectral acquisition: (H, W, C) float32 (rescaled
    by the pixel type's maximum) or the raw sample type with rescale=False"""
    with open(path, "rb") as f:
        buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        entries = read_directory(buf)
        sel = [e for e in entries if e.pyramid_type == 0 and e.start("Z") == z and e.start("T") == t
               and e.dims["X"][1] == e.dims["X"][2] and e.dims["Y"][1] == e.dims["Y"][2]]
        if not sel:
            raise CziError("%s: no level-0 subblocks at z=%d, t=%d" % (path, z, t))
        scene = min(e.start("S") for e in sel)
        sel = [e for e in sel if e.start("S") == scene]
        types = {e.pixel_type for e in sel}
        if len(types) != 1:
            raise CziError("%s: mixed pixel types %s" % (path, sorted(types)))
        ptype = types.pop()
        if ptype not in PIXEL_TYPES:
            raise CziError("pixel type %d is not a grey type this reader handles" % ptype)
        _, dt, scale = PIXEL_TYPES[ptype]
        x0 = min(e.start("X") for e in sel)
        y0 = min(e.start("Y") for e in sel)
        W = max(e.start("X") + e.dims["X"][1] for e in sel) - x0
        H = max(e.start("Y") + e.dims["Y"][1] for e in sel) - y0
        c0 = min(e.start("C") for e in sel)
        C = max(e.start("C") + (e.dims["C"][1] if "C" in e.dims else 1) for e in sel) - c0
        out = np.zeros((H, W, C), dtype=dt)
        for e in sel:
            px = _subblock_pixels(buf, e)
            ys, xs = e.start("Y") - y0, e.start("X") - x0
            out[ys:ys + px.shape[0], xs:xs + px.shape[1], e.start("C") - c0] = px
            del px
    finally:
        try:
            buf.close()
        except BufferError:      # a view survives an exception path; the map closes with it
            pass
    if rescale:
        return (out.astype(np.float32) / np.float32(scale)) if scale != 1.0 else out.astype(np.float32)
    return out
