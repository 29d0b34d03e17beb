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
and C index.  Supported: Gray8 / Gray16 / Gray32Float / Gray32 subblocks, uncompressed (what
ZEN 2.x writes for LSM 880 lambda-mode acquisitions) or zstd-compressed (ZEN 3.x: "Zstd0" = a
bare zstd frame, "Zstd1" = a small header whose chunk 1 flags the low/high byte split of 16-bit
data, then the frame; decoded with the zstd codec pyarrow carries) or JPEG-XR-compressed ("JpegXr",
compression 4: each subblock a JPEG XR file, lossless or lossy, decoded by jxrlib -- Microsoft's
reference implementation of ITU-T T.832, present in this image -- through the in-tree shim
csrc/jxr.c, libhrfjxr.so; the decoded size and grey pixel format must match the directory
entry).  A subblock must hold one plane
(C, Z, T sizes 1 -- what ZEN writes for spectral acquisitions); anything else raises rather than
returning part of it.

The biofilm script's loaders (hiprfish_imaging_biofilm_analysis.py:55-120) are here too:
`load_ztslice(path, z, t, series)`, the z-stacks `load_image_zstack_fixed_t(path, t)` ->
(H, W, Z, C) (np.stack over z on axis 2, `load_image_tile` = t 0) and the z-window
`load_image_zstack_fixed_t_memory_efficient`, the per-tile `load_ztslice_tile` /
`load_image_zstack_fixed_t_tile`, and the OME sizes `get_{x,y,c,z,t}_range` / `get_image_count`
/ `get_tile_size` from the directory.  Series convention: every mosaic tile (M index) is a
series, as in the Bio-Formats of the reference's era (the biofilm script takes
get_tile_size = sqrt(image_count) and stitches the per-tile series itself, :93-96, :1066), so
get_image_count is the tile count and get_x_range / get_y_range are series 0's (one tile's)
size; every loader reads series 0 -- one tile -- unless told otherwise, as bioformats.load_image
does without a series (python-bioformats leaves the reader on series 0), and `series=k` reads tile
k.  `stitch=True` (this reader's extension) places every tile of the scene by its X / Y start
instead; for the single-tile acquisitions the measurement scripts load the two agree.

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


def _zstd(raw, nbytes):
    try:
        import pyarrow as pa
    except ImportError as ex:  # pragma: no cover - pyarrow is in the image
        raise CziError("zstd subblock but no zstd codec importable (%s)" % ex)
    return pa.decompress(bytes(raw), decompressed_size=nbytes, codec="zstd", asbytes=True)


def _decode(buf, off, size, compression, nbytes, itemsize):
    """subblock payload -> nbytes of row-major little-endian samples"""
    if compression == 0:
        return buf, off
    if compression == 5:      # Zstd0: one zstd frame
        return _zstd(memoryview(buf)[off:off + size], nbytes), 0
    if compression == 6:      # Zstd1: header (its own size in byte 0; chunk 1 = hi/lo flag)
        hsize = buf[off]
        if hsize < 1 or hsize > size:
            raise CziError("Zstd1 header size %d" % hsize)
        hilo = False
        q = off + 1
        while q < off + hsize:
            chunk = buf[q]
            if chunk != 1 or q + 1 >= off + hsize:
                raise CziError("Zstd1 header chunk %d not understood" % chunk)
            hilo = bool(buf[q + 1] & 1)
            q += 2
        data = _zstd(memoryview(buf)[off + hsize:off + size], nbytes)
        if hilo and itemsize == 2:  # low bytes of every sample first, then the high bytes
            lo = np.frombuffer(data, np.uint8, nbytes // 2)
            hi = np.frombuffer(data, np.uint8, nbytes // 2, offset=nbytes // 2)
            data = np.stack([lo, hi], axis=1).tobytes()
        elif hilo:
            raise CziError("Zstd1 low/high byte split on %d-byte samples" % itemsize)
        return data, 0
    if compression == 4:
        raise CziError("JpegXrFile subblock reached the byte decoder")   # decoded in _subblock_pixels
    raise CziError("subblock compression %s is not supported (no decoder in this build)"
                   % COMPRESSION.get(compression, compression))


_JXR = None


def _jxr_lib():
    """libhrfjxr.so (built by _build.build_jxr next to libhrf.so)"""
    global _JXR
    if _JXR is None:
        import ctypes
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhrfjxr.so")
        if not os.path.exists(path):
            raise CziError("JpegXrFile subblock but libhrfjxr.so is not built (jxrlib's headers and "
                           "libjxrglue.so were not found at build time; _build.JXR_INC / JXR_LIB)")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:
            raise CziError("JpegXrFile subblock but libhrfjxr.so cannot load jxrlib (libjxrglue.so / libjpegxr.so, "
                           "linked from %s; set LD_LIBRARY_PATH or rebuild with HRF_JXR_LIBDIR): %s"
                           % (os.environ.get("HRF_JXR_LIBDIR", "/opt/conda/lib"), e)) from e
        lib.hrf_jxr_info.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]
        lib.hrf_jxr_decode.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
        _JXR = lib
    return _JXR


def _jpegxr(raw, ys, xs, dt):
    """one JPEG XR subblock -> (ys, xs) array of dt (the directory's pixel type)"""
    import ctypes
    lib = _jxr_lib()
    data = bytes(raw)
    w, h, b = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    r = lib.hrf_jxr_info(data, len(data), ctypes.addressof(w), ctypes.addressof(h), ctypes.addressof(b))
    if r == -100:
        raise CziError("JPEG-XR subblock with a pixel format that is not grey 8/16-bit or 32-bit float")
    if r != 0:
        raise CziError("JPEG-XR subblock: decoder error %d" % r)
    if (h.value, w.value) != (ys, xs) or b.value != np.dtype(dt).itemsize:
        raise CziError("JPEG-XR subblock of %d x %d x %d bytes, the directory says %d x %d x %d"
                       % (h.value, w.value, b.value, ys, xs, np.dtype(dt).itemsize))
    out = np.empty((ys, xs), dtype=dt)
    r = lib.hrf_jxr_decode(data, len(data), out.ctypes.data, xs * np.dtype(dt).itemsize)
    if r != 0:
        raise CziError("JPEG-XR subblock: decoder error %d" % r)
    return out


def _subblock_pixels(buf, e):
    p = _segment(buf, e.file_position, "ZISRAWSUBBLOCK")
    meta_size, _att_size, data_size = struct.unpack_from("<iiq", buf, p)
    _, esize = _parse_entry(buf, p + 16)
    head = max(256, 16 + esize)
    data_off = p + head + meta_size
    for d in ("C", "Z", "T"):
        if d in e.dims and (e.dims[d][1] != 1 or e.dims[d][2] != 1):
            raise CziError("subblock with %s size %d: multi-plane subblocks are not supported"
                           % (d, e.dims[d][1]))
    if e.pixel_type not in PIXEL_TYPES:
        raise CziError("pixel type %d is not a grey type this reader handles" % e.pixel_type)
    _, dt, _ = PIXEL_TYPES[e.pixel_type]
    ys, xs = e.dims["Y"][2], e.dims["X"][2]
    n = xs * ys
    nbytes = n * np.dtype(dt).itemsize
    if e.compression == 4:
        return _jpegxr(memoryview(buf)[data_off:data_off + data_size], ys, xs, dt)
    src, off = _decode(buf, data_off, data_size, e.compression, nbytes, np.dtype(dt).itemsize)
    if len(src) - off < nbytes or (e.compression == 0 and data_size < nbytes):
        raise CziError("subblock data %d bytes, %d x %d pixels expected" % (data_size, ys, xs))
    return np.frombuffer(src, dtype=dt, count=n, offset=off).reshape(ys, xs)


def _open(path):
    with open(path, "rb") as f:
        return mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)


def _close(buf):
    try:
        buf.close()
    except BufferError:      # a view survives an exception path; the map closes with it
        pass


def _level0(entries):
    return [e for e in entries if e.pyramid_type == 0
            and e.dims["X"][1] == e.dims["X"][2] and e.dims["Y"][1] == e.dims["Y"][2]]


def _plane(buf, entries, path, z, t, series, stitch=False):
    sel = [e for e in _level0(entries) if e.start("Z") == z and e.start("T") == t]
    if not sel:
        raise CziError("%s: no level-0 subblocks at z=%d, t=%d" % (path, z, t))
    scene = min(e.start("S") for e in sel)
    sel = [e for e in sel if e.start("S") == scene]
    if not stitch:
        series = 0 if series is None else series
        tiles = sorted({e.start("M") for e in sel})
        if not 0 <= series < len(tiles):
            raise CziError("%s: series %d of %d mosaic tiles" % (path, series, len(tiles)))
        sel = [e for e in sel if e.start("M") == tiles[series]]
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
    return out, scale


def _rescaled(out, scale, rescale):
    if rescale:
        return (out.astype(np.float32) / np.float32(scale)) if scale != 1.0 else out.astype(np.float32)
    return out


def load_image(path, rescale=True, z=0, t=0, series=None, stitch=False):
    """bioformats.load_image(path, z=, t=, series=) for a CZI spectral acquisition: (H, W, C)
    float32 (rescaled by the pixel type's maximum) or the raw sample type with rescale=False.
    series None = series 0 (one mosaic tile), as Bio-Formats; stitch=True: the whole scene"""
    buf = _open(path)
    try:
        out, scale = _plane(buf, read_directory(buf), path, z, t, series, stitch)
    finally:
        _close(buf)
    return _rescaled(out, scale, rescale)


def dims(path):
    """{'X','Y','C','Z','T','M'} sizes of the first scene's level-0 plane set (the OME Pixels
    sizes the biofilm script queries; M = mosaic tiles = Bio-Formats' series count per scene)"""
    buf = _open(path)
    try:
        ent = _level0(read_directory(buf))
    finally:
        _close(buf)
    if not ent:
        raise CziError("%s: no level-0 subblocks" % path)
    scene = min(e.start("S") for e in ent)
    ent = [e for e in ent if e.start("S") == scene]
    out = {}
    for d in ("C", "Z", "T", "M"):
        vals = {e.start(d) for e in ent}
        out[d] = max(vals) - min(vals) + 1
    out["X"] = max(e.start("X") + e.dims["X"][1] for e in ent) - min(e.start("X") for e in ent)
    out["Y"] = max(e.start("Y") + e.dims["Y"][1] for e in ent) - min(e.start("Y") for e in ent)
    return out


def _series0_size(path):
    """(X, Y) of series 0: the first mosaic tile when the scene has several (Bio-Formats of the
    reference's era gives every tile its own series, so ome.image(0).Pixels is one tile), else
    the scene"""
    buf = _open(path)
    try:
        ent = _level0(read_directory(buf))
    finally:
        _close(buf)
    if not ent:
        raise CziError("%s: no level-0 subblocks" % path)
    scene = min(e.start("S") for e in ent)
    ent = [e for e in ent if e.start("S") == scene]
    m0 = min(e.start("M") for e in ent)
    ent = [e for e in ent if e.start("M") == m0]
    x = max(e.start("X") + e.dims["X"][1] for e in ent) - min(e.start("X") for e in ent)
    y = max(e.start("Y") + e.dims["Y"][1] for e in ent) - min(e.start("Y") for e in ent)
    return x, y


def get_x_range(path):
    """ome.image(0).Pixels.SizeX (biofilm :63-67): one tile's width when tiles are series"""
    return _series0_size(path)[0]


def get_y_range(path):
    """ome.image(0).Pixels.SizeY (biofilm :69-73)"""
    return _series0_size(path)[1]


def get_c_range(path):
    return dims(path)["C"]


def get_z_range(path):
    return dims(path)["Z"]


def get_t_range(path):
    return dims(path)["T"]


def get_image_count(path):
    """ome.image_count (biofilm :98-101): the series count = mosaic tiles of the first scene
    (load_image(path, series=k) reads tile k unstitched)"""
    return dims(path)["M"]


def get_tile_size(path):
    """int(sqrt(ome.image_count)) (biofilm :93-96): tiles per side of a square mosaic"""
    return int(np.sqrt(get_image_count(path)))


def load_ztslice_tile(path, z_index, t_index, tile, rescale=True):
    """bioformats.load_image(path, z=, t=, series=tile) (biofilm :59-61)"""
    return load_image(path, rescale=rescale, z=z_index, t=t_index, series=tile)


def load_image_zstack_fixed_t_tile(path, t, tile, rescale=True):
    """(H, W, Z, C) of one tile (biofilm :116-119)"""
    return load_image_zstack_fixed_t_memory_efficient(path, t, 0, get_z_range(path), tile, rescale)


def load_ztslice(path, z_index, t_index, series=0, rescale=True, stitch=False):
    """bioformats.load_image(path, z=, t=) (biofilm :55-57): series 0 -- one tile, the size
    get_x_range / get_y_range report"""
    return load_image(path, rescale=rescale, z=z_index, t=t_index, series=series, stitch=stitch)


def load_image_zstack_fixed_t_memory_efficient(path, t, z_min, z_max, series=0, rescale=True, stitch=False):
    """(H, W, z_max - z_min, C): planes z_min..z_max-1 of series 0 (or `series`, or the stitched
    scene) stacked on axis 2, the file mapped once (biofilm :103-114)"""
    buf = _open(path)
    try:
        ent = read_directory(buf)
        planes = []
        scale = 1.0
        for z in range(z_min, z_max):
            a, scale = _plane(buf, ent, path, z, t, series, stitch)
            planes.append(a)
    finally:
        _close(buf)
    if not planes:
        raise CziError("%s: empty z range [%d, %d)" % (path, z_min, z_max))
    return _rescaled(np.stack(planes, axis=2), scale, rescale)


def load_image_zstack_fixed_t(path, t, series=0, rescale=True, stitch=False):
    """biofilm :75-91: every z plane of series 0 at time t -> (H, W, Z, C)"""
    return load_image_zstack_fixed_t_memory_efficient(path, t, 0, get_z_range(path), series, rescale, stitch)


def load_image_tile(path, rescale=True, stitch=False):
    """biofilm :120-122: the z-stack at t 0 of series 0"""
    return load_image_zstack_fixed_t(path, 0, rescale=rescale, stitch=stitch)
