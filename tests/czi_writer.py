"""Minimal ZISRAW (CZI) writer -- test infrastructure: writes files laid out per the published
ZISRAW specification (file header, subblocks with a 256-byte padded header and metadata,
directory, metadata segment) so the reader in hiprfish_image_analysis_amd/czi.py is exercised
on the structures it parses.  Not part of the product."""
import struct

import numpy as np

SEG = struct.Struct("<16sqq")


def _seg(sid, data):
    pad = (-len(data)) % 32
    return SEG.pack(sid.encode().ljust(16, b"\0"), len(data) + pad, len(data)) + data + b"\0" * pad


def _entry(pixel_type, pos, compression, dims, pyramid=0):
    out = b"DV" + struct.pack("<iqiiB", pixel_type, pos, 0, compression, pyramid) + b"\0" * 5
    out += struct.pack("<i", len(dims))
    for name, start, size, stored in dims:
        out += struct.pack("<4siifi", name.encode().ljust(4, b"\0"), start, size, float(start), stored)
    return out


JXR_ENC = "/opt/conda/bin/JxrEncApp"     # jxrlib's encoder (the image's conda tree)
JXR_DEC = "/opt/conda/bin/JxrDecApp"


def write_tiff(path, a):
    """a minimal baseline TIFF (one strip, uncompressed, BlackIsZero) of a grey uint8 / uint16
    image: JxrEncApp's input format"""
    H, W = a.shape
    data = np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<")).tobytes()
    tags = [(256, 4, W), (257, 4, H), (258, 3, a.dtype.itemsize * 8), (259, 3, 1), (262, 3, 1), (273, 4, 0),
            (277, 3, 1), (278, 4, H), (279, 4, len(data)), (284, 3, 1)]
    data_off = 8 + 2 + 12 * len(tags) + 4
    out = bytearray(b"II*\x00" + struct.pack("<IH", 8, len(tags)))
    for tag, typ, val in tags:
        val = data_off if tag == 273 else val
        out += struct.pack("<HHIHH", tag, typ, 1, val, 0) if typ == 3 else struct.pack("<HHII", tag, typ, 1, val)
    out += struct.pack("<I", 0) + data
    with open(path, "wb") as f:
        f.write(bytes(out))


def read_tiff(path, dtype):
    """the strip of a one-strip grey TIFF written by JxrDecApp (tag 273 / 279)"""
    b = open(path, "rb").read()
    assert b[:4] == b"II*\x00"
    off = struct.unpack_from("<I", b, 4)[0]
    n = struct.unpack_from("<H", b, off)[0]
    vals = {}
    for i in range(n):
        tag, typ, cnt, v = struct.unpack_from("<HHII", b, off + 2 + 12 * i)
        vals[tag] = v & 0xFFFF if typ == 3 else v
    W, H = vals[256], vals[257]
    return np.frombuffer(b, dtype=np.dtype(dtype).newbyteorder("<"), count=W * H, offset=vals[273]).reshape(H, W)


def jxr_encode(a, quality="1"):
    """JPEG XR file of a grey uint8 / uint16 plane by jxrlib's JxrEncApp (-q 1: lossless)"""
    import os
    import subprocess
    import tempfile
    fmt = {np.dtype(np.uint8): "2", np.dtype(np.uint16): "3"}[a.dtype]
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.tif"), os.path.join(d, "out.jxr")
        write_tiff(src, a)
        subprocess.run([JXR_ENC, "-i", src, "-o", dst, "-c", fmt, "-q", str(quality)], check=True,
                       capture_output=True)
        return open(dst, "rb").read()


def jxr_decode_app(codestream, dtype):
    """the same codestream decoded by jxrlib's own JxrDecApp (to a TIFF)"""
    import os
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.jxr"), os.path.join(d, "out.tif")
        open(src, "wb").write(codestream)
        subprocess.run([JXR_DEC, "-i", src, "-o", dst], check=True, capture_output=True)
        return read_tiff(dst, dtype).copy()


def _compress(data, compression, itemsize, hilo, plane=None, jxr_quality=None):
    import pyarrow as pa

    if compression == 4 and jxr_quality is not None:     # JPEG XR file per subblock (jxrlib)
        return jxr_encode(plane, jxr_quality)
    if compression in (0, 4):      # 4 without a quality: marked JPEG-XR, payload left raw (corrupt)
        return data
    if compression == 6 and hilo and itemsize == 2:   # Zstd1 low/high byte split
        a = np.frombuffer(data, np.uint8).reshape(-1, 2)
        data = a[:, 0].tobytes() + a[:, 1].tobytes()
    z = pa.compress(data, codec="zstd", asbytes=True)
    if compression == 5:
        return z
    if compression == 6:
        return (bytes([3, 1, 1]) if hilo else bytes([1])) + z
    raise ValueError(compression)


def write_czi(path, blocks, compression=0, hilo=False, sizes=None, jxr_quality=None):
    """blocks: list of (array (ys, xs) of uint8/uint16/float32, {dim: start}); dims X, Y
    from the array shape, C/Z/T/S/M from the dict (default 0); compression 5/6 = Zstd0/Zstd1
    (pyarrow's zstd); sizes: {dim: size} written for C/Z/T instead of 1 (malformed files)"""
    ptype = {np.dtype(np.uint8): 0, np.dtype(np.uint16): 1, np.dtype(np.float32): 2}
    header_len = 32 + 512
    body = b""
    entries = []
    pos = header_len
    for arr, where in blocks:
        arr = np.ascontiguousarray(arr)
        ys, xs = arr.shape
        dims = [("X", where.get("X", 0), xs, xs), ("Y", where.get("Y", 0), ys, ys)]
        for d in ("C", "Z", "T", "S", "M"):
            sz = (sizes or {}).get(d, 1)
            dims.append((d, where.get(d, 0), sz, sz))
        pt = ptype[arr.dtype]
        e = _entry(pt, pos, compression, dims, where.get("pyramid", 0))
        meta = b"<METADATA><Tags><AcquisitionTime>2018-08-18</AcquisitionTime></Tags></METADATA>"
        data = _compress(arr.astype(arr.dtype.newbyteorder("<")).tobytes(), compression, arr.dtype.itemsize, hilo,
                         arr, jxr_quality)
        head = struct.pack("<iiq", len(meta), 0, len(data)) + e
        head += b"\0" * (max(256, len(head)) - len(head))
        seg = _seg("ZISRAWSUBBLOCK", head + meta + data)
        entries.append(e)
        body += seg
        pos += len(seg)
    dir_pos = pos
    directory = _seg("ZISRAWDIRECTORY", struct.pack("<i", len(entries)) + b"\0" * 124 + b"".join(entries))
    meta_pos = dir_pos + len(directory)
    xml = b"<ImageDocument><Metadata/></ImageDocument>"
    metadata = _seg("ZISRAWMETADATA", struct.pack("<ii", len(xml), 0) + b"\0" * 248 + xml)
    fh = struct.pack("<iiii", 1, 0, 0, 0) + b"\x11" * 16 + b"\x11" * 16 + struct.pack("<iqqiq", 0, dir_pos, meta_pos, 0, 0)
    fh += b"\0" * (512 - len(fh))
    with open(path, "wb") as f:
        f.write(SEG.pack(b"ZISRAWFILE".ljust(16, b"\0"), 512, 512) + fh + body + directory + metadata)


def write_spectral(path, stack_u16, tiles=1, compression=0, hilo=False, jxr_quality=None):
    """(H, W, C) or (H, W, Z, C) uint16 -> one subblock per channel (and z plane; per mosaic
    tile along x when tiles > 1)"""
    if stack_u16.ndim == 3:
        stack_u16 = stack_u16[:, :, None, :]
    H, W, Z, C = stack_u16.shape
    blocks = []
    xs = np.linspace(0, W, tiles + 1).astype(int)
    for z in range(Z):
        for t in range(tiles):
            for c in range(C):
                blocks.append((stack_u16[:, xs[t]:xs[t + 1], z, c],
                               {"X": 100 + xs[t], "Y": 50, "C": c, "M": t, "Z": z}))
    write_czi(path, blocks, compression, hilo, jxr_quality=jxr_quality)
