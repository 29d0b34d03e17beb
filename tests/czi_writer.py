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


def _compress(data, compression, itemsize, hilo):
    import pyarrow as pa

    if compression in (0, 4):      # 4: marked JPEG-XR, payload left raw (the reader must refuse it)
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


def write_czi(path, blocks, compression=0, hilo=False, sizes=None):
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
        data = _compress(arr.astype(arr.dtype.newbyteorder("<")).tobytes(), compression, arr.dtype.itemsize, hilo)
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


def write_spectral(path, stack_u16, tiles=1, compression=0, hilo=False):
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
    write_czi(path, blocks, compression, hilo)
