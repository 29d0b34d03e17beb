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


def write_czi(path, blocks, compression=0):
    """blocks: list of (array (ys, xs) of uint8/uint16/float32, {dim: start}); dims X, Y
    from the array shape, C/Z/T/S/M from the dict (default 0)"""
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
            dims.append((d, where.get(d, 0), 1, 1))
        pt = ptype[arr.dtype]
        e = _entry(pt, pos, compression, dims, where.get("pyramid", 0))
        meta = b"<METADATA><Tags><AcquisitionTime>2018-08-18</AcquisitionTime></Tags></METADATA>"
        data = arr.astype(arr.dtype.newbyteorder("<")).tobytes()
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


def write_spectral(path, stack_u16, tiles=1):
    """(H, W, C) uint16 -> one subblock per channel (per mosaic tile along x when tiles > 1)"""
    H, W, C = stack_u16.shape
    blocks = []
    xs = np.linspace(0, W, tiles + 1).astype(int)
    for t in range(tiles):
        for c in range(C):
            blocks.append((stack_u16[:, xs[t]:xs[t + 1], c], {"X": 100 + xs[t], "Y": 50, "C": c, "M": t}))
    write_czi(path, blocks)
