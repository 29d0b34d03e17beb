"""CZI reader (row f3) on files written to the ZISRAW layout (tests/czi_writer.py): channel
stacking, bioformats' rescale by the pixel type's maximum, mosaic stitching, plane / scene /
pyramid selection, and loud errors for what it does not decode.  CPU only; parity with
Bio-Formats itself is unpinned (absent here)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from czi_writer import write_czi, write_spectral  # noqa: E402

from hiprfish_image_analysis_amd import czi, io  # noqa: E402


def test_spectral_gray16_rescaled(tmp_path):
    rng = np.random.default_rng(1)
    st = rng.integers(0, 65536, (40, 56, 7), dtype=np.uint16)
    p = str(tmp_path / "s_405.czi")
    write_spectral(p, st)
    got = czi.load_image(p)
    assert got.dtype == np.float32 and got.shape == (40, 56, 7)
    assert np.array_equal(got, st.astype(np.float32) / np.float32(65535.0))
    assert np.array_equal(czi.load_image(p, rescale=False), st)
    # the measurement scripts' loader reads the .czi itself
    assert np.array_equal(io.load_laser_stack(p), got)


def test_mosaic_tiles_stitched(tmp_path):
    rng = np.random.default_rng(2)
    st = rng.integers(0, 65536, (24, 60, 3), dtype=np.uint16)
    p = str(tmp_path / "m.czi")
    write_spectral(p, st, tiles=3)
    assert np.array_equal(czi.load_image(p, rescale=False), st)


def test_gray8_float_and_plane_selection(tmp_path):
    rng = np.random.default_rng(3)
    a8 = rng.integers(0, 256, (10, 12), dtype=np.uint8)
    p = str(tmp_path / "g8.czi")
    other = rng.integers(0, 256, (10, 12), dtype=np.uint8)
    write_czi(p, [(other, {"Z": 1}), (a8, {"Z": 0}), (other, {"T": 2}), (other, {"S": 1}),
                  (rng.integers(0, 256, (5, 6), dtype=np.uint8), {"pyramid": 1})])
    got = czi.load_image(p)
    assert got.shape == (10, 12, 1)
    assert np.array_equal(got[:, :, 0], a8.astype(np.float32) / np.float32(255.0))
    assert np.array_equal(czi.load_image(p, rescale=False, z=1)[:, :, 0], other)
    f = rng.random((6, 9)).astype(np.float32)
    pf = str(tmp_path / "f.czi")
    write_czi(pf, [(f, {"C": 0}), (f * 2, {"C": 1})])
    got = czi.load_image(pf)
    assert np.array_equal(got[:, :, 0], f) and np.array_equal(got[:, :, 1], f * 2)


def test_unsupported_raise(tmp_path):
    p = str(tmp_path / "z.czi")
    write_czi(p, [(np.zeros((4, 4), np.uint16), {})], compression=5)
    with pytest.raises(czi.CziError, match="Zstd0"):
        czi.load_image(p)
    bad = tmp_path / "bad.czi"
    bad.write_bytes(b"NOTACZI" + b"\0" * 100)
    with pytest.raises(czi.CziError):
        czi.load_image(str(bad))
