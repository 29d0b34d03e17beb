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
    """a 3-tile mosaic: Bio-Formats' default is series 0 (one tile); stitch=True places all"""
    rng = np.random.default_rng(2)
    st = rng.integers(0, 65536, (24, 60, 3), dtype=np.uint16)
    p = str(tmp_path / "m.czi")
    write_spectral(p, st, tiles=3)
    assert np.array_equal(czi.load_image(p, rescale=False, stitch=True), st)
    assert np.array_equal(czi.load_image(p, rescale=False), st[:, :20])
    # the loaders' arrays have the sizes the OME queries report (biofilm :55-73)
    assert czi.load_ztslice(p, 0, 0).shape[:2] == (czi.get_y_range(p), czi.get_x_range(p)) == (24, 20)


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


@pytest.mark.parametrize("compression,hilo", [(5, False), (6, False), (6, True)])
def test_zstd_subblocks(tmp_path, compression, hilo):
    """ZEN 3.x zstd subblocks: Zstd0 (bare frame) and Zstd1 (header; optional low/high byte
    split of 16-bit samples)"""
    rng = np.random.default_rng(4)
    st = rng.integers(0, 4096, (33, 47, 5), dtype=np.uint16)
    p = str(tmp_path / "zs.czi")
    write_spectral(p, st, tiles=2, compression=compression, hilo=hilo)
    assert np.array_equal(czi.load_image(p, rescale=False, stitch=True), st)
    f = rng.random((6, 9)).astype(np.float32)
    pf = str(tmp_path / "zf.czi")
    write_czi(pf, [(f, {"C": 0})], compression=compression)
    assert np.array_equal(czi.load_image(pf)[:, :, 0], f)


def test_zstack_loaders_and_sizes(tmp_path):
    """biofilm loaders (hiprfish_imaging_biofilm_analysis.py:55-120): (H, W, Z, C) z-stacks,
    z windows, per-tile series and the OME sizes"""
    rng = np.random.default_rng(5)
    vol = rng.integers(0, 65536, (20, 30, 4, 6), dtype=np.uint16)
    p = str(tmp_path / "v.czi")
    write_spectral(p, vol, tiles=2)
    d = czi.dims(p)
    assert (d["X"], d["Y"], d["Z"], d["C"], d["T"], d["M"]) == (30, 20, 4, 6, 1, 2)
    assert czi.get_z_range(p) == 4 and czi.get_c_range(p) == 6 and czi.get_image_count(p) == 2
    # series 0 (ome.image(0)) is one tile: 15 of the 30 columns; get_tile_size = sqrt(count)
    assert (czi.get_x_range(p), czi.get_y_range(p)) == (15, 20) and czi.get_tile_size(p) == 1
    assert np.array_equal(czi.load_image_zstack_fixed_t_tile(p, 0, 1, rescale=False), vol[:, 15:])
    assert np.array_equal(czi.load_ztslice_tile(p, 3, 0, 0, rescale=False), vol[:, :15, 3])
    # the reference-named loaders read series 0, the size get_x_range / get_y_range report
    got = czi.load_image_zstack_fixed_t(p, 0)
    assert got.dtype == np.float32 and got.shape == (20, 15, 4, 6)
    assert got.shape[:2] == (czi.get_y_range(p), czi.get_x_range(p))
    assert np.array_equal(got, vol[:, :15].astype(np.float32) / np.float32(65535.0))
    assert np.array_equal(czi.load_image_tile(p, rescale=False), vol[:, :15])
    assert np.array_equal(czi.load_image_zstack_fixed_t_memory_efficient(p, 0, 1, 3, rescale=False),
                          vol[:, :15, 1:3])
    assert np.array_equal(czi.load_ztslice(p, 2, 0, rescale=False), vol[:, :15, 2])
    assert czi.load_ztslice(p, 2, 0).shape[:2] == (czi.get_y_range(p), czi.get_x_range(p))
    # stitching is explicit
    assert np.array_equal(czi.load_image_tile(p, rescale=False, stitch=True), vol)
    assert np.array_equal(czi.load_ztslice(p, 2, 0, rescale=False, stitch=True), vol[:, :, 2])
    # series = one mosaic tile, unstitched
    assert np.array_equal(czi.load_image(p, rescale=False, z=1, series=1), vol[:, 15:, 1])
    with pytest.raises(czi.CziError, match="series"):
        czi.load_image(p, series=2)


JXR = os.path.exists("/opt/conda/bin/JxrEncApp")


@pytest.mark.skipif(not JXR, reason="jxrlib's encoder is not in this image")
@pytest.mark.parametrize("dtype,tiles", [(np.uint16, 1), (np.uint16, 2), (np.uint8, 1)])
def test_jpegxr_subblocks_lossless(tmp_path, dtype, tiles):
    """JPEG-XR subblocks (ZEN's 'JpegXrFile', compression 4), each a JPEG XR file written by
    jxrlib's own encoder (JxrEncApp, lossless): load_image equals the uncompressed read of the
    same planes, rescale included (ecoli measurement.py:145 bioformats.load_image)"""
    rng = np.random.default_rng(6)
    hi = 4096 if dtype == np.uint16 else 256
    st = rng.integers(0, hi, (29, 46, 4), dtype=dtype)
    pu, pj = str(tmp_path / "u.czi"), str(tmp_path / "j.czi")
    write_spectral(pu, st, tiles=tiles)
    write_spectral(pj, st, tiles=tiles, compression=4, jxr_quality=1)
    got = czi.load_image(pj, stitch=True)
    assert np.array_equal(got, czi.load_image(pu, stitch=True))
    assert np.array_equal(czi.load_image(pj, rescale=False, stitch=True), st)


@pytest.mark.skipif(not JXR, reason="jxrlib's encoder is not in this image")
def test_jpegxr_lossy_equals_reference_decoder(tmp_path):
    """lossy JPEG-XR subblocks: every plane equals jxrlib's own decoder application (JxrDecApp)
    on the same codestream, and is close to the source"""
    from czi_writer import jxr_decode_app, jxr_encode
    rng = np.random.default_rng(7)
    yy, xx = np.mgrid[0:40, 0:52]
    st = np.stack([(2000 + 1500 * np.sin(yy / 5.0 + c) * np.cos(xx / 7.0) + rng.integers(0, 50, yy.shape))
                   for c in range(3)], -1).astype(np.uint16)
    p = str(tmp_path / "lossy.czi")
    write_spectral(p, st, compression=4, jxr_quality=0.8)
    got = czi.load_image(p, rescale=False)
    for c in range(3):
        ref = jxr_decode_app(jxr_encode(st[:, :, c], 0.8), np.uint16)
        assert np.array_equal(got[:, :, c], ref)
    assert 0 < np.abs(got.astype(np.int64) - st).max() < 400


def test_unsupported_raise(tmp_path):
    p = str(tmp_path / "z.czi")
    write_czi(p, [(np.zeros((4, 4), np.uint16), {})], compression=4)
    with pytest.raises(czi.CziError, match="JPEG-XR|JpegXr"):
        czi.load_image(p)            # a corrupt (raw) JPEG-XR payload
    # a multi-channel subblock would be read as its first plane only: refused
    pm = str(tmp_path / "mc.czi")
    write_czi(pm, [(np.zeros((4, 4), np.uint16), {})], sizes={"C": 3})
    with pytest.raises(czi.CziError, match="C size 3"):
        czi.load_image(pm)
    bad = tmp_path / "bad.czi"
    bad.write_bytes(b"NOTACZI" + b"\0" * 100)
    with pytest.raises(czi.CziError):
        czi.load_image(str(bad))


@pytest.mark.gpu
@pytest.mark.skipif(not JXR, reason="jxrlib's encoder is not in this image")
def test_jpegxr_on_the_gpu_box(tmp_path):
    """the lossless JPEG-XR case where the measurement scripts run: the shim loads jxrlib on the
    GPU box, and the decoded acquisition goes through the device channel sum as the
    uncompressed one does (ecoli measurement.py:145, :71)"""
    torch = pytest.importorskip("torch")
    from hiprfish_image_analysis_amd import kernels as K
    rng = np.random.default_rng(8)
    st = rng.integers(0, 4096, (64, 96, 6), dtype=np.uint16)
    pu, pj = str(tmp_path / "u_405.czi"), str(tmp_path / "j_405.czi")
    write_spectral(pu, st)
    write_spectral(pj, st, compression=4, jxr_quality=1)
    a, b = io.load_laser_stack(pj), io.load_laser_stack(pu)
    assert np.array_equal(a, b)
    sa = K.channel_sum(torch.from_numpy(a).cuda())
    sb = K.channel_sum(torch.from_numpy(b).cuda())
    assert torch.equal(sa, sb)
