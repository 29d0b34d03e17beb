"""End-to-end parity: the device pipeline (hiprfish_image_analysis_amd.pipeline) against the
CPU restatement (oracle/pipeline.py) of ecoli measurement.py:44-162 plus classification,
on synthetic tiles.  Label maps bit-exact, spectra within 1e-12 relative."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    import pipeline as OP  # oracle/pipeline.py

    from hiprfish_image_analysis_amd import pipeline as P
    from hiprfish_image_analysis_amd import synthetic as S
    return P, S, OP


def host(t):
    return t.cpu().numpy()


@pytest.mark.parametrize("H,W,seed", [(256, 256, 1), (512, 512, 2), (384, 640, 3)])
def test_measure_ecoli_parity(mods, H, W, seed):
    P, S, OP = mods
    stack, truth, lay, ref = S.tile(H, W, seed=seed)
    keep = {}
    m = P.measure_ecoli(stack, keep=keep)
    okeep = {}
    oseg, olabs, oavg, oavgn = OP.measure_ecoli(host(stack), keep=okeep)
    np.testing.assert_allclose(host(keep["image_cn"]), okeep["image_cn"], rtol=4e-16, atol=0)
    for k in ("rough_mask", "interior", "cell_sm"):
        assert np.array_equal(host(keep[k]).astype(bool), okeep[k]), k
    assert np.array_equal(host(keep["seeds"]), okeep["seeds"])
    assert np.array_equal(host(keep["watershed"]), okeep["watershed"])
    assert np.array_equal(host(m.segmentation), oseg)
    assert np.array_equal(host(m.labels), olabs)
    assert len(olabs) >= 1
    np.testing.assert_allclose(host(m.avgint), oavg, rtol=1e-12)
    np.testing.assert_allclose(host(m.avgint_norm), oavgn, rtol=1e-12)


def test_measure_with_calibration(mods):
    P, S, OP = mods
    stack, truth, lay, ref = S.tile(256, 256, seed=7)
    cal = (0.6 + 0.4 * np.random.default_rng(0).random((256, 256))).astype(np.float32)
    m = P.measure_ecoli(stack, calibration=torch.from_numpy(cal).cuda())
    oseg, olabs, oavg, _ = OP.measure_ecoli(host(stack), calibration=cal)
    assert np.array_equal(host(m.segmentation), oseg)
    np.testing.assert_allclose(host(m.avgint), oavg, rtol=1e-12)


def test_process_tile_classification_and_counts(mods, orc):
    P, S, OP = mods
    stack, truth, lay, ref = S.tile(512, 512, seed=5)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    res = P.process_tile(stack, lib, per_pixel=True)
    o = OP.process_tile(host(stack), ref, S.ECOLI_BOUNDS)
    assert np.array_equal(host(res.meas.segmentation), o["segmentation"])
    # per-cell argmin on spectra equal to 1e-12: identical unless a near tie
    gi, oi = host(res.cell_idx), o["cell_idx"]
    np.testing.assert_allclose(host(res.cell_dist), o["cell_dist"], rtol=1e-9, atol=1e-12)
    assert (gi == oi).mean() == 1.0
    assert np.array_equal(host(res.counts), orc.barcode_counts(gi, lib.R))
    assert np.array_equal(host(res.identification), orc.paint_ids(o["segmentation"], gi + 1))
    # per-pixel mode, spot-checked against the restatement
    P_ = 512 * 512
    sel = np.random.default_rng(0).choice(P_, 400, replace=False)
    x = host(stack).reshape(P_, -1)[sel].astype(np.float64)
    ri, rd = orc.classify(x, ref.astype(np.float64), S.ECOLI_BOUNDS, 0)
    pi, pd = host(res.pixel_idx).ravel()[sel], host(res.pixel_dist).ravel()[sel]
    np.testing.assert_allclose(pd, rd, rtol=1e-5, atol=1e-5)
    assert (pi == ri).mean() > 0.97


# ---- synthetic-community measurement (multispecies measurement.py:78-174) ------------------
@pytest.mark.parametrize("H,W,seed,cal_kind", [(256, 256, 11, "channel"), (320, 384, 12, "full"),
                                              (256, 256, 13, None)])
def test_measure_multispecies_parity(mods, orc, H, W, seed, cal_kind):
    P, S, OP = mods
    stack, truth, lay, ref = S.tile(H, W, bounds=P.MULTI_BOUNDS, seed=seed)
    C = stack.shape[2]
    rng = np.random.default_rng(seed)
    cal = None
    if cal_kind == "channel":
        cal = (0.5 + rng.random(C)).astype(np.float32)
    elif cal_kind == "full":
        cal = (0.5 + rng.random((H, W, C))).astype(np.float32)
    keep = {}
    m = P.measure_multispecies(stack, None if cal is None else torch.from_numpy(cal).cuda(), keep=keep)
    # float stages: channel sum of the calibrated stack bit-exact, NL-means within 1e-12
    okeep = {}
    st64 = OP._calibrated(host(stack), cal)
    s = np.sum(st64, axis=2)
    assert np.array_equal(host(keep["image_sum"]), s)
    np.testing.assert_allclose(host(keep["nl"]), orc.nl_means_skimage(s / s.max(), 7, 11, 0.02, 0.0),
                               rtol=0, atol=1e-12)
    # discrete stages exact once the NL-means image is shared
    oseg, olabs, oavg, oavgn = OP.measure_multispecies(host(stack), cal, keep=okeep, nl=host(keep["nl"]))
    np.testing.assert_allclose(host(keep["final"]), okeep["final"], rtol=1e-12, atol=1e-15)
    for k in ("rough_mask", "bkg_mask"):
        assert np.array_equal(host(keep[k]).astype(bool), okeep[k]), k
    assert np.array_equal(host(keep["seeds"]), okeep["seeds"])
    assert np.array_equal(host(m.segmentation), oseg)
    assert m.maxlab == len(olabs) and len(olabs) >= 1
    assert np.array_equal(host(m.labels), olabs)
    np.testing.assert_allclose(host(m.avgint), oavg, rtol=1e-12)
    np.testing.assert_allclose(host(m.avgint_norm), oavgn, rtol=1e-12)


# ---- native drivers (segment.hip) == the Python composition of the same calls --------------
@pytest.mark.parametrize("H,W,seed", [(256, 256, 21), (384, 640, 22), (1024, 1024, 23)])
def test_native_segmentation_equals_composed(mods, H, W, seed):
    P, S, OP = mods
    stack, _, _, _ = S.tile(H, W, seed=seed)
    seg_n, mx_n = P.segment_ecoli(stack)                 # one native call
    seg_c, mx_c = P.segment_ecoli(stack, keep={})        # composed from Python
    assert mx_n == mx_c and torch.equal(seg_n, seg_c)
    ms, _, _, _ = S.tile(H, W, nbit=7, bounds=P.MULTI_BOUNDS, seed=seed)
    cal = torch.rand(ms.shape[2], device="cuda") + 0.5
    a = P.segment_multispecies(ms, cal)
    b = P.segment_multispecies(ms, cal, keep={})
    assert a[1] == b[1] and torch.equal(a[0], b[0])
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])
    # repeated calls reuse the context
    seg_n2, _ = P.segment_ecoli(stack)
    assert torch.equal(seg_n2, seg_n)


# ---- degenerate tiles: empty, constant, tiny, ragged -----------------------------------------
def _degenerate_tiles(S, C):
    rng = np.random.default_rng(40)
    out = {"zeros": np.zeros((64, 80, C), np.float32),
           "constant": np.full((48, 48, C), 0.25, np.float32),
           "noise_only": (0.01 + 0.005 * rng.standard_normal((96, 64, C))).clip(0).astype(np.float32),
           "tiny": rng.random((12, 17, C)).astype(np.float32)}
    st, _, _, _ = S.tile(160, 96, seed=41, ncells=3)
    out["few_cells_ragged"] = st.cpu().numpy()[:, :, :C] if st.shape[2] >= C else None
    return out


def test_ecoli_degenerate_tiles(mods):
    P, S, OP = mods
    for name, st in _degenerate_tiles(S, 95).items():
        if st is None:
            continue
        d = torch.from_numpy(np.ascontiguousarray(st)).cuda()
        seg_n, mx_n = P.segment_ecoli(d)
        seg_c, mx_c = P.segment_ecoli(d, keep={})
        assert mx_n == mx_c and torch.equal(seg_n, seg_c), name
        oseg, _ = OP.segment_ecoli(st)
        assert np.array_equal(host(seg_n), oseg), name
        m = P.measure_ecoli(d)
        assert m.avgint.shape[1] == 95 and m.avgint.shape[0] == len(np.setdiff1d(np.unique(oseg), [0])), name


def test_multispecies_degenerate_tiles(mods, orc):
    P, S, OP = mods
    for name, st in _degenerate_tiles(S, 63).items():
        if st is None or name == "zeros":
            continue   # an all-zero stack divides 0 by 0 in the reference's sum / max (:106)
        d = torch.from_numpy(np.ascontiguousarray(st)).cuda()
        a = P.segment_multispecies(d)
        keep = {}
        b = P.segment_multispecies(d, keep=keep)
        assert a[1] == b[1] and torch.equal(a[0], b[0]), name
        oseg, on, _, _ = OP.segment_multispecies(st, nl=host(keep["nl"]))
        assert np.array_equal(host(a[0]), oseg) and a[1] == on, name
