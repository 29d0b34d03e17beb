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
    # per-pixel mode: the restatement's argmin and distance on every sampled pixel
    from test_kernels_gpu import check_pixel_argmin
    P_ = 512 * 512
    cells = np.nonzero(host(res.meas.segmentation).ravel() > 0)[0]
    rng = np.random.default_rng(0)
    sel = np.concatenate([rng.choice(cells, 3000, replace=False), rng.choice(P_, 1000, replace=False)])
    x = host(stack).reshape(P_, -1)[sel].astype(np.float64)
    pi, pd = host(res.pixel_idx).ravel()[sel], host(res.pixel_dist).ravel()[sel]
    check_pixel_argmin(orc, pi, pd, x, ref.astype(np.float64), S.ECOLI_BOUNDS, 3000)


def test_concurrent_tiles_equal_isolated(mods):
    """bench.py's configuration: two tiles processed concurrently, each on its own stream
    driven by its own host thread, each tile's classifier on a side stream overlapping its
    segmentation chain.  Every output must equal the same tile processed alone (the LDS-DMA
    race fixed in 2da341b corrupted ~1 % of pixels only under this concurrency)."""
    P, S, OP = mods
    from concurrent.futures import ThreadPoolExecutor
    ref = S.reference_library(10, S.ECOLI_BOUNDS)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    lib.refx()
    tiles = [S.tile(1024, 1024, seed=60 + t)[0] for t in range(4)]

    def outputs(r):   # per-cell sums use f64 atomics (order-dependent last bits): compared apart
        return [r.pixel_idx, r.pixel_dist, r.cell_idx, r.counts, r.meas.segmentation, r.identification,
                r.meas.avgint]

    alone = []
    for st in tiles:
        alone.append([t.clone() for t in outputs(P.process_tile(st, lib))])
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(2)]

    def worker(j):
        res = []
        with torch.cuda.stream(streams[j]):
            for i in range(j, len(tiles), 2):
                res.append((i, [t.clone() for t in outputs(P.process_tile(tiles[i], lib))]))
        streams[j].synchronize()
        return res
    for rep in range(3):
        with ThreadPoolExecutor(2) as ex:
            got = [r for f in [ex.submit(worker, j) for j in range(2)] for r in f.result()]
        torch.cuda.synchronize()
        for i, outs in got:
            for a, b in zip(outs[:-1], alone[i][:-1]):
                assert torch.equal(a, b), (rep, i)
            torch.testing.assert_close(outs[-1], alone[i][-1], rtol=1e-12, atol=0)


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
    # float stages bit-exact: calibrated channel sum, NL-means (the oracle runs the kernel's
    # arithmetic; within 1e-12 of skimage's integral-image algorithm), enhancement
    okeep = {}
    st64 = OP._calibrated(host(stack), cal)
    s = np.sum(st64, axis=2)
    assert np.array_equal(host(keep["image_sum"]), s)
    np.testing.assert_allclose(host(keep["nl"]), orc.nl_means_skimage(s / s.max(), 7, 11, 0.02, 0.0),
                               rtol=0, atol=1e-12)
    # the whole chain, no intermediate handed over
    oseg, olabs, oavg, oavgn = OP.measure_multispecies(host(stack), cal, keep=okeep)
    assert np.array_equal(host(keep["nl"]), okeep["nl"])
    assert np.array_equal(host(keep["final"]), okeep["final"], equal_nan=True)
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


def test_native_segmentation_run_overflow(mods):
    """a bright comb whose 8-connected component has a box above the pixel kernel's capacity and
    more runs than the run kernel holds: the native driver finds the overflow at the
    watershed's synchronisation and redoes the seeds; equal to the composition and the oracle"""
    P, S, OP = mods
    stack, _, _, _ = S.tile(512, 512, seed=24)
    st = host(stack).copy()
    peak = float(st.sum(axis=2).max())
    teeth = np.zeros((512, 512), bool)
    for c in range(250, 480, 6):
        teeth[280:470, c:c + 3] = True
    teeth[280:284, 250:480] = True
    # a second comb whose box fits the pixel kernel (110 x 120) but whose ~2200 runs do not fit
    # the run kernel: handed over on the device (the context's scratch)
    for c in range(40, 160, 6):
        teeth[40:150, c:c + 3] = True
    teeth[40:44, 40:160] = True
    st[teeth] = (3.0 * peak / st.shape[2]) * (1.0 + 0.05 * np.random.default_rng(5).random((int(teeth.sum()), 1)))
    dstack = torch.from_numpy(st).cuda()
    seg_n, mx_n = P.segment_ecoli(dstack)
    seg_c, mx_c = P.segment_ecoli(dstack, keep={})
    assert mx_n == mx_c and torch.equal(seg_n, seg_c)
    oseg, _ = OP.segment_ecoli(st)
    assert np.array_equal(host(seg_n), oseg)


def test_ecoli_nan_input_raises(mods):
    """a NaN in the stack makes image_cn NaN and sklearn's KMeans raise (:73); the native driver
    reads the flag at its next synchronisation and raises the same ValueError; the context
    stays usable"""
    P, S, OP = mods
    stack, _, _, _ = S.tile(128, 160, seed=25)
    bad = stack.clone()
    bad[7, 9, 3] = float("nan")
    with pytest.raises(ValueError):
        P.segment_ecoli(bad)
    with pytest.raises(ValueError):
        P.segment_ecoli(bad, keep={})
    seg_n, mx_n = P.segment_ecoli(stack)
    seg_c, mx_c = P.segment_ecoli(stack, keep={})
    assert mx_n == mx_c and torch.equal(seg_n, seg_c)


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


def test_multispecies_degenerate_tiles(mods):
    P, S, OP = mods
    for name, st in _degenerate_tiles(S, 63).items():
        if st is None or name == "zeros":
            continue   # an all-zero stack divides 0 by 0 in the reference's sum / max (:106)
        d = torch.from_numpy(np.ascontiguousarray(st)).cuda()
        if name == "constant":
            # flat line profiles make `final` NaN (:111-124) and sklearn's KMeans raises on it
            # (:125): the reference stops there, and so do both restatements
            with pytest.raises(ValueError):
                P.segment_multispecies(d)
            with pytest.raises(ValueError):
                OP.segment_multispecies(st)
            continue
        a = P.segment_multispecies(d)
        keep = {}
        b = P.segment_multispecies(d, keep=keep)
        assert a[1] == b[1] and torch.equal(a[0], b[0]), name
        oseg, on, _, _ = OP.segment_multispecies(st)
        assert np.array_equal(host(a[0]), oseg) and a[1] == on, name


# ---- bioformats-like quantised stacks: integer counts / (2^bits - 1) -----------------------
def quantised(stack, q):
    """the stack as bioformats hands it over (integer counts rescaled to [0, 1]), kept f32"""
    return (torch.round(stack.double() * q) / q).float().contiguous()


@pytest.mark.parametrize("H,q,seed", [(512, 4095, 31), (512, 255, 32), (384, 63, 33)])
def test_ecoli_quantised_parity(mods, orc, H, q, seed):
    """ecoli measurement.py:44-162 on a quantised tile: every intermediate and the label map
    bit-exact (ties in image_cn reach the watershed), spectra 1e-12"""
    P, S, OP = mods
    from hiprfish_image_analysis_amd import kernels as K
    stack = quantised(S.tile(H, H, seed=seed)[0], q)
    keep = {}
    m = P.measure_ecoli(stack, keep=keep)
    okeep = {}
    oseg, olabs, oavg, oavgn = OP.measure_ecoli(host(stack), keep=okeep)
    for k in ("rough_mask", "interior", "cell_sm"):
        assert np.array_equal(host(keep[k]).astype(bool), okeep[k]), k
    assert np.array_equal(host(keep["seeds"]), okeep["seeds"])
    # the watershed itself (:113) on the device's log-sum (within 1 ulp of numpy's, same order)
    ties = []
    ws = K.watershed(keep["image_cn"], keep["seeds"], keep["rough_mask"], negate=True, ties=ties)
    assert ties[2] == 0
    assert np.array_equal(host(ws), orc.watershed(-host(keep["image_cn"]), okeep["seeds"], okeep["rough_mask"]))
    assert np.array_equal(host(keep["watershed"]), okeep["watershed"])   # after rso(100) and clear_border
    assert np.array_equal(host(m.segmentation), oseg)
    native, _ = P.segment_ecoli(stack)
    assert np.array_equal(host(native), oseg)
    assert np.array_equal(host(m.labels), olabs) and len(olabs) >= 1
    np.testing.assert_allclose(host(m.avgint), oavg, rtol=1e-12)


@pytest.mark.parametrize("H,q,seed", [(384, 4095, 41), (320, 255, 42)])
def test_multispecies_quantised_parity(mods, H, q, seed):
    """multispecies measurement.py:102-174 on a quantised tile, whole chain vs the oracle"""
    P, S, OP = mods
    stack = quantised(S.tile(H, H, nbit=7, bounds=P.MULTI_BOUNDS, seed=seed)[0], q)
    keep = {}
    m = P.measure_multispecies(stack, keep=keep)
    oseg, olabs, oavg, _ = OP.measure_multispecies(host(stack))
    assert np.array_equal(host(m.segmentation), oseg)
    native = P.segment_multispecies(stack)
    assert np.array_equal(host(native[0]), oseg)
    assert np.array_equal(host(m.labels), olabs) and len(olabs) >= 1
    np.testing.assert_allclose(host(m.avgint), oavg, rtol=1e-12)


def test_concurrent_registered_tiles_equal_isolated(mods):
    """bench.py's current configuration: four tiles in flight, each on its own high-priority
    stream and host thread, starting from the five per-laser acquisitions and the flat field
    (registration with image_cn, calibrated spectra), classifiers on side streams.  Every
    output equals the tile processed alone."""
    P, S, OP = mods
    from concurrent.futures import ThreadPoolExecutor
    ref = S.reference_library(10, S.ECOLI_BOUNDS)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    lib.refx()
    cal = S.flat_field(768, 768)
    tiles = [S.laser_split(S.tile(768, 768, seed=160 + t)[0]) for t in range(8)]

    def run(t):
        r = P.process_tile(P.register_tile(t), lib, calibration=cal)
        return [x.clone() for x in (r.pixel_idx, r.pixel_dist, r.cell_idx, r.counts, r.meas.segmentation,
                                    r.identification, r.meas.avgint)]

    alone = [run(t) for t in tiles]
    torch.cuda.synchronize()
    hi = torch.cuda.Stream.priority_range()[1]
    streams = [torch.cuda.Stream(priority=hi) for _ in range(4)]

    def worker(j):
        res = []
        with torch.cuda.stream(streams[j]):
            for i in range(j, len(tiles), 4):
                res.append((i, run(tiles[i])))
        streams[j].synchronize()
        return res
    for rep in range(2):
        with ThreadPoolExecutor(4) as ex:
            got = [r for f in [ex.submit(worker, j) for j in range(4)] for r in f.result()]
        torch.cuda.synchronize()
        for i, outs in got:
            for a, b in zip(outs[:-1], alone[i][:-1]):
                assert torch.equal(a, b), (rep, i)
            torch.testing.assert_close(outs[-1], alone[i][-1], rtol=1e-12, atol=0)
