"""Full-size parity: BASELINE.json's headline configurations at their own size, the device
pipeline against the CPU restatement (oracle/pipeline.py) end to end -- no intermediate
handed over.

cfg3: one 2048x2048x95 E. coli tile against the 1023-barcode library (process_tile: ecoli
measurement.py:44-162 + image_classification.py:43-71 + collect :92-98), continuous and
bioformats-quantised (k/4095).  cfg2: one 2048x2048x63 synthetic-community tile against the
127-barcode library (multispecies measurement.py:78-174 + classify_spectra.py, _7b_v2 gating).
Label maps, per-cell barcodes, counts and the identification map bit-exact; spectra 1e-12;
the per-pixel argmin exact wherever the restatement separates best and runner-up."""
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


def quantised(stack, q):
    return (torch.round(stack.double() * q) / q).float().contiguous()


@pytest.mark.parametrize("q", [None, 4095])
def test_fullsize_ecoli_tile(mods, orc, q):
    P, S, OP = mods
    from test_kernels_gpu import check_pixel_argmin
    stack, _, _, ref = S.tile(2048, 2048, seed=20190301)
    if q:
        stack = quantised(stack, q)
    assert stack.shape == (2048, 2048, 95) and ref.shape[0] == 1023
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    res = P.process_tile(stack, lib, per_pixel=True)
    st = host(stack)
    o = OP.process_tile(st, ref, S.ECOLI_BOUNDS)
    seg = host(res.meas.segmentation)
    assert np.array_equal(seg, o["segmentation"])
    assert len(o["labels"]) > 500
    np.testing.assert_allclose(host(res.meas.avgint), o["avgint"], rtol=1e-12)
    np.testing.assert_allclose(host(res.cell_dist), o["cell_dist"], rtol=1e-9, atol=1e-12)
    assert np.array_equal(host(res.cell_idx), o["cell_idx"])
    assert np.array_equal(host(res.counts), o["counts"])
    assert np.array_equal(host(res.identification), orc.paint_ids(o["segmentation"], o["cell_idx"] + 1))
    # per pixel: 16384 cell pixels and 4096 anywhere
    rng = np.random.default_rng(1)
    cells = np.nonzero(seg.ravel() > 0)[0]
    sel = np.concatenate([rng.choice(cells, 16384, replace=False), rng.choice(seg.size, 4096, replace=False)])
    x = st.reshape(seg.size, -1)[sel].astype(np.float64)
    check_pixel_argmin(orc, host(res.pixel_idx).ravel()[sel], host(res.pixel_dist).ravel()[sel], x,
                       ref.astype(np.float64), S.ECOLI_BOUNDS, 16384)


def test_fullsize_community_tile(mods, orc):
    P, S, OP = mods
    b = P.MULTI_BOUNDS
    stack, _, _, ref = S.tile(2048, 2048, nbit=7, bounds=b, seed=20190201)
    stack = quantised(stack, 4095)
    assert stack.shape == (2048, 2048, 63) and ref.shape[0] == 127
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), b, 7)
    res = P.process_tile(stack, lib, per_pixel=True, measure=P.measure_multispecies, variant=2)
    st = host(stack)
    oseg, olabs, oavg, oavgn = OP.measure_multispecies(st)
    assert np.array_equal(host(res.meas.segmentation), oseg)
    assert np.array_equal(host(res.meas.labels), olabs) and len(olabs) > 500
    np.testing.assert_allclose(host(res.meas.avgint), oavg, rtol=1e-12)
    oidx, odist = OP.classify_cells(oavgn, ref, b, variant=2)
    np.testing.assert_allclose(host(res.cell_dist), odist, rtol=1e-9, atol=1e-12)
    assert np.array_equal(host(res.cell_idx), oidx)
    assert np.array_equal(host(res.counts), orc.barcode_counts(oidx, 127))
    # per pixel (cfg2's 2048x2048x63 against the 127-row library): the restatement's argmin and
    # distance on every sampled pixel
    from test_kernels_gpu import check_pixel_argmin
    rng = np.random.default_rng(3)
    cells = np.nonzero(oseg.ravel() > 0)[0]
    sel = np.concatenate([rng.choice(cells, 16384, replace=False), rng.choice(oseg.size, 4096, replace=False)])
    x = st.reshape(oseg.size, -1)[sel].astype(np.float64)
    check_pixel_argmin(orc, host(res.pixel_idx).ravel()[sel], host(res.pixel_dist).ravel()[sel], x,
                       ref.astype(np.float64), b, 16384)


@pytest.mark.parametrize("q", [None, 4095, 255])
def test_fullsize_bench_workload(mods, orc, q):
    """bench.py's exact timed workload on one tile at full size (2048x2048x95, R=1023), through the
    native tile call the bench times (and equal to the composed path): the five
    misregistered per-laser acquisitions (bench.py's tile generation; continuous, or
    bioformats-like k/4095 and k/255 samples) + the flat field -> channel-max projections, FFT
    shifts on the device, registered assembly with the coverage mask and image_cn ->
    segmentation -> flat-fielded per-cell spectra -> per-cell and per-pixel classification ->
    counts, identification map.  Against the restatement of ecoli measurement.py:44-162 with
    -c T (estimate_shifts, register_stacks, measure_ecoli(calibration)).  The watershed's
    contest / equal-marker statistics of the tile are printed (DESIGN.md "Watershed")."""
    P, S, OP = mods
    import bench
    from hiprfish_image_analysis_amd import kernels as K
    from test_kernels_gpu import check_pixel_argmin
    H = W = 2048
    ref = S.reference_library(bench.NBIT, S.ECOLI_BOUNDS)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, bench.NBIT)
    seed = 20190101
    lay = S.cell_layout(H, W, S.default_ncells(H, W), lib.R, seed)
    truth, prof = S.render_truth(H, W, lay, with_profile=True)
    stack = S.render_stack(truth, lay, ref, seed=seed, device="cuda", profile=prof)
    lasers = S.laser_split(stack)
    del stack
    if q:
        lasers = [quantised(l, q) for l in lasers]
    cal = S.flat_field(H, W, device="cuda")
    # bench.py's path: one native call per tile (hrf_tile_ecoli), gated per-cell metric
    res = P.process_tile_native(lasers, lib, calibration=cal, per_pixel=True, variant=1)
    torch.cuda.synchronize()
    stats = K.tile_stats(lasers[0].device, H, W)
    print("watershed stats q=%s: %s" % (q, stats))
    # the composed path (register_tile without a stack + process_tile) gives the same tile
    rt = P.register_tile(lasers)
    comp = P.process_tile(rt, lib, calibration=cal, per_pixel=True, variant=1)
    for x, y in ((res.meas.segmentation, comp.meas.segmentation), (res.cell_idx, comp.cell_idx),
                 (res.counts, comp.counts), (res.identification, comp.identification),
                 (res.pixel_idx, comp.pixel_idx), (res.pixel_dist, comp.pixel_dist)):
        assert torch.equal(x, y)
    del comp
    reg, cn = P.register_stack(lasers, want_cn=True)
    assert torch.equal(rt.image_cn, cn)
    del rt

    hl = [host(l) for l in lasers]
    shifts = OP.estimate_shifts(hl, "max", 15)
    assert P.estimate_shifts(lasers) == shifts
    oreg = OP.register_stacks(hl, shifts, True).astype(np.float32)
    del hl
    assert np.array_equal(host(reg), oreg)
    # image_cn bit for bit: the correctly rounded log of numpy's pairwise channel sum; numpy's own
    # log differs from it in the last ulp on a few pixels (reported)
    ssum = np.sum(oreg.astype(np.float64), axis=2) + 1e-2
    want_cn = orc.cr_log(ssum)
    assert np.array_equal(host(cn), want_cn)
    print("image_cn pixels where np.log differs from the correctly rounded log: %d of %d"
          % (int((np.log(ssum) != want_cn).sum()), ssum.size))
    del ssum, want_cn
    o = OP.process_tile(oreg, ref, S.ECOLI_BOUNDS, calibration=host(cal), variant=1)
    seg = host(res.meas.segmentation)
    assert np.array_equal(seg, o["segmentation"])
    assert len(o["labels"]) > 500
    np.testing.assert_allclose(host(res.meas.avgint), o["avgint"], rtol=1e-12)
    np.testing.assert_allclose(host(res.cell_dist), o["cell_dist"], rtol=1e-9, atol=1e-12)
    assert np.array_equal(host(res.cell_idx), o["cell_idx"])
    assert np.array_equal(host(res.counts), o["counts"])
    assert np.array_equal(host(res.identification), orc.paint_ids(o["segmentation"], o["cell_idx"] + 1))
    rng = np.random.default_rng(2)
    cells = np.nonzero(seg.ravel() > 0)[0]
    sel = np.concatenate([rng.choice(cells, 16384, replace=False), rng.choice(seg.size, 4096, replace=False)])
    x = oreg.reshape(seg.size, -1)[sel].astype(np.float64)
    check_pixel_argmin(orc, host(res.pixel_idx).ravel()[sel], host(res.pixel_dist).ravel()[sel], x,
                       ref.astype(np.float64), S.ECOLI_BOUNDS, 16384)


def _enhance_3d_threads(pad, nthreads=16, patch=11):
    """oracle.enhance_3d over x slabs (each output voxel reads only its patch^3 neighbourhood, so
    slabs with a patch - 1 halo are exact); the ctypes call releases the GIL, so threads run the
    slabs in parallel"""
    from concurrent.futures import ThreadPoolExecutor

    import oracle as O
    X = pad.shape[0] - patch + 1
    cuts = np.linspace(0, X, nthreads + 1).astype(int)
    with ThreadPoolExecutor(nthreads) as ex:
        parts = list(ex.map(lambda k: O.enhance_3d(pad[cuts[k]:cuts[k + 1] + patch - 1]), range(nthreads)))
    return np.concatenate(parts, axis=0)


def test_fullsize_volume_chain_full_xy():
    """cfg4 at its own XY size: the biofilm volume chain (biofilm :808-817: channel sum, / max,
    edge pad 5, line_profile_memory_efficient_v2 + post-chain) on a 1024x1024x6x63 volume -- the
    full 1024x1024 plane of the benched 1024x1024x64x63 stack, 6 z planes -- bit-exact against
    the restatement (the bench's 64 planes cost the single-threaded restatement ~11 minutes)."""
    from hiprfish_image_analysis_amd import pipeline as P
    X, Y, Z, C = 1024, 1024, 6, 63
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    vol = torch.rand((X, Y, Z, C), dtype=torch.float32, device="cuda", generator=g)
    got = host(P.enhance_volume(vol))
    s = np.sum(host(vol).astype(np.float64), axis=3)
    del vol
    pad = np.pad(s / np.max(s), 5, mode="edge")
    want = _enhance_3d_threads(pad)
    assert got.shape == want.shape == (X, Y, Z)
    assert np.array_equal(got, want)


def test_fullsize_volume_chain_64_planes():
    """cfg4 at the benched size: the device chain on the whole 1024x1024x64x63 volume bench.py
    times (same generator, same seed), compared with the restatement on three z slabs -- both
    boundaries and the middle -- each computed from the globally normalised, edge-padded array
    with its patch - 1 halo (an output voxel reads only its 11^3 neighbourhood, so a slab is exact)."""
    from hiprfish_image_analysis_amd import pipeline as P
    X, Y, Z, C = 1024, 1024, 64, 63
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    vol = torch.rand((X, Y, Z, C), dtype=torch.float32, device="cuda", generator=g)
    got = P.enhance_volume(vol)
    # numpy's channel sum in f64, streamed over x (the f64 copy of the whole volume is 34 GB)
    s = np.concatenate([np.sum(host(vol[x0:x0 + 64]).astype(np.float64), axis=3) for x0 in range(0, X, 64)], axis=0)
    del vol
    pad = np.pad(s / np.max(s), 5, mode="edge")
    del s
    for z0 in (0, 29, 58):
        want = _enhance_3d_threads(pad[:, :, z0:z0 + 6 + 10])
        part = host(got[:, :, z0:z0 + 6])
        assert part.shape == want.shape == (X, Y, 6)
        assert np.array_equal(part, want), z0


def test_fullsize_community_registered_calibrated(mods, orc):
    """cfg2 as the reference runs it (multispecies generate_2d_segmentation :78-159 +
    measure_biofilm_images_no_reference :161-174): four misregistered 2048x2048 acquisitions
    (23 / 20 / 14 / 6 channels, bioformats-like k/4095 samples) registered on their channel sums
    with no clamp and no coverage-mask multiply (:82-102), divided by a (H, W, C) calibration
    array (:103-104), then the whole segmentation + per-cell chain; against oracle/pipeline.py
    (estimate_shifts 'sum', register_stacks without the mask, measure_multispecies with the
    calibration).  Also the _registered.npy array (:166) bit for bit."""
    P, S, OP = mods
    from hiprfish_image_analysis_amd import kernels as K
    b = P.MULTI_BOUNDS
    H = W = 2048
    stack, _, _, ref = S.tile(H, W, nbit=7, bounds=b, seed=20190205)
    stack = quantised(stack, 4095)
    lasers = S.laser_split(stack, b, S.COMMUNITY_SHIFTS)
    del stack
    cal = S.calibration_stack(H, W, 63)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), b, 7)
    shifts_dev = P.estimate_shifts(lasers, reduce="sum", clamp=None, device=True)
    reg = P.register_multispecies(lasers, shifts_dev)
    res = P.process_tile(reg, lib, calibration=cal, per_pixel=True, measure=P.measure_multispecies, variant=2)
    torch.cuda.synchronize()
    hl = [host(l) for l in lasers]
    shifts = OP.estimate_shifts(hl, "sum", None)
    assert [tuple(int(v) for v in r) for r in host(shifts_dev)] == shifts
    assert shifts[1:] == [tuple(s) for s in S.COMMUNITY_SHIFTS[1:]]
    oreg = OP.register_stacks(hl, shifts, False).astype(np.float32)
    del hl
    assert np.array_equal(host(reg), oreg)
    hcal = host(cal)
    assert np.array_equal(host(K.calibrate(reg, cal)), oreg.astype(np.float64) / hcal.astype(np.float64))   # :166
    oseg, olabs, oavg, oavgn = OP.measure_multispecies(oreg, calibration=hcal)
    assert np.array_equal(host(res.meas.segmentation), oseg)
    assert np.array_equal(host(res.meas.labels), olabs) and len(olabs) > 500
    np.testing.assert_allclose(host(res.meas.avgint), oavg, rtol=1e-12)
    oidx, odist = OP.classify_cells(oavgn, ref, b, variant=2)
    np.testing.assert_allclose(host(res.cell_dist), odist, rtol=1e-9, atol=1e-12)
    assert np.array_equal(host(res.cell_idx), oidx)
    assert np.array_equal(host(res.counts), orc.barcode_counts(oidx, 127))
    from test_kernels_gpu import check_pixel_argmin
    rng = np.random.default_rng(4)
    cells = np.nonzero(oseg.ravel() > 0)[0]
    sel = np.concatenate([rng.choice(cells, 8192, replace=False), rng.choice(oseg.size, 2048, replace=False)])
    x = oreg.reshape(oseg.size, -1)[sel].astype(np.float64)
    check_pixel_argmin(orc, host(res.pixel_idx).ravel()[sel], host(res.pixel_dist).ravel()[sel], x,
                       ref.astype(np.float64), b, 8192)
