"""One E. coli tile as one native call (hrf_tile_ecoli, tile.hip) against the composed path
(pipeline.register_tile + process_tile), which the full-size tests check against the CPU
restatement: label map, per-cell labels, barcodes, counts, identification map and per-pixel
barcodes and distances bit for bit; per-cell spectra and distances within 1e-12 / 1e-9 (f64
atomics in the label sums).  Reference: ecoli
measurement.py:44-162 (-c T), image_classification.py:43-71, collect_measurement_results.py:92-98.
"""
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    from hiprfish_image_analysis_amd import kernels as K
    from hiprfish_image_analysis_amd import pipeline as P
    from hiprfish_image_analysis_amd import synthetic as S
    return K, P, S


def _lib(P, S):
    ref = S.reference_library(10, S.ECOLI_BOUNDS)
    return P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)


def _lasers(S, H, W, seed, q=None):
    lib_ref = S.reference_library(10, S.ECOLI_BOUNDS)
    lay = S.cell_layout(H, W, S.default_ncells(H, W), lib_ref.shape[0], seed)
    truth, prof = S.render_truth(H, W, lay, with_profile=True)
    stack = S.render_stack(truth, lay, lib_ref, seed=seed, device="cuda", profile=prof)
    lasers = S.laser_split(stack)
    if q:
        lasers = [(torch.round(l.double() * q) / q).float().contiguous() for l in lasers]
    return lasers


def _same(a, b):
    return torch.equal(a, b)


def _check(nat, ref, per_pixel=True):
    """integer outputs bit for bit; the spectra within 1e-12 (label sums accumulate with f64
    atomics, so their last bits depend on the order the flushes land in -- the tolerance every
    label-sums test uses) and the per-cell distances with them"""
    assert _same(nat.meas.segmentation, ref.meas.segmentation)
    assert nat.meas.maxlab == ref.meas.maxlab
    assert _same(nat.meas.labels, ref.meas.labels)
    np.testing.assert_allclose(nat.meas.avgint.cpu().numpy(), ref.meas.avgint.cpu().numpy(), rtol=1e-12, atol=0)
    np.testing.assert_allclose(nat.meas.avgint_norm.cpu().numpy(), ref.meas.avgint_norm.cpu().numpy(), rtol=1e-12,
                               atol=0)
    assert _same(nat.cell_idx, ref.cell_idx)
    np.testing.assert_allclose(nat.cell_dist.cpu().numpy(), ref.cell_dist.cpu().numpy(), rtol=1e-9, atol=1e-12)
    assert _same(nat.counts, ref.counts)
    assert _same(nat.identification, ref.identification)
    if per_pixel:
        assert _same(nat.pixel_idx, ref.pixel_idx)
        assert _same(nat.pixel_dist, ref.pixel_dist)


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("calibrated", [False, True])
def test_tile_native_equals_composed(mods, variant, calibrated):
    K, P, S = mods
    H = W = 512
    lib = _lib(P, S)
    lasers = _lasers(S, H, W, 20190107)
    cal = S.flat_field(H, W, device="cuda") if calibrated else None
    nat = P.process_tile_native(lasers, lib, calibration=cal, variant=variant)
    ref = P.process_tile(P.register_tile(lasers), lib, calibration=cal, per_pixel=True, variant=variant)
    torch.cuda.synchronize()
    assert nat.ncells > 20
    _check(nat, ref)


def test_tile_native_non_power_of_two(mods):
    """a 384 x 320 tile (not powers of two): the native call registers through hipFFT per target
    and equals the composed path bit for bit"""
    K, P, S = mods
    H, W = 384, 320
    lib = _lib(P, S)
    lasers = _lasers(S, H, W, 20190114)
    cal = S.flat_field(H, W, device="cuda")
    assert not K.xcorr_supported(5, H, W)
    nat = P.process_tile_native(lasers, lib, calibration=cal, variant=1)
    ref = P.process_tile(P.register_tile(lasers), lib, calibration=cal, per_pixel=True, variant=1)
    torch.cuda.synchronize()
    assert nat.ncells > 10
    _check(nat, ref)


def test_tile_native_no_overlap_no_pixels(mods):
    K, P, S = mods
    H = W = 256
    lib = _lib(P, S)
    lasers = _lasers(S, H, W, 20190108, q=4095)
    cal = S.flat_field(H, W, device="cuda")
    ref = P.process_tile(P.register_tile(lasers), lib, calibration=cal, per_pixel=True, variant=1)
    a = P.process_tile_native(lasers, lib, calibration=cal, variant=1, overlap=False)
    _check(a, ref)
    b = P.process_tile_native(lasers, lib, calibration=cal, variant=1, per_pixel=False)
    _check(b, ref, per_pixel=False)
    assert b.pixel_idx is None


def test_tile_native_cell_capacity_retry(mods):
    """more labels than the per-cell buffers hold: the tail runs again through
    hrf_tile_ecoli_cells with buffers sized for every label"""
    K, P, S = mods
    H = W = 512
    lib = _lib(P, S)
    lasers = _lasers(S, H, W, 20190109)
    cal = S.flat_field(H, W, device="cuda")
    key = (lasers[0].device, H, W)
    K._CELL_CAP[key] = 8
    try:
        nat = P.process_tile_native(lasers, lib, calibration=cal, variant=1)
        assert K._CELL_CAP[key] >= nat.meas.maxlab > 8
    finally:
        K._CELL_CAP.pop(key, None)
    ref = P.process_tile(P.register_tile(lasers), lib, calibration=cal, per_pixel=True, variant=1)
    _check(nat, ref)


def test_tile_native_concurrent_streams(mods):
    """two host threads, each with its own stream (and so its own tile context and side stream),
    as bench.py drives them: equal to the isolated results"""
    K, P, S = mods
    H = W = 512
    lib = _lib(P, S)
    lib.refx()
    lib.presence_flags()
    tiles = [_lasers(S, H, W, 20190110 + i) for i in range(2)]
    cal = S.flat_field(H, W, device="cuda")
    want = [P.process_tile_native(t, lib, calibration=cal) for t in tiles]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in tiles]
    got = [None, None]

    def run(j):
        with torch.cuda.stream(streams[j]):
            for _ in range(3):
                got[j] = P.process_tile_native(tiles[j], lib, calibration=cal)
            streams[j].synchronize()
    th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    torch.cuda.synchronize()
    for g, w in zip(got, want):
        _check(g, w)


def test_tile_native_rejects_bad_input(mods):
    K, P, S = mods
    lib = _lib(P, S)
    lasers = _lasers(S, 256, 256, 20190111)
    with pytest.raises(ValueError):
        P.process_tile_native(lasers[:4], lib)
    with pytest.raises(ValueError):
        K.tile_ecoli(lasers, None, None, lib.spectra, None, variant=1, per_pixel=False)


def test_tile_native_six_streams_fullsize(mods):
    """the bench's schedule at the bench's size: six host threads, six high-priority streams (each
    with its own tile context and classifier side stream), 2048^2 tiles, every tile twice --
    equal to the same tiles run one at a time (bench.py main, DESIGN.md 'Concurrency on one GPU')"""
    K, P, S = mods
    H = W = 2048
    T = 6
    lib = _lib(P, S)
    lib.refx_table()
    lib.presence_flags()
    tiles = [_lasers(S, H, W, 20190301 + i) for i in range(T)]
    cal = S.flat_field(H, W, device="cuda")
    want = [P.process_tile_native(t, lib, calibration=cal, variant=1) for t in tiles]
    torch.cuda.synchronize()
    prio = torch.cuda.Stream.priority_range()[1]
    streams = [torch.cuda.Stream(priority=prio) for _ in range(T)]
    got = [None] * T
    errs = []

    def run(j):
        try:
            with torch.cuda.stream(streams[j]):
                for _ in range(2):
                    got[j] = P.process_tile_native(tiles[j], lib, calibration=cal, variant=1)
                streams[j].synchronize()
        except Exception as e:       # surfaced below
            errs.append(e)
    th = [threading.Thread(target=run, args=(j,)) for j in range(T)]
    [t.start() for t in th]
    [t.join() for t in th]
    torch.cuda.synchronize()
    assert not errs, errs
    for g, w in zip(got, want):
        assert g.ncells > 300
        _check(g, w)


def test_tile_context_cache_bounded(mods):
    """a caller that makes a fresh stream per tile: the contexts stay within the cache's cap and
    device memory does not grow with the number of streams"""
    K, P, S = mods
    H = W = 512
    lib = _lib(P, S)
    lasers = _lasers(S, H, W, 20190112)
    cal = S.flat_field(H, W, device="cuda")
    want = P.process_tile_native(lasers, lib, calibration=cal, variant=1)
    torch.cuda.synchronize()
    cn = P.register_tile(lasers).image_cn
    K.release_contexts()
    cap = K._TILE_CTX.cap

    def one():
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            r = P.process_tile_native(lasers, lib, calibration=cal, variant=1)
            K.segment_ecoli_native(None, image_cn=cn)
        s.synchronize()
        return r
    def free_bytes():
        # torch's caching allocator keeps freed blocks per stream (a fresh stream cannot reuse
        # another's): released before reading what the device has left
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        return torch.cuda.mem_get_info()[0]
    # torch hands out streams from a pool of 32 (the side streams draw on it too); the HIP runtime
    # gives a stream its queue resources (and a queue its scratch) on first use, so every pool
    # stream is used once before memory is read: afterwards each call on the next pool stream
    # misses the cache (the pool cycles through more streams than the cap), makes a context and
    # evicts the least recently used one
    for _ in range(40):
        one()
    assert len(K._TILE_CTX) == cap and len(K._SEG_CTX) == cap
    free_full = free_bytes()
    made = K._TILE_CTX.created
    for _ in range(20):
        r = one()
        assert len(K._TILE_CTX) <= cap and len(K._SEG_CTX) <= cap
    assert K._TILE_CTX.created - made >= 10        # contexts really churned
    grown = free_full - free_bytes()
    assert grown < 64 << 20, "device memory grew by %d bytes over 20 fresh contexts" % grown
    _check(r, want)
    K.release_contexts()
    assert len(K._TILE_CTX) == 0 and len(K._SEG_CTX) == 0


def test_pixel_table_needs_mode2_table(mods):
    """the pixel-table classifier refuses a mode-0/1 prepared library (it would read it as split-fp16
    rows of another pitch); the Library hands it a mode-2 table whatever refx() holds"""
    K, P, S = mods
    H = W = 256
    lib = _lib(P, S)
    lasers = _lasers(S, H, W, 20190113)
    rt = P.register_tile(lasers)
    for mode in (0, 1):
        bad = K.classify_prepare(lib.spectra.to(torch.float32), lib.bounds, mode=mode)
        with pytest.raises(ValueError):
            K.classify_pixels_table(rt.pixtable, bad, lib.R)
        with pytest.raises(ValueError):
            K.tile_ecoli(lasers, None, bad, lib.spectra, lib.presence_flags(), variant=1)
    want = P.process_tile_native(lasers, lib, variant=1)
    lib1 = _lib(P, S)
    lib1._refx = K.classify_prepare(lib1.spectra.to(torch.float32), lib1.bounds, mode=1)
    got = P.process_tile_native(lasers, lib1, variant=1)
    torch.cuda.synchronize()
    _check(got, want)


def test_tile_native_equal_marker_ties(mods, orc):
    """ecoli measurement.py:113 inside the native tile chain (hrf_tile_ecoli) on a tile whose
    watershed decisions come down to equal-valued markers of different labels (synthetic.tie_tile):
    the chain floods the tile again with the heap replay and its label map, cells and barcodes
    equal oracle/pipeline.py's (skimage's heap restated) on the registered lasers -- where the
    order model alone (raw) would label corridor pixels differently"""
    import pipeline as OP
    K, P, S = mods
    H = W = 256
    stack = S.tie_tile(H, W, gap=1)
    lasers = S.laser_split(stack)
    lib = _lib(P, S)
    nat = P.process_tile_native(lasers, lib, variant=1)
    torch.cuda.synchronize()
    st = K.tile_stats(stack.device, H, W)
    assert st["marker_ties"] > 0 and st["contests"] > 0, st
    lh = [l.cpu().numpy() for l in lasers]
    reg = OP.register_stacks(lh, OP.estimate_shifts(lh), True)
    ref = lib.spectra.cpu().numpy()
    keep = {}
    OP.segment_ecoli(reg, keep=keep)
    raw, rs = orc.watershed_ordered(-keep["image_cn"], keep["seeds"], keep["rough_mask"], raw=True)
    assert rs[2] > 0 and (raw != keep["watershed"]).any()   # the layout decides some pixels
    o = OP.process_tile(reg, ref, S.ECOLI_BOUNDS, variant=1)
    assert np.array_equal(nat.meas.segmentation.cpu().numpy(), o["segmentation"])
    assert nat.ncells == len(o["cell_idx"]) and nat.ncells >= 16
    assert np.array_equal(nat.cell_idx.cpu().numpy()[:nat.ncells], o["cell_idx"])
    comp = P.process_tile(P.register_tile(lasers), lib, per_pixel=True, variant=1)
    _check(nat, comp)
