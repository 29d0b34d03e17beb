"""Exact per-pixel classification (§8 a19, north_star's per-pixel mode; round 6).

The MFMA sweeps are a screen; hrf_classify_pixels_refine certifies the screen's row with its f64
distance against the screen's proven error bound, or re-scores every row.  These tests pin:
  * the accumulation model of the f16 MFMAs the bound assumes (hrf_probe_mfma_f16);
  * the bound itself on real screens: every library row's restated score is within it of the
    screen's runner-up report (the certificate's premise), on every screen form;
  * exactness where a screen alone cannot decide: duplicate and near-duplicate library rows,
    all-zero / partly zero / tiny / huge / NaN / inf pixels -- argmin and distance equal to the
    restatement's (oracle_classify_top2, train_reference.py:223-386 ungated) on every pixel.
"""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ECOLI = (0, 32, 55, 75, 89, 95)
MULTI = (0, 23, 43, 57, 63)
U = 2.0 ** -24


@pytest.fixture(scope="module")
def K():
    from hiprfish_image_analysis_amd import kernels
    return kernels


@pytest.fixture(scope="module")
def S():
    from hiprfish_image_analysis_amd import synthetic
    return synthetic


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.detach().cpu().numpy()


def restated_scores(x, ref, bounds):
    """S[i, r] = nseg * (1 - D(x_i, ref_r)) with D the restatement's f64 distance (oracle_segcos
    variant 0), vectorised: per segment 1 - d / sqrt(nx ny), both-zero 0, one-zero 1"""
    x = x.astype(np.float64)
    ref = ref.astype(np.float64)
    nseg = len(bounds) - 1
    D = np.zeros((x.shape[0], ref.shape[0]))
    for s in range(nseg):
        a, b = bounds[s], bounds[s + 1]
        d = x[:, a:b] @ ref[:, a:b].T
        nx = (x[:, a:b] ** 2).sum(1)[:, None]
        ny = (ref[:, a:b] ** 2).sum(1)[None, :]
        with np.errstate(invalid="ignore", divide="ignore"):
            sd = 1.0 - d / np.sqrt(nx * ny)
        sd = np.where((nx == 0) & (ny == 0), 0.0, np.where((nx == 0) | (ny == 0), 1.0, sd))
        D += sd
    return nseg * (1.0 - D / nseg)


def test_mfma_f16_accumulation_model(K):
    """Each f16 MFMA output is within KMFMA = 16 u (|c| + sum |a b|) of the exact sum (the screen
    bound's model, classify.hip screen_eps).  gfx950 measures <= 7.6 (tools/mfma_probe.py); this
    asserts <= 12 on adversarial and random tiles, both MFMA shapes."""
    from hiprfish_image_analysis_amd import _lib
    rng = np.random.default_rng(11)
    worst = 0.0
    for shape, (M, Kd, N) in ((0, (16, 32, 16)), (1, (32, 16, 32))):
        n = 48
        cases = []
        cases.append((np.full((n, M, Kd), 2.0 ** -12), np.full((n, Kd, N), 2.0 ** -13), np.ones((n, M, N))))
        cases.append((rng.random((n, M, Kd)), rng.random((n, Kd, N)), rng.random((n, M, N)) * Kd))
        cases.append((rng.normal(size=(n, M, Kd)), rng.normal(size=(n, Kd, N)), rng.normal(size=(n, M, N))))
        e = rng.integers(-24, 1, (n, M, Kd)).astype(np.float64)
        cases.append((rng.random((n, M, Kd)) * 2.0 ** e, rng.random((n, Kd, N)), rng.random((n, M, N)) * 4))
        A = rng.random((n, M, Kd)) * 2.0 ** -11
        A[:, :, 0] = 1.0
        cases.append((A, rng.random((n, Kd, N)), np.zeros((n, M, N))))
        # the screen's own operand statistics: hi / lo splits of unit-segment values
        v = rng.random((n, M, Kd)) / math.sqrt(Kd)
        hi = v.astype(np.float16).astype(np.float64)
        cases.append((np.concatenate([hi[:, :, :Kd // 2], (v - hi)[:, :, :Kd // 2]], 2), rng.random((n, Kd, N)) / 4,
                      rng.random((n, M, N)) * 5))
        for A, B, Cm in cases:
            a = torch.from_numpy(A.astype(np.float16)).cuda()
            b = torch.from_numpy(B.astype(np.float16)).cuda()
            c = torch.from_numpy(Cm.astype(np.float32)).cuda()
            d = torch.empty_like(c)
            _lib.call("hrf_probe_mfma_f16", shape, a.data_ptr(), b.data_ptr(), c.data_ptr(), d.data_ptr(), n,
                      torch.cuda.current_stream().cuda_stream)
            a64, b64 = host(a).astype(np.float64), host(b).astype(np.float64)
            c64, d64 = host(c).astype(np.float64), host(d).astype(np.float64)
            prods = a64[:, :, :, None] * b64[:, None, :, :]           # (n, M, K, N), exact
            exact = c64 + prods.sum(2)                                # within 2^-50 relative of exact
            mag = np.abs(c64) + np.abs(prods).sum(2)
            ok = mag > 0
            ratio = np.abs(d64 - exact)[ok] / (U * mag[ok])
            worst = max(worst, float(ratio.max()))
    print("f16 MFMA accumulation: max error %.3f u (|c| + sum |ab|) (bound model 16, asserted <= 12)" % worst)
    assert worst <= 12.0


def _library(S, nbit, bounds, near=False, dup=False):
    ref = S.reference_library(nbit, bounds).astype(np.float32).copy()
    R = ref.shape[0]
    rng = np.random.default_rng(5)
    pairs = []
    if dup or near:
        pairs = [(3, 70), (10, 11), (40, 104), (0, R - 1)]
        if R > 500:
            pairs += [(5, 900), (130, 513), (600, 601)]
        for a, b in pairs:
            ref[b] = ref[a]
            if near:   # a relative perturbation far below the screen's resolution
                ref[b] *= (1 + rng.normal(0, 3e-7, ref.shape[1])).astype(np.float32)
    return ref, pairs


def _pixels(ref, pairs, n, rng):
    """pixels near the paired rows (both about equally close), plus noisy library multiples"""
    C = ref.shape[1]
    out = []
    for i in range(n):
        if pairs and i % 2 == 0:
            a, b = pairs[(i // 2) % len(pairs)]
            x = 0.5 * (ref[a].astype(np.float64) + ref[b]) * rng.uniform(0.5, 1.0)
            x = x * (1 + rng.normal(0, 1e-3, C))
        else:
            r = rng.integers(0, ref.shape[0])
            x = ref[r] * rng.uniform(0.5, 1.0) + rng.normal(0, 0.02, C)
        out.append(np.clip(x, 0, None))
    return np.array(out, dtype=np.float32)


@pytest.mark.parametrize("screen", [0, 1, 2, 3])
@pytest.mark.parametrize("nbit,bounds", [(10, ECOLI), (7, MULTI)])
def test_screen_bound_holds(K, S, screen, nbit, bounds):
    """the certificate's premise on real screens: for every pixel and every library row r other
    than the screen's best row, the restated score S(r) <= second + eps (+ eps_zero per all-zero
    segment of the pixel).  Reports how much of eps the observed excess uses."""
    if screen == 2 and 2 not in K.classify_modes(bounds):
        pytest.skip("mode 2: reference layouts only")
    ref, pairs = _library(S, nbit, bounds, near=True)
    rng = np.random.default_rng(screen)
    x = _pixels(ref, pairs, 4096, rng)
    x[:64] = 0.0                                          # all-zero pixels
    x[64:128, bounds[0]:bounds[1]] = 0.0                  # one zero segment
    R, C = ref.shape
    mode = 2 if screen == 3 else screen
    refx = K.classify_prepare(dev(ref), bounds, mode=mode)
    st = dev(x.reshape(64, 64, C))
    if screen == 3:
        idx, dist, sec = K.classify_pixels_table_screen(K.pixtable_prepare(st, bounds), refx, R)
    else:
        idx, dist, sec = K.classify_pixels_screen(st, refx, R, bounds, mode=mode)
    idx, sec = host(idx).ravel(), host(sec).ravel().astype(np.float64)
    base, zero, _ = K.classify_screen_eps(C, bounds, R, screen)
    Sx = restated_scores(x, ref, bounds)
    nseg = len(bounds) - 1
    nz = np.zeros(x.shape[0], dtype=np.int64)
    for s in range(nseg):
        nz += (np.abs(x[:, bounds[s]:bounds[s + 1]]).sum(1) == 0)
    eps = base + zero * nz
    Sx[np.arange(x.shape[0]), idx] = -np.inf
    over = Sx.max(1) - sec                                # must be <= eps
    live = nz < nseg                                      # all-zero pixels: answered from the library
    used = float((over[live] / eps[live]).max())
    print("screen %d: max (S(r) - second) / eps over rows r != best = %.4f (eps %.3e)" % (screen, used, base))
    assert used <= 1.0


@pytest.mark.parametrize("mode", [0, 1, 2, "table"])
@pytest.mark.parametrize("nbit,bounds", [(10, ECOLI), (7, MULTI)])
@pytest.mark.parametrize("lib", ["near", "dup"])
def test_near_ties_exact(K, S, orc, mode, nbit, bounds, lib):
    """duplicate rows (exact ties: the lowest row) and rows perturbed by ~3e-7 relative (ties no
    MFMA screen resolves): every pixel gets the restatement's argmin and distance"""
    if mode == 2 and 2 not in K.classify_modes(bounds):
        pytest.skip("mode 2: reference layouts only")
    from test_kernels_gpu import check_pixel_argmin
    ref, pairs = _library(S, nbit, bounds, near=lib == "near", dup=lib == "dup")
    rng = np.random.default_rng(17)
    x = _pixels(ref, pairs, 64 * 48, rng)
    R, C = ref.shape
    st = dev(x.reshape(64, 48, C))
    if mode == "table":
        refx = K.classify_prepare(dev(ref), bounds, mode=2)
        gi, gd = K.classify_pixels_table(K.pixtable_prepare(st, bounds), refx, R)
    else:
        refx = K.classify_prepare(dev(ref), bounds, mode=mode)
        gi, gd = K.classify_pixels(st, refx, R, bounds)
    near, _ = check_pixel_argmin(orc, host(gi).ravel(), host(gd).ravel(), x.astype(np.float64),
                                 ref.astype(np.float64), bounds)
    assert near > 64 * 48 // 4     # the pairs are exercised


@pytest.mark.parametrize("mode", [0, 1, 2, "table"])
def test_special_pixels_exact(K, S, orc, mode):
    """pixels outside the screen bound's premises -- all-zero, partly zero, f32-underflowing,
    f32-overflowing, NaN and inf values -- and a library with an all-zero segment row: the
    restatement's answer (NaN anywhere: row 0 at distance inf, oracle_classify's loop)"""
    from test_kernels_gpu import check_pixel_argmin
    bounds = ECOLI
    ref = S.reference_library(10, bounds).astype(np.float32).copy()
    ref[7, 0:32] = 0.0
    ref[9, 89:95] = 0.0
    R, C = ref.shape
    rng = np.random.default_rng(3)
    x = (ref[rng.integers(0, R, 2048)] * rng.uniform(0.5, 1, (2048, 1)) + rng.normal(0, 0.02, (2048, C)))
    x = np.clip(x, 0, None).astype(np.float32)
    x[0:16] = 0.0
    x[16:32, 0:32] = 0.0
    x[32:48, 55:75] = 0.0
    x[48:64, 89:95] = 0.0
    x[64:80, 32:55] *= 1e-24                          # segment sums of squares ~1e-50: f32 underflow
    x[80:96] *= np.float32(1e-22)
    x[96:112, 0:32] *= np.float32(3e19)               # f32 overflow of the sum of squares
    x[112, 5] = np.nan
    x[113, 40] = np.inf
    x[114, 90] = -np.inf
    x[115:120, 93] = 1e-42                           # f32 subnormal values
    st = dev(x.reshape(32, 64, C))
    if mode == "table":
        refx = K.classify_prepare(dev(ref), bounds, mode=2)
        gi, gd = K.classify_pixels_table(K.pixtable_prepare(st, bounds), refx, R)
    else:
        refx = K.classify_prepare(dev(ref), bounds, mode=mode)
        gi, gd = K.classify_pixels(st, refx, R, bounds)
    check_pixel_argmin(orc, host(gi).ravel(), host(gd).ravel(), x.astype(np.float64), ref.astype(np.float64), bounds)


def test_refine_from_lasers_equals_stack(K, S, orc):
    """a registered tile's table refined from the five shifted acquisitions (LaserSource, the
    bench path) -- sweep + certificate pass, the certificate fused into the sweep, and the Python
    composition of screen + refine -- = the registered stack refined as a plain stack = the
    restatement, with the coverage mask and a ragged width"""
    from hiprfish_image_analysis_amd import pipeline as P
    from test_kernels_gpu import check_pixel_argmin
    for H, W in ((128, 192), (96, 80)):
        stack, _, _, ref = S.tile(H, W, seed=H * W)
        lasers = S.laser_split(stack)
        shifts = P.estimate_shifts(lasers, device=True)
        reg, _ = K.register_assemble(lasers, shifts, True, cn_mode=1)
        cn, pt, _ = K.register_assemble_pixtable(lasers, shifts, True)
        refx = K.classify_prepare(torch.from_numpy(ref).cuda(), ECOLI, mode=2)
        a = K.classify_pixels_table(pt, refx, ref.shape[0])                 # sweep, then the certificate kernel
        f = K.classify_pixels_table(pt, refx, ref.shape[0], fused=True)     # the certificate in the sweep
        u = K.classify_pixels_table(pt, refx, ref.shape[0], composed=True)  # screen + classify_refine
        b = K.classify_pixels(reg, refx, ref.shape[0], ECOLI, mode=2)
        for v in (a, f, u):
            assert torch.equal(v[0], b[0]) and torch.equal(v[1], b[1])
        x = host(reg).reshape(H * W, -1).astype(np.float64)
        check_pixel_argmin(orc, host(a[0]).ravel(), host(a[1]).ravel(), x, ref.astype(np.float64), ECOLI)


@pytest.mark.parametrize("mode", [2, "table"])
def test_largest_library_exact(K, S, orc, mode):
    """R = 4095 (12-bit barcodes, LIST_RMAX = 4096: the list pass's 128 KB of LDS scores) with
    near-duplicate rows, so the list pass runs at the largest library the refine accepts; one
    row more is refused"""
    from test_kernels_gpu import check_pixel_argmin
    bounds = ECOLI
    ref = S.reference_library(12, bounds).astype(np.float32).copy()
    R, C = ref.shape
    assert R == 4095
    rng = np.random.default_rng(5)
    ref[R // 2:R // 2 + 64] = ref[:64] * np.float32(1 + 3e-7)   # near ties the screen cannot separate
    x = ref[rng.integers(0, R, 4096)] * rng.uniform(0.5, 1, (4096, 1)) + rng.normal(0, 0.01, (4096, C))
    x = np.clip(x, 0, None).astype(np.float32)
    st = dev(x.reshape(64, 64, C))
    if mode == "table":
        refx = K.classify_prepare(dev(ref), bounds, mode=2)
        gi, gd, n = K.classify_pixels_table(K.pixtable_prepare(st, bounds), refx, R, want_listed=True)
        assert n > 0
    else:
        refx = K.classify_prepare(dev(ref), bounds, mode=2)
        gi, gd = K.classify_pixels(st, refx, R, bounds)
    check_pixel_argmin(orc, host(gi).ravel(), host(gd).ravel(), x.astype(np.float64), ref.astype(np.float64), bounds)
    big = np.concatenate([ref, ref[:2]])
    with pytest.raises(Exception):
        K.classify_prepare(dev(big), bounds, mode=2)


@pytest.mark.parametrize("npx", [1, 5, 63, 65, 191, 193, 257])
def test_small_and_ragged_pixel_counts(K, S, orc, npx):
    """pixel counts that end inside a 16-pixel group, a 64-pixel certificate wave, a 192-pixel screen
    workgroup and a 256-pixel table block: both screens and the exact answers on every pixel"""
    from test_kernels_gpu import check_pixel_argmin
    bounds = ECOLI
    ref = S.reference_library(10, bounds).astype(np.float32)
    R, C = ref.shape
    rng = np.random.default_rng(npx)
    x = ref[rng.integers(0, R, npx)] * rng.uniform(0.5, 1, (npx, 1)) + rng.normal(0, 0.02, (npx, C))
    x = np.clip(x, 0, None).astype(np.float32)
    st = dev(x.reshape(1, npx, C))
    refx = K.classify_prepare(dev(ref), bounds, mode=2)
    a = K.classify_pixels(st, refx, R, bounds)
    b = K.classify_pixels_table(K.pixtable_prepare(st, bounds), refx, R)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    check_pixel_argmin(orc, host(a[0]).ravel(), host(a[1]).ravel(), x.astype(np.float64), ref.astype(np.float64), bounds)
