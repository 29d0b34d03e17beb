"""Pin the CPU restatement (oracle/) against fixtures generated from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest


def test_tables(orc, golden):
    g2 = golden("neighbor2d")
    assert np.array_equal(orc.lp_table_2d(11, 9), g2["table"])
    g3 = golden("neighbor3d")
    assert np.array_equal(orc.lp_table_3d(11, 9, 9), g3["table"])
    # the centre tap is always the pixel itself
    assert (g2["table"][:, 5] == 5).all() and (g3["table"][:, 5] == 5).all()


@pytest.mark.parametrize("case", ["a", "d"])
def test_line_profile_2d(orc, golden, case):
    g = golden("neighbor2d")
    assert np.array_equal(orc.line_profile_2d(g["pad_" + case]), g["lp_" + case])


@pytest.mark.parametrize("case", ["a", "b", "c", "d"])
def test_enhance_2d_bitexact(orc, golden, case):
    g = golden("neighbor2d")
    got = orc.enhance_2d(g["pad_" + case])
    ref = g["final_" + case]
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(got[~np.isnan(ref)], ref[~np.isnan(ref)])
    if case == "c":
        assert np.isnan(ref).any()  # the flat-window NaN path is exercised


def test_line_profile_3d(orc, golden):
    g = golden("neighbor3d")
    assert np.array_equal(orc.line_profile_3d(g["pad_small"]), g["lp_small"])
    assert np.array_equal(orc.line_profile_3d_norm(g["pad"]), g["lp_norm"])


def test_enhance_3d_bitexact(orc, golden):
    g = golden("neighbor3d")
    assert np.array_equal(orc.enhance_3d(g["pad"]), g["final"])


@pytest.mark.parametrize("case", ["a", "b", "c"])
def test_memory_efficient_v3_on_defined_voxels(orc, golden, case):
    """neighbor.line_profile_memory_efficient_v3 (reference Cython output): bit-exact wherever
    the reference's unchecked reads stay inside the padded array"""
    g = golden("neighbor3d_v3")
    pad, want = g["pad_" + case], g["final_" + case]
    ok = orc.v3_defined(pad.shape)
    assert ok.any()
    assert np.array_equal(orc.enhance_3d_v3(pad)[ok], want[ok])


def test_v3_table_matches_generated_constants(orc):
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "hiprfish_image_analysis_amd", "csrc"))
    import gen_tables
    assert np.array_equal(orc.lp_table_3d_v3(), np.array(gen_tables.table_3d_v3()))


def test_metric_channel_cosine_intensity(orc, golden):
    g = golden("metrics")
    b = [0, 32, 55, 75, 89, 95]
    for i in range(len(g["d95"])):
        x, y = g["x95"][i], g["y95"][i]
        d = orc.segcos(x[:95], y[:95], b, 1, x[95:100], y[95:100])
        assert d == pytest.approx(g["d95"][i], rel=1e-12, abs=1e-12)


def test_metric_7b_v2(orc, golden):
    g = golden("metrics")
    b = [0, 23, 43, 57, 63]
    for i in range(len(g["d7b"])):
        x, y = g["x67"][i], g["y67"][i]
        d = orc.segcos(x[:63], y[:63], b, 2, x[63:67], y[63:67])
        assert d == pytest.approx(g["d7b"][i], rel=1e-12, abs=1e-12)


def test_metric_violet_derivative_segments(orc, golden):
    """_violet_derivative_v2 returns a 6-tuple (train_reference.py:731); its 5 spectral
    segment distances equal the gated per-segment distances of the 95-channel metric."""
    g = golden("metrics")
    b = [0, 32, 55, 75, 89, 95]
    for i in range(len(g["dvd"])):
        x, y = g["x132"][i], g["y132"][i]
        tup = g["dvd"][i]
        gate = np.sum(np.abs(x[126:132] - y[126:132])) < 0.01
        for s in range(5):
            single = [b[s], b[s + 1]]
            d = orc.segcos(x[:95], y[:95], single, 0)
            if gate and x[126 + s] == 0:
                d = 0.0
            assert d == pytest.approx(tup[1 + s], rel=1e-12, abs=1e-12)
        assert tup[0] == (0.0 if gate else 1.0)


def test_label_raster_numbering(orc, golden):
    g = golden("label")
    l8, _ = orc.label(g["mask"].astype(np.int32), conn=2)
    l4, _ = orc.label(g["mask"].astype(np.int32), conn=1)
    assert np.array_equal(l8, g["l8"])
    assert np.array_equal(l4, g["l4"])


@pytest.mark.parametrize("shape,h,sigma", [((40, 52), 0.02, 0.0), ((33, 29), 0.1, 0.0), ((7, 5), 0.05, 0.01),
                                           ((1, 9), 0.05, 0.0)])
def test_nl_means_restatement_equals_integral_image_algorithm(orc, shape, h, sigma):
    """a4: the per-pixel formulation libhrf computes (oracle_nl_means) equals skimage's
    integral-image / symmetric-pair algorithm (oracle_nl_means_skimage) to rounding.
    skimage itself is absent: parity to skimage is unpinned."""
    rng = np.random.default_rng(sum(shape))
    yy, xx = np.mgrid[0:shape[0], 0:shape[1]]
    img = 0.5 + 0.3 * np.sin(yy / 6.0) * np.cos(xx / 5.0) + 0.01 * rng.standard_normal(shape)
    a = orc.nl_means(img, 7, 11, h, sigma)
    b = orc.nl_means_skimage(img, 7, 11, h, sigma)
    np.testing.assert_allclose(a, b, rtol=1e-11, atol=0)
    assert np.abs(a - img).max() > 1e-4          # it actually denoises


def test_register_translation_restatement(orc):
    """f1: numpy restatement of skimage.feature.register_translation recovers known shifts"""
    rng = np.random.default_rng(1)
    img = rng.random((64, 80))
    for dr, dc in [(3, -5), (-7, 2), (0, 0), (15, 15)]:
        moved = np.roll(img, (dr, dc), axis=(0, 1))
        assert tuple(orc.register_translation(img, moved)) == (-dr, -dc)


def _same_partition(a, b):
    pairs = set(zip(a.tolist(), b.tolist()))
    return len(pairs) == len(set(a.tolist())) == len(set(b.tolist()))


@pytest.mark.parametrize("name", ["bimodal", "logsum", "trimodal"])
def test_kmeans_matches_sklearn(orc, golden, name):
    """a8: the sklearn restatement (kmeans_sk.c, numpy's random stream replayed) returns
    sklearn 1.7.2's own labels -- the cluster ids, not only the partition"""
    g = golden("kmeans")
    x = g["x_" + name]
    k = int(g["k_" + name])
    lab, cen, info = orc.kmeans_sk(x, k)
    assert np.array_equal(lab, g["lab_" + name])
    lab3, _, _ = orc.kmeans_sk(x, 3)
    assert np.array_equal(lab3, g["lab3_" + name])


@pytest.mark.parametrize("block", range(4))
def test_watershed_order_model_equals_heap(orc, block):
    """a12: the flow libhrf's watershed implements (oracle/ws_order.c: keys (lambda, h),
    candidate strings, and -- when a decision comes down to equal-valued markers of different
    labels, which skimage settles by its binary heap's layout -- the heap flood again) gives the
    heap flood's label map (oracle_watershed, skimage's (value, age) binary heap) on
    plateau-heavy integer images, unconditionally.  Both the ordered walk and the fallback
    are exercised (the even seeds carry equal-valued markers)."""
    decided_by_layout = 0
    for seed in range(block * 150, (block + 1) * 150):
        rng = np.random.default_rng(seed)
        H, W = 10 + seed % 37, 10 + (seed * 7) % 41
        f = rng.integers(0, 2 + seed % 5, (H, W)).astype(np.float64)
        mask = rng.random((H, W)) < 0.85 if seed % 4 else None
        markers = np.zeros((H, W), np.int32)
        idx = rng.choice(H * W, max(2, H * W // 60), replace=False)
        markers.flat[idx] = rng.integers(1, 6, idx.size)
        if seed % 2:
            f = f + 1e-3 * markers       # no equal-valued markers of different labels
        ref = orc.watershed(f, markers, mask)
        got, st = orc.watershed_ordered(f, markers, mask)
        assert np.array_equal(got, ref), seed
        if st[2]:
            assert seed % 2 == 0
            decided_by_layout += 1
    assert 0 < decided_by_layout < 150


@pytest.mark.parametrize("key", ["2_ecoli_a", "3_ecoli_a", "2_ecoli_q", "3_ecoli_q", "2_community_final",
                                 "2_community_nl"])
def test_kmeans_matches_sklearn_on_images(orc, golden, key):
    """a8 on the images the reference clusters (ecoli image_cn k=2/3 :73-94, community final and
    NL-means k=2 :125/:141; 256^2 synthetic tiles, one 12-bit quantised whose k=3 fit a
    deterministic init gets wrong): sklearn's labels, ids included"""
    g = golden("kmeans_images")
    k = int(key[0])
    name = key[2:]
    lab, cen, info = orc.kmeans_sk(g["x_" + name].ravel(), k)
    assert np.array_equal(lab, g["lab%d_%s" % (k, name)].ravel().astype(np.int32))


def test_kmeans_random_stream_matches_numpy(orc):
    """the restatement's random stream is numpy's RandomState(0) as sklearn's KMeans.fit draws it"""
    first, draws = orc.kmeans_draws(1000, 3)
    rs = np.random.RandomState(0)
    for r in range(10):
        assert first[r] == rs.choice(1000, p=np.ones(1000) / 1000)
        assert np.array_equal(draws[r * 6:(r + 1) * 6], np.concatenate([rs.uniform(size=3), rs.uniform(size=3)]))


@pytest.mark.parametrize("block", range(3))
def test_kmeans_matches_sklearn_random(orc, block):
    """sklearn KMeans(k, random_state=0, n_init=10) on assorted 1-D data, labels equal (values
    jittered below 1e-9: an exact midpoint tie is decided by sklearn's rounding of its centred
    expansion, which the restatement does not reproduce -- DESIGN.md)"""
    from sklearn.cluster import KMeans
    rng = np.random.default_rng(block)
    for t in range(12):
        n = int(rng.integers(30, 4000))
        k = int(rng.integers(1, 6))
        kind = t % 4
        if kind == 0:
            x = rng.normal(size=n)
        elif kind == 1:
            x = np.concatenate([rng.normal(0, 1, n // 2), rng.normal(5, 0.5, n - n // 2)])
        elif kind == 2:
            x = np.round(rng.gamma(2, 1, n) * 4) / 4 + rng.random(n) * 1e-9
        else:
            x = np.log(rng.integers(0, 40, n) + 0.01) + rng.random(n) * 1e-10
        lab, cen, info = orc.kmeans_sk(x, k)
        sk = KMeans(n_clusters=k, random_state=0, n_init=10).fit(x.reshape(-1, 1))
        assert np.array_equal(lab, sk.labels_), (block, t, n, k)


# ---- a9 / a11 / a13 morphology pinned to scipy.ndimage (make_golden.py morphology) -----------
def _morph_names(g):
    return sorted(k[2:] for k in g.files if k.startswith("m_"))


def test_morphology_primitives_match_scipy(orc, golden):
    """skimage 0.14's binary morphology is scipy.ndimage underneath: binary_erosion(cross,
    border_value=True) (ecoli :107, :122), binary_dilation, binary_opening = dilation(erosion)
    (:95, multispecies :136), remove_small_objects / remove_small_holes as ndi.label + bincount
    sieves (:95-96, :108, :111), binary_fill_holes (multispecies :138-139)"""
    g = golden("morphology")
    names = _morph_names(g)
    assert len(names) >= 10
    for n in names:
        m = g["m_" + n]
        assert np.array_equal(orc.erode(m, 1), g["ero_" + n]), n
        assert np.array_equal(orc.dilate(m), g["dil_" + n]), n
        assert np.array_equal(orc.opening(m), g["open_" + n]), n
        assert np.array_equal(orc.remove_small_objects_mask(m, 50, 1), g["rso50c1_" + n]), n
        assert np.array_equal(orc.remove_small_objects_mask(m, 10, 1), g["rso10c1_" + n]), n
        assert np.array_equal(orc.remove_small_objects_mask(m, 10, 2), g["rso10c2_" + n]), n
        assert np.array_equal(orc.remove_small_holes(m, 64, 1), g["rsh64_" + n]), n
        assert np.array_equal(orc.fill_holes(m), g["fill_" + n]), n
        cs = orc.remove_small_objects_mask(orc.opening(orc.remove_small_holes(m, 64, 1)), 50, 1)
        assert np.array_equal(cs, g["cellsm_" + n]), n


def test_erosion_seed_loop_matches_scipy(orc, golden):
    """ecoli :97-112 (freeze < 600 px, erode, sieve < 10 px, repeat; then
    label(rso(label(dist_be), 10))) composed from scipy.ndimage equals the restatement"""
    import pipeline as OP
    g = golden("morphology")
    seen = 0
    for n in _morph_names(g):
        if "be_" + n not in g.files:
            continue
        be = OP.erosion_seeds(g["m_" + n])
        assert np.array_equal(be, g["be_" + n]), n
        seeds, _ = orc.label(orc.remove_small_objects_mask(be, 10, 2).astype(np.int32), 2)
        assert np.array_equal(seeds, g["seeds_" + n]), n
        seen += int(g["seeds_" + n].max())
    assert seen > 80


def test_cr_log_is_correctly_rounded(orc):
    """detmath.h hrf_cr_log / hrf_cr_log10 (image_cn, ecoli :72; biofilm :831) against Python's
    decimal ln / log10 at 50 digits, on the image_cn range, near 1, at the table knots, across
    the exponent range and on subnormals"""
    import decimal
    decimal.getcontext().prec = 50
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(0.01, 96.0, 6000), np.exp(rng.uniform(-744, 709, 2000)),
                        1 + rng.uniform(-1e-3, 1e-3, 1000), 1 + rng.uniform(-1e-13, 1e-13, 300),
                        np.arange(96, 193) / 128.0, np.nextafter(np.arange(96, 193) / 128.0, 0),
                        2.0 ** np.arange(-1074, 1024, 11.0), [5e-324, 2.2e-308, 1.7976931348623157e308, 1.0,
                                                             0.01, 10.0, 100.0, 1e-2 + 1.0]])
    got = orc.cr_log(x)
    want = np.array([float(decimal.Decimal(v).ln()) for v in x])
    assert np.array_equal(got, want)
    got10 = orc.cr_log10(x)
    want10 = np.array([float(decimal.Decimal(v).log10()) for v in x])
    assert np.array_equal(got10, want10)
    assert orc.cr_log(np.array([0.0]))[0] == -np.inf and np.isnan(orc.cr_log(np.array([-1.0]))[0])


def test_flat_field_division_through_reciprocal(orc):
    """detmath.h hrf_div_rcp (the lasers label sums' flat-field division, ecoli :41 image /
    calibration_norm, with both operands float32 values): equal to the IEEE quotient on 2e7
    random and directed float pairs"""
    import ctypes
    f = orc.lib().oracle_div_rcp_check
    f.restype = ctypes.c_int64
    assert f(ctypes.c_uint64(7), ctypes.c_int64(20_000_000)) == 0


def test_nl_means_widened_exp_table(orc):
    """nlmeans.hip's exponential (hrf_exp_neg_tabw: 740-entry table, no ldexp) equals the
    oracle's hrf_exp_neg_tab bit for bit over [-8, 0] and at every rounding boundary of k"""
    import ctypes
    f = orc.lib().oracle_exp_tabw_check
    f.restype = ctypes.c_int64
    assert f(ctypes.c_int64(4_000_000)) == 0
