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
                       ref.astype(np.float64), S.ECOLI_BOUNDS, 0.5)


def test_fullsize_community_tile(mods, orc):
    P, S, OP = mods
    b = P.MULTI_BOUNDS
    stack, _, _, ref = S.tile(2048, 2048, nbit=7, bounds=b, seed=20190201)
    stack = quantised(stack, 4095)
    assert stack.shape == (2048, 2048, 63) and ref.shape[0] == 127
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), b, 7)
    res = P.process_tile(stack, lib, per_pixel=False, measure=P.measure_multispecies, variant=2)
    oseg, olabs, oavg, oavgn = OP.measure_multispecies(host(stack))
    assert np.array_equal(host(res.meas.segmentation), oseg)
    assert np.array_equal(host(res.meas.labels), olabs) and len(olabs) > 500
    np.testing.assert_allclose(host(res.meas.avgint), oavg, rtol=1e-12)
    oidx, odist = OP.classify_cells(oavgn, ref, b, variant=2)
    np.testing.assert_allclose(host(res.cell_dist), odist, rtol=1e-9, atol=1e-12)
    assert np.array_equal(host(res.cell_idx), oidx)
    assert np.array_equal(host(res.counts), orc.barcode_counts(oidx, 127))
