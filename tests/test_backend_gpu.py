"""The classifier back-end on the device (backend.hip through libhrf.so) against sklearn's
outputs (backend.npz) and the oracle.  SVC predict, the scaler, the kNN search and the
feature tables are exact-order f64 restatements: class decisions bit-exact, decision values
and distances within 1e-12 (exp/tanh/sqrt of the device libm vs glibc).  UMAP initialisation
against the oracle only (parity unpinned, umap-learn absent)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from hiprfish_image_analysis_amd import backend as B  # noqa: E402
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402

SVC_CASES = ["rbf5", "lin2", "poly3", "sig2", "rbf40"]


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()


def model(g, name):
    return B.SvcModel.from_npz(g, name + "_")


@pytest.mark.parametrize("name", SVC_CASES)
def test_svc_predict(golden, orc, name):
    g = golden("backend")
    m = model(g, name)
    x = g[name + "_x"]
    pred, dec = K.svc_predict(dev(x), m, want_dec=True)
    pred = pred.cpu().numpy()
    assert np.array_equal(g[name + "_classes"][pred], g[name + "_pred"])
    want = g[name + "_dec"]
    if m.n_class == 2:
        want = -want.reshape(-1, 1)
    np.testing.assert_allclose(dec.cpu().numpy(), want, rtol=1e-12, atol=1e-12)
    # and bit-equal class decisions with the oracle
    opred = orc.svc_predict(x, m.sv.cpu().numpy(), m.coef.cpu().numpy(), m.intercept.cpu().numpy(),
                            m.start.cpu().numpy(), m.kernel, m.gamma, m.coef0, m.degree)
    assert np.array_equal(pred, opred)


def test_svc_predict_into_column_of_wider_table(golden):
    """the flag-column path: input a column slice, output written into another column"""
    g = golden("backend")
    m = model(g, "poly3")
    x = g["poly3_x"]
    table = torch.zeros((len(x), 12), dtype=torch.float64, device="cuda")
    table[:, 2:8] = dev(x)
    pred = m.predict(table[:, 2:8], out_column=table[:, 10])
    t = table.cpu().numpy()
    assert np.array_equal(t[:, 10], g["poly3_pred"])
    assert np.array_equal(t[:, 2:8], x) and not t[:, [0, 1, 8, 9, 11]].any()
    assert np.array_equal(g["poly3_classes"][pred.cpu().numpy()], g["poly3_pred"])


def test_svc_empty_and_mismatch(golden):
    g = golden("backend")
    m = model(g, "rbf5")
    assert K.svc_predict(torch.empty((0, 3), dtype=torch.float64, device="cuda"), m).numel() == 0
    with pytest.raises(ValueError):
        K.svc_predict(dev(np.zeros((4, 5))), m)


def test_standard_scale(golden):
    g = golden("backend")
    wide = torch.zeros((50, 70), dtype=torch.float64, device="cuda")
    wide[:, 3:66] = dev(g["scaler_x"])
    out = K.standard_scale(wide[:, 3:66], dev(g["scaler_mean"]), dev(g["scaler_scale"]))
    np.testing.assert_allclose(out.cpu().numpy(), g["scaler_out"], rtol=0, atol=1e-15)


@pytest.mark.parametrize("name,metric", [("knn7b", "channel_cosine_intensity_7b_v2"),
                                         ("knnviolet", "channel_cosine_intensity_violet_derivative_v2")])
def test_knn_matches_sklearn(golden, orc, name, metric):
    g = golden("backend")
    trT = dev(g[name + "_train"].T)
    idx, dist = K.knn(dev(g[name + "_q"]), trT, metric, 15)
    dist = dist.cpu().numpy()
    np.testing.assert_allclose(dist, g[name + "_dist"], rtol=0, atol=1e-13)
    from test_backend_oracle import assert_same_neighbours
    assert_same_neighbours(idx.cpu().numpy(), dist, g[name + "_idx"])
    # the lower-row tie rule the oracle states, exactly
    oi, _ = orc.knn(g[name + "_q"], g[name + "_train"], 1 if "7b" in name else 2, 15)
    assert np.array_equal(idx.cpu().numpy(), oi)


@pytest.mark.parametrize("metric", [0, 1, 2])
@pytest.mark.parametrize("k", [1, 15, 64])
def test_knn_random_vs_oracle(orc, metric, k):
    rng = np.random.default_rng(100 + metric * 7 + k)
    f = (20, 67, 132)[metric]
    tr = rng.random((3000, f))
    q = rng.random((700, f))
    if metric:
        fl = (63, 67) if metric == 1 else (126, 132)
        tr[:, fl[0]:fl[1]] = (rng.random((3000, fl[1] - fl[0])) < 0.8)
        q[:, fl[0]:fl[1]] = (rng.random((700, fl[1] - fl[0])) < 0.8)
    idx, dist = K.knn(dev(q), dev(tr.T), metric, k)
    oi, od = orc.knn(q, tr, metric, k)
    np.testing.assert_allclose(dist.cpu().numpy(), od, rtol=0, atol=1e-13)
    # ties (metric 1 returns exactly 1.0 for a flag mismatch) resolve to the lower row
    assert np.array_equal(idx.cpu().numpy(), oi)


def test_knn_fewer_train_rows_than_k(orc):
    rng = np.random.default_rng(5)
    tr, q = rng.random((5, 8)), rng.random((9, 8))
    idx, dist = K.knn(dev(q), dev(tr.T), 0, 8)
    oi, od = orc.knn(q, tr, 0, 8)
    assert np.array_equal(idx.cpu().numpy(), oi)
    assert np.array_equal(np.isinf(dist.cpu().numpy()), np.isinf(od))


@pytest.mark.parametrize("lc", [0.0, 1.0, 1.5])
def test_umap_init_vs_oracle(orc, golden, lc):
    g = golden("backend")
    idx, dist = orc.knn(g["knnviolet_q"], g["knnviolet_train"], 2, 15)
    rng = np.random.default_rng(11)
    emb = rng.normal(size=(len(g["knnviolet_train"]), 2)).astype(np.float32)
    out, memb = K.umap_init_transform(torch.from_numpy(idx).cuda(), dev(dist), torch.from_numpy(emb).cuda(), 15, lc,
                                      want_memb=True)
    want, wmemb = orc.umap_init(idx, dist, emb, 15.0, lc, want_memb=True)
    # exp written out in IEEE operations on both sides (csrc/detmath.h): bit-exact
    assert np.array_equal(memb.cpu().numpy(), wmemb)
    assert np.array_equal(out.cpu().numpy(), want)


def test_umap_refine_vs_oracle(orc, golden):
    """the layout refinement on the same float32 inputs: same per-cell streams, same schedule,
    float32 state with f64 gradients, pow from csrc/detmath.h on both sides: bit-exact"""
    g = golden("backend")
    idx, dist = orc.knn(g["knn7b_q"], g["knn7b_train"], 1, 15)
    rng = np.random.default_rng(12)
    emb = (rng.normal(size=(len(g["knn7b_train"]), 2)) * 4).astype(np.float32)
    init, memb = orc.umap_init(idx, dist, emb, 15.0, 0.0, want_memb=True)
    for ne, seed in ((100, 0), (30, 77)):
        want = orc.umap_refine(idx, memb, init, emb, ne, 1.577, 0.8951, 1.0, 0.25, 5.0, seed=seed)
        got = K.umap_refine(torch.from_numpy(idx).cuda(), torch.from_numpy(memb).cuda(), torch.from_numpy(init).cuda(),
                            torch.from_numpy(emb).cuda(), ne, 1.577, 0.8951, 1.0, 0.25, 5.0, seed=seed).cpu().numpy()
        assert np.array_equal(got, want)


def _random_svc(rng, ncls, f, kernel="rbf"):
    nsv = rng.integers(3, 8, ncls)
    sv = rng.random((int(nsv.sum()), f))
    dual = rng.normal(size=(ncls - 1, int(nsv.sum())))
    inter = rng.normal(size=ncls * (ncls - 1) // 2) * 0.1
    return B.SvcModel.from_arrays(sv, dual, inter, nsv, np.arange(ncls, dtype=np.float64), kernel, gamma=0.5)


def test_features_and_classify_chain(orc):
    """E. coli bundle: features (diff + check flags), kNN under the violet-derivative metric,
    UMAP init, SVC on the embedding -- each stage against the oracle on the same inputs"""
    rng = np.random.default_rng(21)
    n = 500
    avg = rng.random((n, 95))
    avg /= avg.max(axis=1, keepdims=True)
    checks = [_random_svc(rng, 2, hi - lo) for lo, hi in B.ECOLI_SEGMENTS]
    feats = B.features_ecoli(dev(avg), checks).cpu().numpy()
    want = np.zeros((n, 132))
    want[:, :95] = avg
    want[:, 95:126] = np.diff(avg[:, :32], axis=1)
    for k, (lo, hi) in enumerate(B.ECOLI_SEGMENTS):
        c = checks[k]
        p = orc.svc_predict(want[:, lo:hi], c.sv.cpu().numpy(), c.coef.cpu().numpy(), c.intercept.cpu().numpy(),
                            c.start.cpu().numpy(), c.kernel, c.gamma, c.coef0, c.degree)
        want[:, 126 + k] = p
    np.testing.assert_array_equal(feats, want)
    assert 0 < want[:, 126:].mean() < 1     # both flag values occur

    tr = np.vstack([want[:200] + 0.0, rng.random((300, 132))])
    tr[200:, 126:] = (rng.random((300, 6)) < 0.5)
    emb = rng.normal(size=(500, 2)).astype(np.float32)
    um = B.UmapModel(dev(tr.T), torch.from_numpy(emb).cuda(), 15, 1.0, "channel_cosine_intensity_violet_derivative_v2")
    svc = _random_svc(rng, 7, 2)
    bundle = B.ClassifierModel(checks, um, svc)
    cls, classes, f2 = bundle.classify(dev(avg))
    oi, od = orc.knn(want, tr, 2, 15)
    e, memb = orc.umap_init(oi, od, emb, 15.0, 0.0, want_memb=True)
    e = orc.umap_refine(oi, memb, e, emb, 100, um.a, um.b, 1.0, 0.25, 5.0, seed=0).astype(np.float64)
    op = orc.svc_predict(e, svc.sv.cpu().numpy(), svc.coef.cpu().numpy(), svc.intercept.cpu().numpy(),
                         svc.start.cpu().numpy(), svc.kernel, svc.gamma, svc.coef0, svc.degree)
    got = cls.cpu().numpy()
    # every stage in the same operation order with the same exp / pow: the embedding and the
    # SVC decisions are bit-equal, so every cell's class is
    assert np.array_equal(got, op)


def test_features_multi_with_scaler(orc):
    rng = np.random.default_rng(22)
    n = 300
    avg = rng.random((n, 63))
    mean, scale = rng.random(63), rng.uniform(0.5, 2, 63)
    checks = [_random_svc(rng, 2, hi - lo, "linear") for lo, hi in B.MULTI_SEGMENTS]
    feats = B.features_multi(dev(avg), dev(mean), dev(scale), checks).cpu().numpy()
    sc = (avg - mean) / scale
    assert np.array_equal(feats[:, :63], avg)
    for k, (lo, hi) in enumerate(B.MULTI_SEGMENTS):
        c = checks[k]
        p = orc.svc_predict(sc[:, lo:hi], c.sv.cpu().numpy(), c.coef.cpu().numpy(), c.intercept.cpu().numpy(),
                            c.start.cpu().numpy(), c.kernel, c.gamma, c.coef0, c.degree)
        assert np.array_equal(feats[:, 63 + k], p.astype(np.float64))


@pytest.mark.parametrize("name", ["prob2", "prob6", "prob30"])
def test_svc_predict_proba(golden, orc, name):
    """biofilm :1229 predict_proba against sklearn itself (its libsvm sums kernel values with
    BLAS ddot, so agreement is to ~1e-15, not bit for bit) and the oracle's libsvm restatement"""
    g = golden("backend")
    m = model(g, name)
    x = g[name + "_x"]
    prob = m.predict_proba(dev(x)).cpu().numpy()
    np.testing.assert_allclose(prob, g[name + "_proba"], rtol=0, atol=1e-12)
    op = orc.svc_proba(x, m.sv.cpu().numpy(), m.coef.cpu().numpy(), m.intercept.cpu().numpy(), m.start.cpu().numpy(),
                       m.kernel, m.gamma, m.coef0, m.degree, m.probA.cpu().numpy(), m.probB.cpu().numpy())
    np.testing.assert_allclose(prob, op, rtol=0, atol=1e-13)
    np.testing.assert_allclose(prob.sum(axis=1), 1.0, atol=1e-12)


def test_biofilm_typing_and_filtered_adjacency(orc):
    """biofilm :1259-1295: debris typing (area, epithelial overlap, max probability) and the raw
    and cell-filtered barcode adjacency matrices, against the restatement (rag_boundary edges
    counted from both endpoints; filtered = the same count over 'cell' rows only)"""
    from hiprfish_image_analysis_amd import pipeline as P
    H = W = 256
    rng = np.random.default_rng(6)
    # a packed biofilm-like field: nearest-seed cells, background where no seed is near
    pts = rng.uniform(0, 256, (150, 2))
    yy, xx = np.mgrid[0:H, 0:W]
    d = (yy.ravel()[:, None] - pts[:, 0]) ** 2 + (xx.ravel()[:, None] - pts[:, 1]) ** 2
    seg = (np.argmin(d, axis=1) + 1).astype(np.int32)
    seg[np.min(d, axis=1) > 12.0 ** 2] = 0
    seg = seg.reshape(H, W)
    labs = np.unique(seg)
    labs = labs[labs > 0]
    remap = np.zeros(seg.max() + 1, np.int32)       # sequential labels, as the reference assumes
    remap[labs] = np.arange(1, len(labs) + 1)
    seg = remap[seg]
    N = len(labs)
    bc = rng.integers(0, 31, N).astype(np.int32)
    prob = rng.uniform(0.8, 1.0, N)
    prob[::7] = np.nan
    epi = np.zeros((H, W), np.uint8)
    epi[:40, :] = 1
    area = np.bincount(seg.ravel(), minlength=N + 1)[1:].astype(np.float64)
    area_max = float(np.percentile(area, 90))
    res = P.biofilm_typing_and_adjacency(torch.from_numpy(seg).cuda(), torch.from_numpy(seg).cuda(),
                                         torch.from_numpy(bc).cuda(), 31, dev(prob), torch.from_numpy(epi).cuda(),
                                         area_max=area_max)
    debris_labels = set(np.unique(seg * epi)) - {0}
    want_cell = np.array([not (area[i] > area_max or (i + 1) in debris_labels or prob[i] <= 0.95)
                          for i in range(N)])
    assert np.array_equal(res.is_cell.cpu().numpy().astype(bool), want_cell)
    assert 0 < want_cell.sum() < N
    e = orc.rag_edges(seg, N)
    bcl = np.concatenate([[-1], bc]).astype(np.int32)
    assert np.array_equal(res.adjacency.cpu().numpy(), orc.barcode_adjacency(e, bcl, 31))
    bcf = np.where(np.concatenate([[False], want_cell]), bcl, -1).astype(np.int32)
    assert np.array_equal(res.adjacency_filtered.cpu().numpy(), orc.barcode_adjacency(e, bcf, 31))
    assert res.adjacency_filtered.sum() < res.adjacency.sum()
