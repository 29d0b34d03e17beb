"""The biofilm per-cell report (biofilm :1214-1295) on a synthetic community field with a
classifier bundle fitted here (sklearn SVCs with probability=True, a stand-in UMAP): file
layouts, predict_proba / max_probability against sklearn, debris typing and both adjacency
matrices against the restatement."""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _field(H, W, rng, n=120):
    pts = rng.uniform(0, H, (n, 2))
    yy, xx = np.mgrid[0:H, 0:W]
    d = (yy.ravel()[:, None] - pts[:, 0]) ** 2 + (xx.ravel()[:, None] - pts[:, 1]) ** 2
    seg = (np.argmin(d, axis=1) + 1).astype(np.int32)
    seg[np.min(d, axis=1) > 11.0 ** 2] = 0
    seg = seg.reshape(H, W)
    labs = np.unique(seg)
    labs = labs[labs > 0]
    remap = np.zeros(seg.max() + 1, np.int32)
    remap[labs] = np.arange(1, len(labs) + 1)
    return remap[seg], len(labs)


def test_cell_report(tmp_path, orc):
    from types import SimpleNamespace

    from sklearn.preprocessing import StandardScaler
    from sklearn.svm import SVC
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tools.export_classifier import export_bundle
    from hiprfish_image_analysis_amd import backend as B, biofilm, kernels as K
    rng = np.random.default_rng(31)
    H = W = 192
    seg, N = _field(H, W, rng)
    spectra = rng.random((6, 63)) ** 2 + 0.05
    kind = rng.integers(0, 6, N + 1)
    stack = (spectra[kind[seg]] * (seg > 0)[..., None] + 0.01 * rng.random((H, W, 63))).astype(np.float32)
    # training set of the bundle
    y = np.repeat(np.arange(6), 30)
    xt = spectra[y] * rng.uniform(0.8, 1.2, (len(y), 1)) + rng.normal(0, 0.02, (len(y), 63))
    xt /= xt.max(axis=1, keepdims=True)
    sc = StandardScaler().fit(xt)
    xs = sc.transform(xt)
    feats = np.zeros((len(y), 67))
    feats[:, :63] = xt
    checks = []
    for k, (lo, hi) in enumerate(B.MULTI_SEGMENTS):
        seg_max = xt[:, lo:hi].max(axis=1)
        lab = np.zeros(len(y))
        lab[np.argsort(seg_max, kind="stable")[len(y) // 2:]] = 1.0      # two classes always
        checks.append(SVC(kernel="linear", C=1.0).fit(xs[:, lo:hi], lab))
        feats[:, 63 + k] = checks[-1].predict(xs[:, lo:hi])
    emb = (rng.normal(0, 5, (6, 2))[y] + rng.normal(0, 0.4, (len(y), 2))).astype(np.float32)
    codes = np.array([format(v + 1, "07b") for v in y])
    clf_umap = SVC(kernel="rbf", gamma=0.5, C=10.0, probability=True, random_state=0).fit(emb.astype(float), codes)
    um = SimpleNamespace(_raw_data=feats, embedding_=emb, n_neighbors=15, local_connectivity=1.0,
                         metric=SimpleNamespace(__name__="channel_cosine_intensity_7b_v2"), _a=1.577, _b=0.8951,
                         repulsion_strength=1.0, negative_sample_rate=5, n_epochs=None, _initial_alpha=1.0)
    path = str(tmp_path / "bundle.npz")
    export_bundle(path, um, clf_umap, checks, sc)
    model = B.ClassifierModel.load(path)
    taxon_codes = [format(v + 1, "07b") for v in range(5)]        # one class missing from the lookup
    epi = np.zeros((H, W), np.uint8)
    epi[:20] = 1
    sample = str(tmp_path / "bf")
    first = biofilm.cell_report(sample, torch.from_numpy(stack).cuda(), torch.from_numpy(seg).cuda(),
                                torch.from_numpy(seg).cuda(), model, taxon_codes, torch.from_numpy(epi).cuda(),
                                write=False)
    # the reference's 0.95 cut, moved to this model's median so both types occur
    prob_min = float(np.median(first["cell_info"].max_probability))
    out = biofilm.cell_report(sample, torch.from_numpy(stack).cuda(), torch.from_numpy(seg).cuda(),
                              torch.from_numpy(seg).cuda(), model, taxon_codes, torch.from_numpy(epi).cuda(),
                              prob_min=prob_min)
    ci = out["cell_info"]
    assert list(ci.columns[:63]) == ["channel_{}".format(i) for i in range(63)]
    assert list(ci.columns[63:69]) == ["intensity_classification_{}".format(i) for i in range(4)] + [
        "cell_barcode", "max_probability"]
    assert list(ci.columns[-12:]) == ["sample", "label", "centroid_x", "centroid_y", "major_axis", "minor_axis",
                                      "eccentricity", "orientation", "area", "epithelial_distance",
                                      "max_intensity", "type"]
    assert len(ci) == N and list(ci.label) == list(range(1, N + 1))
    # predict_proba of the device embedding, by sklearn itself
    feats_dev = model.features(K.cell_table(*K.label_sums(torch.from_numpy(stack).cuda(), torch.from_numpy(seg).cuda(),
                                                          N), N)[3])
    e = model.umap.transform(feats_dev).double().cpu().numpy()
    np.testing.assert_allclose(ci[[c + "_prob" for c in clf_umap.classes_]].values, clf_umap.predict_proba(e),
                               rtol=0, atol=1e-12)
    # typing (area > 10000 never here; epithelial overlap; max probability <= 0.95)
    debris = set(np.unique(seg * epi)) - {0}
    want = np.array([not ((i + 1) in debris or ci.max_probability[i] <= prob_min) for i in range(N)])
    assert np.array_equal(ci.type.values == "cell", want)
    assert 0 < want.sum() < N
    fil = out["cell_info_filtered"]
    assert list(fil.label) == [i + 1 for i in range(N) if want[i]]
    # adjacency: rows / columns the taxon codes, counts from both endpoints, barcodes outside
    # the lookup not counted
    idx = {c: i for i, c in enumerate(taxon_codes)}
    bc = np.array([-1] + [idx.get(c, -1) for c in ci.cell_barcode], np.int32)
    e_ = orc.rag_edges(seg, N)
    assert np.array_equal(out["adjacency"].values.astype(np.int64), orc.barcode_adjacency(e_, bc, 5))
    bcf = np.where(np.concatenate([[False], want]), bc, -1).astype(np.int32)
    assert np.array_equal(out["adjacency_filtered"].values.astype(np.int64), orc.barcode_adjacency(e_, bcf, 5))
    for suffix in ("_cell_information.csv", "_cell_information_filtered.csv", "_avgint.csv", "_avgint_filtered.csv",
                   "_adjacency_matrix.csv", "_adjacency_matrix_filtered.csv"):
        assert os.path.exists(sample + suffix)
    import pandas as pd
    adj = pd.read_csv(sample + "_adjacency_matrix.csv", index_col=0, dtype={0: str})
    assert list(adj.columns) == taxon_codes
