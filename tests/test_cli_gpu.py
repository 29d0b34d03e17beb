"""The drop-in stage scripts (hiprfish_image_analysis_amd/scripts/) end to end on synthetic
per-laser images written as {stem}.npy: registration estimate -> measurement -> files, then
classification of the written spectra; outputs checked against the oracle restatement."""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprfish_image_analysis_amd", "scripts"))


def split_lasers(stack, bounds, shifts):
    """(H, W, C) -> per-laser stacks, laser i displaced so that the reference registration
    (dst[r] = src[r - shift]) undoes it"""
    out = []
    for i, (dr, dc) in enumerate(shifts):
        out.append(np.ascontiguousarray(np.roll(stack[:, :, bounds[i]:bounds[i + 1]], (-dr, -dc), axis=(0, 1))))
    return out


def test_ecoli_measurement_cli(tmp_path, orc):
    import pipeline as OP
    import hiprfish_imaging_spectral_image_measurement as cli

    from hiprfish_image_analysis_amd import synthetic as S
    stack, _, _, _ = S.tile(256, 256, seed=31)
    lasers = split_lasers(stack.cpu().numpy(), S.ECOLI_BOUNDS, [(0, 0), (2, -1), (0, 3), (-1, 0), (1, 1)])
    files = []
    for i, l in enumerate(lasers):
        np.save(tmp_path / ("s_%d.npy" % (i + 1)), l)
        files.append(str(tmp_path / ("s_%d.czi" % (i + 1))))
    cal = (0.7 + 0.3 * np.random.default_rng(1).random((256, 256))).astype(np.float32)
    np.save(tmp_path / "cal.npy", cal)
    cli.main(['-i'] + files + ['-c', 'T', '-cf', str(tmp_path / "cal.npy")])
    sample = str(tmp_path / "s")
    shifts = OP.estimate_shifts(lasers, "max", 15)
    reg = OP.register_stacks(lasers, shifts, True).astype(np.float32)
    oseg, olabs, oavg, oavgn = OP.measure_ecoli(reg, calibration=cal)
    assert np.array_equal(np.load(sample + "_seg.npy"), oseg)
    np.testing.assert_allclose(np.loadtxt(sample + "_avgint.csv", delimiter=',', ndmin=2), oavg, rtol=1e-12)
    np.testing.assert_allclose(np.loadtxt(sample + "_avgint_norm.csv", delimiter=',', ndmin=2), oavgn, rtol=1e-12)


def test_multispecies_measure_and_classify_cli(tmp_path, orc):
    import pandas as pd
    import pipeline as OP
    import hiprfish_imaging_classify_spectra as ccli
    import hiprfish_imaging_multispecies_spectral_image_measurement as mcli

    from hiprfish_image_analysis_amd import kernels as K
    from hiprfish_image_analysis_amd import pipeline as P
    from hiprfish_image_analysis_amd import synthetic as S
    stack, _, _, ref = S.tile(256, 256, nbit=7, bounds=S.MULTI_BOUNDS, seed=32)
    lasers = split_lasers(stack.cpu().numpy(), S.MULTI_BOUNDS, [(0, 0), (3, 2), (-2, 0), (1, -4)])
    for x, l in zip(mcli.EXCITATIONS, lasers):
        np.save(tmp_path / ("m_%s.npy" % x), l)
    C = stack.shape[2]
    cal = (0.5 + np.random.default_rng(2).random(C)).astype(np.float32)
    np.save(tmp_path / "cal.npy", cal)
    m = mcli.main(['-i', str(tmp_path / "m_488.czi"), '-c', str(tmp_path / "cal.npy")])
    sample = str(tmp_path / "m")
    shifts = OP.estimate_shifts(lasers, "sum", None)
    reg = OP.register_stacks(lasers, shifts, False).astype(np.float32)
    # the script's measurement equals the pipeline on the oracle-registered stack ...
    dreg = torch.from_numpy(reg).cuda()
    dcal = torch.from_numpy(cal).cuda()
    keep = {}
    m2 = P.measure_multispecies(dreg, dcal, keep=keep)
    seg = np.load(sample + "_seg.npy")
    assert np.array_equal(seg, m2.segmentation.cpu().numpy())
    # ... and the oracle restatement of the whole chain
    oseg, olabs, oavg, oavgn = OP.measure_multispecies(reg, cal)
    assert np.array_equal(seg, oseg) and len(olabs) >= 1
    csv = pd.read_csv(sample + "_avgint_norm.csv")
    assert list(csv.columns) == [str(i) for i in range(C)]
    np.testing.assert_allclose(csv.values, oavgn, rtol=1e-12)
    np.testing.assert_array_equal(np.load(sample + "_registered.npy"), reg.astype(np.float64) / cal.astype(np.float64))
    # classification of the written spectra
    np.save(tmp_path / "lib.npy", ref)
    info = ccli.main(['-i', sample + "_avgint_norm.csv", '-r', str(tmp_path / "lib.npy")])
    out = pd.read_csv(sample + "_cell_information.csv", header=None)
    assert out.shape == (len(olabs), 77)
    x = csv.values / csv.values.max(axis=1)[:, None]
    lib = ref.astype(np.float64) / ref.astype(np.float64).max(axis=1, keepdims=True)
    b = S.MULTI_BOUNDS
    fx = np.stack([x[:, b[k]:b[k + 1]].max(axis=1) > 0.1 for k in range(4)], 1).astype(np.float64)
    fr = np.stack([lib[:, b[k]:b[k + 1]].max(axis=1) > 0.1 for k in range(4)], 1).astype(np.float64)
    idx, _ = orc.classify(x, lib, b, 2, fx, fr)
    assert [str(v).zfill(7) for v in out[67]] == [format(i + 1, "07b") for i in idx]
    np.testing.assert_allclose(out.iloc[:, 63:67].values.astype(np.float64), fx)
    assert (out[68] == sample).all()
    assert np.array_equal(out[69].values, olabs)
    stats = orc.region_stats(oseg)
    np.testing.assert_allclose(out.iloc[:, 70:76].values.astype(np.float64), stats[olabs][:, 1:7], rtol=1e-9, atol=1e-9)
    assert np.array_equal(out[76].values, stats[olabs][:, 0].astype(np.int64))
    assert info is not None and m is not None
    del K


def test_collect_measurement_results_cli(tmp_path):
    """collect_measurement_results.py -t R / -t M on hand-made result folders"""
    import pandas as pd
    import hiprfish_imaging_collect_measurement_results as cli
    rng = np.random.default_rng(4)
    rows = []
    for s, img, enc in [("S1", "08_18_2018_enc_5_fov_1", 5), ("S1", "08_18_2018_enc_5_fov_2", 5),
                        ("S2", "09_01_2018_enc_1023_fov_3", 1023)]:
        d = tmp_path / s
        d.mkdir(exist_ok=True)
        n = int(rng.integers(5, 40))
        np.savetxt(d / (img + "_avgint.csv"), rng.random((n, 4)), delimiter=",")
        codes = [format(enc, "010b")] * n
        for j in rng.choice(n, 4, replace=False):     # 1-, 2- and 3-bit errors
            flip = rng.choice(10, int(rng.integers(1, 4)), replace=False)
            c = list(codes[j])
            for f in flip:
                c[f] = "1" if c[f] == "0" else "0"
            codes[j] = "".join(c)
        (d / (img + "_cell_ids.txt")).write_text("\n".join(codes) + "\n")
        rows.append((s, img, codes, n, enc))
    pd.DataFrame({"SAMPLE": [r[0] for r in rows], "IMAGES": [r[1] for r in rows]}).to_csv(tmp_path / "tab.csv",
                                                                                       index=False)
    out = str(tmp_path / "res.csv")
    cli.main([str(tmp_path), str(tmp_path / "tab.csv"), out, "-t", "R"])
    r = pd.read_csv(out, float_precision="round_trip")
    for i, (_, _, codes, n, enc) in enumerate(rows):
        ref = format(enc, "010b")
        nb = [sum(a != b for a, b in zip(c, ref)) for c in codes]
        assert r.NCells[i] == n and r.Barcodes[i] == enc and r.BarcodeComplexity[i] == ref.count("1")
        wrong = sum(x > 0 for x in nb)
        assert r.ErrorRate[i] == (1 - (n - wrong) / n if wrong else 1 / n)
        assert r.OneBitError[i] == sum(x == 1 for x in nb) / n
        assert r.TwoBitError[i] == sum(x == 2 for x in nb) / n
        assert r.MultipleBitError[i] == sum(x > 2 for x in nb) / n
    cli.main([str(tmp_path), str(tmp_path / "tab.csv"), out, "-t", "M"])
    a = pd.read_csv(str(tmp_path / "res_abundance.csv"))
    assert list(a.columns) == ["Barcodes", "FOV1", "FOV2", "FOV3"] and a.shape[0] == 1023
    for i, (_, _, codes, n, enc) in enumerate(rows):
        want = np.zeros(1023)
        for c in codes:
            if int(c, 2) >= 1:
                want[int(c, 2) - 1] += 1
        assert np.array_equal(a["FOV%d" % (i + 1)].values, want)
    m = pd.read_csv(out)
    assert list(m.FOV) == [1, 2, 3] and list(m.NCells) == [r[3] for r in rows]


def test_ecoli_image_classification_cli(tmp_path, orc):
    """image_classification.py drop-in on measured spectra: barcodes (gated metric) against the
    restated classifier, the _avgint_ids.csv column layout and the identification image"""
    import pandas as pd
    import hiprfish_imaging_image_classification as ccli
    import hiprfish_imaging_spectral_image_measurement as mcli

    from hiprfish_image_analysis_amd import synthetic as S
    stack, _, _, ref = S.tile(256, 256, seed=33)
    lasers = split_lasers(stack.cpu().numpy(), S.ECOLI_BOUNDS, [(0, 0)] * 5)
    files = []
    for i, l in enumerate(lasers):
        np.save(tmp_path / ("e_%d.npy" % (i + 1)), l)
        files.append(str(tmp_path / ("e_%d.czi" % (i + 1))))
    mcli.main(['-i'] + files + ['-c', 'F'])
    sample = str(tmp_path / "e")
    np.save(tmp_path / "lib.npy", ref)
    codes = ccli.main([sample + "_avgint.csv", "-rf", str(tmp_path / "lib.npy")])
    avg = np.loadtxt(sample + "_avgint.csv", delimiter=",", ndmin=2)
    x = avg / avg.max(axis=1)[:, None]
    lib = ref.astype(np.float64) / ref.astype(np.float64).max(axis=1, keepdims=True)
    b = S.ECOLI_BOUNDS
    fx = np.stack([x[:, b[k]:b[k + 1]].max(axis=1) > 0.1 for k in range(5)], 1).astype(np.float64)
    fr = np.stack([lib[:, b[k]:b[k + 1]].max(axis=1) > 0.1 for k in range(5)], 1).astype(np.float64)
    idx, _ = orc.classify(x, lib, b, 1, fx, fr)
    want = [format(i + 1, "010b") for i in idx]
    assert list(codes) == want
    assert [l.strip() for l in open(sample + "_cell_ids.txt")] == want
    ids = pd.read_csv(sample + "_avgint_ids.csv", header=None, dtype=str)
    assert ids.shape == (len(want), 135)
    assert list(ids[132]) == want and (ids[133] == sample).all()
    np.testing.assert_allclose(ids.iloc[:, 95:126].values.astype(np.float64), np.diff(x[:, :32], axis=1),
                               rtol=1e-15, atol=1e-15)
    seg = np.load(sample + "_seg.npy")
    assert list(ids[134].astype(int)) == sorted(set(np.unique(seg)) - {0})


def _bundle(tmp_path, lib95, rng):
    """A classifier bundle of the reference's shape fitted here with sklearn (synthetic training
    spectra from 12 library barcodes; a stand-in UMAP whose embedding puts each barcode in its
    own cluster), exported with tools/export_classifier.py"""
    from types import SimpleNamespace

    from sklearn.svm import SVC
    sys.path.insert(0, ROOT)
    from tools.export_classifier import export_bundle
    from hiprfish_image_analysis_amd import backend as B
    rows = rng.choice(len(lib95), 12, replace=False)
    y = np.repeat(rows, 25)
    x = lib95[y] * rng.uniform(0.8, 1.2, (len(y), 1)) + rng.normal(0, 0.02, (len(y), 95))
    x = np.clip(x, 1e-3, None)
    x /= x.max(axis=1, keepdims=True)
    feats = np.zeros((len(x), 132))
    feats[:, :95] = x
    feats[:, 95:126] = np.diff(x[:, :32], axis=1)
    checks = []
    for k, (lo, hi) in enumerate(B.ECOLI_SEGMENTS):
        seg = np.abs(feats[:, lo:hi]).max(axis=1)
        lab = (seg > np.median(seg)).astype(np.float64)
        checks.append(SVC(kernel="rbf", gamma=2.0, C=5.0).fit(feats[:, lo:hi], lab))
        feats[:, 126 + k] = checks[-1].predict(feats[:, lo:hi])
    centres = rng.normal(0, 6, (12, 2))
    emb = (centres[np.repeat(np.arange(12), 25)] + rng.normal(0, 0.5, (len(y), 2))).astype(np.float32)
    codes = np.array([format(r + 1, "010b") for r in y])
    clf_umap = SVC(kernel="rbf", gamma=0.5, C=10.0).fit(emb.astype(np.float64), codes)
    um = SimpleNamespace(_raw_data=feats, embedding_=emb, n_neighbors=15, local_connectivity=1.0,
                         metric=SimpleNamespace(__name__="channel_cosine_intensity_violet_derivative_v2"),
                         _a=1.577, _b=0.8951, repulsion_strength=1.0, negative_sample_rate=5, n_epochs=None,
                         _initial_alpha=1.0)
    path = str(tmp_path / "bundle.npz")
    export_bundle(path, um, clf_umap, checks)
    return path, checks, feats, emb, clf_umap


def test_ecoli_image_classification_cli_with_bundle(tmp_path, orc):
    """image_classification.py with an exported classifier bundle: the reference's chain
    (:47-56) -- check-SVC flags, UMAP transform, barcode SVC -- on the device, against the
    oracle restatement of every stage on the same spectra"""
    import pandas as pd
    import hiprfish_imaging_image_classification as ccli
    import hiprfish_imaging_spectral_image_measurement as mcli

    from hiprfish_image_analysis_amd import synthetic as S
    stack, _, _, ref = S.tile(256, 256, seed=34)
    lasers = split_lasers(stack.cpu().numpy(), S.ECOLI_BOUNDS, [(0, 0)] * 5)
    files = []
    for i, l in enumerate(lasers):
        np.save(tmp_path / ("b_%d.npy" % (i + 1)), l)
        files.append(str(tmp_path / ("b_%d.czi" % (i + 1))))
    mcli.main(['-i'] + files + ['-c', 'F'])
    sample = str(tmp_path / "b")
    lib95 = ref.astype(np.float64) / ref.astype(np.float64).max(axis=1, keepdims=True)
    path, checks, tfeats, temb, clf_umap = _bundle(tmp_path, lib95, np.random.default_rng(9))
    codes = ccli.main([sample + "_avgint.csv", "-rf", path])

    avg = np.loadtxt(sample + "_avgint.csv", delimiter=",", ndmin=2)
    x = avg / avg.max(axis=1)[:, None]
    f = np.zeros((len(x), 132))
    f[:, :95] = x
    f[:, 95:126] = np.diff(x[:, :32], axis=1)
    from hiprfish_image_analysis_amd import backend as B
    for k, (lo, hi) in enumerate(B.ECOLI_SEGMENTS):
        c = checks[k]
        f[:, 126 + k] = c.predict(f[:, lo:hi])                # sklearn itself for the flags
    oi, od = orc.knn(f, tfeats, 2, 15)
    e, memb = orc.umap_init(oi, od, temb, 15.0, 0.0, want_memb=True)
    e = orc.umap_refine(oi, memb, e, temb, 100, 1.577, 0.8951, 1.0, 0.25, 5.0, seed=0)
    want = clf_umap.predict(e.astype(np.float64))             # and for the barcode
    assert list(codes) == list(want)
    ids = pd.read_csv(sample + "_avgint_ids.csv", header=None, dtype=str)
    assert ids.shape == (len(want), 135)
    np.testing.assert_array_equal(ids.iloc[:, 126:132].values.astype(np.float64), f[:, 126:132])
    assert list(ids[132]) == list(want)
    assert len(set(want)) > 1
