"""Generate the committed golden fixtures in tests/golden/*.npz from the REFERENCE itself.

Runs only in the build container (needs /root/reference).  Nothing here ships to the GPU
box except the .npz data it writes.  Reference code is executed, never copied:

* neighbor2d.line_profile_2d_v2 / neighbor.line_profile_v2 / line_profile_memory_efficient_v2
  -- the reference's own Cython, compiled from /root/reference by oracle/build_ref.sh.
* the 2-D enhancement post-chain -- lines 111-124 of
  hiprfish-image-analysis-synthetic-community/hiprfish_imaging_multispecies_spectral_image_measurement.py
  read from the reference file at run time and exec'd on the Cython output.
* the 3-D post-chain -- lines 812-817 of hiprfish-image-analysis-biofilm/hiprfish_imaging_biofilm_analysis.py.
* the segmented-cosine metrics -- the functions channel_cosine_intensity,
  channel_cosine_intensity_7b_v2 and channel_cosine_intensity_violet_derivative_v2 AST-extracted
  from hiprfish-image-analysis-reference-training/hiprfish_imaging_train_reference.py with the
  @numba.njit decorator dropped (numba is absent), run as plain Python.
* CC labelling against scipy.ndimage.label (raster-first numbering, the semantics skimage.label
  shares), and the partition sklearn 1.7.2 KMeans(random_state=0, n_init=10) finds on 1-D data.
* the binary morphology skimage 0.14 wraps (scipy.ndimage binary_erosion / dilation /
  fill_holes, label + bincount sieves) and the erosion-seed loop composed from them
  (`make_golden.py morphology` -> morphology.npz).

Usage: python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
import ast
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
MULTI = REF + "/hiprfish-image-analysis-synthetic-community/hiprfish_imaging_multispecies_spectral_image_measurement.py"
BIOF = REF + "/hiprfish-image-analysis-biofilm/hiprfish_imaging_biofilm_analysis.py"
TRAIN = REF + "/hiprfish-image-analysis-reference-training/hiprfish_imaging_train_reference.py"


def ref_lines(path, lo, hi):
    with open(path) as f:
        lines = f.readlines()
    return "".join(l.lstrip() for l in lines[lo - 1:hi])


def ref_functions(path, names):
    src = open(path).read()
    tree = ast.parse(src)
    ns = {"np": np}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            node.decorator_list = []
            mod = ast.Module(body=[node], type_ignores=[])
            exec(compile(mod, path, "exec"), ns)
    return {n: ns[n] for n in names}


def edge_pad(img, w=5):
    return np.pad(img, w, mode="edge")


def main_v3():
    """neighbor3d_v3.npz: the reference's line_profile_memory_efficient_v3 (neighbor.pyx:268-349)
    on small edge-padded volumes (kept separate so the other fixtures are not regenerated)."""
    subprocess.check_call([os.path.join(REPO, "oracle", "build_ref.sh")])
    sys.path.insert(0, os.path.join(REPO, "oracle", "_ref"))
    import neighbor
    rng = np.random.default_rng(20190102)
    out = {}
    # the reference's v3 table reaches up to 18 voxels along x and z (neighbor.pyx:304-307
    # floor with the signed interval), i.e. past the 11-voxel patch: its reads are flat-address
    # arithmetic on the padded array and leave the buffer for voxels near the far x face.
    # Volumes here are long in x so that the first X-9 slices only read inside the array.
    for name, vol in [("a", rng.random((14, 5, 4))), ("b", rng.random((12, 6, 2)) ** 3),
                      ("c", np.full((11, 4, 3), 0.5))]:
        if name == "c":
            vol[1:3, 1:3, 1] = rng.random((2, 2))
        pad = edge_pad(vol)
        out["pad_" + name] = pad
        with np.errstate(all="ignore"):
            out["final_" + name] = neighbor.line_profile_memory_efficient_v3(pad, 11, 9, 9)
    np.savez_compressed(os.path.join(HERE, "neighbor3d_v3.npz"), **out)


def main():
    subprocess.check_call([os.path.join(REPO, "oracle", "build_ref.sh")])
    sys.path.insert(0, os.path.join(REPO, "oracle", "_ref"))
    import neighbor2d  # reference Cython
    import neighbor

    rng = np.random.default_rng(20190101)

    # ---- offset tables (decoded from index images) ---------------------------------
    H = W = 25
    idx = np.arange(H * W, dtype=np.float64).reshape(H, W)
    v = neighbor2d.line_profile_2d_v2(idx, 11, 9)[0, 0].astype(np.int64)
    table2d = np.stack([v // W, v % W], -1).astype(np.int32)
    X = Y = Z = 13
    idx3 = np.arange(X * Y * Z, dtype=np.float64).reshape(X, Y, Z)
    v = neighbor.line_profile_v2(idx3, 11, 9, 9)[0, 0, 0].astype(np.int64)
    table3d = np.stack([v // (Y * Z), (v // Z) % Y, v % Z], -1).astype(np.int32)

    # ---- 2-D line profiles + enhancement chain --------------------------------------
    chain2d = ref_lines(MULTI, 111, 124)
    cases = {}
    img_a = rng.random((18, 23))                       # ragged, generic
    img_b = rng.random((12, 12)) ** 3                  # skewed intensities
    img_c = np.full((14, 16), 0.25)                    # flat -> NaN path
    img_c[4:9, 6:11] = rng.random((5, 5))
    img_d = rng.random((1, 7))                         # single row
    for name, img in [("a", img_a), ("b", img_b), ("c", img_c), ("d", img_d)]:
        pad = edge_pad(img)
        lp = neighbor2d.line_profile_2d_v2(pad.astype(np.float64), 11, 9)
        ns = {"np": np, "image_lp": lp.copy()}
        with np.errstate(all="ignore"):
            exec(chain2d, ns)
        cases["pad_" + name] = pad
        cases["final_" + name] = ns["image_final"]
        if name in ("a", "d"):
            cases["lp_" + name] = lp
    np.savez_compressed(os.path.join(HERE, "neighbor2d.npz"), table=table2d, **cases)

    # ---- 3-D -----------------------------------------------------------------------
    chain3d = ref_lines(BIOF, 812, 817)
    vol = rng.random((8, 7, 5))
    pad3 = edge_pad(vol)
    lp3n = neighbor.line_profile_memory_efficient_v2(pad3, 11, 9, 9)
    ns = {"np": np, "image_lp": lp3n.copy()}
    with np.errstate(all="ignore"):
        exec(chain3d, ns)
    vol_s = rng.random((4, 3, 3))
    pad3s = edge_pad(vol_s)
    lp3 = neighbor.line_profile_v2(pad3s, 11, 9, 9)
    np.savez_compressed(os.path.join(HERE, "neighbor3d.npz"), table=table3d, pad=pad3, lp_norm=lp3n,
                        final=ns["image_final"], pad_small=pad3s, lp_small=lp3)

    # ---- segmented cosine metrics ---------------------------------------------------
    fns = ref_functions(TRAIN, ["channel_cosine_intensity", "channel_cosine_intensity_7b_v2",
                                "channel_cosine_intensity_violet_derivative_v2"])
    n = 160
    # 95-ch + 5 flags (channel_cosine_intensity), flags agree on half of the pairs
    x95 = rng.random((n, 100))
    y95 = rng.random((n, 100))
    fl = (rng.random((n, 5)) > 0.3).astype(np.float64)
    x95[:, 95:100] = fl
    y95[:, 95:100] = np.where(rng.random((n, 1)) < 0.5, fl, (rng.random((n, 5)) > 0.3).astype(np.float64))
    x95[:20, 32:55] = 0.0                 # zero-norm segments
    y95[10:30, 32:55] = 0.0
    d95 = np.array([fns["channel_cosine_intensity"](x95[i], y95[i]) for i in range(n)])
    x67 = rng.random((n, 67))
    y67 = rng.random((n, 67))
    fl = (rng.random((n, 4)) > 0.3).astype(np.float64)
    x67[:, 63:67] = fl
    y67[:, 63:67] = np.where(rng.random((n, 1)) < 0.5, fl, (rng.random((n, 4)) > 0.3).astype(np.float64))
    x67[:15, 57:63] = 0.0
    y67[5:25, 57:63] = 0.0
    d7b = np.array([float(fns["channel_cosine_intensity_7b_v2"](x67[i], y67[i])) for i in range(n)])
    x132 = rng.random((n, 132))
    y132 = rng.random((n, 132))
    fl = (rng.random((n, 6)) > 0.3).astype(np.float64)
    x132[:, 126:132] = fl
    y132[:, 126:132] = np.where(rng.random((n, 1)) < 0.5, fl, (rng.random((n, 6)) > 0.3).astype(np.float64))
    dvd = np.array([fns["channel_cosine_intensity_violet_derivative_v2"](x132[i], y132[i]) for i in range(n)])
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), x95=x95, y95=y95, d95=d95, x67=x67, y67=y67,
                        d7b=d7b, x132=x132, y132=y132, dvd=dvd)

    # ---- connected components (scipy raster numbering) ------------------------------
    from scipy import ndimage as ndi
    m = rng.random((64, 80)) > 0.55
    l8, n8 = ndi.label(m, structure=np.ones((3, 3), int))
    l4, n4 = ndi.label(m)
    np.savez_compressed(os.path.join(HERE, "label.npz"), mask=m, l8=l8.astype(np.int32), l4=l4.astype(np.int32))

    # ---- 1-D KMeans partitions (sklearn, 2019 defaults forced) ----------------------
    from sklearn.cluster import KMeans
    km = {}
    for k, (name, x) in enumerate([
        ("bimodal", np.concatenate([rng.normal(0.1, 0.03, 3000), rng.normal(0.7, 0.1, 2000)])),
        ("logsum", np.log(np.concatenate([rng.gamma(2.0, 0.01, 4000), rng.gamma(9.0, 0.5, 1500)]) + 1e-2)),
        ("trimodal", np.concatenate([rng.normal(0, 0.1, 2000), rng.normal(2, 0.2, 1500), rng.normal(5, 0.3, 800)])),
    ]):
        kk = 3 if name == "trimodal" else 2
        lab = KMeans(n_clusters=kk, random_state=0, n_init=10).fit_predict(x.reshape(-1, 1))
        km["x_" + name] = x
        km["lab_" + name] = lab.astype(np.int32)
        km["k_" + name] = np.int32(kk)
        lab3 = KMeans(n_clusters=3, random_state=0, n_init=10).fit_predict(x.reshape(-1, 1))
        km["lab3_" + name] = lab3.astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "kmeans.npz"), **km)
    print("golden fixtures written to", HERE)


def main_kmeans_images():
    """sklearn KMeans(k, random_state=0, n_init=10) partitions of the images the reference
    actually clusters: E. coli image_cn = log(sum + 1e-2) (ecoli :71-94, k = 2 and 3) and the
    community final / NL-means images (multispecies :125, :141, k = 2), from synthetic 256^2
    tiles (plain and 12-bit quantised) computed by the oracle pipeline."""
    import torch
    from sklearn.cluster import KMeans
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, REPO)
    import pipeline as OP
    from hiprfish_image_analysis_amd import synthetic as S
    out = {}
    for name, seed, q in [("ecoli_a", 201, None), ("ecoli_q", 202, 4095)]:
        st = S.tile(256, 256, seed=seed, device="cpu")[0]
        if q:
            st = torch.round(st.double() * q) / q
        x = np.log(np.sum(st.float().numpy().astype(np.float64), axis=2) + 1e-2)
        out["x_" + name] = x
        for k in (2, 3):
            out["lab%d_%s" % (k, name)] = KMeans(n_clusters=k, random_state=0, n_init=10).fit_predict(
                x.reshape(-1, 1)).astype(np.int8)
    for name, seed in [("community", 203)]:
        st = S.tile(256, 256, nbit=7, bounds=S.MULTI_BOUNDS, seed=seed, device="cpu")[0].numpy()
        keep = {}
        OP.segment_multispecies(st, keep=keep)
        for im in ("final", "nl"):
            x = keep[im]
            out["x_%s_%s" % (name, im)] = x
            out["lab2_%s_%s" % (name, im)] = KMeans(n_clusters=2, random_state=0, n_init=10).fit_predict(
                x.reshape(-1, 1)).astype(np.int8)
    np.savez_compressed(os.path.join(HERE, "kmeans_images.npz"), **out)
    print("kmeans_images.npz written")


def _seg_cos_py(x, y, lo, hi):
    r = nx = ny = 0.0
    for i in range(lo, hi):
        r += x[i] * y[i]
        nx += x[i] ** 2
        ny += y[i] ** 2
    if nx == 0.0 and ny == 0.0:
        return 0.0
    if nx == 0.0 or ny == 0.0:
        return 1.0
    return 1.0 - r / np.sqrt(nx * ny)


def metric_7b_v2(x, y):
    """channel_cosine_intensity_7b_v2 (train_reference.py:994-1072), restated for sklearn's
    brute-force neighbour search"""
    if np.sum(np.abs(x[63:67] - y[63:67])) < 0.01:
        b = (0, 23, 43, 57, 63)
        c = [0.0 if x[63 + s] == 0 else _seg_cos_py(x, y, b[s], b[s + 1]) for s in range(4)]
        return 0.5 * (c[0] + c[1] + c[2] + c[3]) / 4
    return 1.0


def metric_violet_v2(x, y):
    """the scalar (d + c1..c5) / 6 of channel_cosine_intensity_violet_derivative_v2 (:569-731)"""
    b = (0, 32, 55, 75, 89, 95)
    if np.sum(np.abs(x[126:132] - y[126:132])) < 0.01:
        d = 0.0
        c = [0.0 if x[126 + s] == 0 else _seg_cos_py(x, y, b[s], b[s + 1]) for s in range(5)]
    else:
        d = 1.0
        c = [_seg_cos_py(x, y, b[s], b[s + 1]) for s in range(5)]
    return (d + c[0] + c[1] + c[2] + c[3] + c[4]) / 6


def main_backend():
    """sklearn SVC (predict, ovo decision_function), StandardScaler and brute-force
    NearestNeighbors on synthetic data: the a17/a18/f2 back-end fixtures (backend.npz)"""
    from sklearn.neighbors import NearestNeighbors
    from sklearn.preprocessing import StandardScaler
    from sklearn.svm import SVC
    rng = np.random.default_rng(7)
    out = {}
    cases = [("rbf5", dict(kernel="rbf", gamma=0.7, C=3.0), 5, 3), ("lin2", dict(kernel="linear", C=0.5), 2, 32),
             ("poly3", dict(kernel="poly", degree=3, gamma=0.4, coef0=1.0, C=2.0), 3, 6),
             ("sig2", dict(kernel="sigmoid", gamma=0.05, coef0=0.1, C=1.0), 2, 23),
             ("rbf40", dict(kernel="rbf", gamma=2.0, C=10.0), 40, 2)]
    for name, kw, ncls, f in cases:
        centres = rng.normal(0, 1.5, (ncls, f))
        y = rng.integers(0, ncls, 600)
        x = centres[y] + rng.normal(0, 1.0, (600, f))
        clf = SVC(decision_function_shape="ovo", **kw).fit(x, y)
        xt = centres[rng.integers(0, ncls, 300)] + rng.normal(0, 1.2, (300, f))
        out[name + "_sv"] = clf.support_vectors_
        out[name + "_dual_coef"] = clf.dual_coef_
        out[name + "_intercept"] = clf.intercept_
        out[name + "_n_support"] = clf.n_support_.astype(np.int32)
        out[name + "_classes"] = clf.classes_.astype(np.float64)
        out[name + "_gamma"] = np.float64(clf._gamma)
        out[name + "_coef0"] = np.float64(clf.coef0)
        out[name + "_degree"] = np.int32(clf.degree)
        out[name + "_kernel"] = np.int32({"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}[kw["kernel"]])
        out[name + "_x"] = xt
        out[name + "_pred"] = clf.predict(xt).astype(np.float64)
        out[name + "_dec"] = clf.decision_function(xt)
    x = rng.normal(3, 2, (200, 63)) * rng.uniform(0.1, 4, 63)
    sc = StandardScaler().fit(x)
    out["scaler_x"] = x[:50] + 0.3
    out["scaler_mean"] = sc.mean_
    out["scaler_scale"] = sc.scale_
    out["scaler_out"] = sc.transform(x[:50] + 0.3)
    for name, f, flags, metric in (("knn7b", 67, (63, 67), metric_7b_v2), ("knnviolet", 132, (126, 132), metric_violet_v2)):
        proto = rng.random((12, f))
        tr = proto[rng.integers(0, 12, 400)] + 0.05 * rng.random((400, f))
        qs = proto[rng.integers(0, 12, 40)] + 0.05 * rng.random((40, f))
        for a in (tr, qs):   # flag columns 0/1, a few mismatching
            a[:, flags[0]:flags[1]] = (rng.random((len(a), flags[1] - flags[0])) < 0.7).astype(np.float64)
        nn = NearestNeighbors(n_neighbors=15, algorithm="brute", metric=metric).fit(tr)
        d, i = nn.kneighbors(qs)
        out[name + "_train"] = tr
        out[name + "_q"] = qs
        out[name + "_idx"] = i.astype(np.int32)
        out[name + "_dist"] = d
    # SVC(probability=True): predict_proba (Platt pairs + libsvm's coupling) -- drawn after the
    # cases above so their data stay as they were
    for name, kw, ncls, f in [("prob2", dict(kernel="rbf", gamma=0.5, C=2.0), 2, 4),
                              ("prob6", dict(kernel="rbf", gamma=0.3, C=4.0), 6, 5),
                              ("prob30", dict(kernel="linear", C=1.0), 30, 3)]:
        centres = rng.normal(0, 2.0, (ncls, f))
        y = rng.integers(0, ncls, 900)
        x = centres[y] + rng.normal(0, 1.0, (900, f))
        clf = SVC(probability=True, random_state=0, **kw).fit(x, y)
        xt = centres[rng.integers(0, ncls, 200)] + rng.normal(0, 1.3, (200, f))
        out[name + "_sv"] = clf.support_vectors_
        out[name + "_dual_coef"] = clf.dual_coef_
        out[name + "_intercept"] = clf.intercept_
        out[name + "_n_support"] = clf.n_support_.astype(np.int32)
        out[name + "_classes"] = clf.classes_.astype(np.float64)
        out[name + "_gamma"] = np.float64(clf._gamma)
        out[name + "_coef0"] = np.float64(clf.coef0)
        out[name + "_degree"] = np.int32(clf.degree)
        out[name + "_kernel"] = np.int32({"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}[kw["kernel"]])
        out[name + "_probA"] = clf.probA_
        out[name + "_probB"] = clf.probB_
        out[name + "_x"] = xt
        out[name + "_proba"] = clf.predict_proba(xt)
        out[name + "_pred"] = clf.predict(xt).astype(np.float64)
    np.savez_compressed(os.path.join(HERE, "backend.npz"), **out)
    print("backend.npz written")


CROSS = np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]], bool)
SQUARE = np.ones((3, 3), bool)


def _rso_bool(m, min_size, conn):
    """skimage.morphology.remove_small_objects(bool image, min_size, connectivity) (0.14-era source):
    ndi.label with generate_binary_structure(2, conn), bincount of the labels, components with
    size < min_size set to False"""
    from scipy import ndimage as ndi
    ccs, _ = ndi.label(m, CROSS if conn == 1 else SQUARE)
    sizes = np.bincount(ccs.ravel())
    out = m.copy()
    out[sizes[ccs] < min_size] = False
    return out


def _seeds_scipy(cell_sm):
    """ecoli measurement.py:97-112 composed from scipy.ndimage primitives: skimage's label
    (8-connected), regionprops areas (bincount), binary_erosion (cross, border_value=True),
    remove_small_objects(., 10) (4-connected), then label(rso(label(dist_be), 10)).  The loop is
    capped as libhrf's (4 (H + W) + 8 rounds; the fixtures never reach the cap)."""
    from scipy import ndimage as ndi
    H, W = cell_sm.shape
    lab, _ = ndi.label(cell_sm, SQUARE)
    be = np.zeros(cell_sm.shape, bool)
    rounds = 0
    while lab.max() > 0:
        assert rounds < 4 * (H + W) + 8
        rounds += 1
        sizes = np.bincount(lab.ravel())
        small = (lab > 0) & (sizes[lab] < 600)
        be |= small
        lab[small] = 0
        er = ndi.binary_erosion(lab > 0, CROSS, border_value=1)
        lab, _ = ndi.label(_rso_bool(er, 10, 1), SQUARE)
    lb, _ = ndi.label(be, SQUARE)
    sizes = np.bincount(lb.ravel())
    lb[sizes[lb] < 10] = 0
    seeds, n = ndi.label(lb > 0, SQUARE)
    return be, seeds.astype(np.int32), rounds


def main_morphology():
    """morphology.npz: the a9 / a11 / a13 primitives on E. coli-like masks, computed by
    scipy.ndimage (the functions skimage 0.14's binary morphology wraps): binary_erosion with
    the cross and border_value=1 (skimage.morphology.binary_erosion), binary_dilation,
    skimage's binary_opening = dilation(erosion), remove_small_objects / remove_small_holes as
    ndi.label + a bincount sieve, binary_fill_holes, and the erosion-seed loop of ecoli :97-112.
    Masks: the interior / cell_sm / rough masks of synthetic 256^2 E. coli tiles (plain and
    12-bit quantised; the oracle pipeline only makes the INPUTS), thresholded smooth noise with
    holes on ragged shapes, and degenerate cases."""
    import torch
    from scipy import ndimage as ndi
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, REPO)
    import pipeline as OP
    from hiprfish_image_analysis_amd import synthetic as S
    rng = np.random.default_rng(20190401)
    masks = {}
    for name, seed, q in [("ecoli_a", 301, None), ("ecoli_q", 302, 4095)]:
        st = S.tile(256, 256, seed=seed, device="cpu")[0]
        if q:
            st = (torch.round(st.double() * q) / q).float()
        keep = {}
        OP.segment_ecoli(st.numpy(), keep=keep)
        masks[name + "_interior"] = keep["interior"]
        masks[name + "_cellsm"] = keep["cell_sm"]
        masks[name + "_rough"] = keep["rough_mask"]
    for name, shape, thr in [("blob_a", (96, 112), 0.55), ("blob_b", (61, 47), 0.5), ("blob_c", (128, 128), 0.6)]:
        f = ndi.gaussian_filter(rng.random(shape), 2.0)
        masks[name] = f > np.quantile(f, thr)
    edge = np.zeros((20, 24), bool)
    edge[:, :3] = True
    edge[5:9, 10:15] = True
    edge[6, 12] = False
    masks["edge"] = edge
    masks["empty"] = np.zeros((9, 13), bool)
    masks["full"] = np.ones((7, 5), bool)
    one = np.zeros((8, 8), bool)
    one[3, 4] = True
    masks["one"] = one
    out = {}
    for name, m in masks.items():
        m = np.ascontiguousarray(m, bool)
        ero = ndi.binary_erosion(m, CROSS, border_value=1)
        out["m_" + name] = m
        out["ero_" + name] = ero
        out["dil_" + name] = ndi.binary_dilation(m, CROSS)
        out["open_" + name] = ndi.binary_dilation(ero, CROSS)
        out["rso50c1_" + name] = _rso_bool(m, 50, 1)
        out["rso10c1_" + name] = _rso_bool(m, 10, 1)
        out["rso10c2_" + name] = _rso_bool(m, 10, 2)
        out["rsh64_" + name] = ~_rso_bool(~m, 64, 1)
        out["fill_" + name] = ndi.binary_fill_holes(m)
        # ecoli :95-96 cell_sm = rso(opening(rsh(interior)), 50)
        out["cellsm_" + name] = _rso_bool(ndi.binary_dilation(ndi.binary_erosion(~_rso_bool(~m, 64, 1), CROSS,
                                                                                     border_value=1), CROSS), 50, 1)
    for name in ("ecoli_a_cellsm", "ecoli_q_cellsm", "blob_a", "blob_c", "edge", "one", "empty"):
        be, seeds, rounds = _seeds_scipy(out["m_" + name])
        out["be_" + name] = be
        out["seeds_" + name] = seeds
        print("seeds", name, "rounds", rounds, "n", int(seeds.max()))
    np.savez_compressed(os.path.join(HERE, "morphology.npz"), **out)
    print("morphology.npz written")


if __name__ == "__main__":
    if sys.argv[1:] == ["morphology"]:
        main_morphology()
    elif sys.argv[1:] == ["v3"]:
        main_v3()
    elif sys.argv[1:] == ["kmeans_images"]:
        main_kmeans_images()
    elif sys.argv[1:] == ["backend"]:
        main_backend()
    else:
        main()
