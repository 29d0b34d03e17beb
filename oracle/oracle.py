"""ctypes wrapper over oracle/liboracle.so -- the CPU restatement of the reference path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product package never imports this module.
Each function names the reference code it restates (see hrf_oracle.c for the full
citations).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    srcs = [os.path.join(_HERE, f) for f in ("hrf_oracle.c", "ws_order.c", "kmeans_sk.c", "backend.c",
                                              "../hiprfish_image_analysis_amd/csrc/detmath.h")]
    if not os.path.exists(_LIB) or max(os.path.getmtime(s) for s in srcs) > os.path.getmtime(_LIB):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB)
        _lib.oracle_segcos.restype = ctypes.c_double
        _lib.oracle_label.restype = ctypes.c_int32
        _lib.oracle_relabel_sequential.restype = ctypes.c_int32
        _lib.oracle_kmeans_scale.restype = ctypes.c_int
        _lib.oracle_kmeans_scale.argtypes = [ctypes.c_double, ctypes.c_int64]
        _lib.oracle_knn_metric.restype = ctypes.c_double
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


I64 = ctypes.c_int64


# ---- a3 ---------------------------------------------------------------------------------
def cr_log(x):
    """correctly rounded natural log (detmath.h hrf_cr_log, the function libhrf's image_cn uses):
    image_cn = log(sum + 1e-2), ecoli measurement.py:72.  numpy's log differs from it in the last
    ulp on ~1e-4 of inputs (SVML on AVX-512 hosts)"""
    a = _c(x, np.float64)
    out = np.empty_like(a)
    lib().oracle_cr_log(_p(a), I64(a.size), 0, _p(out))
    return out


def libm_log(x, base10=False):
    """the C library's log (glibc on the host), one call per element: numpy 1.16's np.log (the
    reference era's numpy called libm); tests/test_image_cn_log.py"""
    a = _c(x, np.float64)
    out = np.empty_like(a)
    lib().oracle_libm_log(_p(a), I64(a.size), 1 if base10 else 0, _p(out))
    return out


def cr_log10(x):
    """correctly rounded log10 (hrf_cr_log10): log10(sum + 1), biofilm :831"""
    a = _c(x, np.float64)
    out = np.empty_like(a)
    lib().oracle_cr_log(_p(a), I64(a.size), 1, _p(out))
    return out


# ---- a5/a7 ---------------------------------------------------------------------------
def lp_table_2d(patch=11, nphi=9):
    """neighbor2d.pyx:32-55 -> int32 [nphi, patch, 2]"""
    out = np.zeros((nphi, patch, 2), np.int32)
    lib().oracle_lp_table_2d(patch, nphi, _p(out))
    return out


def lp_table_3d(patch=11, ntheta=9, nphi=9):
    """neighbor.pyx:209-243 -> int32 [(ntheta-1)*nphi, patch, 3]"""
    out = np.zeros(((ntheta - 1) * nphi, patch, 3), np.int32)
    lib().oracle_lp_table_3d(patch, ntheta, nphi, _p(out))
    return out


def line_profile_2d(pad, patch=11, nphi=9):
    """neighbor2d.line_profile_2d_v2 (neighbor2d.pyx:8-64)"""
    pad = _c(pad, np.float64)
    hp, wp = pad.shape
    out = np.zeros((hp - patch + 1, wp - patch + 1, nphi, patch), np.float64)
    lib().oracle_line_profile_2d(_p(pad), I64(hp), I64(wp), patch, nphi, _p(out))
    return out


def enhance_2d(pad, patch=11, nphi=9):
    """multispecies_spectral_image_measurement.py:110-124 -> final (H, W) f64"""
    pad = _c(pad, np.float64)
    hp, wp = pad.shape
    out = np.zeros((hp - patch + 1, wp - patch + 1), np.float64)
    lib().oracle_enhance_2d(_p(pad), I64(hp), I64(wp), patch, nphi, _p(out))
    return out


def line_profile_3d(pad, patch=11, ntheta=9, nphi=9):
    """neighbor.line_profile_v2 (neighbor.pyx:115-181)"""
    pad = _c(pad, np.float64)
    xp, yp, zp = pad.shape
    nd = (ntheta - 1) * nphi
    out = np.zeros((xp - patch + 1, yp - patch + 1, zp - patch + 1, nd, patch), np.float64)
    lib().oracle_line_profile_3d(_p(pad), I64(xp), I64(yp), I64(zp), patch, ntheta, nphi, _p(out))
    return out


def line_profile_3d_norm(pad, patch=11, ntheta=9, nphi=9):
    """neighbor.line_profile_memory_efficient_v2 (neighbor.pyx:186-263)"""
    pad = _c(pad, np.float64)
    xp, yp, zp = pad.shape
    nd = (ntheta - 1) * nphi
    out = np.zeros((xp - patch + 1, yp - patch + 1, zp - patch + 1, nd), np.float64)
    lib().oracle_line_profile_3d_norm(_p(pad), I64(xp), I64(yp), I64(zp), patch, ntheta, nphi, _p(out))
    return out


def enhance_3d(pad, patch=11, ntheta=9, nphi=9):
    """biofilm_analysis.py:811-817 -> final (X, Y, Z) f64"""
    pad = _c(pad, np.float64)
    xp, yp, zp = pad.shape
    out = np.zeros((xp - patch + 1, yp - patch + 1, zp - patch + 1), np.float64)
    lib().oracle_enhance_3d(_p(pad), I64(xp), I64(yp), I64(zp), patch, ntheta, nphi, _p(out))
    return out


def lp_table_3d_v3(patch=11, ntheta=9, nphi=9):
    off = np.zeros(((ntheta - 1) * nphi, patch, 3), np.int32)
    lib().oracle_lp_table_3d_v3(patch, ntheta, nphi, _p(off))
    return off


def enhance_3d_v3(pad, patch=11, ntheta=9, nphi=9):
    """neighbor.line_profile_memory_efficient_v3 (neighbor.pyx:268-349)"""
    pad = _c(pad, np.float64)
    xp, yp, zp = pad.shape
    out = np.zeros((xp - patch + 1, yp - patch + 1, zp - patch + 1), np.float64)
    lib().oracle_enhance_3d_v3(_p(pad), I64(xp), I64(yp), I64(zp), patch, ntheta, nphi, _p(out))
    return out


def v3_defined(shape, patch=11, ntheta=9, nphi=9):
    """voxels of line_profile_memory_efficient_v3 whose reads stay inside the padded array"""
    xp, yp, zp = shape
    ok = np.zeros((xp - patch + 1, yp - patch + 1, zp - patch + 1), np.uint8)
    lib().oracle_v3_defined(I64(xp), I64(yp), I64(zp), patch, ntheta, nphi, _p(ok))
    return ok.astype(bool)


# ---- a4 -------------------------------------------------------------------------------
def nl_means(img, patch_size=7, patch_distance=11, h=0.1, sigma=0.0):
    """skimage.restoration.denoise_nl_means (fast 2-D) in libhrf's summation order"""
    im = _c(img, np.float64)
    out = np.zeros(im.shape, np.float64)
    lib().oracle_nl_means(_p(im), I64(im.shape[0]), I64(im.shape[1]), patch_size, patch_distance,
                          ctypes.c_double(h), ctypes.c_double(sigma), _p(out))
    return out


def nl_means_skimage(img, patch_size=7, patch_distance=11, h=0.1, sigma=0.0):
    """skimage's fast 2-D NL-means algorithm itself (integral images, symmetric pair credit)"""
    im = _c(img, np.float64)
    out = np.zeros(im.shape, np.float64)
    lib().oracle_nl_means_skimage(_p(im), I64(im.shape[0]), I64(im.shape[1]), patch_size, patch_distance,
                                  ctypes.c_double(h), ctypes.c_double(sigma), _p(out))
    return out


def register_translation(src, target):
    """skimage.feature.register_translation(src, target)[0] with its defaults (upsample_factor 1):
    argmax |ifft(F(src) conj(F(target)))|, wrapped to (-n/2, n/2] per axis (numpy FFT)."""
    src = np.asarray(src, np.float64)
    target = np.asarray(target, np.float64)
    cc = np.fft.ifftn(np.fft.fftn(src) * np.fft.fftn(target).conj())
    maxima = np.unravel_index(np.argmax(np.abs(cc)), cc.shape)
    shifts = np.array(maxima, dtype=np.float64)
    mid = np.array([np.fix(n / 2) for n in cc.shape])
    big = shifts > mid
    shifts[big] -= np.array(cc.shape)[big]
    return shifts


# ---- a9/a10/a12/a13 ------------------------------------------------------------------
def label(img, conn=2):
    """skimage.measure.label(img, connectivity=conn) (background 0, equal-value components)"""
    img = _c(img, np.int32)
    out = np.zeros(img.shape, np.int32)
    n = lib().oracle_label(_p(img), I64(img.shape[0]), I64(img.shape[1]), conn, _p(out))
    return out, int(n)


def erode(mask, border=1):
    m = _c(mask, np.uint8)
    out = np.zeros(m.shape, np.uint8)
    lib().oracle_erode(_p(m), I64(m.shape[0]), I64(m.shape[1]), border, _p(out))
    return out.astype(bool)


def dilate(mask):
    m = _c(mask, np.uint8)
    out = np.zeros(m.shape, np.uint8)
    lib().oracle_dilate(_p(m), I64(m.shape[0]), I64(m.shape[1]), _p(out))
    return out.astype(bool)


def opening(mask):
    return dilate(erode(mask))


def remove_small_objects_mask(mask, min_size, conn=1):
    m = _c(mask, np.uint8)
    out = np.zeros(m.shape, np.uint8)
    lib().oracle_rso_mask(_p(m), I64(m.shape[0]), I64(m.shape[1]), I64(min_size), conn, _p(out))
    return out.astype(bool)


def remove_small_objects_labels(lab, min_size):
    l = _c(lab, np.int32)
    out = np.zeros(l.shape, np.int32)
    lib().oracle_rso_labels(_p(l), I64(l.shape[0]), I64(l.shape[1]), I64(min_size), _p(out))
    return out


def remove_small_holes(mask, thr=64, conn=1):
    m = _c(mask, np.uint8)
    out = np.zeros(m.shape, np.uint8)
    lib().oracle_remove_small_holes(_p(m), I64(m.shape[0]), I64(m.shape[1]), I64(thr), conn, _p(out))
    return out.astype(bool)


def fill_holes(mask):
    m = _c(mask, np.uint8)
    out = np.zeros(m.shape, np.uint8)
    lib().oracle_fill_holes(_p(m), I64(m.shape[0]), I64(m.shape[1]), _p(out))
    return out.astype(bool)


def clear_border(lab):
    l = _c(lab, np.int32)
    out = np.zeros(l.shape, np.int32)
    lib().oracle_clear_border(_p(l), I64(l.shape[0]), I64(l.shape[1]), _p(out))
    return out


def relabel_sequential(lab):
    l = _c(lab, np.int32)
    out = np.zeros(l.shape, np.int32)
    n = lib().oracle_relabel_sequential(_p(l), I64(l.size), _p(out))
    return out, int(n)


def watershed(img, markers, mask=None):
    im = _c(img, np.float64)
    mk = _c(markers, np.int32)
    out = np.zeros(mk.shape, np.int32)
    mp = None
    if mask is not None:
        m = _c(mask, np.uint8)
        mp = _p(m)
    lib().oracle_watershed(_p(im), _p(mk), mp, I64(im.shape[0]), I64(im.shape[1]), _p(out))
    return out


def watershed_ordered(img, markers, mask=None, raw=False):
    """ws_order.c: the tie-exact formulation libhrf's watershed implements (NOT a reference
    restatement; checked against watershed() above).  -> (labels, stats) with stats =
    [contested pixels, walk steps, heap-layout decisions, label rounds].  Where a decision came
    down to the heap's layout (stats[2] > 0) the labels are the heap flood's, as in libhrf;
    raw=True keeps the resolution's own labels there (the order model alone)."""
    im = _c(img, np.float64)
    mk = _c(markers, np.int32)
    out = np.zeros(mk.shape, np.int32)
    st = np.zeros(4, np.int64)
    mp = None
    if mask is not None:
        m = _c(mask, np.uint8)
        mp = _p(m)
    fn = lib().oracle_watershed_ordered_raw if raw else lib().oracle_watershed_ordered
    fn(_p(im), _p(mk), mp, I64(im.shape[0]), I64(im.shape[1]), _p(out), _p(st))
    return out, st


# ---- a14/a15/a20 ---------------------------------------------------------------------
def region_stats(lab, nlab=None):
    """-> [(nlab+1), 8]: area, cen_r, cen_c, major, minor, ecc, orient, present"""
    l = _c(lab, np.int32)
    if nlab is None:
        nlab = int(l.max()) if l.size else 0
    out = np.zeros((nlab + 1, 8), np.float64)
    lib().oracle_region_stats(_p(l), I64(l.shape[0]), I64(l.shape[1]), ctypes.c_int32(nlab), _p(out))
    return out


def label_sums(stack, lab, nlab=None):
    s = _c(stack, np.float32)
    l = _c(lab, np.int32)
    C = s.shape[-1]
    if nlab is None:
        nlab = int(l.max()) if l.size else 0
    sums = np.zeros((nlab + 1, C), np.float64)
    counts = np.zeros(nlab + 1, np.int64)
    lib().oracle_label_sums(_p(s), _p(l), I64(l.size), C, ctypes.c_int32(nlab), _p(sums), _p(counts))
    return sums, counts


# ---- a19 -----------------------------------------------------------------------------
def segcos(x, y, bounds, variant=0, fx=None, fy=None):
    x = _c(x, np.float64)
    y = _c(y, np.float64)
    b = _c(bounds, np.int32)
    nseg = len(b) - 1
    fxp = fyp = None
    if fx is not None:
        fxa = _c(fx, np.float64)
        fya = _c(fy, np.float64)
        fxp, fyp = _p(fxa), _p(fya)
    return lib().oracle_segcos(_p(x), _p(y), _p(b), nseg, variant, fxp, fyp)


def classify_top2(x, ref, bounds):
    """ungated argmin (first minimum) with the best and runner-up distances"""
    x = _c(x, np.float64)
    ref = _c(ref, np.float64)
    b = _c(bounds, np.int32)
    n, C = x.shape
    arg = np.zeros(n, np.int32)
    d1 = np.zeros(n, np.float64)
    d2 = np.zeros(n, np.float64)
    lib().oracle_classify_top2(_p(x), I64(n), _p(ref), ref.shape[0], C, _p(b), len(b) - 1, _p(arg), _p(d1), _p(d2))
    return arg, d1, d2


def classify(x, ref, bounds, variant=0, fx=None, fr=None):
    x = _c(x, np.float64)
    ref = _c(ref, np.float64)
    b = _c(bounds, np.int32)
    n, C = x.shape
    R = ref.shape[0]
    arg = np.zeros(n, np.int32)
    dmin = np.zeros(n, np.float64)
    if variant and (fx is None or fr is None):
        raise ValueError("classify: the gated variants need the presence flags fx and fr")
    fxa = _c(fx, np.float64) if fx is not None else None
    fra = _c(fr, np.float64) if fr is not None else None
    lib().oracle_classify(_p(x), I64(n), _p(ref), R, C, _p(b), len(b) - 1, variant,
                          _p(fxa) if fxa is not None else None, _p(fra) if fra is not None else None,
                          _p(arg), _p(dmin))
    return arg, dmin


# ---- a8 ------------------------------------------------------------------------------
def kmeans_draws(nv, k, n_init=10, seed=0):
    """sklearn 1.7.2 KMeans(random_state=seed, n_init).fit's random stream on nv unit-weight
    samples: per run the first centre (RandomState.choice(nv, p=1/nv)) and the k-means++
    trial draws (RandomState.uniform(size=2 + int(log k)) per further centre), in call order"""
    rs = np.random.RandomState(seed)
    p = np.ones(nv) / np.ones(nv).sum()
    nt = 2 + int(np.log(k))
    first, draws = [], []
    for _ in range(n_init):
        first.append(int(rs.choice(nv, p=p)))
        for _c in range(1, k):
            draws.extend(rs.uniform(size=nt).tolist())
    return np.array(first, np.int64), np.array(draws if draws else [0.0], np.float64)


def kmeans_sk(x, k, valid=None, n_init=10, max_iter=300, seed=0):
    """sklearn KMeans(k, random_state=0, n_init=10).fit_predict(x.reshape(-1,1)) restated
    (kmeans_sk.c) -> labels (sklearn's cluster ids, -1 where not valid), centres, info
    [winning run, its iterations, strict convergence, empty-cluster relocations]"""
    xv = _c(x, np.float64).ravel()
    if np.isnan(xv if valid is None else xv[_c(valid, np.uint8).ravel().astype(bool)]).any():
        raise ValueError("Input contains NaN")          # sklearn's check_array
    vp = None
    nv = xv.size
    if valid is not None:
        va = _c(valid, np.uint8).ravel()
        vp = _p(va)
        nv = int(va.astype(bool).sum())
    first, draws = kmeans_draws(max(nv, 1), k, n_init, seed)
    lab = np.zeros(xv.size, np.int32)
    cen = np.zeros(k, np.float64)
    info = np.zeros(4, np.int64)
    lib().oracle_kmeans_sk(_p(xv), vp, I64(xv.size), k, n_init, max_iter, _p(first), _p(draws), _p(lab), _p(cen),
                           _p(info))
    return lab.reshape(np.shape(x)), cen, info


# ---- a21/a22/a23 ---------------------------------------------------------------------
def rag_edges(lab, nlab=None):
    l = _c(lab, np.int32)
    if nlab is None:
        nlab = int(l.max())
    e = np.zeros((nlab + 1, nlab + 1), np.uint8)
    lib().oracle_rag_edges(_p(l), I64(l.shape[0]), I64(l.shape[1]), ctypes.c_int32(nlab), _p(e))
    return e


def barcode_adjacency(edge, bc_of_label, R):
    e = _c(edge, np.uint8)
    nlab = e.shape[0] - 1
    bc = _c(bc_of_label, np.int32)
    adj = np.zeros((R, R), np.int64)
    lib().oracle_barcode_adjacency(_p(e), ctypes.c_int32(nlab), _p(bc), R, _p(adj))
    return adj


def barcode_counts(bc, R):
    b = _c(bc, np.int32)
    out = np.zeros(R, np.int64)
    lib().oracle_barcode_counts(_p(b), I64(b.size), R, _p(out))
    return out


def paint_ids(lab, code):
    l = _c(lab, np.int32)
    c = _c(code, np.int32)
    out = np.zeros(l.shape, np.int32)
    lib().oracle_paint_ids(_p(l), I64(l.size), _p(c), ctypes.c_int32(c.size), _p(out))
    return out


def shape_filter(lab, stats, lo=15.0, hi=35.0):
    l = _c(lab, np.int32)
    st = _c(stats, np.float64)
    out = np.zeros(l.shape, np.int32)
    lib().oracle_shape_filter(_p(l), I64(l.shape[0]), I64(l.shape[1]), _p(st), ctypes.c_int32(st.shape[0] - 1),
                              ctypes.c_double(lo), ctypes.c_double(hi), _p(out))
    return out


# ---- a17, a18, f2: classifier back-end (backend.c) -------------------------------------------
def svc_predict(x, sv, coef, intercept, start, kernel, gamma=1.0, coef0=0.0, degree=3, want_dec=False):
    """libsvm one-vs-one predict (coef / intercept in libsvm's sign convention) -> class index
    (and the pair decision values)"""
    x = _c(x, np.float64)
    sv = _c(sv, np.float64)
    coef = _c(coef, np.float64)
    intercept = _c(intercept, np.float64)
    start = _c(start, np.int32)
    n, f = x.shape
    nc = len(start) - 1
    pred = np.zeros(n, np.int32)
    dec = np.zeros((n, nc * (nc - 1) // 2), np.float64) if want_dec else None
    lib().oracle_svc_predict(_p(x), I64(n), I64(f), f, _p(sv), sv.shape[0], _p(coef), _p(intercept), _p(start), nc,
                             int(kernel), ctypes.c_double(gamma), ctypes.c_double(coef0), int(degree), _p(pred),
                             _p(dec) if dec is not None else None)
    return (pred, dec) if want_dec else pred


def svc_proba(x, sv, coef, intercept, start, kernel, gamma, coef0, degree, probA, probB):
    """libsvm svm_predict_probability (coef / intercept in libsvm's sign convention)"""
    x = _c(x, np.float64)
    n, f = x.shape
    start = _c(start, np.int32)
    nc = len(start) - 1
    prob = np.zeros((n, nc), np.float64)
    sv, coef, intercept = _c(sv, np.float64), _c(coef, np.float64), _c(intercept, np.float64)
    pa, pb = _c(probA, np.float64), _c(probB, np.float64)
    lib().oracle_svc_proba(_p(x), I64(n), I64(f), f, _p(sv), sv.shape[0], _p(coef), _p(intercept), _p(start), nc,
                           int(kernel), ctypes.c_double(gamma), ctypes.c_double(coef0), int(degree), _p(pa), _p(pb),
                           _p(prob))
    return prob


def knn_metric(x, y, metric):
    x = _c(x, np.float64)
    y = _c(y, np.float64)
    return lib().oracle_knn_metric(int(metric), _p(x), _p(y), x.shape[0])


def knn(q, train, metric, k):
    q = _c(q, np.float64)
    train = _c(train, np.float64)
    nq, f = q.shape
    idx = np.zeros((nq, k), np.int32)
    dist = np.zeros((nq, k), np.float64)
    lib().oracle_knn(_p(q), I64(nq), I64(f), _p(train), I64(train.shape[0]), f, int(metric), int(k), _p(idx),
                     _p(dist))
    return idx, dist


def umap_init(idx, dist, embedding, n_neighbors, local_connectivity=0.0, want_memb=False):
    idx = _c(idx, np.int32)
    dist = _c(dist, np.float64)
    emb = _c(embedding, np.float32)
    nq, k = idx.shape
    out = np.zeros((nq, emb.shape[1]), np.float32)
    memb = np.zeros((nq, k), np.float32)
    lib().oracle_umap_init(_p(idx), _p(dist), I64(nq), k, ctypes.c_double(n_neighbors),
                           ctypes.c_double(local_connectivity), _p(emb), emb.shape[1], _p(memb), _p(out))
    return (out, memb) if want_memb else out


def umap_refine(idx, memb, init, tail, n_epochs, a, b, gamma=1.0, alpha=0.25, neg_rate=5.0, seed=0):
    idx = _c(idx, np.int32)
    memb = _c(memb, np.float32)
    tail = _c(tail, np.float32)
    emb = np.array(init, dtype=np.float32, order="C", copy=True)
    nq, k = idx.shape
    lib().oracle_umap_refine(_p(idx), _p(memb), I64(nq), k, int(n_epochs), _p(tail), I64(tail.shape[0]),
                             tail.shape[1], ctypes.c_double(a), ctypes.c_double(b), ctypes.c_double(gamma),
                             ctypes.c_double(alpha), ctypes.c_double(neg_rate), ctypes.c_uint64(seed), _p(emb))
    return emb
