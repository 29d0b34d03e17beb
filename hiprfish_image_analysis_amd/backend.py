"""The per-cell classifier back-end on the device.

Reference: ecoli hiprfish_imaging_image_classification.py:43-56 and synthetic-community
hiprfish_imaging_classify_spectra.py:27-35 classify the max-normalised cell spectra with
pickled sklearn/umap models (StandardScaler, per-laser "check" SVCs, a UMAP transform under
the segmented-cosine metric and an SVC on the embedding).  The pickles are not shipped and are
never unpickled here: a model is a plain .npz of arrays (np.load(allow_pickle=False)) whose
keys are listed in INTEGRATION.md -- an exporter would write the fitted estimators' public
attributes (support_vectors_, dual_coef_, intercept_, n_support_, classes_, _gamma, coef0,
degree, kernel; mean_, scale_; the UMAP training table _raw_data, embedding_, n_neighbors,
local_connectivity, metric name).

Stages (kernels.py -> backend.hip):
  features   avgint_norm | np.diff(channels 0..31) | check flags  (E. coli, 132 columns)
             avgint_norm | check flags on the scaled segments         (community, 67 columns)
  flags      SVC.predict per laser segment (libsvm one-vs-one)
  embedding  umap-learn transform (umap_.py, 0.4 era): exact kNN under the reference metric,
             smooth_knn_dist, membership strengths, l1 rows, init_transform, then the layout
             refinement epochs with the training embedding fixed.  The reference runs the
             refinement unseeded (random_state None, parallel numba: not reproducible run to
             run); here the negative samples come from seeded per-cell streams.  umap-learn is
             absent here: parity unpinned for this stage
  barcode    SVC.predict on the embedding
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import kernels as K

ECOLI_SEGMENTS = ((0, 32), (32, 55), (55, 75), (75, 89), (89, 95), (95, 126))   # :49-54
MULTI_SEGMENTS = ((0, 23), (23, 43), (43, 57), (57, 63))                        # classify_spectra.py:30-33
KERNELS = {"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}


@dataclass
class SvcModel:
    """An sklearn SVC as device arrays in libsvm's one-vs-one convention."""
    sv: torch.Tensor            # (nsv, f) f64
    coef: torch.Tensor          # (n_class - 1, nsv) f64, pair (a, b) votes a when its sum > 0
    intercept: torch.Tensor     # (pairs,) f64
    start: torch.Tensor         # (n_class + 1,) int32
    class_values: torch.Tensor  # (n_class,) f64 (classes_ as numbers)
    classes: np.ndarray         # classes_ as given (e.g. barcode strings)
    kernel: int
    gamma: float
    coef0: float
    degree: int
    probA: torch.Tensor | None = None   # (pairs,) f64: probA_ / probB_ (probability=True)
    probB: torch.Tensor | None = None

    @property
    def n_class(self):
        return int(self.start.numel()) - 1

    @classmethod
    def from_arrays(cls, support_vectors, dual_coef, intercept, n_support, classes, kernel="rbf", gamma=1.0,
                    coef0=0.0, degree=3, device="cuda", probA=None, probB=None):
        """sklearn's public attributes (support_vectors_, dual_coef_, intercept_, n_support_,
        classes_, kernel, _gamma, coef0, degree).  sklearn flips the sign of dual_coef_ and
        intercept_ for two classes; libsvm's own signs are restored here."""
        dual = np.asarray(dual_coef, np.float64)
        inter = np.asarray(intercept, np.float64).ravel()
        ns = np.asarray(n_support, np.int64).ravel()
        if len(ns) == 2:
            dual, inter = -dual, -inter
        start = np.concatenate([[0], np.cumsum(ns)]).astype(np.int32)
        classes = np.asarray(classes)
        try:
            cv = classes.astype(np.float64)
        except (TypeError, ValueError):
            cv = np.arange(len(classes), dtype=np.float64)
        k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        pa = None if probA is None else t(np.asarray(probA, np.float64).ravel())
        pb = None if probB is None else t(np.asarray(probB, np.float64).ravel())
        return cls(t(np.asarray(support_vectors, np.float64)), t(dual), t(inter), t(start), t(cv), classes, k,
                   float(gamma), float(coef0), int(degree), pa, pb)

    @classmethod
    def from_npz(cls, z, prefix, device="cuda"):
        g = lambda key, default=None: z[prefix + key] if (prefix + key) in z.files else default  # noqa: E731
        kernel = g("kernel", np.array("rbf"))
        kernel = kernel.item() if kernel.shape == () else kernel
        if isinstance(kernel, bytes):
            kernel = kernel.decode()
        sv = g("support_vectors")
        return cls.from_arrays(g("sv") if sv is None else sv, g("dual_coef"), g("intercept"), g("n_support"), g("classes"),
                               kernel if isinstance(kernel, str) else int(kernel), float(g("gamma", 1.0)),
                               float(g("coef0", 0.0)), int(g("degree", 3)), device, g("probA"), g("probB"))

    def predict(self, x, out_column=None):
        return K.svc_predict(x, self, out_column)

    def predict_proba(self, x):
        return K.svc_predict_proba(x, self)


@dataclass
class UmapModel:
    """The parts of a fitted umap.UMAP that transform() reads."""
    trainT: torch.Tensor        # (f, n_train) f64: the training table (_raw_data), feature-major
    embedding: torch.Tensor     # (n_train, d) float32 (embedding_)
    n_neighbors: int
    local_connectivity: float
    metric: str
    a: float = 1.577           # _a, _b: umap's curve for min_dist 0.1, spread 1 (find_ab_params)
    b: float = 0.8951
    repulsion_strength: float = 1.0
    negative_sample_rate: int = 5
    n_epochs: int = -1          # the fitted n_epochs (-1: None, transform's 100 / 30 rule)
    initial_alpha: float = 1.0  # _initial_alpha (learning_rate)
    refine: bool = True         # False: stop at the initial embedding
    seed: int = 0

    @classmethod
    def from_npz(cls, z, prefix="umap_", device="cuda"):
        g = lambda key, default=None: z[prefix + key] if (prefix + key) in z.files else default  # noqa: E731
        train = np.asarray(g("raw_data"), np.float64)
        metric = g("metric", np.array("euclidean")).item()
        if isinstance(metric, bytes):
            metric = metric.decode()
        return cls(torch.from_numpy(np.ascontiguousarray(train.T)).to(device),
                   torch.from_numpy(np.ascontiguousarray(np.asarray(g("embedding"), np.float32))).to(device),
                   int(g("n_neighbors")), float(g("local_connectivity", 1.0)), metric,
                   float(g("a", 1.577)), float(g("b", 0.8951)), float(g("repulsion_strength", 1.0)),
                   int(g("negative_sample_rate", 5)), int(g("n_epochs", -1)), float(g("initial_alpha", 1.0)))

    def transform_epochs(self, nq):
        """umap_.py transform: 100 epochs up to 10000 queries, else 30; a fitted n_epochs / 3"""
        if self.n_epochs is None or self.n_epochs < 0:
            return 100 if nq <= 10000 else 30
        return int(self.n_epochs // 3.0)

    def transform(self, features):
        """umap-learn transform (see module doc): float32 (nq, d)"""
        idx, dist = K.knn(features, self.trainT, self.metric, self.n_neighbors)
        init, memb = K.umap_init_transform(idx, dist, self.embedding, self.n_neighbors,
                                           max(0.0, self.local_connectivity - 1.0), want_memb=True)
        ne = self.transform_epochs(features.shape[0])
        if not self.refine or ne < 1:
            return init
        return K.umap_refine(idx, memb, init, self.embedding, ne, self.a, self.b, self.repulsion_strength,
                             self.initial_alpha / 4.0, self.negative_sample_rate, self.seed)


def features_ecoli(avgint_norm, checks):
    """image_classification.py:47-54: the 132-column table, flags 126..131 from the six check
    SVCs on their segments"""
    f = K.features_ecoli(avgint_norm)
    for k, (lo, hi) in enumerate(ECOLI_SEGMENTS):
        checks[k].predict(f[:, lo:hi], out_column=f[:, 126 + k])
    return f


def features_multi(avgint_norm, scaler_mean, scaler_scale, checks):
    """classify_spectra.py:27-33: the 67-column table, flags 63..66 from the four check SVCs
    on the StandardScaler-scaled segments"""
    f = K.features_multi(avgint_norm)
    scaled = K.standard_scale(f[:, 0:63], scaler_mean, scaler_scale)
    for k, (lo, hi) in enumerate(MULTI_SEGMENTS):
        checks[k].predict(scaled[:, lo:hi], out_column=f[:, 63 + k])
    return f


@dataclass
class ClassifierModel:
    """The reference's classifier bundle as arrays (ecoli: 6 checks, no scaler; community: 4
    checks + scaler)."""
    checks: list
    umap: UmapModel
    svc: SvcModel
    scaler_mean: torch.Tensor | None = None
    scaler_scale: torch.Tensor | None = None

    @classmethod
    def load(cls, path, device="cuda"):
        z = np.load(path, allow_pickle=False)
        nchk = int(z["n_checks"])
        checks = [SvcModel.from_npz(z, "check%d_" % k, device) for k in range(nchk)]
        sm = ss = None
        if "scaler_mean" in z.files:
            sm = torch.from_numpy(np.asarray(z["scaler_mean"], np.float64)).to(device)
            ss = torch.from_numpy(np.asarray(z["scaler_scale"], np.float64)).to(device)
        return cls(checks, UmapModel.from_npz(z, "umap_", device), SvcModel.from_npz(z, "svc_", device), sm, ss)

    def features(self, avgint_norm):
        if len(self.checks) == 6:
            return features_ecoli(avgint_norm, self.checks)
        return features_multi(avgint_norm, self.scaler_mean, self.scaler_scale, self.checks)

    def classify(self, avgint_norm):
        """-> (class index per cell (int32 device), the classes_ array, the feature table)"""
        feats = self.features(avgint_norm)
        emb = self.umap.transform(feats).double()     # sklearn reads the float32 embedding as f64
        return self.svc.predict(emb), self.svc.classes, feats
