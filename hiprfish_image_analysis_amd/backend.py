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
  embedding  exact kNN under the reference metric + umap-learn's transform initialisation
             (smooth_knn_dist, membership strengths, l1 rows, init_transform); the layout
             optimisation epochs umap-learn runs after it are not restated (stochastic, and
             umap-learn is absent here: parity unpinned for this stage)
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

    @property
    def n_class(self):
        return int(self.start.numel()) - 1

    @classmethod
    def from_arrays(cls, support_vectors, dual_coef, intercept, n_support, classes, kernel="rbf", gamma=1.0,
                    coef0=0.0, degree=3, device="cuda"):
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
        return cls(t(np.asarray(support_vectors, np.float64)), t(dual), t(inter), t(start), t(cv), classes, k,
                   float(gamma), float(coef0), int(degree))

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
                               float(g("coef0", 0.0)), int(g("degree", 3)), device)

    def predict(self, x, out_column=None):
        return K.svc_predict(x, self, out_column)


@dataclass
class UmapModel:
    """The parts of a fitted umap.UMAP that transform() reads."""
    trainT: torch.Tensor        # (f, n_train) f64: the training table, feature-major
    embedding: torch.Tensor     # (n_train, d) f64
    n_neighbors: int
    local_connectivity: float
    metric: str

    @classmethod
    def from_npz(cls, z, prefix="umap_", device="cuda"):
        train = np.asarray(z[prefix + "raw_data"], np.float64)
        metric = z[prefix + "metric"].item() if (prefix + "metric") in z.files else "euclidean"
        if isinstance(metric, bytes):
            metric = metric.decode()
        return cls(torch.from_numpy(np.ascontiguousarray(train.T)).to(device),
                   torch.from_numpy(np.ascontiguousarray(np.asarray(z[prefix + "embedding"], np.float64))).to(device),
                   int(z[prefix + "n_neighbors"]), float(z[prefix + "local_connectivity"])
                   if (prefix + "local_connectivity") in z.files else 1.0, metric)

    def transform(self, features):
        """umap-learn transform's neighbour graph and initial embedding (see module doc)"""
        idx, dist = K.knn(features, self.trainT, self.metric, self.n_neighbors)
        return K.umap_init_transform(idx, dist, self.embedding, self.n_neighbors,
                                     max(0.0, self.local_connectivity - 1.0))


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
        emb = self.umap.transform(feats)
        return self.svc.predict(emb), self.svc.classes, feats
