"""Write a fitted classifier bundle as plain arrays (.npz) for backend.ClassifierModel.load.

The reference loads four joblib pickles per run (ecoli image_classification.py:44-46,
synthetic-community classify_spectra.py:56-59): the UMAP transform, the barcode SVC, the list
of per-laser check SVCs and (community) the StandardScaler.  A maintainer who owns those
pickles loads them once in their own environment and passes the objects to export_bundle;
nothing here unpickles anything, and the .npz it writes loads with allow_pickle=False.

    from tools.export_classifier import export_bundle
    export_bundle("ecoli_classifier.npz", umap_transform, clf_umap, clf, scaler=None)

Keys (INTEGRATION.md lists them): n_checks; check{k}_* and svc_* (sv, dual_coef, intercept,
n_support, classes, kernel, gamma, coef0, degree; probA / probB when fitted with probability=True); scaler_mean / scaler_scale; umap_raw_data,
umap_embedding, umap_n_neighbors, umap_local_connectivity, umap_metric, umap_a, umap_b,
umap_repulsion_strength, umap_negative_sample_rate, umap_n_epochs (-1 = umap's default rule),
umap_initial_alpha.
"""
import numpy as np

KERNEL_CODES = {"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}


def svc_arrays(clf, prefix):
    """sklearn SVC public attributes under `prefix`"""
    kernel = clf.kernel if isinstance(clf.kernel, str) else None
    if kernel not in KERNEL_CODES:
        raise ValueError("only the built-in SVC kernels are supported, got %r" % (clf.kernel,))
    classes = np.asarray(clf.classes_)
    if classes.dtype == object:
        classes = classes.astype(str)
    return {prefix + "sv": np.asarray(clf.support_vectors_, np.float64),
            prefix + "dual_coef": np.asarray(clf.dual_coef_, np.float64),
            prefix + "intercept": np.asarray(clf.intercept_, np.float64),
            prefix + "n_support": np.asarray(clf.n_support_, np.int32),
            prefix + "classes": classes,
            prefix + "kernel": np.int32(KERNEL_CODES[kernel]),
            prefix + "gamma": np.float64(clf._gamma),
            prefix + "coef0": np.float64(clf.coef0),
            prefix + "degree": np.int32(clf.degree),
            **({prefix + "probA": np.asarray(clf.probA_, np.float64), prefix + "probB": np.asarray(clf.probB_, np.float64)}
               if getattr(clf, "probability", False) else {})}


def umap_arrays(um):
    metric = um.metric if isinstance(um.metric, str) else getattr(um.metric, "__name__", "")
    n_epochs = getattr(um, "n_epochs", None)
    return {"umap_raw_data": np.asarray(um._raw_data, np.float64),
            "umap_embedding": np.asarray(um.embedding_, np.float64),
            "umap_n_neighbors": np.int32(getattr(um, "_n_neighbors", um.n_neighbors)),
            "umap_local_connectivity": np.float64(um.local_connectivity),
            "umap_metric": np.array(metric),
            "umap_a": np.float64(um._a), "umap_b": np.float64(um._b),
            "umap_repulsion_strength": np.float64(um.repulsion_strength),
            "umap_negative_sample_rate": np.int32(um.negative_sample_rate),
            "umap_n_epochs": np.int32(-1 if n_epochs is None else n_epochs),
            "umap_initial_alpha": np.float64(getattr(um, "_initial_alpha", getattr(um, "learning_rate", 1.0)))}


def bundle_arrays(umap_transform, clf_umap, checks, scaler=None):
    out = {"n_checks": np.int32(len(checks))}
    for k, c in enumerate(checks):
        out.update(svc_arrays(c, "check%d_" % k))
    out.update(svc_arrays(clf_umap, "svc_"))
    if scaler is not None:
        out["scaler_mean"] = np.asarray(scaler.mean_, np.float64)
        out["scaler_scale"] = np.asarray(scaler.scale_, np.float64)
    out.update(umap_arrays(umap_transform))
    return out


def export_bundle(path, umap_transform, clf_umap, checks, scaler=None):
    np.savez(path, **bundle_arrays(umap_transform, clf_umap, checks, scaler))
    return path
