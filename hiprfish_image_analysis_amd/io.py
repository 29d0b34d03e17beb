"""File surface of the reference stages (inputs and the CSV/npy/png outputs they write).

CZI input: the reference reads it through bioformats + a JVM (ecoli measurement.py:15-16,31,145);
here `czi.py` reads the ZISRAW file natively (uncompressed, Zstd and JPEG-XR grey subblocks as
czi.py documents).  When only an array is at hand, a stage given `{stem}.czi` reads the
(H, W, C_l) array from `{stem}.npy` next to it instead; everything written keeps the reference's
names and formats.
"""
from __future__ import annotations

import os
import re

import numpy as np


def load_laser_stack(path: str) -> np.ndarray:
    """One laser's (H, W, C) float32 acquisition, as bioformats.load_image returns it (ecoli
    measurement.py:145): a .czi is read by czi.load_image; otherwise (or when only the array is
    at hand) {stem}.npy holds the (H, W, C) float array."""
    stem, ext = os.path.splitext(path)
    if ext.lower() == ".czi" and os.path.exists(path):
        from . import czi
        a = czi.load_image(path)
    else:
        cand = path if ext == ".npy" else stem + ".npy"
        if not os.path.exists(cand):
            raise FileNotFoundError("%s: neither the CZI file nor %s exists" % (path, cand))
        a = np.load(cand, allow_pickle=False)
    if a.ndim == 2:
        a = a[:, :, None]
    return np.ascontiguousarray(a, dtype=np.float32)


def sample_name_ecoli(first_image: str) -> str:
    """ecoli measurement.py:143  re.sub('_[0-9]*.czi', '', image_name[0])"""
    return re.sub('_[0-9]*.czi', '', first_image)


def sample_name_multispecies(first_image: str) -> str:
    """multispecies measurement.py:182  re.sub('_[0-9][0-9][0-9].czi', '', ...)"""
    return re.sub('_[0-9][0-9][0-9].czi', '', first_image)


def savetxt_like_reference(path: str, arr: np.ndarray):
    """np.savetxt(path, arr, delimiter=',') with numpy's default fmt '%.18e' (ecoli :160-161)"""
    np.savetxt(path, arr, delimiter=',')


def label_color_image(lab: np.ndarray) -> np.ndarray:
    """Deterministic label -> RGB colouring, background black (stand-in for skimage
    color.label2rgb(seg, bg_label=0, bg_color=(0,0,0)) used by the figure writers)."""
    lab = np.asarray(lab)
    rng = np.random.default_rng(0)
    n = int(lab.max()) + 1 if lab.size else 1
    pal = rng.uniform(0.2, 1.0, (max(n, 1), 3))
    pal[0] = 0.0
    return pal[np.clip(lab, 0, n - 1)]


def save_figure(img: np.ndarray, path: str, cmap=None):
    """5x5 inch, 300 dpi, frameless (save_segmentation ecoli :129-140)"""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # figures are optional products
        return
    fig = plt.figure(frameon=False)
    fig.set_size_inches(5, 5)
    ax = plt.Axes(fig, [0, 0, 1, 1])
    fig.add_axes(ax)
    ax.imshow(img, cmap=cmap)
    fig.savefig(path, dpi=300)
    plt.close(fig)


def load_library(path: str, nbit: int | None = None):
    """Reference barcode library for the restated classifier.  `path` is
    * a .npy / .csv (R, C) array of per-barcode mean spectra (row r = barcode r + 1), or
    * a directory of per-barcode measurement outputs `*_enc_<N>_avgint.csv`: the library row of
      barcode N is the column mean of that file (train_reference.py:1395-1397).
    Rows are max-normalised.  -> (spectra (R, C) f64, nbit)"""
    if os.path.isdir(path):
        import glob
        files = glob.glob(os.path.join(path, "*_avgint.csv"))
        rows = {}
        for f in files:
            m = re.search('enc_[0-9]*', f)
            if not m:
                continue
            enc = int(re.sub('enc_', '', m.group(0)))
            rows[enc] = np.average(np.loadtxt(f, delimiter=',', ndmin=2), axis=0)
        if not rows:
            raise FileNotFoundError("no *_enc_N_avgint.csv files in %s" % path)
        R = max(rows)
        C = len(next(iter(rows.values())))
        lib = np.zeros((R, C))
        for enc, v in rows.items():
            lib[enc - 1] = v
    elif path.endswith(".npy"):
        lib = np.load(path, allow_pickle=False).astype(np.float64)
    else:
        lib = np.loadtxt(path, delimiter=',', ndmin=2).astype(np.float64)
    mx = lib.max(axis=1, keepdims=True)
    mx[mx == 0] = 1.0
    lib = lib / mx
    if nbit is None:
        nbit = int(np.ceil(np.log2(lib.shape[0] + 1)))
    return lib, nbit
