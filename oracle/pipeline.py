"""CPU restatement of the reference pipelines, built from the oracle primitives.

TEST INFRASTRUCTURE ONLY (the checker for tests/, smoke() and bench.py's cpu_baseline).
Mirrors hiprfish-image-analysis-ecoli/hiprfish_imaging_spectral_image_measurement.py
segment_images (:44-127) and measure_reference_images (:142-162), and the restated
classification (train_reference.py metrics), step for step.
"""
from __future__ import annotations

import numpy as np

import oracle as O


def erosion_seeds(cell_sm, area_max=600, min_obj=10):
    """ecoli measurement.py:97-110"""
    m = cell_sm.astype(bool).copy()
    be = np.zeros_like(m)
    while m.any():
        lab, n = O.label(m.astype(np.int32), 2)
        area = np.bincount(lab.ravel(), minlength=n + 1)
        small = (lab > 0) & (area[lab] < area_max)
        be |= small
        m = (lab > 0) & ~small
        m = O.erode(m, 1)
        m = O.remove_small_objects_mask(m, min_obj, 1)
    return be


def segment_ecoli(stack, keep=None, image_cn=None):
    """ecoli measurement.py:44-127 on the registered (H, W, C) stack"""
    if image_cn is None:
        image_cn = np.log(np.sum(stack.astype(np.float64), axis=2) + 1e-2)         # :71-72
    l2, c2, _ = O.kmeans_1d(image_cn, 2)                                          # :73-84
    rough_mask = l2 == int(np.argmax(c2))
    l3, c3, _ = O.kmeans_1d(image_cn, 3)                                          # :85-94
    interior = l3 == int(np.argmax(c3))
    opened = O.opening(O.remove_small_holes(interior, 64, 1))                     # :95
    cell_sm = O.remove_small_objects_mask(opened, 50, 1)                          # :96
    be = erosion_seeds(cell_sm)                                                   # :97-110
    seeds, nseeds = O.label(O.remove_small_objects_mask(be, 10, 2).astype(np.int32), 2)   # :111-112
    seg = O.watershed(-image_cn, seeds, rough_mask)                              # :113
    seg = O.remove_small_objects_labels(seg, 100)                                # :114
    seg = O.clear_border(seg)                                                    # :115
    stats = O.region_stats(seg, nseeds)                                          # :116
    final = O.shape_filter(seg, stats, 15.0, 35.0)                               # :117-126
    if keep is not None:
        keep.update(image_cn=image_cn, rough_mask=rough_mask, interior=interior, cell_sm=cell_sm, seeds=seeds,
                    watershed=seg)
    return final, nseeds


def measure_ecoli(stack, calibration=None, keep=None, image_cn=None):
    """ecoli measurement.py:142-162 -> (segmentation, labels, avgint, avgint_norm)"""
    seg, nseeds = segment_ecoli(stack, keep, image_cn)
    st = stack.astype(np.float64)
    if calibration is not None:
        st = st.copy()
        st[..., :32] /= calibration.astype(np.float64)[..., None]                # :147-150
    labs = np.unique(seg)
    labs = labs[labs > 0]
    avgint = np.stack([st[seg == l].mean(axis=0) for l in labs]) if len(labs) else np.zeros((0, st.shape[2]))
    avgint_norm = avgint / avgint.max(axis=1, keepdims=True) if len(labs) else avgint
    return seg, labs.astype(np.int32), avgint, avgint_norm


def classify_cells(avgint_norm, library, bounds, variant=0):
    return O.classify(avgint_norm, library.astype(np.float64), bounds, variant)


def process_tile(stack, library, bounds, calibration=None):
    seg, labs, avgint, avgint_norm = measure_ecoli(stack, calibration)
    idx, dist = classify_cells(avgint_norm, library, bounds)
    counts = O.barcode_counts(idx, library.shape[0])
    return dict(segmentation=seg, labels=labs, avgint=avgint, avgint_norm=avgint_norm, cell_idx=idx,
                cell_dist=dist, counts=counts)
