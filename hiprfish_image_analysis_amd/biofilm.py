"""Biofilm per-cell report (hiprfish_imaging_biofilm_analysis.py measure_biofilm_images_2d
:1214-1295, after the segmentation): per-cell spectra, the classifier chain with
predict_proba, regionprops shape columns, debris typing and the raw / cell-filtered barcode
adjacency matrices -- written with the reference's file names and layouts:

  {sample}_avgint.csv                  per-cell mean spectra, header 0..C-1 (:1219)
  {sample}_cell_information.csv        channel_*, intensity_classification_*, cell_barcode,
                                       max_probability, {class}_prob, sample, label, centroid_x,
                                       centroid_y, major_axis, minor_axis, eccentricity,
                                       orientation, area, epithelial_distance, max_intensity,
                                       type (:1231-1246)
  {sample}_cell_information_filtered.csv   the rows typed 'cell' (:1271-1273)
  {sample}_avgint_filtered.csv         their spectra (:1274-1275)
  {sample}_adjacency_matrix.csv / _filtered.csv   taxon code x taxon code counts (:1276-1295)

Every per-pixel and per-cell computation runs on the device (label_sums, cell_table,
backend.ClassifierModel, region_props, biofilm_typing_and_adjacency); pandas only writes.
The identification images (:1247-1258, :1260-1270: colour renderings) are not written.
The reference's script does not run as shipped (SyntaxError at :1254-1255), so
the layouts follow its source text.
"""
from __future__ import annotations

import numpy as np
import torch

from . import kernels as K
from . import pipeline as P


def cell_report(sample: str, registered: torch.Tensor, segmentation: torch.Tensor, adjacency_seg: torch.Tensor,
                model, taxon_codes, epithelial_area: torch.Tensor | None = None, calibration=None,
                write: bool = True, area_max: float = 10000.0, prob_min: float = 0.95):
    """-> dict of DataFrames (cell_info, cell_info_filtered, avgint, avgint_filtered, adjacency,
    adjacency_filtered); `model` a backend.ClassifierModel whose barcode SVC carries probA/probB;
    `calibration` folds the flat field into the spectra as the registered image's division does"""
    import pandas as pd
    seg = segmentation.to(torch.int32).contiguous()
    maxlab = int(seg.max().item()) if seg.numel() else 0
    sums, counts = K.label_sums(registered, seg, maxlab, cal=calibration)                # :1215-1218
    _, labels, avgint, avgint_norm = K.cell_table(sums, counts, maxlab)
    feats = model.features(avgint_norm)                                                   # :1220-1226
    emb = model.umap.transform(feats).double()                                            # :1227
    cls = model.svc.predict(emb)                                                          # :1228
    prob = model.svc.predict_proba(emb)                                                   # :1229
    classes = np.asarray(model.svc.classes).astype(str)
    codes = classes[cls.cpu().numpy()]
    maxp = prob.max(dim=1).values
    props = K.region_props(seg, maxlab)[labels.long()]                                    # :1234-1241
    code_index = {c: i for i, c in enumerate(np.asarray(taxon_codes).astype(str))}
    bc_idx = torch.tensor([code_index.get(c, -1) for c in codes], dtype=torch.int32, device=seg.device)
    typ = P.biofilm_typing_and_adjacency(seg, adjacency_seg, bc_idx, len(code_index), maxp, epithelial_area,
                                         area_max, prob_min)                              # :1263-1269

    f = feats.cpu().numpy()
    C = f.shape[1] - 4
    cell_info = pd.DataFrame(f[:, :C], columns=["channel_{}".format(i) for i in range(C)])
    for i in range(4):
        cell_info["intensity_classification_{}".format(i)] = f[:, C + i]
    cell_info["cell_barcode"] = codes
    cell_info["max_probability"] = maxp.cpu().numpy()
    pr = prob.cpu().numpy()
    for k, c in enumerate(classes):
        cell_info["{}_prob".format(c)] = pr[:, k]
    cell_info["sample"] = sample
    pp = props.cpu().numpy()
    cell_info["label"] = labels.cpu().numpy()
    cell_info["centroid_x"] = pp[:, 1]
    cell_info["centroid_y"] = pp[:, 2]
    cell_info["major_axis"] = pp[:, 3]
    cell_info["minor_axis"] = pp[:, 4]
    cell_info["eccentricity"] = pp[:, 5]
    cell_info["orientation"] = pp[:, 6]
    cell_info["area"] = pp[:, 0].astype(np.int64)
    cell_info["epithelial_distance"] = 0                                                  # :1243
    cell_info["max_intensity"] = f[:, :C].max(axis=1)                                     # :1244
    is_cell = typ.is_cell.cpu().numpy().astype(bool)
    cell_info["type"] = np.where(is_cell, "cell", "debris")                               # :1245, :1268
    av = avgint.cpu().numpy()
    codes_all = np.asarray(taxon_codes).astype(str)
    out = {
        "cell_info": cell_info,
        "cell_info_filtered": cell_info.loc[is_cell, :].copy(),
        "avgint": pd.DataFrame(av),
        "avgint_filtered": pd.DataFrame(av[is_cell, :]),
        "adjacency": pd.DataFrame(typ.adjacency.cpu().numpy().astype(np.float64), index=codes_all,
                                  columns=codes_all),
        "adjacency_filtered": pd.DataFrame(typ.adjacency_filtered.cpu().numpy().astype(np.float64),
                                           index=codes_all, columns=codes_all),
    }
    if write:
        out["avgint"].to_csv("{}_avgint.csv".format(sample), index=None)                   # :1219
        out["cell_info"].to_csv(sample + "_cell_information.csv", index=None)            # :1246
        out["cell_info_filtered"].to_csv(sample + "_cell_information_filtered.csv", index=None)
        out["avgint_filtered"].to_csv("{}_avgint_filtered.csv".format(sample), index=None)
        out["adjacency"].to_csv(sample + "_adjacency_matrix.csv")                         # :1294
        out["adjacency_filtered"].to_csv(sample + "_adjacency_matrix_filtered.csv")       # :1295
    return out
