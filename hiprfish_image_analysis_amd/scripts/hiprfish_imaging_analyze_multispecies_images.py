"""Drop-in for hiprfish-image-analysis-synthetic-community/hiprfish_imaging_analyze_multispecies_images.py
(the consumer of the _cell_information.csv files classify_spectra writes):
same CLI (positional input_folder, -p/--probe_design_filename x3).

summarize_error_rate (:34-121) restated on the host (pandas; no GPU work): for each encoding set
B, C, A the *_{set}_*_cell_information.csv files of the folder, their taxon from the file name,
the taxon's barcode from the probe design, the fraction of cells whose barcode (column 67)
differs (ErrorRate; 1 / n_cells with UpperLimit = 1 when none does), the per-cell Hamming
distances of the cells brighter than 0.75 x the mode of their max channel intensity.  The
reference only plots these; this script also writes them, as multispecies_error_rate.csv
(one row per set x taxon) and multispecies_hamming_distance.csv (one row per kept cell), and
draws the reference's two-panel figure (multispecies_error_rate.pdf) when matplotlib is
importable.  plot_representative_cell_image (:123-) is a figure of cell crops and is not
reproduced (plotting is out of scope).
"""
import argparse
import glob
import os
import re

import numpy as np

ENCODING_SETS = ("B", "C", "A")          # :38
SET_LABELS = ("Least Complex", "Most Complex", "Random")
SCI_NAME = {564: "E. coli", 1718: "C. glutamicum", 1590: "L. plantarum", 140100: "V. albensis",
            1580: "L. brevis", 438: "A. plantarum", 104102: "A. tropicalis", 108981: "A. schindleri",
            285: "C. testosteroni", 1353: "E. gallinarum", 56459: "X. vasicola"}   # :46-57


def hamming2(s1, s2):
    """:28-31"""
    assert len(s1) == len(s2)
    return sum(c1 != c2 for c1, c2 in zip(s1, s2))


def _mode(values):
    """scipy.stats.mode(values, axis=None)[0][0]: the most frequent value, the smallest on ties"""
    u, c = np.unique(values, return_counts=True)
    return u[np.argmax(c)]


def summarize_error_rate(input_folder, probe_design_filename):
    """-> (summary DataFrame, hamming DataFrame) in the reference's per-set order"""
    import pandas as pd
    rows, ham = [], []
    for k, enc_set in enumerate(ENCODING_SETS):
        filenames = sorted(glob.glob("{}/*_{}_*_cell_information.csv".format(input_folder, enc_set)))   # :40-41
        samples = [re.sub("_cell_information.csv", "", f) for f in filenames]
        probes = pd.read_csv(probe_design_filename[k], dtype={"code": str})                           # :43
        summary = probes.loc[:, ["target_taxon", "code"]].drop_duplicates().reset_index(drop=True)
        summary["ErrorRate"] = 0.0
        summary["UpperLimit"] = 0
        summary["samples"] = None
        taxid_list = [re.sub("_", "", re.sub("_fov_1", "", re.search("_.[0-9]*_fov_1", f).group(0)))
                      for f in filenames]                                                              # :60
        for s, taxid in zip(samples, taxid_list):
            cell_info = pd.read_csv("{}_cell_information.csv".format(s), header=None, dtype={67: str})  # :64
            maxint = cell_info.iloc[:, 0:63].values.max(axis=1)
            sel = summary.target_taxon.values == int(taxid)
            assignment = summary.loc[sel, "code"].values[0]
            mode = _mode(maxint)
            n_all = cell_info.shape[0]
            error_rate = 1 - np.sum(cell_info.iloc[:, 67].values == assignment) / n_all               # :70
            hd = np.array([hamming2(c, assignment) for c in cell_info[67].values])
            keep = maxint > 0.75 * mode                                                               # :72
            for c, d in zip(cell_info[67].values[keep], hd[keep]):
                ham.append({"set": enc_set, "target_taxon": int(taxid), "sample": s, "barcode": c,
                            "hamming_distance": int(d)})
            summary.loc[sel, "samples"] = s
            if error_rate > 0:
                summary.loc[sel, "ErrorRate"] = error_rate
            else:                                                                                    # :77-79
                summary.loc[sel, "ErrorRate"] = 1 / int(keep.sum())
                summary.loc[sel, "UpperLimit"] = 1
        summary = summary.sort_values(["samples"])
        summary["sci_name"] = [SCI_NAME.get(int(t)) for t in summary.target_taxon.values]
        summary.insert(0, "set", enc_set)
        rows.append(summary)
    return pd.concat(rows, ignore_index=True), pd.DataFrame(ham)


def plot(summary, ham, path):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    colors = ("darkviolet", "dodgerblue", "orangered")
    fig, axes = plt.subplots(2, 1, figsize=(8.75 * 0.393701, 7.25 * 0.393701))
    for k, enc_set in enumerate(ENCODING_SETS):
        s = summary[summary["set"] == enc_set]
        x = np.arange(len(s))
        up = s.UpperLimit.values == 1
        axes[0].plot(x[~up], s.ErrorRate.values[~up], "o", color=colors[k], markersize=4, alpha=0.8)
        axes[0].plot(x[up], s.ErrorRate.values[up], "v", color=colors[k], markersize=4, alpha=0.8)
        h = ham[ham["set"] == enc_set] if len(ham) else ham
        data = [h.loc[h["sample"] == smp, "hamming_distance"].values for smp in s.samples.values] if len(h) else []
        data = [d if len(d) else np.zeros(1) for d in data]
        if data:
            axes[1].violinplot(data, np.arange(1, len(data) + 1) + (k - 1) * 0.1, showmeans=True, showextrema=False,
                               widths=0.5)
    axes[0].set_yscale("log")
    axes[0].set_ylabel("Error Rate", fontsize=8)
    axes[1].set_ylabel("Hamming distance", fontsize=8)
    fig.savefig(path, dpi=300, transparent=True)
    plt.close(fig)


def main(argv=None):
    parser = argparse.ArgumentParser('Summarize multispecies synthetic community measurement results')
    parser.add_argument('input_folder', type=str)
    parser.add_argument('-p', '--probe_design_filename', dest='probe_design_filename', type=str, nargs='*')
    args = parser.parse_args(argv)
    summary, ham = summarize_error_rate(args.input_folder, args.probe_design_filename)
    summary.to_csv(os.path.join(args.input_folder, "multispecies_error_rate.csv"), index=False)
    ham.to_csv(os.path.join(args.input_folder, "multispecies_hamming_distance.csv"), index=False)
    try:
        plot(summary, ham, os.path.join(args.input_folder, "multispecies_error_rate.pdf"))
    except ImportError:
        pass
    return summary, ham


if __name__ == '__main__':
    main()
