"""analyze_multispecies_images.py summarize_error_rate (:34-121) on hand-made result folders:
error rates, the 1/n upper limit when no cell is wrong, the Hamming distances of the cells
above 0.75 x the max-intensity mode.  CPU only (host code)."""
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprfish_image_analysis_amd", "scripts"))


def _cells(path, codes, maxint):
    n = len(codes)
    x = np.full((n, 63), 0.1)
    x[:, 5] = maxint
    df = pd.DataFrame(x)
    for c in range(63, 67):
        df[c] = 1.0
    df[67] = codes
    df[68] = "s"
    df.to_csv(path, header=False, index=False)


def test_summarize_error_rate(tmp_path):
    import hiprfish_imaging_analyze_multispecies_images as cli
    designs = []
    truth = {}
    for k, enc in enumerate(("B", "C", "A")):
        pd.DataFrame({"target_taxon": [564, 1718, 564], "code": ["0000011", "0000101", "0000011"],
                      "probe": ["p1", "p2", "p3"]}).to_csv(tmp_path / ("design_%s.csv" % enc), index=False)
        designs.append(str(tmp_path / ("design_%s.csv" % enc)))
        # taxon 564: 1 of 4 cells wrong (2 bits); taxon 1718: none wrong
        _cells(tmp_path / ("03_14_2019_DSGN_%s_wb_564_fov_1_cell_information.csv" % enc),
               ["0000011", "0000011", "0000110", "0000011"], [1.0, 1.0, 1.0, 0.5])
        _cells(tmp_path / ("03_14_2019_DSGN_%s_wb_1718_fov_1_cell_information.csv" % enc),
               ["0000101"] * 5, [1.0, 1.0, 1.0, 1.0, 0.2])
        truth[enc] = {564: (0.25, 0), 1718: (1 / 4, 1)}    # 1718: 1 / (cells above 0.75 x mode)
    summary, ham = cli.main([str(tmp_path), "-p"] + designs)
    assert list(summary["set"].unique()) == ["B", "C", "A"]
    for _, row in summary.iterrows():
        er, up = truth[row["set"]][row.target_taxon]
        assert abs(row.ErrorRate - er) < 1e-15 and row.UpperLimit == up
        assert row.sci_name == {564: "E. coli", 1718: "C. glutamicum"}[row.target_taxon]
    h = ham[(ham["set"] == "B") & (ham.target_taxon == 564)]
    assert sorted(h.hamming_distance.tolist()) == [0, 0, 2]      # the 0.5-intensity cell is dropped
    assert (tmp_path / "multispecies_error_rate.csv").exists()
    assert (tmp_path / "multispecies_error_rate.pdf").exists()
