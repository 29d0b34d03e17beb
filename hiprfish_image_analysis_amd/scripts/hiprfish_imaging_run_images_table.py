"""Run the measurement stage over an image table, as the reference's Snakefiles do.

The reference drives every stage from an image table (examples/images_table_*.csv: SAMPLE,
IMAGES, CALIBRATION, CALIBRATION_FILENAME, ...) and a DATA_DIR (hiprfish_config_imaging.json).
Its rule measure_image / measure_reference_image (ecoli Snakefile:67-82, reference
Snakefile:92-107, synthetic-community Snakefile:92-103) call the measurement script per row on

    {DATA_DIR}/{SAMPLE}/{IMAGES}_{exc}.czi   for exc in 405 488 514 561 633   (ecoli, reference)
                                             for exc in 488 514 561 633       (multispecies)
    -c {CALIBRATION} -cf {DATA_DIR}/{CALIBRATION_FILENAME}                    (ecoli, reference)
    -c {DATA_DIR}/{CALIBRATION_FILENAME}                                      (multispecies)

and write {DATA_DIR}/{SAMPLE}/{IMAGES}_avgint.csv, _avgint_norm.csv, _seg.npy, _seg.png.  This
driver does the same rows in one process (one device context for the whole table) with the
drop-in measurement scripts; it is not a workflow engine (no DAG, no up-to-date checks).

    python hiprfish_imaging_run_images_table.py TABLE DATA_DIR [-t E|R|M] [--dry-run]
"""
import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))

EXCITATIONS = {"E": ("405", "488", "514", "561", "633"), "R": ("405", "488", "514", "561", "633"),
               "M": ("488", "514", "561", "633")}


def read_table(path):
    """the image table (CRLF or LF, as the examples are)"""
    import pandas as pd
    return pd.read_csv(path)


def plan(table, data_dir, kind="E"):
    """-> [(IMAGES, argv for the measurement script, output stem)] in table order"""
    if kind not in EXCITATIONS:
        raise ValueError("image type must be E (ecoli), R (reference) or M (multispecies)")
    rows = []
    for i in table.index.tolist():
        folder, sample = str(table.loc[i, "SAMPLE"]), str(table.loc[i, "IMAGES"])
        images = ["{}/{}/{}_{}.czi".format(data_dir, folder, sample, exc) for exc in EXCITATIONS[kind]]
        calfile = "{}/{}".format(data_dir, table.loc[i, "CALIBRATION_FILENAME"])
        if kind == "M":
            argv = ["-i", *images, "-c", calfile]
        else:
            argv = ["-i", *images, "-c", str(table.loc[i, "CALIBRATION"]), "-cf", calfile]
        rows.append((sample, argv, "{}/{}/{}".format(data_dir, folder, sample)))
    return rows


def main(argv=None):
    parser = argparse.ArgumentParser("Run the HiPR-FISH measurement stage over an image table")
    parser.add_argument("image_list_table", type=str)
    parser.add_argument("data_dir", type=str)
    parser.add_argument("-t", "--image_type", dest="image_type", type=str, default="E",
                        help="E: ecoli measurement, R: reference measurement, M: multispecies")
    parser.add_argument("--dry-run", action="store_true", help="print the per-row commands only")
    args = parser.parse_args(argv)
    rows = plan(read_table(args.image_list_table), args.data_dir, args.image_type)
    if args.dry_run:
        for _, a, _ in rows:
            print(" ".join(a))
        return rows
    if args.image_type == "M":
        import hiprfish_imaging_multispecies_spectral_image_measurement as cli
    else:
        import hiprfish_imaging_spectral_image_measurement as cli
    results = []
    for sample, a, stem in rows:
        results.append((stem, cli.main(a)))
    return results


if __name__ == "__main__":
    main()
