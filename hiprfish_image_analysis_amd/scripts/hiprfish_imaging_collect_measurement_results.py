"""Drop-in for hiprfish-image-analysis-ecoli/hiprfish_imaging_collect_measurement_results.py:
same positional arguments and -t/--type (main :110-128), same output tables.

  data_dir simulation_table simulation_results [-t R|M]

-t R (reference libraries, :18-69): per image the cell count, the encoding's bit count and
the single/double/multiple bit error rates of its `_cell_ids.txt` against the encoding.
-t M (mixtures, :71-102): per image the cell count and, per field of view, the number of
cells of every barcode 1..1023 -- the per-barcode histogram runs
on the MI355X (hrf_barcode_counts), the table around it is host bookkeeping.  Files are
written at the same points of the loop as the reference writes them, so partial inputs give
the same partial outputs.
"""
import argparse
import os
import re
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))

import numpy as np  # noqa: E402

NBIT = 10


def _code(enc):
    """format(enc, '#012b') without the 0b prefix (:34, :43)"""
    return format(enc, '0%db' % NBIT)


def _read_ids(path):
    import pandas as pd
    ids = pd.read_csv(path, header=None, dtype=str)
    ids.columns = ['Barcodes']
    return ids


def collect_reference(data_dir, table, out):
    import pandas as pd
    sim = pd.read_csv(table)
    for col in ('NCells', 'BarcodeComplexity', 'Barcodes', 'MostCommonSingleErrorBit'):
        sim[col] = 0
    for i in range(sim.shape[0]):
        folder, name = sim.SAMPLE.values[i], sim.IMAGES.values[i]
        enc = int(re.search('enc_[0-9]*', name).group(0)[4:])
        sim.loc[i, 'Barcodes'] = enc
        code = _code(enc)
        sim.loc[i, 'BarcodeComplexity'] = code.count('1')
        avg = '{}/{}/{}_avgint.csv'.format(data_dir, folder, name)
        idf = '{}/{}/{}_cell_ids.txt'.format(data_dir, folder, name)
        if os.path.exists(avg):
            sim.loc[i, 'NCells'] = pd.read_csv(avg, header=None).shape[0]
        else:
            print('Sample result file %s does not exist' % avg)
        if not os.path.exists(idf):
            continue
        ids = _read_ids(idf).Barcodes.values
        n = ids.shape[0]
        wrong = ids[ids != code]
        err = 1 - (n - wrong.shape[0]) / n
        sim.loc[i, 'ErrorRate'] = 1 / n if err == 0 else err
        sim.loc[i, 'ErrorRateUpperLimit'] = 'T' if err == 0 else 'F'
        nbits = np.array([sum(a != b for a, b in zip(w, code)) for w in wrong], dtype=np.int64)
        sim.loc[i, 'OneBitError'] = np.count_nonzero(nbits == 1) / n
        sim.loc[i, 'TwoBitError'] = np.count_nonzero(nbits == 2) / n
        sim.loc[i, 'MultipleBitError'] = np.count_nonzero(nbits > 2) / n
        sim.to_csv(out, index=False, header=True)


def collect_mix(data_dir, table, out):
    import pandas as pd
    import torch

    from hiprfish_image_analysis_amd import kernels as K
    sim = pd.read_csv(table)
    sim['NCells'] = 0
    sim['FOV'] = 0
    R = 2 ** NBIT - 1
    abundance = pd.DataFrame(np.arange(1, R + 1), columns=['Barcodes'])
    for i in range(sim.shape[0]):
        folder, name = sim.SAMPLE.values[i], sim.IMAGES.values[i]
        sim.loc[i, 'FOV'] = int(re.search('fov_[0-9]*', name).group(0)[4:])
        avg = '{}/{}/{}_avgint.csv'.format(data_dir, folder, name)
        idf = '{}/{}/{}_cell_ids.txt'.format(data_dir, folder, name)
        if os.path.exists(avg):
            sim.loc[i, 'NCells'] = pd.read_csv(avg, header=None).shape[0]
        else:
            print('Sample result file %s does not exist' % avg)
        if os.path.exists(idf):
            bc = np.array([int(x, 2) for x in _read_ids(idf).Barcodes.values], dtype=np.int32)
            # barcode b counts in slot b - 1; hrf_barcode_counts ignores ids outside 0..R-1
            counts = K.barcode_counts(torch.from_numpy(bc - 1).cuda(), R).cpu().numpy()
            col = 'FOV{}'.format(i + 1)
            present = counts > 0        # value_counts lists the barcodes that occur
            fov = pd.DataFrame({col: counts[present].astype(np.int64), 'Barcodes': np.nonzero(present)[0] + 1})
            abundance = abundance.merge(fov, on='Barcodes', how='left').fillna(0)
        sim.to_csv(out, index=False, header=True)
        abundance.to_csv(re.sub('.csv', '_abundance.csv', out), index=False, header=True)


def main(argv=None):
    parser = argparse.ArgumentParser('Collect summary statistics of HiPRFISH probes for a complex microbial community')
    parser.add_argument('data_dir', type=str)
    parser.add_argument('simulation_table', type=str)
    parser.add_argument('simulation_results', type=str)
    parser.add_argument('-t', '--type', dest='type', type=str, default='R')
    args = parser.parse_args(argv)
    if args.type == 'R':
        collect_reference(args.data_dir, args.simulation_table, args.simulation_results)
    else:
        collect_mix(args.data_dir, args.simulation_table, args.simulation_results)


if __name__ == '__main__':
    main()
