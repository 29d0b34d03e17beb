"""Drop-in for hiprfish-image-analysis-synthetic-community/hiprfish_imaging_classify_spectra.py:
same flags (-i/--input_spectra {s}_avgint_norm.csv, -r/--ref_clf), same output
({s}_cell_information.csv, no header, no index).

The UMAP/SVC pickles (:56-59) are never unpickled here.  -r names either
  * a classifier bundle exported to arrays (.npz with scaler, four check SVCs, UMAP and barcode
    SVC): the reference's chain (:27-35) on the device (backend.py);
  * or a reference library for the restated classifier (a (R, C) .npy/.csv of per-barcode mean
    spectra or a directory of *_enc_N_avgint.csv measurements, see io.load_library): the
    barcode is the argmin of the segmented-cosine metric (default: the _7b_v2 gated variant,
    train_reference.py:993-1072) and the flags are segment max > 0.1 presence flags.
Columns follow the reference (:27-46): 0-62 max-normalised spectrum, 63-66 per-laser flags, 67 barcode,
68 sample, 69 label, 70-71 centroid, 72 major, 73 minor, 74 eccentricity, 75 orientation,
76 area (regionprops order: ascending label).
"""
import argparse
import os
import re
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))

import numpy as np  # noqa: E402


def main(argv=None):
    import pandas as pd
    import torch

    from hiprfish_image_analysis_amd import io, kernels as K, pipeline as P
    parser = argparse.ArgumentParser('Classify single cell spectra')
    parser.add_argument('-i', '--input_spectra', dest='input_spectra', type=str, default='')
    parser.add_argument('-r', '--ref_clf', dest='ref_clf', type=str, default='')
    parser.add_argument('--variant', type=int, default=2, help='0 ungated, 1 channel_cosine_intensity, 2 _7b_v2')
    args = parser.parse_args(argv)
    sample = re.sub('_avgint_norm.csv', '', args.input_spectra)                   # :24
    dev = torch.device("cuda", 0)
    avgint = pd.read_csv(args.input_spectra)                                      # :25
    segmentation = np.load('{}_seg.npy'.format(sample), allow_pickle=False)       # :26
    avgint_norm = avgint.values / np.max(avgint.values, axis=1)[:, None]          # :27
    x = torch.from_numpy(np.ascontiguousarray(avgint_norm, dtype=np.float64)).to(dev)
    if args.ref_clf.endswith('.npz'):
        from hiprfish_image_analysis_amd import backend as B
        model = B.ClassifierModel.load(args.ref_clf, dev)                         # :56-59 as arrays
        cls, classes, feats_t = model.classify(x)                                 # :28-35
        codes = np.asarray(classes)[cls.cpu().numpy()].astype(str)
        feats = feats_t.cpu().numpy()
    else:
        libspec, nbit = io.load_library(args.ref_clf)
        bounds = P.MULTI_BOUNDS if avgint_norm.shape[1] == 63 else (0, avgint_norm.shape[1])
        lib = P.Library(torch.from_numpy(libspec).to(dev), bounds, nbit)
        nseg = len(bounds) - 1
        feats = np.concatenate((avgint_norm, np.zeros((avgint_norm.shape[0], nseg))), axis=1)   # :28
        feats[:, -nseg:] = P.segment_flags(x, bounds).cpu().numpy()               # :30-33
        idx, _ = P.classify_cells(x, lib, variant=args.variant)                   # :34-35
        codes = np.array(P.barcode_strings(idx.cpu().numpy(), nbit))
    cell_info = pd.DataFrame(np.concatenate((feats, codes[:, None]), axis=1))    # :36
    cell_info[68] = sample                                                        # :37
    seg = torch.from_numpy(segmentation.astype(np.int32)).to(dev)
    maxlab = int(segmentation.max()) if segmentation.size else 0
    props = K.region_props(seg, maxlab).cpu().numpy()                             # :38 regionprops
    props = props[1:][props[1:, 7] > 0]
    labels = np.nonzero(np.bincount(segmentation.ravel().astype(np.int64), minlength=maxlab + 1)[1:])[0] + 1
    cell_info[69] = labels                                                        # :39
    cell_info[70] = props[:, 1]                                                   # :40 centroid row
    cell_info[71] = props[:, 2]                                                   # :41 centroid col
    cell_info[72] = props[:, 3]                                                   # :42 major_axis_length
    cell_info[73] = props[:, 4]                                                   # :43 minor_axis_length
    cell_info[74] = props[:, 5]                                                   # :44 eccentricity
    cell_info[75] = props[:, 6]                                                   # :45 orientation
    cell_info[76] = props[:, 0].astype(np.int64)                                  # :46 area
    cell_info.to_csv('{}_cell_information.csv'.format(sample), index=None, header=None)   # :47-48
    return cell_info


if __name__ == '__main__':
    main()
