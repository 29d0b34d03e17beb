"""Drop-in for hiprfish-image-analysis-ecoli/hiprfish_imaging_image_classification.py:
same CLI (positional input_spectra = {s}_avgint.csv, -rf/--reference_clf), same outputs
({s}_cell_ids.txt, {s}_avgint_ids.csv, {s}_identification.png).

-rf names either
  * a classifier bundle exported to arrays (.npz, see INTEGRATION.md and
    tools/export_classifier.py): the reference's own chain (:47-56) on the device -- six
    check-SVC flags, the UMAP transform (exact kNN under the violet-derivative metric and the
    transform's initial embedding) and the barcode SVC (backend.py).  Pickles are never
    unpickled here;
  * or a reference library (a (R, C) .npy/.csv of per-barcode mean spectra, or a directory of
    *_enc_N_avgint.csv reference measurements): the barcode is then the argmin of the
    reference's segmented-cosine metric over it and the flags 126-131
    are segment max > 0.1 presence flags.
Columns of _avgint_ids.csv follow the reference (:47-64): 0-94 max-normalised spectrum,
95-125 violet derivative, 126-131 per-laser flags, 132 barcode, 133 sample, 134 label.
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
    parser = argparse.ArgumentParser('Design FISH probes for a complex microbial community')
    parser.add_argument('input_spectra', type=str, default='')
    parser.add_argument('-rf', '--reference_clf', dest='ref_clf', type=str, default='')
    parser.add_argument('--variant', type=int, default=1, help='0 ungated, 1 channel_cosine_intensity gating')
    args = parser.parse_args(argv)
    sample = re.sub('_avgint.csv', '', args.input_spectra)
    print('Classifying sample {}...'.format(sample))
    dev = torch.device("cuda", 0)
    segmentation = np.load('{}_seg.npy'.format(sample), allow_pickle=False)
    avgint = pd.read_csv(args.input_spectra, header=None).values
    avgint_norm = avgint / np.max(avgint, axis=1)[:, None]                        # :43
    x = torch.from_numpy(np.ascontiguousarray(avgint_norm)).to(dev)
    if args.ref_clf.endswith('.npz'):
        from hiprfish_image_analysis_amd import backend as B
        model = B.ClassifierModel.load(args.ref_clf, dev)                         # :44-46 as arrays
        cls, classes, feats_t = model.classify(x)                                 # :47-56
        codes = np.asarray(classes)[cls.cpu().numpy()].astype(str)
        feats = feats_t.cpu().numpy()
        paint = np.array([int(c, 2) for c in codes], dtype=np.int32)              # :66-71 int(id, 2)
    else:
        libspec, nbit = io.load_library(args.ref_clf)
        bounds = P.ECOLI_BOUNDS if avgint.shape[1] == 95 else (0, avgint.shape[1])
        lib = P.Library(torch.from_numpy(libspec).to(dev), bounds, nbit)
        idx, dist = P.classify_cells(x, lib, variant=args.variant)
        idx = idx.cpu().numpy()
        codes = np.array(P.barcode_strings(idx, nbit))
        paint = (idx + 1).astype(np.int32)
        feats = np.concatenate((avgint_norm, np.zeros((avgint_norm.shape[0], 37))), axis=1)
        if avgint.shape[1] == 95:
            feats[:, 95:126] = np.diff(avgint_norm[:, 0:32], axis=1)              # :48
            feats[:, 126:131] = P.segment_flags(x, bounds).cpu().numpy()
            feats[:, 131] = (np.abs(feats[:, 95:126]).max(axis=1) > 0.01)
    np.savetxt(sample + '_cell_ids.txt', codes, fmt='%s')                         # :63
    ids = pd.DataFrame(np.concatenate((feats, codes[:, None]), axis=1))
    ids[133] = sample
    labels = np.unique(segmentation)
    ids[134] = labels[labels > 0][:len(ids)]
    ids.to_csv(sample + '_avgint_ids.csv', header=None, index=None)               # :64
    seg = torch.from_numpy(segmentation.astype(np.int32)).to(dev)
    ident = K.paint_ids(seg, torch.from_numpy(paint).to(dev)).cpu().numpy()   # :65-71
    io.save_figure(io.label_color_image(ident), sample + '_identification.png')
    return codes


if __name__ == '__main__':
    main()
