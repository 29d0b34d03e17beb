"""Drop-in for hiprfish-image-analysis-synthetic-community/
hiprfish_imaging_multispecies_spectral_image_measurement.py: same flags (main :176-184), same
outputs ({s}_seg.npy, {s}_seg.png, {s}_sum.png, {s}_enhanced.png, {s}_registered.npy,
{s}_avgint_norm.csv), computed on the MI355X.

  -i/--image_name FILE...   any one of the sample's images; as the reference (:79-81) the
                            stage reads {s}_488, {s}_514, {s}_561 and {s}_633
  -c/--calibration FILE     calibration .npy dividing the registered stack (:103-104):
                            (H, W, C), (C,) or (H, W) (every channel)
  --shifts dr,dc ...        override the registration estimate (:82-84) for lasers 2..4
"""
import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))

import numpy as np  # noqa: E402

EXCITATIONS = ['488', '514', '561', '633']


def main(argv=None):
    import pandas as pd
    import torch

    from hiprfish_image_analysis_amd import io, kernels as K, pipeline as P
    parser = argparse.ArgumentParser('Measure multispecies synthetic spectral images')
    parser.add_argument('-i', '--image_name', dest='image_name', nargs='*', default=[], type=str)
    parser.add_argument('-c', '--calibration', dest='calibration', type=str, default='')
    parser.add_argument('--shifts', nargs='*', default=None)
    args = parser.parse_args(argv)
    if not args.image_name:
        parser.error("no images given")
    sample = io.sample_name_multispecies(args.image_name[0])                     # :182
    dev = torch.device("cuda", 0)
    lasers = [torch.from_numpy(io.load_laser_stack('{}_{}.czi'.format(sample, x))).to(dev)
              for x in EXCITATIONS]                                              # :79-81
    if args.shifts:
        shifts = [(0, 0)] + [tuple(int(v) for v in s.split(',')) for s in args.shifts]
    else:
        shifts = P.estimate_shifts(lasers, reduce="sum", clamp=None)             # :82-84
    for r, c in shifts:
        print(r, c)                                                              # :91
    stack = K.register_assemble(lasers, shifts, apply_mask=False)                # :85-102
    del lasers
    cal = None
    if args.calibration:
        cal = torch.from_numpy(np.load(args.calibration, allow_pickle=False).astype(np.float32)).to(dev)   # :39-41
    m = P.measure_multispecies(stack, cal)
    seg = m.segmentation.cpu().numpy().astype(np.int64)
    io.save_figure(io.label_color_image(seg), sample + '_seg.png')               # :43-53
    np.save(sample + '_seg', seg)
    io.save_figure(m.extras["image_sum"].cpu().numpy(), sample + '_sum.png', cmap='jet')            # :163
    io.save_figure(m.extras["final_bkg"].cpu().numpy(), sample + '_enhanced.png', cmap='jet')      # :164
    registered = K.calibrate(stack, cal) if cal is not None else stack.to(torch.float64)
    np.save('{}_registered.npy'.format(sample), registered.cpu().numpy())       # :166
    del registered
    pd.DataFrame(m.avgint_norm.cpu().numpy()).to_csv('{}_avgint_norm.csv'.format(sample), index=None)   # :173
    return m


if __name__ == '__main__':
    main()
