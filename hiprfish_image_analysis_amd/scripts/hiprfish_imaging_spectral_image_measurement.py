"""Drop-in for hiprfish-image-analysis-ecoli/hiprfish_imaging_spectral_image_measurement.py
(and hiprfish-image-analysis-reference/hiprfish_imaging_reference_image_measurement.py):
same flags (main :164-169), same outputs ({s}_avgint.csv, {s}_avgint_norm.csv, {s}_seg.npy,
{s}_seg.png), computed on the MI355X.

  -i/--image_name FILE...   per-laser images in 405, 488, 514, 561, 633 nm order
  -c/--calibration T|F       flat-field correction (default T)
  -cf/--calibration_images_filename  (H, W) calibration .npy applied to channels 0-31
  --shifts dr,dc ...         per-laser registration shifts overriding the estimate of
                             :45-57 (register_translation of the channel-max images)
"""
import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))

import numpy as np  # noqa: E402


def main(argv=None):
    import torch

    from hiprfish_image_analysis_amd import io, kernels as K, pipeline as P
    parser = argparse.ArgumentParser('Design FISH probes for a complex microbial community')
    parser.add_argument('-i', '--image_name', dest='image_name', nargs='*', default=[], type=str)
    parser.add_argument('-c', '--calibration', dest='cal_toggle', type=str, default='T')
    parser.add_argument('-cf', '--calibration_images_filename', dest='calibration_images_filename', type=str,
                        default='')
    parser.add_argument('--shifts', nargs='*', default=None)
    args = parser.parse_args(argv)
    if not args.image_name:
        parser.error("no images given")
    sample = io.sample_name_ecoli(args.image_name[0])
    print('Analyzing sample {}...'.format(sample))
    dev = torch.device("cuda", 0)
    lasers = [torch.from_numpy(io.load_laser_stack(f)).to(dev) for f in args.image_name]
    if args.shifts:
        shifts = [tuple(int(v) for v in s.split(',')) for s in args.shifts]
    else:
        shifts = P.estimate_shifts(lasers, reduce="max", clamp=15)               # :45-47
    # ecoli :54-57: shifts beyond 15 px are discarded
    shifts = [(r if abs(r) <= 15 else 0, c if abs(c) <= 15 else 0) for r, c in shifts]
    stack = K.register_assemble(lasers, shifts, apply_mask=True)          # :51-70
    cal = None
    if args.cal_toggle == 'T':
        cal = torch.from_numpy(np.load(args.calibration_images_filename, allow_pickle=False)
                               .astype(np.float32)).to(dev)               # :33-38
    m = P.measure_ecoli(stack, cal)
    seg = m.segmentation.cpu().numpy().astype(np.int64)
    io.save_figure(io.label_color_image(seg), sample + '_seg.png')
    np.save(sample + '_seg', seg)                                        # :139
    io.savetxt_like_reference(sample + '_avgint.csv', m.avgint.cpu().numpy())            # :160
    io.savetxt_like_reference(sample + '_avgint_norm.csv', m.avgint_norm.cpu().numpy())  # :161
    return m


if __name__ == '__main__':
    main()
