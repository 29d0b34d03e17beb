"""Drop-in for the reference's Cython module `neighbor` (hiprfish-image-analysis-biofilm/
neighbor.pyx).  line_profile_v2 (:115-181) and line_profile_memory_efficient_v2 (:186-263)
run on the MI355X through libhrf.so; the fused enhance_3d returns the biofilm :811-817
result without materialising the (X, Y, Z, 72) intermediate.
line_profile_memory_efficient_v3 (:268-349, imported by biofilm :40) runs on the MI355X too
(parameters 11, 9, 9; its table reaches past the patch and the reference reads those taps
unchecked -- see DESIGN.md).  neighbor_average (:8-37: a double array viewed as float, which
raises a buffer dtype mismatch on every call) and line_profile (:42-110: prints inside its
inner loop and samples the same window for every voxel) are unused and not provided.
"""
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))
sys.path.insert(0, _HERE)

from hiprfish_image_analysis_amd import kernels as _K  # noqa: E402
from neighbor2d import _check  # noqa: E402


def line_profile_v2(image_padded, patch_size, theta_range, phi_range):
    import torch
    a = _check(image_padded, 3)
    return _K.line_profile_3d(torch.from_numpy(a).cuda(), int(patch_size), int(theta_range),
                              int(phi_range)).cpu().numpy()


def line_profile_memory_efficient_v2(image_padded, patch_size, theta_range, phi_range):
    import torch
    a = _check(image_padded, 3)
    return _K.line_profile_3d_norm(torch.from_numpy(a).cuda(), int(patch_size), int(theta_range),
                                   int(phi_range)).cpu().numpy()


def enhance_3d(image_padded):
    import torch
    a = _check(image_padded, 3)
    return _K.enhance_3d(torch.from_numpy(a).cuda()).cpu().numpy()


def line_profile_memory_efficient_v3(image_padded, patch_size, theta_range, phi_range):
    import torch
    a = _check(image_padded, 3)
    if (int(patch_size), int(theta_range), int(phi_range)) != (11, 9, 9):
        raise ValueError("line_profile_memory_efficient_v3: only (11, 9, 9) is provided")
    return _K.enhance_3d_v3(torch.from_numpy(a).cuda()).cpu().numpy()
