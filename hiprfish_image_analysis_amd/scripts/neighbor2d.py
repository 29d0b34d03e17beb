"""Drop-in for the reference's Cython module `neighbor2d` (neighbor2d.pyx:8-64).

`from neighbor2d import line_profile_2d_v2` (multispecies measurement.py:30) keeps working
with this directory on sys.path; the gather runs on the MI355X through libhrf.so.  Same
signature, same dtype contract (float64 only; a float32 buffer raises ValueError as the
typed memoryview does), same output: a new (H, W, phi_range, patch_size) float64 array.
"""
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))

from hiprfish_image_analysis_amd import kernels as _K  # noqa: E402


def _check(a, ndim):
    if not isinstance(a, np.ndarray):
        a = np.asarray(a)
    if a.dtype != np.float64:
        raise ValueError("Buffer dtype mismatch, expected 'double' but got '%s'" % a.dtype)
    if a.ndim != ndim:
        raise ValueError("Buffer has wrong number of dimensions (expected %d, got %d)" % (ndim, a.ndim))
    return np.ascontiguousarray(a)


def line_profile_2d_v2(image_padded, patch_size, phi_range):
    import torch
    a = _check(image_padded, 2)
    out = _K.line_profile_2d(torch.from_numpy(a).cuda(), int(patch_size), int(phi_range))
    return out.cpu().numpy()


def enhance_2d(image_padded):
    """Fused line_profile_2d_v2(pad, 11, 9) + the numpy chain of
    multispecies measurement.py:111-124 -> image_final (H, W) float64."""
    import torch
    a = _check(image_padded, 2)
    return _K.enhance_2d(torch.from_numpy(a).cuda()).cpu().numpy()
