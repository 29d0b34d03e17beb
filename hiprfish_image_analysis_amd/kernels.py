"""Torch-tensor wrappers over the libhrf.so C ABI.

Device tensors in, device tensors out; every call is queued on torch's current HIP stream.
No CPU fallback exists: a CPU tensor or a missing libhrf.so raises.
"""
from __future__ import annotations

import torch

from . import _lib


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dev(t: torch.Tensor, dtype: torch.dtype, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError("%s must be a device (cuda/HIP) tensor" % name)
    if t.dtype != dtype:
        raise ValueError("%s: expected dtype %s, got %s" % (name, dtype, t.dtype))
    return t.contiguous()


def _ptr(t):
    return t.data_ptr() if t is not None else None


# ---- a5/a6/a7: line-profile enhancement ---------------------------------------------------
def line_profile_2d(pad: torch.Tensor, patch: int = 11, nphi: int = 9) -> torch.Tensor:
    """neighbor2d.line_profile_2d_v2 (neighbor2d.pyx:8-64) -> (H, W, nphi, patch) f64"""
    pad = _dev(pad, torch.float64, "image_padded")
    hp, wp = pad.shape
    H, W = hp - (patch - 1), wp - (patch - 1)
    if H < 0 or W < 0:
        raise ValueError("negative dimensions are not allowed")
    out = torch.empty((H, W, nphi, patch), dtype=torch.float64, device=pad.device)
    _lib.call("hrf_line_profile_2d", _ptr(pad), hp, wp, wp, patch, nphi, _ptr(out), _stream())
    return out


def enhance_2d(pad: torch.Tensor) -> torch.Tensor:
    """multispecies_spectral_image_measurement.py:110-124 -> final (H, W) f64"""
    pad = _dev(pad, torch.float64, "image_padded")
    hp, wp = pad.shape
    if hp < 10 or wp < 10:
        raise ValueError("negative dimensions are not allowed")
    out = torch.empty((hp - 10, wp - 10), dtype=torch.float64, device=pad.device)
    _lib.call("hrf_enhance_2d", _ptr(pad), hp, wp, wp, 11, 9, _ptr(out), _stream())
    return out


def line_profile_3d(pad: torch.Tensor, patch: int = 11, ntheta: int = 9, nphi: int = 9) -> torch.Tensor:
    """neighbor.line_profile_v2 (neighbor.pyx:115-181) -> (X, Y, Z, ndir, patch) f64"""
    pad = _dev(pad, torch.float64, "image_padded")
    xp, yp, zp = pad.shape
    X, Y, Z = xp - patch + 1, yp - patch + 1, zp - patch + 1
    if min(X, Y, Z) < 0:
        raise ValueError("negative dimensions are not allowed")
    out = torch.empty((X, Y, Z, (ntheta - 1) * nphi, patch), dtype=torch.float64, device=pad.device)
    _lib.call("hrf_line_profile_3d", _ptr(pad), xp, yp, zp, patch, ntheta, nphi, _ptr(out), _stream())
    return out


def line_profile_3d_norm(pad: torch.Tensor, patch: int = 11, ntheta: int = 9, nphi: int = 9) -> torch.Tensor:
    """neighbor.line_profile_memory_efficient_v2 (neighbor.pyx:186-263) -> (X, Y, Z, ndir) f64"""
    pad = _dev(pad, torch.float64, "image_padded")
    xp, yp, zp = pad.shape
    X, Y, Z = xp - patch + 1, yp - patch + 1, zp - patch + 1
    if min(X, Y, Z) < 0:
        raise ValueError("negative dimensions are not allowed")
    out = torch.empty((X, Y, Z, (ntheta - 1) * nphi), dtype=torch.float64, device=pad.device)
    _lib.call("hrf_line_profile_3d_norm", _ptr(pad), xp, yp, zp, patch, ntheta, nphi, _ptr(out), _stream())
    return out


def enhance_3d(pad: torch.Tensor) -> torch.Tensor:
    """biofilm_analysis.py:811-817 -> final (X, Y, Z) f64"""
    pad = _dev(pad, torch.float64, "image_padded")
    xp, yp, zp = pad.shape
    if min(xp, yp, zp) < 10:
        raise ValueError("negative dimensions are not allowed")
    out = torch.empty((xp - 10, yp - 10, zp - 10), dtype=torch.float64, device=pad.device)
    _lib.call("hrf_enhance_3d", _ptr(pad), xp, yp, zp, 11, 9, 9, _ptr(out), _stream())
    return out
