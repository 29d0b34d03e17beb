"""Torch-tensor wrappers over the libhrf.so C ABI.

Device tensors in, device tensors out; every call is queued on torch's current HIP stream.
No CPU fallback exists: a CPU tensor or a missing libhrf.so raises.
"""
from __future__ import annotations

import os

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


def enhance_3d_v3(pad: torch.Tensor) -> torch.Tensor:
    """neighbor.line_profile_memory_efficient_v3(pad, 11, 9, 9) (neighbor.pyx:268-349)"""
    pad = _dev(pad, torch.float64, "image_padded")
    xp, yp, zp = pad.shape
    if min(xp, yp, zp) < 10:
        raise ValueError("negative dimensions are not allowed")
    out = torch.empty((xp - 10, yp - 10, zp - 10), dtype=torch.float64, device=pad.device)
    _lib.call("hrf_enhance_3d_v3", _ptr(pad), xp, yp, zp, 11, 9, 9, _ptr(out), _stream())
    return out


# ---- helpers --------------------------------------------------------------------------------
def _u8(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError("%s must be a device tensor" % name)
    if t.dtype == torch.bool:
        t = t.contiguous().view(torch.uint8)
    elif t.dtype != torch.uint8:
        t = (t != 0).to(torch.uint8)
    return t.contiguous()


def _i32(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError("%s must be a device tensor" % name)
    return t.contiguous() if t.dtype == torch.int32 else t.to(torch.int32).contiguous()


def _scalar_i32(dev):
    return int(dev.item())


def _i32_host(seq):
    import numpy as np
    return np.ascontiguousarray(np.asarray(seq, dtype=np.int32))


# ---- a1-a3 ----------------------------------------------------------------------------------
def register_assemble(srcs, shifts, apply_mask=True, cn_mode=None):
    """ecoli measurement.py:51-70: shift each (H,W,C_l) laser stack, concatenate on C.
    shifts: [(dr, dc), ...] on the host, or an (nlaser, 2) int32 device tensor (read by the
    kernel: no synchronisation).  With cn_mode (device shifts only) also the channel sum of
    the assembled stack from the same pass (0 sum, 1 log(sum + 1e-2) = image_cn, 2 log10(sum
    + 1)) -> (stack, sum image f64)."""
    import ctypes
    srcs = [_dev(s, torch.float32, "laser stack") for s in srcs]
    H, W = srcs[0].shape[:2]
    ch = _i32_host([s.shape[2] for s in srcs])
    ptrs = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    out = torch.empty((H, W, int(ch.sum())), dtype=torch.float32, device=srcs[0].device)
    if isinstance(shifts, torch.Tensor) and shifts.is_cuda:
        sd = _dev(shifts, torch.int32, "shifts")
        if sd.numel() != 2 * len(srcs):
            raise ValueError("register_assemble: one (dr, dc) pair per laser expected")
        if cn_mode is not None:
            cn = torch.empty((H, W), dtype=torch.float64, device=out.device)
            _lib.call("hrf_register_assemble_cn_dev", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data, _ptr(sd),
                      len(srcs), H, W, int(bool(apply_mask)), _ptr(out), _ptr(cn), int(cn_mode), _stream())
            return out, cn
        _lib.call("hrf_register_assemble_dev", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data, _ptr(sd),
                  len(srcs), H, W, int(bool(apply_mask)), _ptr(out), _stream())
        return out
    if cn_mode is not None:
        raise ValueError("register_assemble: cn_mode needs device shifts")
    sh = _i32_host([v for d in shifts for v in (int(d[0]), int(d[1]))])
    _lib.call("hrf_register_assemble", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data, sh.ctypes.data,
              len(srcs), H, W, int(bool(apply_mask)), _ptr(out), _stream())
    return out


def _cal_layout(cal, H, W, C, cal_range=None):
    """calibration tensor -> (f32 tensor, pixel stride, channel stride, c0, c1) following numpy
    broadcasting of stack (H, W, C) / cal: (H, W) or (H, W, 1) per pixel, (C,) or (1, 1, C) per
    channel, (H, W, C) full; cal_range limits the divided channels (ecoli: 0..32)."""
    c = _dev(cal, torch.float32, "calibration")
    c0, c1 = cal_range if cal_range is not None else (0, C)
    if c.shape in ((H, W), (H, W, 1)):
        return c, 1, 0, c0, c1
    if c.shape in ((C,), (1, C), (1, 1, C)):
        return c, 0, 1, c0, c1
    if c.shape == (H, W, C):
        return c, C, 1, c0, c1
    raise ValueError("calibration of shape %s does not broadcast against the (%d, %d, %d) stack"
                     % (tuple(c.shape), H, W, C))


def channel_sum(stack, mask=None, mode=0, negate=False, cal=None, cal_range=None, out=None):
    """np.sum(stack, axis=2) (f64, numpy pairwise order); mode 1 -> log(s+1e-2), 2 -> log10(s+1);
    cal: np.sum(stack / cal, axis=2) (multispecies measurement.py:104-105); out: a contiguous
    (H, W) f64 tensor to write into"""
    stack = _dev(stack, torch.float32, "stack")
    H, W, C = stack.shape
    if out is None:
        out = torch.empty((H, W), dtype=torch.float64, device=stack.device)
    elif out.dtype != torch.float64 or tuple(out.shape) != (H, W) or not out.is_contiguous() \
            or out.device != stack.device:
        raise ValueError("channel_sum: out must be a contiguous (%d, %d) f64 tensor on the stack's device" % (H, W))
    if cal is not None:
        if mask is not None or negate:
            raise ValueError("channel_sum: calibration with mask/negate is not supported")
        c, sp, sc, c0, c1 = _cal_layout(cal, H, W, C, cal_range)
        _lib.call("hrf_channel_sum_cal", _ptr(stack), H * W, C, _ptr(c), sp, sc, c0, c1, mode, _ptr(out), _stream())
        return out
    m = _u8(mask, "mask") if mask is not None else None
    _lib.call("hrf_channel_sum", _ptr(stack), H * W, C, _ptr(m), mode, int(negate), _ptr(out), _stream())
    return out


def channel_max(stack):
    """np.max(stack, axis=2) as f64 (ecoli measurement.py:45)"""
    stack = _dev(stack, torch.float32, "stack")
    H, W, C = stack.shape
    out = torch.empty((H, W), dtype=torch.float64, device=stack.device)
    _lib.call("hrf_channel_max", _ptr(stack), H * W, C, _ptr(out), _stream())
    return out


def channel_max_multi(stacks, stacked=False, max_workgroups=0):
    """[np.max(s, axis=2) for s in stacks] (f64) in one launch; the stacks share H x W.
    stacked: return them as one (n, H, W) tensor instead of a list; max_workgroups: the launch's
    workgroup budget (0: the default; the native tile path uses 512)"""
    import ctypes
    stacks = [_dev(s, torch.float32, "stack") for s in stacks]
    H, W = stacks[0].shape[:2]
    if any(s.shape[:2] != (H, W) for s in stacks):
        raise ValueError("channel_max_multi: the stacks must share H x W")
    buf = torch.empty((len(stacks), H, W), dtype=torch.float64, device=stacks[0].device)
    outs = list(buf.unbind(0))
    src = (ctypes.c_void_p * len(stacks))(*[s.data_ptr() for s in stacks])
    dst = (ctypes.c_void_p * len(stacks))(*[o.data_ptr() for o in outs])
    ch = _i32_host([s.shape[2] for s in stacks])
    _lib.call("hrf_channel_max_multi_grid", ctypes.cast(src, ctypes.c_void_p), ch.ctypes.data, len(stacks), H * W,
              ctypes.cast(dst, ctypes.c_void_p), int(max_workgroups), _stream())
    return buf if stacked else outs


def calibrate(stack, cal, cal_range=None):
    """stack / cal as f64 (multispecies measurement.py:104, saved as _registered.npy :166)"""
    stack = _dev(stack, torch.float32, "stack")
    H, W, C = stack.shape
    out = torch.empty((H, W, C), dtype=torch.float64, device=stack.device)
    if cal is None:
        _lib.call("hrf_calibrate_f64", _ptr(stack), H * W, C, None, 0, 0, 0, 0, _ptr(out), _stream())
        return out
    c, sp, sc, c0, c1 = _cal_layout(cal, H, W, C, cal_range)
    _lib.call("hrf_calibrate_f64", _ptr(stack), H * W, C, _ptr(c), sp, sc, c0, c1, _ptr(out), _stream())
    return out


def register_translation(src, target):
    """skimage.feature.register_translation(src, target)[0] (upsample_factor 1): integer
    (row, col) shift, via hipFFT (ecoli measurement.py:45-46, multispecies :82-83)"""
    import ctypes
    import numpy as np
    src = _dev(src, torch.float64, "src")
    target = _dev(target, torch.float64, "target")
    if src.shape != target.shape or src.dim() != 2:
        raise ValueError("register_translation: two equal-shape 2-D images expected")
    H, W = src.shape
    nb = int(_lib.lib().hrf_register_workspace_bytes(H, W))
    work = torch.empty(nb, dtype=torch.uint8, device=src.device)
    sh = np.zeros(2, np.int32)
    _lib.call("hrf_register_translation", _ptr(src), _ptr(target), H, W, _ptr(work), sh.ctypes.data, _stream())
    return int(sh[0]), int(sh[1])


def register_translations_dev(ref, targets, clamp=None):
    """register_translation(ref, t) for every target, into an (1 + len(targets), 2) int32 device
    tensor whose row 0 is (0, 0): the reference's transform is taken once, nothing synchronises.
    clamp: |component| > clamp -> 0 (ecoli measurement.py:47-57), None keeps it."""
    ref = _dev(ref, torch.float64, "src")
    H, W = ref.shape
    nb = int(_lib.lib().hrf_register_workspace_bytes(H, W))
    work = torch.empty(nb, dtype=torch.uint8, device=ref.device)
    out = torch.zeros((1 + len(targets), 2), dtype=torch.int32, device=ref.device)
    cl = -1 if clamp is None else int(clamp)
    for i, t in enumerate(targets):
        t = _dev(t, torch.float64, "target")
        if t.shape != ref.shape:
            raise ValueError("register_translation: two equal-shape 2-D images expected")
        _lib.call("hrf_register_translation_dev", _ptr(ref) if i == 0 else None, _ptr(t), H, W, _ptr(work), cl,
                  _ptr(out[1 + i]), _stream())
    return out


def register_translations_batch_dev(imgs, clamp=None):
    """register_translations_dev(imgs[0], imgs[1:], clamp) from one (n, H, W) f64 tensor in one
    batch (batched hipFFT transforms, one product, argmax and shift launch each)"""
    imgs = _dev(imgs, torch.float64, "imgs")
    n, H, W = imgs.shape
    if n < 2:
        raise ValueError("register_translations_batch: a reference and at least one target expected")
    nb = int(_lib.lib().hrf_register_batch_workspace_bytes(n, H, W))
    if nb <= 0:
        raise ValueError("register_translations_batch: unsupported size")
    work = torch.empty(nb, dtype=torch.uint8, device=imgs.device)
    out = torch.empty((n, 2), dtype=torch.int32, device=imgs.device)
    _lib.call("hrf_register_translations_batch_dev", _ptr(imgs), n, H, W, _ptr(work), -1 if clamp is None else int(clamp),
              _ptr(out), _stream())
    return out


def xcorr_supported(n, H, W):
    return int(_lib.lib().hrf_xcorr_workspace_bytes(n, H, W)) > 0


def xcorr_shifts_dev(imgs, clamp=None):
    """register_translations_dev(imgs[0], imgs[1:], clamp) from one (n, H, W) f64 tensor through
    the hand-written FFT pipeline (xcorr.hip; power-of-two sizes) -> (n, 2) int32 device tensor"""
    imgs = _dev(imgs, torch.float64, "imgs")
    n, H, W = imgs.shape
    nb = int(_lib.lib().hrf_xcorr_workspace_bytes(n, H, W))
    if nb <= 0:
        raise ValueError("xcorr_shifts: unsupported size %d x %d x %d" % (n, H, W))
    work = torch.empty(nb, dtype=torch.uint8, device=imgs.device)
    out = torch.empty((n, 2), dtype=torch.int32, device=imgs.device)
    _lib.call("hrf_xcorr_shifts_dev", _ptr(imgs), n, H, W, _ptr(work), -1 if clamp is None else int(clamp), _ptr(out),
              _stream())
    return out


def xcorr_surfaces(imgs):
    """the cross-correlation surfaces of xcorr_shifts_dev: (n - 1, H, W) f64, H * W / 2 times
    numpy.fft.ifft2(F(imgs[0]) * conj(F(imgs[t]))).real (tests)"""
    imgs = _dev(imgs, torch.float64, "imgs")
    n, H, W = imgs.shape
    nb = int(_lib.lib().hrf_xcorr_workspace_bytes(n, H, W))
    if nb <= 0:
        raise ValueError("xcorr_surfaces: unsupported size %d x %d x %d" % (n, H, W))
    work = torch.empty(nb, dtype=torch.uint8, device=imgs.device)
    out = torch.empty((n - 1, H, W), dtype=torch.float64, device=imgs.device)
    _lib.call("hrf_xcorr_surfaces_dev", _ptr(imgs), n, H, W, _ptr(work), _ptr(out), _stream())
    return out


def pad_edge_3d(a, width=5):
    """skimage.util.pad(a, width, mode='edge') of an (X, Y, Z) f64 volume (biofilm :810)"""
    a = _dev(a, torch.float64, "a")
    X, Y, Z = a.shape
    out = torch.empty((X + 2 * width, Y + 2 * width, Z + 2 * width), dtype=torch.float64, device=a.device)
    _lib.call("hrf_pad_edge3_f64", _ptr(a), X, Y, Z, width, _ptr(out), _stream())
    return out


def max_f64(a):
    a = _dev(a, torch.float64, "a")
    out = torch.empty(1, dtype=torch.float64, device=a.device)
    _lib.call("hrf_max_f64", _ptr(a), a.numel(), _ptr(out), _stream())
    return out


def div_scalar(a, d):
    a = _dev(a, torch.float64, "a")
    out = torch.empty_like(a)
    _lib.call("hrf_div_scalar_f64", _ptr(a), a.numel(), _ptr(_dev(d, torch.float64, "d")), _ptr(out), _stream())
    return out


def pad_edge(a, width=5):
    a = _dev(a, torch.float64, "a")
    H, W = a.shape
    out = torch.empty((H + 2 * width, W + 2 * width), dtype=torch.float64, device=a.device)
    _lib.call("hrf_pad_edge_f64", _ptr(a), H, W, width, _ptr(out), _stream())
    return out


def and_mask(a, b):
    """a AND b on masks -> u8 (multispecies measurement.py:140, :153)"""
    x, y = _u8(a, "a"), _u8(b, "b")
    out = torch.empty_like(x)
    _lib.call("hrf_and_u8", _ptr(x), _ptr(y), x.numel(), _ptr(out), _stream())
    return out


def mask_labels(labels, mask):
    """labels * mask (multispecies measurement.py:152)"""
    l = _i32(labels, "labels")
    m = _u8(mask, "mask")
    out = torch.empty_like(l)
    _lib.call("hrf_mask_labels", _ptr(l), _ptr(m), l.numel(), _ptr(out), _stream())
    return out


def mask_mul(a, mask):
    a = _dev(a, torch.float64, "a")
    m = _u8(mask, "mask")
    out = torch.empty_like(a)
    _lib.call("hrf_mask_mul_f64", _ptr(a), _ptr(m), a.numel(), _ptr(out), _stream())
    return out


# ---- a4 -------------------------------------------------------------------------------------
def nl_means_2d(img, patch_size=7, patch_distance=11, h=0.1, sigma=0.0):
    """skimage.restoration.denoise_nl_means(img, patch_size, patch_distance, h, sigma=sigma)
    on a 2-D f64 image (multispecies measurement.py:108)"""
    img = _dev(img, torch.float64, "image")
    if img.dim() != 2:
        raise ValueError("nl_means_2d: 2-D image expected")
    H, W = img.shape
    out = torch.empty_like(img)
    _lib.call("hrf_nl_means_2d", _ptr(img), H, W, int(patch_size), int(patch_distance), float(h), float(sigma),
              _ptr(out), _stream())
    return out


# ---- a8 -------------------------------------------------------------------------------------


def kmeans_1d(x, k, valid=None, max_iter=300, want_labels=True, share=None, rule=0, n_init=10):
    """sklearn KMeans(k, random_state=0, n_init=10).fit_predict on the values of x (kmeans.hip)
    -> labels int32 (sklearn's cluster ids, or None), top-cluster mask u8 (by `rule`, see
    include/hrf.h), centres (list, sklearn order), iterations.
    share: a dict passed to successive calls on the SAME x / valid so the sort is done once."""
    import ctypes
    import numpy as np
    x = _dev(x, torch.float64, "x")
    n = x.numel()
    dev = x.device
    v = _u8(valid, "valid") if valid is not None else None
    labels = torch.empty(x.shape, dtype=torch.int32, device=dev) if want_labels else None
    top = torch.empty(x.shape, dtype=torch.uint8, device=dev)
    cen = np.zeros(k, np.float64)
    it = ctypes.c_int32(0)
    ident = (x.data_ptr(), n, v.data_ptr() if v is not None else 0)
    reuse = share is not None and share.get("ident") == ident
    if reuse:
        ws = share["ws"]
    else:
        nb = int(_lib.lib().hrf_kmeans_sorted_workspace_bytes(n))
        if nb <= 0:
            raise _lib.HrfError("hrf_kmeans_sorted_workspace_bytes failed")
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        if share is not None:
            share.update(ident=ident, ws=ws, x=x, valid=v)   # keep the inputs alive with the sort
    _lib.call("hrf_kmeans_1d_sorted", _ptr(x), _ptr(v), n, k, max_iter, n_init, rule, _ptr(labels), _ptr(top),
              cen.ctypes.data, ctypes.addressof(it), _ptr(ws), ws.numel(), int(reuse), _stream())
    return labels, top, cen.tolist(), it.value


def kmeans_1d_pair(x, k1, k2, valid=None, max_iter=300, rules=(2, 0), n_init=10):
    """top-cluster masks of KMeans(k1) and KMeans(k2) on the same x with one sort and one host
    synchronisation (ecoli measurement.py:73-94: k = 2 and k = 3 on image_cn)"""
    x = _dev(x, torch.float64, "x")
    n = x.numel()
    v = _u8(valid, "valid") if valid is not None else None
    top1 = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    top2 = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    nb = int(_lib.lib().hrf_kmeans_sorted_workspace_bytes(n))
    if nb <= 0:
        raise _lib.HrfError("hrf_kmeans_sorted_workspace_bytes failed")
    ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    _lib.call("hrf_kmeans_1d_sorted_pair", _ptr(x), _ptr(v), n, k1, k2, max_iter, n_init, rules[0], rules[1],
              _ptr(top1), _ptr(top2), _ptr(ws), ws.numel(), _stream())
    return top1, top2


def kmeans_draws(nv, k, n_init=10):
    """the fit's random stream as libhrf replays it (host): first-centre ranks, trial draws"""
    import numpy as np
    nt = 2 + int(np.log(k))
    first = np.zeros(n_init, np.int64)
    draws = np.zeros(max(1, n_init * (k - 1) * nt), np.float64)
    _lib.call("hrf_kmeans_draws", nv, k, n_init, first.ctypes.data, draws.ctypes.data)
    return first, draws[:n_init * (k - 1) * nt]


# ---- a9/a10/a13 -----------------------------------------------------------------------------
def _img(img):
    if img.dtype == torch.int32:
        return img.contiguous(), 1
    return _u8(img, "img"), 0


def cc_roots(img, conn=2):
    t, dt = _img(img)
    H, W = t.shape
    parent = torch.empty((H, W), dtype=torch.int32, device=t.device)
    _lib.call("hrf_cc_roots", _ptr(t), dt, H, W, conn, _ptr(parent), _stream())
    return parent


def label(img, conn=2, return_num=True):
    """skimage.measure.label(img, connectivity=conn): raster-first numbering"""
    t, dt = _img(img)
    H, W = t.shape
    dev = t.device
    labels = torch.empty((H, W), dtype=torch.int32, device=dev)
    parent = torch.empty((H, W), dtype=torch.int32, device=dev)
    blk = torch.empty((H * W + 1023) // 1024 + 1, dtype=torch.int32, device=dev)
    nlab = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("hrf_label", _ptr(t), dt, H, W, conn, _ptr(labels), _ptr(parent), _ptr(blk), _ptr(nlab), _stream())
    if return_num:
        return labels, _scalar_i32(nlab)
    return labels, nlab


def remove_small_objects(img, min_size=64, conn=1, maxlab=None):
    """skimage.morphology.remove_small_objects: bool -> components, int32 -> label sizes"""
    if img.dtype == torch.int32:
        H, W = img.shape
        if maxlab is None:
            maxlab = max_i32(img)
        cnt = torch.empty(maxlab + 1, dtype=torch.int32, device=img.device)
        out = torch.empty_like(img)
        _lib.call("hrf_remove_small_objects_labels", _ptr(img.contiguous()), H * W, maxlab, min_size, _ptr(out),
                  _ptr(cnt), _stream())
        return out
    m = _u8(img, "mask")
    H, W = m.shape
    out = torch.empty_like(m)
    parent = torch.empty((H, W), dtype=torch.int32, device=m.device)
    size = torch.empty((H, W), dtype=torch.int32, device=m.device)
    _lib.call("hrf_remove_small_objects_mask", _ptr(m), H, W, min_size, conn, _ptr(out), _ptr(parent), _ptr(size),
              _stream())
    return out


def remove_small_holes(mask, area_threshold=64, conn=1):
    m = _u8(mask, "mask")
    H, W = m.shape
    out = torch.empty_like(m)
    parent = torch.empty((H, W), dtype=torch.int32, device=m.device)
    size = torch.empty((H, W), dtype=torch.int32, device=m.device)
    _lib.call("hrf_remove_small_holes", _ptr(m), H, W, area_threshold, conn, _ptr(out), _ptr(parent), _ptr(size),
              _stream())
    return out


def fill_holes(mask):
    m = _u8(mask, "mask")
    H, W = m.shape
    out = torch.empty_like(m)
    parent = torch.empty((H, W), dtype=torch.int32, device=m.device)
    flag = torch.empty((H, W), dtype=torch.int32, device=m.device)
    _lib.call("hrf_fill_holes", _ptr(m), H, W, _ptr(out), _ptr(parent), _ptr(flag), _stream())
    return out


def clear_border(labels):
    l = _i32(labels, "labels")
    H, W = l.shape
    out = torch.empty_like(l)
    parent = torch.empty((H, W), dtype=torch.int32, device=l.device)
    flag = torch.empty((H, W), dtype=torch.int32, device=l.device)
    _lib.call("hrf_clear_border", _ptr(l), H, W, _ptr(out), _ptr(parent), _ptr(flag), _stream())
    return out


def relabel_sequential(labels, maxlab=None):
    l = _i32(labels, "labels")
    if maxlab is None:
        maxlab = max_i32(l)
    out = torch.empty_like(l)
    m = torch.empty(maxlab + 1, dtype=torch.int32, device=l.device)
    n = torch.zeros(1, dtype=torch.int32, device=l.device)
    _lib.call("hrf_relabel_sequential", _ptr(l), l.numel(), maxlab, _ptr(out), _ptr(m), _ptr(n), _stream())
    return out, _scalar_i32(n)


def binary_erosion(mask, border_value=1):
    m = _u8(mask, "mask")
    H, W = m.shape
    out = torch.empty_like(m)
    _lib.call("hrf_binary_erosion", _ptr(m), H, W, int(border_value), _ptr(out), _stream())
    return out


def binary_dilation(mask):
    m = _u8(mask, "mask")
    H, W = m.shape
    out = torch.empty_like(m)
    _lib.call("hrf_binary_dilation", _ptr(m), H, W, _ptr(out), _stream())
    return out


def binary_opening(mask):
    """skimage.morphology.binary_opening (cross): dilation(erosion(border=True))"""
    return binary_dilation(binary_erosion(mask, 1))


def count_nonzero(mask, sync=True):
    m = _u8(mask, "mask")
    c = torch.zeros(1, dtype=torch.int64, device=m.device)
    _lib.call("hrf_count_nonzero_u8", _ptr(m), m.numel(), _ptr(c), _stream())
    return int(c.item()) if sync else c


def max_i32(a, sync=True):
    a = _i32(a, "a")
    m = torch.zeros(1, dtype=torch.int32, device=a.device)
    _lib.call("hrf_max_i32", _ptr(a), a.numel(), _ptr(m), _stream())
    return int(m.item()) if sync else m


# ---- a12 ------------------------------------------------------------------------------------
def watershed(image, markers, mask=None, negate=False, max_passes=100000, ties: list | None = None):
    """skimage.morphology.watershed(+/-image, markers, mask=mask), 4-connectivity, with the
    heap's (value, age) order on ties.  `ties` (a list) receives [pixels that needed the exact
    order, resolution rounds, equal-valued-marker decisions] (hrf_watershed_ex); a tile with
    such a decision is flooded again by skimage's binary heap on the device (watershed_heap)."""
    import ctypes
    image = _dev(image, torch.float64, "image")
    mk = _i32(markers, "markers")
    H, W = image.shape
    m = _u8(mask, "mask") if mask is not None else None
    out = torch.empty((H, W), dtype=torch.int32, device=image.device)
    nb = _lib.lib().hrf_watershed_workspace_bytes(H, W)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=image.device)
    fl = torch.empty(8, dtype=torch.int32, device=image.device)
    passes = ctypes.c_int32(0)
    st = (ctypes.c_int32 * 3)()
    _lib.call("hrf_watershed_ex", _ptr(image), int(negate), _ptr(mk), _ptr(m), H, W, _ptr(out), _ptr(ws), _ptr(fl),
              max_passes, ctypes.addressof(passes), ctypes.addressof(st), _stream())
    if ties is not None:
        ties[:] = list(st)
    return out


def watershed_heap(image, markers, mask=None, negate=False):
    """skimage's heap flood itself on the device, one workgroup (hrf_watershed_heap): the exact
    tie path of watershed(); serial, for tests and small images"""
    image = _dev(image, torch.float64, "image")
    mk = _i32(markers, "markers")
    H, W = image.shape
    m = _u8(mask, "mask") if mask is not None else None
    out = torch.empty((H, W), dtype=torch.int32, device=image.device)
    _lib.call("hrf_watershed_heap", _ptr(image), int(negate), _ptr(mk), _ptr(m), H, W, _ptr(out), _stream())
    return out


# ---- a14-a16, a20, a21, a23 -----------------------------------------------------------------
def label_sums(stack, labels, maxlab, cal=None, cal_range=None):
    """per-label channel sums of stack (/ cal) and pixel counts (ecoli measurement.py:147-155)"""
    stack = _dev(stack, torch.float32, "stack")
    l = _i32(labels, "labels")
    H, W, C = stack.shape
    npix = l.numel()
    sums = torch.empty((maxlab + 1, C), dtype=torch.float64, device=stack.device)
    counts = torch.empty(maxlab + 1, dtype=torch.int64, device=stack.device)
    calp, sp, sc, c0, c1 = None, 1, 0, 0, C
    if cal is not None:
        c, sp, sc, c0, c1 = _cal_layout(cal, H, W, C, cal_range)
        calp = _ptr(c)
    _lib.call("hrf_label_sums_cal", _ptr(stack), _ptr(l), npix, C, maxlab, calp, sp, sc, c0, c1, _ptr(sums),
              _ptr(counts), _stream())
    return sums, counts


def _laser_args(lasers, shifts_dev):
    import ctypes
    srcs = [_dev(s, torch.float32, "laser stack") for s in lasers]
    ch = _i32_host([s.shape[2] for s in srcs])
    ptrs = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    sd = _dev(shifts_dev, torch.int32, "shifts")
    if sd.numel() != 2 * len(srcs):
        raise ValueError("one (dr, dc) pair per laser expected")
    return srcs, ch, ptrs, sd


def register_assemble_pixtable(lasers, shifts_dev, apply_mask=True, cn_mode=1, bounds=(0, 32, 55, 75, 89, 95),
                               want_stack=False):
    """the E. coli registered assembly writing image_cn and the classifier's prepared pixel table
    from one pass over the lasers (the registered stack itself only with want_stack)
    -> (image_cn f64 (H, W), PixTable, stack or None)"""
    import ctypes
    srcs, ch, ptrs, sd = _laser_args(lasers, shifts_dev)
    H, W = srcs[0].shape[:2]
    dev = srcs[0].device
    pt = pixtable_alloc((H, W), int(ch.sum()), bounds, dev)
    pt.source = LaserSource(srcs, sd, apply_mask)
    cn = torch.empty((H, W), dtype=torch.float64, device=dev)
    stack = torch.empty((H, W, int(ch.sum())), dtype=torch.float32, device=dev) if want_stack else None
    _lib.call("hrf_register_assemble_pixtable", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data, _ptr(sd), len(srcs),
              H, W, int(bool(apply_mask)), _ptr(stack) if stack is not None else None, _ptr(cn), int(cn_mode),
              _ptr(pt.table), _ptr(pt.flags), _stream())
    return cn, pt, stack


def register_assemble_cn_only(lasers, shifts_dev, apply_mask=True, cn_mode=1):
    """the E. coli registered assembly writing image_cn only (hrf_register_assemble_pixtable with
    no table: the tile path without the per-pixel classifier) -> image_cn f64 (H, W)"""
    import ctypes
    srcs, ch, ptrs, sd = _laser_args(lasers, shifts_dev)
    H, W = srcs[0].shape[:2]
    cn = torch.empty((H, W), dtype=torch.float64, device=srcs[0].device)
    _lib.call("hrf_register_assemble_pixtable", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data, _ptr(sd), len(srcs),
              H, W, int(bool(apply_mask)), None, _ptr(cn), int(cn_mode), None, None, _stream())
    return cn


def label_sums_lasers(lasers, shifts_dev, labels, maxlab, apply_mask=True, cal=None, cal_range=(0, 32)):
    """label_sums of the registered stack, read from the per-laser acquisitions (no stack);
    cal: a per-pixel (H, W) flat field on channels cal_range"""
    import ctypes
    srcs, ch, ptrs, sd = _laser_args(lasers, shifts_dev)
    l = _i32(labels, "labels")
    H, W = srcs[0].shape[:2]
    C = int(ch.sum())
    sums = torch.empty((maxlab + 1, C), dtype=torch.float64, device=l.device)
    counts = torch.empty(maxlab + 1, dtype=torch.int64, device=l.device)
    calp = None
    if cal is not None:
        c = _dev(cal, torch.float32, "calibration")
        if tuple(c.shape) != (H, W):
            raise ValueError("label_sums_lasers: the flat field must be an (H, W) plane")
        calp = _ptr(c)
    _lib.call("hrf_label_sums_lasers", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data, _ptr(sd), len(srcs), H, W,
              int(bool(apply_mask)), _ptr(l), maxlab, calp, int(cal_range[0]), int(cal_range[1]), _ptr(sums),
              _ptr(counts), _stream())
    return sums, counts


def cell_table(sums, counts, maxlab, max_rows=None):
    C = sums.shape[1]
    dev = sums.device
    if max_rows is None:
        max_rows = maxlab
    rol = torch.empty(maxlab + 1, dtype=torch.int32, device=dev)
    lor = torch.empty(max(max_rows, 1), dtype=torch.int32, device=dev)
    avg = torch.empty((max(max_rows, 1), C), dtype=torch.float64, device=dev)
    avgn = torch.empty((max(max_rows, 1), C), dtype=torch.float64, device=dev)
    nrows = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("hrf_cell_table", _ptr(sums), _ptr(counts), maxlab, C, max_rows, _ptr(rol), _ptr(lor), _ptr(avg),
              _ptr(avgn), _ptr(nrows), _stream())
    n = _scalar_i32(nrows)
    return rol, lor[:n], avg[:n], avgn[:n]


def region_props(labels, maxlab):
    l = _i32(labels, "labels")
    H, W = l.shape
    mom = torch.empty((maxlab + 1, 6), dtype=torch.int64, device=l.device)
    props = torch.empty((maxlab + 1, 8), dtype=torch.float64, device=l.device)
    _lib.call("hrf_region_moments", _ptr(l), H, W, maxlab, _ptr(mom), _stream())
    _lib.call("hrf_region_props", _ptr(mom), maxlab, _ptr(props), _stream())
    return props


def barcode_counts(bc, R):
    b = _i32(bc, "bc")
    out = torch.empty(R, dtype=torch.int64, device=b.device)
    _lib.call("hrf_barcode_counts", _ptr(b), b.numel(), R, _ptr(out), _stream())
    return out


def paint_ids(labels, code):
    l = _i32(labels, "labels")
    c = _i32(code, "code")
    out = torch.empty_like(l)
    _lib.call("hrf_paint_ids", _ptr(l), l.numel(), _ptr(c), c.numel(), _ptr(out), _stream())
    return out


# ---- a19 ------------------------------------------------------------------------------------
CLASSIFY_MODE = None   # None: 2 on the reference layouts, else 1; 1: split-fp16 MFMA; 0: f32 MFMA
REFERENCE_LAYOUTS = ((0, 32, 55, 75, 89, 95), (0, 23, 43, 57, 63))   # train_reference.py:1401, :1488


def classify_modes(bounds):
    """the per-pixel classifier modes available for a channel layout, fastest first"""
    return (2, 1, 0) if tuple(int(b) for b in bounds) in REFERENCE_LAYOUTS else (1, 0)


def _mode(bounds, mode):
    if mode is None:
        mode = CLASSIFY_MODE
    return classify_modes(bounds)[0] if mode is None else mode


def classify_geometry(C, nseg, R, mode=1):
    import ctypes
    kp, rp = ctypes.c_int32(0), ctypes.c_int32(0)
    _lib.call("hrf_classify_geometry", C, nseg, R, mode, ctypes.addressof(kp), ctypes.addressof(rp))
    return kp.value, rp.value


def classify_table_row_bytes(C, bounds, mode):
    import ctypes
    b = _i32_host(bounds)
    rb = ctypes.c_int32(0)
    _lib.call("hrf_classify_table_row_bytes", C, b.ctypes.data, len(b) - 1, mode, ctypes.addressof(rb))
    return rb.value


def classify_refx_bytes(C, bounds, R, mode):
    b = _i32_host(bounds)
    n = int(_lib.lib().hrf_classify_refx_bytes(C, b.ctypes.data, len(b) - 1, R, mode))
    if n < 0:
        raise ValueError("classify_refx_bytes: bad layout")
    return n


def classify_prepare(ref, bounds, mode=None):
    """-> prepared reference table for classify_pixels (mode 0: f32; 1: fp16 hi/lo with
    zero-segment indicator columns; 2: fp16 hi/lo, reference layouts, indicators in the epilogue),
    rows of the mode's pitch; past the MFMA table's Rpad rows the exact section the f64 refine
    reads (hrf_classify_refx_bytes)"""
    mode = _mode(bounds, mode)
    ref = _dev(ref, torch.float32, "ref")
    R, C = ref.shape
    b = _i32_host(bounds)
    kp, rp = classify_geometry(C, len(b) - 1, R, mode)
    nbytes = classify_refx_bytes(C, bounds, R, mode)
    if mode == 0:
        rows = -(-nbytes // (4 * kp))
        refx = torch.empty((rows, kp), dtype=torch.float32, device=ref.device)
    else:
        rowh = classify_table_row_bytes(C, bounds, mode) // 2                            # hi | lo | pad
        rows = -(-nbytes // (2 * rowh))
        refx = torch.empty((rows, rowh), dtype=torch.float16, device=ref.device)
    _lib.call("hrf_classify_prepare_refs", _ptr(ref), R, C, b.ctypes.data, len(b) - 1, mode, _ptr(refx), _stream())
    return refx


def refx_mode(refx, C, bounds):
    """which mode a prepared table was built for (its dtype and row width tell)"""
    if refx.dtype == torch.float32:
        return 0
    if 2 in classify_modes(bounds):
        if refx.shape[1] * 2 == classify_table_row_bytes(C, bounds, 2):
            return 2
    return 1


def _check_refx(refx, R, C, bounds, mode, where):
    if not isinstance(refx, torch.Tensor) or not refx.is_cuda or not refx.is_contiguous():
        raise ValueError("%s: the prepared library must be a contiguous device tensor" % where)
    need = classify_refx_bytes(C, bounds, R, mode)
    if refx.numel() * refx.element_size() < need:
        raise ValueError("%s: prepared library holds %d bytes, %d rows of mode %d need %d (classify_prepare)"
                         % (where, refx.numel() * refx.element_size(), R, mode, need))


def classify_pixels(stack, refx, R, bounds, mode=None):
    """per-pixel classification, exact: the restatement's argmin (lowest row on ties) and its
    f64 distance rounded to f32 (hrf_classify_pixels = MFMA screen + f64 refine)"""
    stack = _dev(stack, torch.float32, "stack")
    C = stack.shape[-1]
    if mode is None:
        mode = refx_mode(refx, C, bounds)
    _check_refx(refx, R, C, bounds, mode, "classify_pixels")
    P = stack.numel() // C
    b = _i32_host(bounds)
    idx = torch.empty(stack.shape[:-1], dtype=torch.int32, device=stack.device)
    dist = torch.empty(stack.shape[:-1], dtype=torch.float32, device=stack.device)
    _lib.call("hrf_classify_pixels", _ptr(stack), P, C, _ptr(refx), R, b.ctypes.data, len(b) - 1, mode, _ptr(idx),
              _ptr(dist), _stream())
    return idx, dist


def classify_pixels_screen(stack, refx, R, bounds, mode=None):
    """the MFMA screen alone -> (device argmax, device distance, runner-up score bound)"""
    stack = _dev(stack, torch.float32, "stack")
    C = stack.shape[-1]
    if mode is None:
        mode = refx_mode(refx, C, bounds)
    _check_refx(refx, R, C, bounds, mode, "classify_pixels_screen")
    P = stack.numel() // C
    b = _i32_host(bounds)
    idx = torch.empty(stack.shape[:-1], dtype=torch.int32, device=stack.device)
    dist = torch.empty(stack.shape[:-1], dtype=torch.float32, device=stack.device)
    sec = torch.empty(stack.shape[:-1], dtype=torch.float32, device=stack.device)
    _lib.call("hrf_classify_pixels_screen", _ptr(stack), P, C, _ptr(refx), R, b.ctypes.data, len(b) - 1, mode,
              _ptr(idx), _ptr(dist), _ptr(sec), _stream())
    return idx, dist, sec


def classify_screen_eps(C, bounds, R, screen):
    """the refine's bounds for `screen` (hrf_classify_screen_eps) -> (base, per zero segment, f32 pass)"""
    import ctypes
    b = _i32_host(bounds)
    out = (ctypes.c_double * 3)()
    _lib.call("hrf_classify_screen_eps", C, b.ctypes.data, len(b) - 1, R, int(screen), ctypes.addressof(out))
    return tuple(out)


class StackSource:
    """the pixels' f32 values for the refine: a plain (..., C) stack"""

    def __init__(self, stack):
        self.stack = _dev(stack, torch.float32, "stack")


class LaserSource:
    """the pixels' f32 values for the refine: the per-laser acquisitions at their device shifts
    (register_assemble's registered stack, never materialised)"""

    def __init__(self, lasers, shifts, apply_mask=True):
        self.lasers, self.shifts, self.apply_mask = list(lasers), shifts, bool(apply_mask)


def classify_refine(source, refx, R, bounds, screen, idx, dist, second, want_listed=False):
    """hrf_classify_pixels_refine in place on a screen's (idx, dist, second).  source: StackSource
    or LaserSource.  screen: 0/1/2 = classify_pixels_screen mode, 3 = classify_pixels_table.
    -> the number of pixels the certificate did not settle (want_listed; synchronises), with
    want_listed="stats" also the list pass's sparse candidates and its pixels scored in full, or None"""
    import ctypes
    if isinstance(source, StackSource):
        st = source.stack
        C = st.shape[-1]
        P = st.numel() // C
        ptrs = (ctypes.c_void_p * 1)(st.data_ptr())
        ch = _i32_host([C])
        n, H, W, sd, mask = 1, 1, P, None, 0
    elif isinstance(source, LaserSource):
        srcs, ch, ptrs, sd = _laser_args(source.lasers, source.shifts)
        C = int(ch.sum())
        n = len(srcs)
        H, W = srcs[0].shape[:2]
        P, mask = H * W, int(source.apply_mask)
    else:
        raise ValueError("classify_refine: a StackSource or LaserSource is required")
    if idx.numel() != P:
        raise ValueError("classify_refine: %d screened pixels, the source holds %d" % (idx.numel(), P))
    _check_refx(refx, R, C, bounds, 2 if screen == 3 else screen, "classify_refine")
    b = _i32_host(bounds)
    wb = int(_lib.lib().hrf_classify_refine_work_bytes(P))
    work = torch.empty(wb, dtype=torch.uint8, device=idx.device)
    _lib.call("hrf_classify_pixels_refine", ctypes.cast(ptrs, ctypes.c_void_p), ch.ctypes.data,
              _ptr(sd) if sd is not None else None, n, H, W, mask, _ptr(refx), R, b.ctypes.data, len(b) - 1,
              int(screen), _ptr(second), _ptr(idx), _ptr(dist), _ptr(work), wb, _stream())
    if want_listed == "stats":  # (listed pixels, sparse candidates scored in f64, pixels scored in full)
        return tuple(int(v) for v in work[:12].view(torch.int32).tolist())
    if want_listed:
        return int(work[:4].view(torch.int32).item())
    return None


class PixTable:
    """the per-pixel classifier's prepared operands (pixtable.hpp): split-fp16 segment-normalised
    pixels in the MFMA register layout + a flag byte per pixel; `source` (StackSource or
    LaserSource) holds the f32 values the table was made from (the refine reads them)"""

    def __init__(self, table, flags, shape, C, bounds, source=None):
        self.table, self.flags, self.shape, self.C, self.bounds = table, flags, tuple(shape), C, tuple(bounds)
        self.source = source

    @property
    def P(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


def pixtable_alloc(shape, C, bounds, device):
    P = 1
    for s in shape:
        P *= s
    b = _i32_host(bounds)
    nb = int(_lib.lib().hrf_pixtable_bytes(P, C, b.ctypes.data, len(b) - 1))
    if nb < 0:
        raise ValueError("pixtable: the E. coli or multispecies channel layout only")
    return PixTable(torch.empty(max(nb, 16), dtype=torch.uint8, device=device),
                    torch.empty(max(P, 1), dtype=torch.uint8, device=device), shape, C, bounds)


def pixtable_prepare(stack, bounds):
    """the prepared operands of an (..., C) stack (standalone pass; the E. coli assembly writes them
    in its own pass: register_assemble(..., pixtable=...))"""
    stack = _dev(stack, torch.float32, "stack")
    C = stack.shape[-1]
    pt = pixtable_alloc(stack.shape[:-1], C, bounds, stack.device)
    pt.source = StackSource(stack)
    b = _i32_host(bounds)
    _lib.call("hrf_pixtable_prepare", _ptr(stack), pt.P, C, b.ctypes.data, len(b) - 1, _ptr(pt.table), _ptr(pt.flags),
              _stream())
    return pt


def check_refx_table(refx, R, C, bounds, where):
    """the pixel-table classifier (w16t) reads a mode-2 table of Rpad rows of the mode-2 pitch; a
    mode-0/1 table (f32, or rows of another width) would be read as split-fp16 rows, past its end"""
    if not isinstance(refx, torch.Tensor) or not refx.is_cuda:
        raise ValueError("%s: the prepared library must be a device tensor" % where)
    if 2 not in classify_modes(bounds) or refx_mode(refx, C, bounds) != 2:
        raise ValueError("%s: a mode-2 prepared library (classify_prepare(..., mode=2)) is required" % where)
    _check_refx(refx, R, C, bounds, 2, where)


def classify_pixels_table_screen(pt, refx, R):
    """the mode-2 screen from a PixTable: classify_pixels_screen(mode=2)'s device scores bit for
    bit -> (device argmax, device distance, runner-up bound)"""
    check_refx_table(refx, R, pt.C, pt.bounds, "classify_pixels_table")
    b = _i32_host(pt.bounds)
    idx = torch.empty(pt.shape, dtype=torch.int32, device=pt.table.device)
    dist = torch.empty(pt.shape, dtype=torch.float32, device=pt.table.device)
    sec = torch.empty(pt.shape, dtype=torch.float32, device=pt.table.device)
    _lib.call("hrf_classify_pixels_table", _ptr(pt.table), _ptr(pt.flags), pt.P, pt.C, _ptr(refx), R, b.ctypes.data,
              len(b) - 1, _ptr(idx), _ptr(dist), _ptr(sec), _stream())
    return idx, dist, sec


def _source_args(source):
    """(ptrs, channels, shifts, nlaser, H, W, apply_mask, C) of a StackSource / LaserSource"""
    import ctypes
    if isinstance(source, StackSource):
        st = source.stack
        C = st.shape[-1]
        return (ctypes.c_void_p * 1)(st.data_ptr()), _i32_host([C]), None, 1, 1, st.numel() // C, 0, C
    if isinstance(source, LaserSource):
        srcs, ch, ptrs, sd = _laser_args(source.lasers, source.shifts)
        H, W = srcs[0].shape[:2]
        return ptrs, ch, sd, len(srcs), H, W, int(source.apply_mask), int(ch.sum())
    raise ValueError("a StackSource or LaserSource is required")


def classify_pixels_table(pt, refx, R, fused=False, composed=False, want_listed=False):
    """exact per-pixel classification from a PixTable, reading the pixels' values from the table's
    source: hrf_classify_pixels_table_exact (sweep, certificate pass, list pass), its _fused form
    (the sweep certifies its own rows) or, composed, classify_pixels_table_screen + classify_refine
    -- the same results bit for bit.
    -> (idx, dist), and the number of listed pixels with want_listed (synchronises)"""
    import ctypes
    if pt.source is None:
        raise ValueError("classify_pixels_table: the table has no source values for the exact refine")
    if composed:
        idx, dist, sec = classify_pixels_table_screen(pt, refx, R)
        n = classify_refine(pt.source, refx, R, pt.bounds, 3, idx, dist, sec, want_listed=want_listed)
        return (idx, dist, n) if want_listed else (idx, dist)
    check_refx_table(refx, R, pt.C, pt.bounds, "classify_pixels_table")
    ptrs, ch, sd, n, H, W, mask, C = _source_args(pt.source)
    if H * W != pt.P or C != pt.C:
        raise ValueError("classify_pixels_table: the source does not match the table")
    b = _i32_host(pt.bounds)
    idx = torch.empty(pt.shape, dtype=torch.int32, device=pt.table.device)
    dist = torch.empty(pt.shape, dtype=torch.float32, device=pt.table.device)
    wb = int(_lib.lib().hrf_classify_refine_work_bytes(pt.P))
    work = torch.empty(wb, dtype=torch.uint8, device=idx.device)
    _lib.call("hrf_classify_pixels_table_exact_fused" if fused else "hrf_classify_pixels_table_exact", _ptr(pt.table), _ptr(pt.flags), ctypes.cast(ptrs, ctypes.c_void_p),
              ch.ctypes.data, _ptr(sd) if sd is not None else None, n, H, W, mask, _ptr(refx), R, b.ctypes.data,
              len(b) - 1, _ptr(idx), _ptr(dist), _ptr(work), wb, _stream())
    if want_listed:
        return idx, dist, int(work[:4].view(torch.int32).item())
    return idx, dist


def segment_flags(x, bounds, thr=0.1):
    """(N, C) f64 -> (N, nseg) f64 presence flags: max over each segment > thr (NaN -> 0)"""
    x = _dev(x, torch.float64, "x")
    N, C = x.shape
    b = _i32_host(bounds)
    out = torch.empty((N, len(b) - 1), dtype=torch.float64, device=x.device)
    _lib.call("hrf_segment_flags", _ptr(x), N, C, b.ctypes.data, len(b) - 1, float(thr), _ptr(out), _stream())
    return out


def classify_cells(x, ref, bounds, variant=0, fx=None, fr=None):
    x = _dev(x, torch.float64, "x")
    ref = _dev(ref, torch.float64, "ref")
    N, C = x.shape
    R = ref.shape[0]
    b = _i32_host(bounds)
    fxp = _ptr(_dev(fx, torch.float64, "fx")) if fx is not None else None
    frp = _ptr(_dev(fr, torch.float64, "fr")) if fr is not None else None
    arg = torch.empty(N, dtype=torch.int32, device=x.device)
    dmin = torch.empty(N, dtype=torch.float64, device=x.device)
    _lib.call("hrf_classify_cells", _ptr(x), N, _ptr(ref), R, C, b.ctypes.data, len(b) - 1, variant, fxp, frp,
              _ptr(arg), _ptr(dmin), _stream())
    return arg, dmin


# ---- a22 ------------------------------------------------------------------------------------
def rag_edges(labels, maxlab):
    l = _i32(labels, "labels")
    H, W = l.shape
    e = torch.empty((maxlab + 1, maxlab + 1), dtype=torch.uint8, device=l.device)
    _lib.call("hrf_rag_edges", _ptr(l), H, W, maxlab, _ptr(e), _stream())
    return e


def barcode_adjacency(edge, bc_of_label, R):
    maxlab = edge.shape[0] - 1
    bc = _i32(bc_of_label, "bc_of_label")
    adj = torch.empty((R, R), dtype=torch.int64, device=edge.device)
    _lib.call("hrf_barcode_adjacency", _ptr(edge.contiguous()), maxlab, _ptr(bc), R, _ptr(adj), _stream())
    return adj


def barcode_adjacency_filtered(edge, bc_of_label, keep_of_label, R):
    """-> (raw, cell-filtered) (R, R) int64 adjacency counts in one pass"""
    maxlab = edge.shape[0] - 1
    bc = _i32(bc_of_label, "bc_of_label")
    keep = _u8(keep_of_label, "keep_of_label")
    if bc.numel() < maxlab + 1 or keep.numel() < maxlab + 1:
        raise ValueError("barcode_adjacency_filtered: per-label arrays shorter than max label + 1")
    adj = torch.empty((R, R), dtype=torch.int64, device=edge.device)
    adjf = torch.empty((R, R), dtype=torch.int64, device=edge.device)
    _lib.call("hrf_barcode_adjacency_filtered", _ptr(edge.contiguous()), maxlab, _ptr(bc), _ptr(keep), R, _ptr(adj),
              _ptr(adjf), _stream())
    return adj, adjf


def label_overlap(labels, mask, maxlab):
    l = _i32(labels, "labels")
    m = _u8(mask, "mask")
    H, W = l.shape
    out = torch.empty(maxlab + 1, dtype=torch.uint8, device=l.device)
    _lib.call("hrf_label_overlap", _ptr(l), _ptr(m), H, W, maxlab, _ptr(out), _stream())
    return out


def cell_typing(label, area, maxprob=None, overlap=None, maxlab=0, area_max=10000.0, prob_min=0.95):
    lab = _i32(label, "label")
    ar = _dev(area, torch.float64, "area")
    mp = None if maxprob is None else _dev(maxprob, torch.float64, "maxprob")
    ov = None if overlap is None else _u8(overlap, "overlap")
    out = torch.empty(lab.numel(), dtype=torch.uint8, device=lab.device)
    _lib.call("hrf_cell_typing", _ptr(lab), _ptr(ar), _ptr(mp) if mp is not None else None,
              _ptr(ov) if ov is not None else None, int(maxlab), lab.numel(), float(area_max), float(prob_min),
              _ptr(out), _stream())
    return out


def shape_filter(labels, props, maxlab, minor_lo=15.0, minor_hi=35.0):
    l = _i32(labels, "labels")
    H, W = l.shape
    out = torch.empty_like(l)
    _lib.call("hrf_shape_filter", _ptr(l), H, W, _ptr(props.contiguous()), maxlab, float(minor_lo), float(minor_hi),
              _ptr(out), _stream())
    return out


def split_by_size(mask, thr, small_or, conn=2):
    """freeze components smaller than thr into small_or (in place); returns the rest"""
    m = _u8(mask, "mask")
    H, W = m.shape
    large = torch.empty_like(m)
    parent = torch.empty((H, W), dtype=torch.int32, device=m.device)
    size = torch.empty((H, W), dtype=torch.int32, device=m.device)
    _lib.call("hrf_split_by_size", _ptr(m), H, W, conn, thr, _ptr(small_or), _ptr(large), _ptr(parent), _ptr(size),
              _stream())
    return large


def label_boxes(labels, maxlab):
    l = _i32(labels, "labels")
    H, W = l.shape
    box = torch.empty((maxlab + 1, 4), dtype=torch.int32, device=l.device)
    _lib.call("hrf_label_boxes", _ptr(l), H, W, maxlab, _ptr(box), _stream())
    return box


def erosion_seeds(cell_sm, area_max=600, min_obj=10):
    """ecoli measurement.py:97-110 in one launch (per-component workgroups) -> dist_be u8"""
    labels, n = label(cell_sm, conn=2)
    H, W = labels.shape
    box = label_boxes(labels, n)
    be = torch.empty((H, W), dtype=torch.uint8, device=labels.device)
    _lib.call("hrf_erosion_seeds", _ptr(labels), H, W, n, _ptr(box), area_max, min_obj, _ptr(be), _stream())
    return be


# ---- native segmentation drivers (segment.hip) ------------------------------------------------
class _CtxCache:
    """Native contexts (hrf_seg_ctx / hrf_tile_ctx) keyed by (device, stream handle, H, W), at most
    `cap` alive (HRF_CTX_CACHE, default 8; a 2048^2 tile context holds ~2 GB of HBM).  The least
    recently used idle one beyond the cap is destroyed once the event recorded behind its last call
    has completed -- an event outlives the stream it was recorded on, so a caller that makes a
    stream per image and drops it does not leak the context (the reference runs one process per
    FOV, ecoli Snakefile:67-82; a long-lived driver must not grow).  Thread-safe: a context in use
    by a call on another host thread is never evicted."""

    def __init__(self, create, destroy):
        import threading
        from collections import OrderedDict
        self._create, self._destroy = create, destroy
        self._d = OrderedDict()       # key -> [handle, last-use event or None, calls in flight]
        self._lock = threading.Lock()
        self.cap = max(1, int(os.environ.get("HRF_CTX_CACHE", "8")))
        self.created = 0              # contexts made so far (tests: churn under the cap)

    def use(self, dev, H, W):
        """context manager: the (device, current stream, H, W) context for one native call"""
        import contextlib
        import ctypes
        key = (torch.device(dev), _stream(), H, W)

        @contextlib.contextmanager
        def cm():
            evict = []
            with self._lock:
                ent = self._d.get(key)
                if ent is None:
                    h = ctypes.c_void_p()
                    _lib.call(self._create, H, W, ctypes.addressof(h))
                    ent = self._d[key] = [h, None, 0]
                    self.created += 1
                else:
                    self._d.move_to_end(key)
                ent[2] += 1
                over = len(self._d) - self.cap
                for k in list(self._d):
                    if over <= 0:
                        break
                    if self._d[k][2] == 0:
                        evict.append(self._d.pop(k))
                        over -= 1
            for e in evict:
                self._free(e)
            try:
                yield ent[0]
            finally:
                with self._lock:
                    if ent[1] is None:
                        ent[1] = torch.cuda.Event()
                    ent[1].record(torch.cuda.current_stream())
                    ent[2] -= 1
        return cm()

    def _free(self, ent):
        h, ev, _ = ent
        if ev is not None:
            ev.synchronize()
        _lib.call(self._destroy, h)

    def clear(self):
        """destroy every idle context (after its last queued use)"""
        with self._lock:
            idle = [k for k, e in self._d.items() if e[2] == 0]
            ents = [self._d.pop(k) for k in idle]
        for e in ents:
            self._free(e)

    def __len__(self):
        return len(self._d)


_SEG_CTX = _CtxCache("hrf_seg_ctx_create", "hrf_seg_ctx_destroy")
_TILE_CTX = _CtxCache("hrf_tile_ctx_create", "hrf_tile_ctx_destroy")


def release_contexts():
    """destroy the cached native segmentation and tile contexts (each after its last queued call)"""
    _SEG_CTX.clear()
    _TILE_CTX.clear()


def tile_stats(device, H, W):
    """seg_stats of the last native tile (tile_ecoli) run on the current stream's (H, W) context"""
    import ctypes
    seg = ctypes.c_void_p()
    out = (ctypes.c_int32 * 4)()
    with _TILE_CTX.use(device, H, W) as ctx:
        _lib.call("hrf_tile_ctx_seg", ctx, ctypes.addressof(seg))
        _lib.call("hrf_seg_ctx_stats", seg, ctypes.addressof(out))
    return dict(zip(("passes", "contests", "rounds", "marker_ties"), list(out)))


def tile_pixel_listed(device, H, W):
    """pixels of the last native tile whose per-pixel certificate failed (scored in full by the
    refine's list pass); synchronises"""
    import ctypes
    n = ctypes.c_int32(0)
    with _TILE_CTX.use(device, H, W) as ctx:
        _lib.call("hrf_tile_ctx_pixel_listed", ctx, ctypes.addressof(n))
    return n.value


_CELL_CAP = {}


def tile_ecoli(lasers, cal, refx, lib, lib_flags, variant=1, flag_thr=0.1, per_pixel=True, side=None,
               pix_events=None):
    """one E. coli tile in one native call (hrf_tile_ecoli).  lasers: the five (H, W, C_l) f32
    acquisitions; cal: (H, W) f32 flat field or None; refx: classify_prepare(library) (mode 2);
    lib: (R, 95) f64 library; lib_flags: its presence flags (R, 5) f64 (gated variants).
    -> dict of device tensors: seg, ident, counts, ncells (int32[1]), maxlab, and per-cell rows
    (labels, avgint, avgint_norm, cell_idx, cell_dist; first ncells rows valid), pixel_idx /
    pixel_dist.  side: the stream the per-pixel classifier runs on (default: the current one)."""
    import ctypes
    srcs = [_dev(l, torch.float32, "laser stack") for l in lasers]
    if len(srcs) != 5 or [int(l.shape[2]) for l in srcs] != [32, 23, 20, 14, 6]:
        raise ValueError("tile_ecoli: the five E. coli laser stacks (32, 23, 20, 14, 6 channels) expected")
    H, W = srcs[0].shape[:2]
    if any(tuple(l.shape[:2]) != (H, W) for l in srcs):
        raise ValueError("tile_ecoli: the laser stacks must share H x W")
    dev = srcs[0].device
    lib = _dev(lib, torch.float64, "library")
    R = lib.shape[0]
    if lib.shape[1] != 95:
        raise ValueError("tile_ecoli: a 95-channel library expected")
    fl = _dev(lib_flags, torch.float64, "library flags") if lib_flags is not None else None
    if variant and fl is None:
        raise ValueError("tile_ecoli: the gated variants need the library's presence flags")
    if per_pixel:
        check_refx_table(refx, R, 95, REFERENCE_LAYOUTS[0], "tile_ecoli")
    calp = None
    if cal is not None:
        c = _dev(cal, torch.float32, "calibration")
        if tuple(c.shape) != (H, W):
            raise ValueError("tile_ecoli: the flat field must be an (H, W) plane")
        calp = _ptr(c)
    ptrs = (ctypes.c_void_p * 5)(*[l.data_ptr() for l in srcs])
    key = (dev, H, W)
    cap = _CELL_CAP.get(key, 4096)
    i32, f64 = torch.int32, torch.float64
    seg = torch.empty((H, W), dtype=i32, device=dev)
    ident = torch.empty((H, W), dtype=i32, device=dev)
    counts = torch.empty(R, dtype=torch.int64, device=dev)
    ncells = torch.empty(1, dtype=i32, device=dev)
    pix_idx = torch.empty((H, W), dtype=i32, device=dev) if per_pixel else None
    pix_dist = torch.empty((H, W), dtype=torch.float32, device=dev) if per_pixel else None

    def rows(n):
        return (torch.empty(n, dtype=i32, device=dev), torch.empty((n, 95), dtype=f64, device=dev),
                torch.empty((n, 95), dtype=f64, device=dev), torch.empty(n, dtype=i32, device=dev),
                torch.empty(n, dtype=f64, device=dev))
    labs, avg, avgn, cidx, cdist = rows(cap)
    mx = ctypes.c_int32(0)
    e0 = e1 = None
    if pix_events is not None and per_pixel:
        st = side if side is not None else torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)        # creates the events (recorded again inside the call)
        e1.record(st)
        pix_events.append((e0, e1))
    with _TILE_CTX.use(dev, H, W) as ctx:
        _lib.call("hrf_tile_ecoli", ctx, ctypes.cast(ptrs, ctypes.c_void_p), calp, _ptr(refx) if per_pixel else None,
                  _ptr(lib), _ptr(fl) if fl is not None else None, R, int(variant), float(flag_thr),
                  int(bool(per_pixel)), _ptr(seg), _ptr(pix_idx) if per_pixel else None,
                  _ptr(pix_dist) if per_pixel else None, cap, _ptr(labs), _ptr(avg), _ptr(avgn), _ptr(cidx),
                  _ptr(cdist), _ptr(ident), _ptr(counts), _ptr(ncells), ctypes.addressof(mx), _stream(),
                  ctypes.c_void_p(side.cuda_stream) if side is not None else None,
                  ctypes.c_void_p(e0.cuda_event) if e0 is not None else None,
                  ctypes.c_void_p(e1.cuda_event) if e1 is not None else None)
    maxlab = mx.value
    if maxlab > cap:            # the per-cell part was left for buffers that hold every label
        cap = 1 << max(12, (maxlab - 1).bit_length())
        _CELL_CAP[key] = cap
        labs, avg, avgn, cidx, cdist = rows(cap)
        with _TILE_CTX.use(dev, H, W) as ctx:
            _lib.call("hrf_tile_ecoli_cells", ctx, _ptr(seg), _ptr(lib), _ptr(fl) if fl is not None else None, R,
                      int(variant), float(flag_thr), cap, _ptr(labs), _ptr(avg), _ptr(avgn), _ptr(cidx),
                      _ptr(cdist), _ptr(ident), _ptr(counts), _ptr(ncells), _stream())
    return dict(seg=seg, ident=ident, counts=counts, ncells=ncells, maxlab=maxlab, labels=labs, avgint=avg,
                avgint_norm=avgn, cell_idx=cidx, cell_dist=cdist, pixel_idx=pix_idx, pixel_dist=pix_dist)


def seg_stats(device, H, W):
    """the watershed of the last native chain run on the current stream's (H, W) context:
    {passes, contests, rounds, marker_ties} (hrf_seg_ctx_stats; marker_ties = decisions between
    equal-valued markers of different labels, DESIGN.md "Watershed")"""
    import ctypes
    out = (ctypes.c_int32 * 4)()
    with _SEG_CTX.use(device, H, W) as ctx:
        _lib.call("hrf_seg_ctx_stats", ctx, ctypes.addressof(out))
    return dict(zip(("passes", "contests", "rounds", "marker_ties"), list(out)))


def segment_ecoli_native(stack, image_cn=None):
    """ecoli measurement.py:44-127 in one native call -> (segmentation int32, max label);
    with image_cn (log(sum + 1e-2), f64 H x W, e.g. from register_assemble(cn_mode=1)) the
    channel sum is not recomputed"""
    import ctypes
    mx = ctypes.c_int32(0)
    if image_cn is not None:
        cn = _dev(image_cn, torch.float64, "image_cn")
        H, W = cn.shape
        seg = torch.empty((H, W), dtype=torch.int32, device=cn.device)
        with _SEG_CTX.use(cn.device, H, W) as ctx:
            _lib.call("hrf_segment_ecoli_cn", ctx, _ptr(cn), _ptr(seg), ctypes.addressof(mx), _stream())
        return seg, mx.value
    stack = _dev(stack, torch.float32, "stack")
    H, W, C = stack.shape
    seg = torch.empty((H, W), dtype=torch.int32, device=stack.device)
    with _SEG_CTX.use(stack.device, H, W) as ctx:
        _lib.call("hrf_segment_ecoli", ctx, _ptr(stack), C, _ptr(seg), ctypes.addressof(mx), _stream())
    return seg, mx.value


def segment_multispecies_native(stack, cal=None):
    """multispecies measurement.py:102-157 in one native call
    -> (segmentation relabelled 1..n, n, image_sum f64, final_bkg f64)"""
    import ctypes
    stack = _dev(stack, torch.float32, "stack")
    H, W, C = stack.shape
    calp, sp, sc, c0, c1 = None, 1, 0, 0, C
    if cal is not None:
        cal_t, sp, sc, c0, c1 = _cal_layout(cal, H, W, C)
        calp = _ptr(cal_t)
    seg = torch.empty((H, W), dtype=torch.int32, device=stack.device)
    s = torch.empty((H, W), dtype=torch.float64, device=stack.device)
    fb = torch.empty((H, W), dtype=torch.float64, device=stack.device)
    n = ctypes.c_int32(0)
    with _SEG_CTX.use(stack.device, H, W) as ctx:
        _lib.call("hrf_segment_multispecies", ctx, _ptr(stack), C, calp, sp, sc, c0, c1, _ptr(seg),
                  ctypes.addressof(n), _ptr(s), _ptr(fb), _stream())
    return seg, n.value, s, fb


# ---- a17, a18, f2: classifier back-end ----------------------------------------------------
def features_ecoli(avgint_norm):
    """(n, 95) -> (n, 132): avgint_norm | np.diff(avgint_norm[:, 0:32]) | 6 zero flag columns
    (ecoli image_classification.py:47-48)"""
    x = _dev(avgint_norm, torch.float64, "avgint_norm")
    out = torch.empty((x.shape[0], 132), dtype=torch.float64, device=x.device)
    _lib.call("hrf_features_ecoli", _ptr(x), x.shape[0], _ptr(out), _stream())
    return out


def features_multi(avgint_norm):
    """(n, 63) -> (n, 67): avgint_norm | 4 zero flag columns (classify_spectra.py:27-28)"""
    x = _dev(avgint_norm, torch.float64, "avgint_norm")
    out = torch.empty((x.shape[0], 67), dtype=torch.float64, device=x.device)
    _lib.call("hrf_features_multi", _ptr(x), x.shape[0], _ptr(out), _stream())
    return out


def standard_scale(x, mean, scale):
    """sklearn StandardScaler.transform on the columns of x (a column slice of a wider table
    is read in place)"""
    if x.stride(1) != 1:
        raise ValueError("standard_scale: rows must be contiguous")
    n, f = x.shape
    out = torch.empty((n, f), dtype=torch.float64, device=x.device)
    m = None if mean is None else _dev(mean, torch.float64, "mean")
    s = None if scale is None else _dev(scale, torch.float64, "scale")
    _lib.call("hrf_standard_scale", _ptr(x), n, f, x.stride(0), _ptr(m) if m is not None else None,
              _ptr(s) if s is not None else None, _ptr(out), _stream())
    return out


def svc_predict(x, model, out_column=None, want_dec=False):
    """sklearn SVC.predict with the arrays of `model` (backend.SvcModel).  x may be a column
    slice of a wider f64 table (rows contiguous).  -> class index (int32, n); with out_column
    (a column view of an f64 table) the class values are also written there; with want_dec the
    one-vs-one decision values (n, pairs) too."""
    if x.dtype != torch.float64 or not x.is_cuda or x.stride(1) != 1:
        raise ValueError("svc_predict: an f64 device table with contiguous rows expected")
    n, f = x.shape
    if f != model.sv.shape[1]:
        raise ValueError("svc_predict: %d features, the model has %d" % (f, model.sv.shape[1]))
    pred = torch.empty(n, dtype=torch.int32, device=x.device)
    nc = model.n_class
    dec = torch.empty((n, nc * (nc - 1) // 2), dtype=torch.float64, device=x.device) if want_dec else None
    vo, vs = (None, 0) if out_column is None else (out_column, out_column.stride(0))
    _lib.call("hrf_svc_predict", _ptr(x), n, x.stride(0), f, _ptr(model.sv), model.sv.shape[0], _ptr(model.coef),
              _ptr(model.intercept), _ptr(model.start), nc, model.kernel, float(model.gamma), float(model.coef0),
              int(model.degree), _ptr(pred), _ptr(dec) if dec is not None else None,
              _ptr(vo) if vo is not None else None, vs, _ptr(model.class_values), _stream())
    return (pred, dec) if want_dec else pred


def svc_predict_proba(x, model):
    """sklearn SVC.predict_proba with the arrays of `model` (a backend.SvcModel carrying
    probA / probB) -> (n, n_class) f64 in class order"""
    if model.probA is None:
        raise ValueError("svc_predict_proba: the model has no probA_ / probB_ (fitted without probability=True)")
    if x.dtype != torch.float64 or not x.is_cuda or x.stride(1) != 1:
        raise ValueError("svc_predict_proba: an f64 device table with contiguous rows expected")
    n, f = x.shape
    if f != model.sv.shape[1]:
        raise ValueError("svc_predict_proba: %d features, the model has %d" % (f, model.sv.shape[1]))
    nc = model.n_class
    prob = torch.empty((n, nc), dtype=torch.float64, device=x.device)
    _lib.call("hrf_svc_predict_proba", _ptr(x), n, x.stride(0), f, _ptr(model.sv), model.sv.shape[0],
              _ptr(model.coef), _ptr(model.intercept), _ptr(model.start), nc, model.kernel, float(model.gamma),
              float(model.coef0), int(model.degree), _ptr(model.probA), _ptr(model.probB), _ptr(prob), _stream())
    return prob


KNN_METRICS = {"euclidean": 0, "channel_cosine_intensity_7b_v2": 1, "channel_cosine_intensity_violet_derivative_v2": 2}


def knn(q, trainT, metric, k):
    """exact k nearest training rows; trainT = the training table transposed (f, nt),
    contiguous.  -> (idx int32 (nq, k), dist f64 (nq, k))"""
    if q.dtype != torch.float64 or q.stride(1) != 1:
        raise ValueError("knn: f64 queries with contiguous rows expected")
    trainT = _dev(trainT, torch.float64, "trainT")
    nq, f = q.shape
    if trainT.shape[0] != f:
        raise ValueError("knn: the training table has %d features, the queries %d" % (trainT.shape[0], f))
    m = KNN_METRICS[metric] if isinstance(metric, str) else int(metric)
    idx = torch.empty((nq, k), dtype=torch.int32, device=q.device)
    dist = torch.empty((nq, k), dtype=torch.float64, device=q.device)
    _lib.call("hrf_knn", _ptr(q), nq, q.stride(0), _ptr(trainT), trainT.shape[1], f, m, int(k), _ptr(idx), _ptr(dist),
              _stream())
    return idx, dist


def umap_init_transform(idx, dist, embedding, n_neighbors, local_connectivity=0.0, want_memb=False):
    """umap-learn transform's initial embedding of the queries from their kNN (the mean knn
    distance stays on the device).  embedding: the training embedding, float32 (umap's dtype).
    -> float32 (nq, d) [, the float32 membership strengths (nq, k) in knn order]"""
    idx = _i32(idx, "idx")
    dist = _dev(dist, torch.float64, "dist")
    emb = _dev(embedding, torch.float32, "embedding")
    nq, k = idx.shape
    mean = dist.mean().reshape(1) if dist.numel() else torch.zeros(1, dtype=torch.float64, device=dist.device)
    out = torch.empty((nq, emb.shape[1]), dtype=torch.float32, device=dist.device)
    memb = torch.empty((nq, k), dtype=torch.float32, device=dist.device) if want_memb else None
    _lib.call("hrf_umap_init_transform", _ptr(idx), _ptr(dist), nq, k, float(n_neighbors), float(local_connectivity),
              _ptr(mean), _ptr(emb), emb.shape[1], _ptr(memb) if memb is not None else None, _ptr(out), _stream())
    return (out, memb) if want_memb else out


def umap_refine(idx, memb, init, tail_embedding, n_epochs, a, b, repulsion_strength=1.0, initial_alpha=0.25,
                negative_sample_rate=5.0, seed=0):
    """transform()'s layout refinement of `init` (float32, nq x d, refined in a copy) against the
    fixed training embedding; initial_alpha is the rate transform passes (umap's
    _initial_alpha / 4).  Deterministic per-query negative-sample streams (see hrf.h)."""
    idx = _i32(idx, "idx")
    memb = _dev(memb, torch.float32, "memb")
    tail = _dev(tail_embedding, torch.float32, "tail_embedding")
    emb = _dev(init, torch.float32, "init").clone()
    nq, k = idx.shape
    if memb.shape != idx.shape or emb.shape[0] != nq or emb.shape[1] != tail.shape[1]:
        raise ValueError("umap_refine: shapes disagree")
    wmax = memb.amax().reshape(1) if memb.numel() else torch.zeros(1, dtype=torch.float32, device=memb.device)
    _lib.call("hrf_umap_refine", _ptr(idx), _ptr(memb), nq, k, _ptr(wmax), int(n_epochs), _ptr(tail), tail.shape[0],
              tail.shape[1], float(a), float(b), float(repulsion_strength), float(initial_alpha),
              float(negative_sample_rate), int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(emb), _stream())
    return emb
