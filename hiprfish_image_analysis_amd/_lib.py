"""ctypes binding to libhrf.so (the C ABI declared in include/hrf.h).

The library is built in-tree (hiprfish_image_analysis_amd/libhrf.so).  Loading fails loudly
when it is missing: there is no CPU fallback for any entry point.
"""
from __future__ import annotations

import ctypes
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HRF_LIB") or os.path.join(_PKG, "libhrf.so")   # HRF_LIB: A/B builds
HEADER = os.path.join(os.path.dirname(_PKG), "include", "hrf.h")

_lib = None

_CT = {
    "const double *": ctypes.c_void_p, "double *": ctypes.c_void_p,
    "const float *": ctypes.c_void_p, "float *": ctypes.c_void_p,
    "const int32_t *": ctypes.c_void_p, "int32_t *": ctypes.c_void_p,
    "const int64_t *": ctypes.c_void_p, "int64_t *": ctypes.c_void_p,
    "const uint8_t *": ctypes.c_void_p, "uint8_t *": ctypes.c_void_p,
    "const int16_t *": ctypes.c_void_p, "int16_t *": ctypes.c_void_p,
    "void *": ctypes.c_void_p, "const void *": ctypes.c_void_p,
    "hrf_stream_t": ctypes.c_void_p, "size_t": ctypes.c_size_t,
    "int64_t": ctypes.c_int64, "int32_t": ctypes.c_int32, "double": ctypes.c_double,
    "float": ctypes.c_float, "uint32_t": ctypes.c_uint32, "uint64_t": ctypes.c_uint64, "int": ctypes.c_int,
    "const float *const *": ctypes.c_void_p, "double *const *": ctypes.c_void_p,
    "hrf_seg_ctx *": ctypes.c_void_p, "hrf_seg_ctx * *": ctypes.c_void_p, "const hrf_seg_ctx *": ctypes.c_void_p,
    "hrf_tile_ctx *": ctypes.c_void_p, "hrf_tile_ctx * *": ctypes.c_void_p, "hrf_event_t": ctypes.c_void_p,
}


def declared_functions():
    """Parse include/hrf.h -> {name: (restype, [argtypes])}.  Also used by the export test."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"^HRF_API (hrf_status|int32_t|int64_t|const char \*)\s*(hrf_\w+)\s*\(([^)]*)\)\s*;", src, re.M):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        argtypes = []
        args = " ".join(args.split())
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                typ = re.sub(r"\s*\w+$", "", a).strip()
                typ = typ.replace("*", " *").replace("  ", " ").strip()
                typ = re.sub(r"\s+\*", " *", typ)
                if typ not in _CT:
                    raise TypeError("unmapped C type %r in %s" % (typ, name))
                argtypes.append(_CT[typ])
        restype = (ctypes.c_char_p if ret.startswith("const char") else
                   ctypes.c_int64 if ret == "int64_t" else ctypes.c_int32)
        out[name] = (restype, argtypes)
    return out


class HrfError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HrfError("libhrf.so not built (%s); run `python -m hiprfish_image_analysis_amd._build`" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in declared_functions().items():
            fn = getattr(L, name, None)
            if fn is None:
                if os.environ.get("HRF_LIB"):   # an older A/B build may predate newer entries
                    continue
                raise HrfError("%s does not export %s (declared in include/hrf.h)" % (LIB_PATH, name))
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def call(name, *args):
    L = lib()
    st = getattr(L, name)(*args)
    if st != 0:
        msg = L.hrf_last_error().decode(errors="replace")
        if st == 1:
            raise ValueError("%s: %s" % (name, msg))
        raise HrfError("%s failed (status %d): %s" % (name, st, msg))
    return st
