"""In-tree build of libhrf.so (hipcc, gfx950 only).  Incremental by mtime.

python -m hiprfish_image_analysis_amd._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libhrf.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off",
          "-fvisibility=hidden", "-Wno-unused-result", "-I" + os.path.join(REPO, "include")] + \
    os.environ.get("HRF_EXTRA_CFLAGS", "").split()   # A/B variants (tools/build_variant.sh)
HEADERS = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(CSRC, "*.h")) + \
    glob.glob(os.path.join(CSRC, "*.inc")) + \
    [os.path.join(REPO, "include", "hrf.h")]


def _newer(src, dst, extra=()):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(p) > t for p in (src, *extra) if os.path.exists(p))


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if _newer(src, obj, HEADERS):
        cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr[-6000:]))
        return obj, True
    return obj, False


JXR_INC = os.environ.get("HRF_JXR_INCLUDE", "/opt/conda/include/jxrlib")
JXR_LIB = os.environ.get("HRF_JXR_LIBDIR", "/opt/conda/lib")
JXR_SO = os.path.join(PKG, "libhrfjxr.so")


def build_jxr(verbose: bool = True):
    """libhrfjxr.so: the host-side JPEG-XR shim (csrc/jxr.c) over jxrlib, when the image carries
    jxrlib's headers and libraries (czi.py decodes JPEG-XR subblocks through it)"""
    src = os.path.join(CSRC, "jxr.c")
    if not (os.path.isdir(JXR_INC) and os.path.exists(os.path.join(JXR_LIB, "libjxrglue.so"))):
        if verbose:
            print("jxrlib not found (%s, %s): libhrfjxr.so not built" % (JXR_INC, JXR_LIB))
        return None
    if _newer(src, JXR_SO):
        cmd = ["gcc", "-O2", "-fPIC", "-shared", "-fvisibility=hidden", "-D__ANSI__", "-DDISABLE_PERF_MEASUREMENT",
               "-Wno-endif-labels", "-I" + JXR_INC, src, "-o", JXR_SO, "-L" + JXR_LIB, "-ljxrglue", "-ljpegxr",
               "-Wl,-rpath," + JXR_LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("jxr shim build failed:\n%s" % r.stderr[-4000:])
        if verbose:
            print("built", JXR_SO)
    return JXR_SO


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    gen = os.path.join(CSRC, "gen_tables.py")
    inc = os.path.join(CSRC, "lp_tables.inc")
    if _newer(gen, inc):
        subprocess.check_call([sys.executable, gen])
    if force:
        for o in glob.glob(os.path.join(OBJ, "*.o")):
            os.remove(o)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        res = list(ex.map(_compile, srcs))
    objs = [o for o, _ in res]
    if any(ch for _, ch in res) or not os.path.exists(LIB) or force:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lhipfft", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s" % r.stderr[-4000:])
        if verbose:
            print("built", LIB)
    build_jxr(verbose)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    build(a.force, a.j)
