"""KMeans(k) on the image_cn of one registered cfg3 tile: time per k and per-run Lloyd
iterations / relocations.  Dev tool (also a rocprofv3 target)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import _lib, kernels as K, pipeline as P, synthetic as S  # noqa: E402

seed = int(os.environ.get("HRF_PROF_SEED", "20190101"))
st, _, _, _ = S.tile(2048, 2048, seed=seed)
for name, x in (("raw", st), ("registered", P.register_stack(S.laser_split(st)))):
    keep = {}
    P.segment_ecoli(x, keep=keep)
    cn = keep["image_cn"]
    for k in (2, 3):
        share = {}
        K.kmeans_1d(cn, k, share=share)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        _, _, cen, it = K.kmeans_1d(cn, k, share=share)
        b.record()
        torch.cuda.synchronize()
        iters = (ctypes.c_int32 * 10)()
        reloc = (ctypes.c_int32 * 10)()
        strict = (ctypes.c_int32 * 10)()
        _lib.call("hrf_kmeans_last_runs", ctypes.addressof(iters), ctypes.addressof(reloc), ctypes.addressof(strict), 10)
        print("%-10s k=%d %.3f ms (sort reused) centres %s iters %s reloc %s strict %s" %
              (name, k, a.elapsed_time(b), np.round(cen, 4).tolist(), list(iters), list(reloc), list(strict)),
              flush=True)
