"""Segmentation timing on one cfg3 tile, raw vs registered stack (zero borders), with the
component statistics that drive erosion_seed_kernel.  Dev tool (also a rocprofv3 target)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import kernels as K, pipeline as P, synthetic as S  # noqa: E402

seed = int(os.environ.get("HRF_PROF_SEED", "20190101"))
st, _, _, _ = S.tile(2048, 2048, seed=seed)
reg = P.register_stack(S.laser_split(st))


def ms(fn, n=3):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for name, x in (("raw", st), ("registered", reg)):
    keep = {}
    P.segment_ecoli(x, keep=keep)
    cs = keep["cell_sm"]
    lab, n = K.label(cs, conn=2)
    sizes = np.bincount(lab.cpu().numpy().ravel())[1:]
    t_seg = ms(lambda: P.segment_ecoli(x))
    t_ero = ms(lambda: K.erosion_seeds(cs, 600, 10))
    print("%-10s segment %.3f ms  erosion_seeds %.3f ms  components %d  largest %d  >600: %d" %
          (name, t_seg, t_ero, n, sizes.max() if len(sizes) else 0, int((sizes > 600).sum())), flush=True)
