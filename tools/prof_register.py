"""Registration stage timing on one cfg3 tile (five per-laser acquisitions): projections, the
device shift estimate, the assembly.  Dev tool (also a rocprofv3 target)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import kernels as K, pipeline as P, synthetic as S  # noqa: E402

st, _, _, _ = S.tile(2048, 2048, seed=20190101)
lasers = S.laser_split(st)


def ms(fn, n=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


proj = [K.channel_max(s) for s in lasers]
print("projections  %.3f ms" % ms(lambda: [K.channel_max(s) for s in lasers]))
print("shifts (dev) %.3f ms" % ms(lambda: K.register_translations_dev(proj[0], proj[1:], 15)))
sh = P.estimate_shifts(lasers, device=True)
print("assemble     %.3f ms" % ms(lambda: K.register_assemble(lasers, sh)))
print("register_stack %.3f ms" % ms(lambda: P.register_stack(lasers)))
print("shifts", sh.cpu().tolist())
