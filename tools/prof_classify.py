"""Per-pixel classifier timing by mode on one synthetic cfg3 tile (2048x2048x95, R=1023).
Dev tool (also a rocprofv3 target): HRF_PROF_MODES=2,1 ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import kernels as K, synthetic as S  # noqa: E402

H = W = int(os.environ.get("HRF_PROF_HW", "2048"))
st, truth, lay, ref = S.tile(H, W, seed=20190101)
if os.environ.get("HRF_PROF_REG", "0") == "1":   # the registered stack (zero borders: all-zero pixels)
    from hiprfish_image_analysis_amd import pipeline as P
    st = P.register_stack(S.laser_split(st))
b = S.ECOLI_BOUNDS
R, C = ref.shape
first = None
for mode in [int(m) for m in os.environ.get("HRF_PROF_MODES", "2").split(",")]:
    refx = K.classify_prepare(torch.from_numpy(ref).cuda(), b, mode=mode)
    for it in range(4):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        idx, dist = K.classify_pixels(st, refx, R, b, mode=mode)
        e.record()
        torch.cuda.synchronize()
        print("mode %d: %.3f ms" % (mode, a.elapsed_time(e)), flush=True)
    if first is None:
        first = idx.clone()
    else:
        print("  index agreement with the first mode: %.6f" % (idx == first).float().mean().item())
