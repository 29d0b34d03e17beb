"""The E. coli assembly writing image_cn + the pixel table, alone on one 2048x2048 cfg3 tile
(HIP events, mean of 10): the driver for its kernel-trace / PMC passes.  Dev tool."""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K, pipeline as P, synthetic as S  # noqa: E402

st, _, _, _ = S.tile(2048, 2048, seed=20190101)
lasers = S.laser_split(st)
del st
shifts = P.estimate_shifts(lasers, device=True)
K.register_assemble_pixtable(lasers, shifts, True)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    K.register_assemble_pixtable(lasers, shifts, True)
b.record()
torch.cuda.synchronize()
print("assemble cn + pixtable %.4f ms" % (a.elapsed_time(b) / 10))
