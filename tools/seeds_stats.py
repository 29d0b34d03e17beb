"""Erosion-seeding dispatch statistics on the bench's registered tiles (HRF_SEEDS_DEBUG=1):
components per class and how many the run kernel hands to the pixel kernel.  Dev tool."""
import os
import sys

os.environ["HRF_SEEDS_DEBUG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiprfish_image_analysis_amd import pipeline as P, synthetic as S  # noqa: E402

ref = S.reference_library(10, S.ECOLI_BOUNDS)
for t in range(8):
    seed = 20190101 + t
    lay = S.cell_layout(2048, 2048, S.default_ncells(2048, 2048), 1023, seed)
    truth, prof = S.render_truth(2048, 2048, lay, with_profile=True)
    stack = S.render_stack(truth, lay, ref, seed=seed, device="cuda", profile=prof)
    reg = P.register_stack(S.laser_split(stack))
    keep = {}
    P.segment_ecoli(reg, keep=keep)
    torch.cuda.synchronize()
