"""Time hrf_classify_pixels (isolated) on the bench's cfg3 tile in its different forms: the
pre-assembled synthetic stack, the registered stack (zeroed wrap borders), the registered stack
with its zero pixels filled, and uniform random data of the same shape -- separates the
data-dependent paths of the sweep (zero-segment epilogue, keyed argmax) from the MFMA sweep.

python tools/time_classify_tile.py
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def ms_of(fn, n=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    H = W = 2048
    bounds = S.ECOLI_BOUNDS
    ref = S.reference_library(10, bounds)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), bounds, 10)
    refx = lib.refx()
    seed = 20190101
    lay = S.cell_layout(H, W, S.default_ncells(H, W), lib.R, seed)
    truth, prof = S.render_truth(H, W, lay, with_profile=True)
    stack = S.render_stack(truth, lay, ref, seed=seed, device="cuda", profile=prof)
    reg = P.register_stack(S.laser_split(stack))
    zero_px = (reg == 0).all(dim=-1)
    print("registered: %.4f of pixels all-zero, %.4f with a zero value" %
          (zero_px.float().mean().item(), (reg == 0).any(dim=-1).float().mean().item()))
    filled = torch.where(reg == 0, torch.full_like(reg, 1e-3), reg)
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    rnd = torch.rand((H, W, 95), generator=g, device="cuda")
    for name, x in (("preassembled", stack), ("registered", reg), ("registered, zeros filled", filled),
                    ("uniform random", rnd)):
        ms = ms_of(lambda: K.classify_pixels(x, refx, lib.R, bounds))
        print("%-26s %.3f ms  %.1f TF/s algorithmic" % (name, ms, 2.0 * H * W * lib.R * 95 / ms / 1e9))


if __name__ == "__main__":
    main()
