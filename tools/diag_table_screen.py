"""which screen output differs between the in-kernel (w16) and table (w16t) sweeps, where"""
import numpy as np
import torch

from hiprfish_image_analysis_amd import kernels as K, synthetic as S

bounds = (0, 32, 55, 75, 89, 95)
H, W = 96, 80
ref = S.reference_library(10, bounds).copy()
ref[3, bounds[0]:bounds[1]] = 0.0
stack = S.tile(H, W, nbit=10, bounds=bounds, seed=5, ncells=6)[0]
st = stack.cpu().numpy().reshape(-1, ref.shape[1])
st[:7] = 0.0
st[7:20, bounds[0]:bounds[1]] = 0.0
st[20:23, bounds[1]:bounds[2]] = 1e-25
print("negative values in the plain stack:", int((st < 0).sum()))
refx = K.classify_prepare(torch.from_numpy(ref).cuda(), bounds, mode=2)
for case in ("plain", "nonneg"):
    s2 = st if case == "plain" else np.maximum(st, 0)
    d = torch.from_numpy(s2.reshape(H, W, -1)).cuda()
    pt = K.pixtable_prepare(d, bounds)
    sw = K.classify_pixels_screen(d, refx, ref.shape[0], bounds, mode=2)
    sg = K.classify_pixels_table_screen(pt, refx, ref.shape[0])
    for name, a, b in zip(("idx", "dist", "second"), sw, sg):
        bad = torch.nonzero((a != b).ravel()).ravel().cpu().numpy()
        print(case, name, "differ on", bad.size, "pixels; first", bad[:10])
