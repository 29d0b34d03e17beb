"""Does v_mfma_f32_16x16x32_f16 return C exactly when every product is zero (B = 0)?  (the
indicator step of the screen's zero-segment workgroups runs it on pixels without zero segments)"""
import numpy as np
import torch

from hiprfish_image_analysis_amd import _lib

rng = np.random.default_rng(3)
n = 64
for shape, (M, Kd, N) in ((0, (16, 32, 16)), (1, (32, 16, 32))):
    A = rng.random((n, M, Kd))
    B = np.zeros((n, Kd, N))
    for name, Cm in (("unit", rng.random((n, M, N)) * 5), ("wide", rng.random((n, M, N)) * 2.0 ** rng.integers(-40, 40, (n, M, N))),
                     ("neg", rng.normal(size=(n, M, N)))):
        a = torch.from_numpy(A.astype(np.float16)).cuda()
        b = torch.from_numpy(B.astype(np.float16)).cuda()
        c = torch.from_numpy(Cm.astype(np.float32)).cuda()
        d = torch.empty_like(c)
        _lib.call("hrf_probe_mfma_f16", shape, a.data_ptr(), b.data_ptr(), c.data_ptr(), d.data_ptr(), n,
                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        diff = (d != c).sum().item()
        print("shape %d %-5s: %d of %d outputs differ from C; max rel %.3g" % (
            shape, name, diff, c.numel(), ((d - c).abs() / c.abs().clamp_min(1e-30)).max().item()))
