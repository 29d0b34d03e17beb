"""Isolated timing on one resident 2048x2048x95 tile (R = 1023): the in-kernel classifier (w16)
against the standalone pixel-table pass + the table classifier (w16t).  Dev tool."""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K, synthetic as S  # noqa: E402


def ev(fn, n=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


st, _, _, ref = S.tile(2048, 2048, seed=20190101)
b = S.ECOLI_BOUNDS
refx = K.classify_prepare(torch.from_numpy(ref).cuda(), b)
R = ref.shape[0]
pt = K.pixtable_prepare(st, b)
print("w16 in-kernel      %.4f ms" % ev(lambda: K.classify_pixels(st, refx, R, b)))
print("pixtable prepare   %.4f ms" % ev(lambda: K.pixtable_prepare(st, b)))
print("w16t from table    %.4f ms" % ev(lambda: K.classify_pixels_table(pt, refx, R)))
a = K.classify_pixels(st, refx, R, b)
c = K.classify_pixels_table(pt, refx, R)
print("equal", torch.equal(a[0], c[0]) and torch.equal(a[1], c[1]))
