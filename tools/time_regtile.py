"""Isolated kernel times of the two registered-tile paths on one 2048x2048 cfg3 tile: assembly
(stack + image_cn) vs assembly writing image_cn + pixel table; label sums from the stack vs from
the lasers; the classifier's in-kernel operand build vs the table.  Dev tool."""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K, pipeline as P, synthetic as S  # noqa: E402


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
lasers = S.laser_split(st)
shifts = P.estimate_shifts(lasers, device=True)
cal = S.flat_field(2048, 2048)
reg, cn = K.register_assemble(lasers, shifts, True, cn_mode=1)
seg, maxlab = P.segment_ecoli(reg, image_cn=cn)
lib = P.Library(torch.from_numpy(ref).double().cuda(), S.ECOLI_BOUNDS, 10)
refx = lib.refx()
print("assemble stack + cn        %.4f ms" % ev(lambda: K.register_assemble(lasers, shifts, True, cn_mode=1)))
print("assemble cn + pixtable     %.4f ms" % ev(lambda: K.register_assemble_pixtable(lasers, shifts, True)))
print("label_sums (stack, cal)    %.4f ms" % ev(lambda: K.label_sums(reg, seg, maxlab, cal=cal, cal_range=(0, 32))))
print("label_sums_lasers (cal)    %.4f ms" % ev(lambda: K.label_sums_lasers(lasers, shifts, seg, maxlab, True, cal=cal)))
pt = K.register_assemble_pixtable(lasers, shifts, True)[1]
print("classify w16 (stack)       %.4f ms" % ev(lambda: K.classify_pixels(reg, refx, lib.R, lib.bounds)))
print("classify w16t (table)      %.4f ms" % ev(lambda: K.classify_pixels_table(pt, refx, lib.R)))
print("channel_max_multi          %.4f ms" % ev(lambda: K.channel_max_multi(lasers, stacked=True)))
proj = K.channel_max_multi(lasers, stacked=True)
print("xcorr shifts               %.4f ms" % ev(lambda: K.xcorr_shifts_dev(proj, 15)))
cells = P.process_tile(pt and P.register_tile(lasers), lib, calibration=cal, per_pixel=False, variant=1)
xn = cells.meas.avgint_norm
fr = lib.presence_flags()
fx = K.segment_flags(xn, lib.bounds)
print("classify_cells (%d cells)  %.4f ms" % (xn.shape[0], ev(lambda: K.classify_cells(xn, lib.spectra, lib.bounds, 1, fx, fr))))
