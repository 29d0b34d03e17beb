"""Per-pixel classifier on one bench-like 2048^2 x 95 tile (R = 1023): the w16t screen from the
assembly's pixel table, the f64 refine reading the five shifted acquisitions, and the number of
pixels the certificate left to the list pass.  HIP events on the current stream.
python tools/time_classify_exact.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def ev(fn, n):
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    stack, _, _, ref = S.tile(2048, 2048, seed=20190301)
    lasers = S.laser_split(stack)
    rt = P.register_tile(lasers)
    R = ref.shape[0]
    refx = K.classify_prepare(torch.from_numpy(ref).cuda(), S.ECOLI_BOUNDS, mode=2)
    pt = rt.pixtable
    idx, dist, sec = K.classify_pixels_table_screen(pt, refx, R)
    t_screen = ev(lambda: K.classify_pixels_table_screen(pt, refx, R), n)
    i2, d2 = idx.clone(), dist.clone()

    def refine():
        i2.copy_(idx)
        d2.copy_(dist)
        K.classify_refine(pt.source, refx, R, S.ECOLI_BOUNDS, 3, i2, d2, sec)
    t_copy = ev(lambda: (i2.copy_(idx), d2.copy_(dist)), n)
    t_ref = ev(refine, n) - t_copy
    i2.copy_(idx)
    d2.copy_(dist)
    listed = K.classify_refine(pt.source, refx, R, S.ECOLI_BOUNDS, 3, i2, d2, sec, want_listed=True)
    t_unf = ev(lambda: K.classify_pixels_table(pt, refx, R), n)
    t_full = ev(lambda: K.classify_pixels_table(pt, refx, R, fused=True), n)
    for fu in (False, True):
        fi, fd, flisted = K.classify_pixels_table(pt, refx, R, fused=fu, want_listed=True)
        assert torch.equal(fi, i2) and torch.equal(fd, d2) and flisted == listed, "exact paths differ"
    Pn = 2048 * 2048
    changed = int((i2 != idx).sum().item())
    print("w16t screen %.3f ms | refine %.3f ms | exact unfused %.3f ms | exact fused %.3f ms | listed %d of %d "
          "pixels (%.3f %%) | screen row changed on %d pixels" % (t_screen, t_ref, t_unf, t_full, listed, Pn,
                                                                  100.0 * listed / Pn, changed))
    i2.copy_(idx)
    d2.copy_(dist)
    st = K.classify_refine(pt.source, refx, R, S.ECOLI_BOUNDS, 3, i2, d2, sec, want_listed="stats")
    print("list pass: %d pixels, %d sparse f64 candidates (%.1f per pixel), %d pixels scored in full"
          % (st[0], st[1], st[1] / max(st[0], 1), st[2]))
    eps = K.classify_screen_eps(95, S.ECOLI_BOUNDS, R, 3)
    print("bounds (score units): screen %.3e, per zero segment %.3e, list pass %.3e" % eps)


if __name__ == "__main__":
    main()
