"""Time hrf_classify_pixels on a resident 2048x2048x95 stack for several library sizes
(separates the per-workgroup prologue from the per-reference sweep).

python tools/time_classify.py [mode] [R ...]     (mode default: the fastest for the layout;
                                                 mode "t": the pixel-table kernel, w16t)
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    args = sys.argv[1:]
    mode = args.pop(0) if args else None
    table = mode == "t"
    mode = None if (mode is None or table) else int(mode)
    H = W = 2048
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    stack = torch.rand((H, W, 95), generator=g, device="cuda")
    pt = K.pixtable_prepare(stack, S.ECOLI_BOUNDS) if table else None
    for R in [int(a) for a in (args or ["64", "256", "1023"])]:
        ref = torch.rand((R, 95), generator=g, device="cuda")
        refx = K.classify_prepare(ref, S.ECOLI_BOUNDS, mode)
        m = K.refx_mode(refx, 95, S.ECOLI_BOUNDS)
        kp, _ = K.classify_geometry(95, 5, R, m)
        def once():
            # the MFMA screen (the roofline's kernel); the exact path adds the f64 refine
            # (tools/time_classify_exact.py)
            if table:
                K.classify_pixels_table_screen(pt, refx, R)
            else:
                K.classify_pixels_screen(stack, refx, R, S.ECOLI_BOUNDS, mode=m)
        for _ in range(2):
            once()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 5
        e0.record()
        for _ in range(n):
            once()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        tf = 2.0 * H * W * R * 95 / ms / 1e9
        print(("table " if table else "") + "mode %d R=%5d  %.3f ms  %.1f TF/s algorithmic  %.1f TF/s executed" % (m, R, ms, tf,
                                                                                   3 * tf * kp / 95 if m else tf))


if __name__ == "__main__":
    t = time.time()
    main()
