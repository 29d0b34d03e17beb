"""Per-pixel classifier on one cfg2-like community tile (2048^2 x 63, R = 127): the mode-2 screen
(classify_pixels_lay_kernel, 32x32x16) and the exact path (screen + f64 refine from the stack),
and the list pass's statistics.  python tools/time_classify_exact_multi.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402
from time_classify_exact import ev  # noqa: E402

MULTI = (0, 23, 43, 57, 63)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    stack, _, _, ref = S.tile(2048, 2048, nbit=7, bounds=MULTI, seed=20190301)
    R = ref.shape[0]
    refx = K.classify_prepare(torch.from_numpy(ref).cuda(), MULTI, mode=2)
    t_screen = ev(lambda: K.classify_pixels_screen(stack, refx, R, MULTI, mode=2), n)
    t_exact = ev(lambda: K.classify_pixels(stack, refx, R, MULTI), n)
    idx, dist, sec = K.classify_pixels_screen(stack, refx, R, MULTI, mode=2)
    st = K.classify_refine(K.StackSource(stack), refx, R, MULTI, 2, idx, dist, sec, want_listed="stats")
    P = 2048 * 2048
    print("community screen %.3f ms | exact %.3f ms | listed %d (%.3f %%), %d f64 candidates, %d in full"
          % (t_screen, t_exact, st[0], 100.0 * st[0] / P, st[1], st[2]))
    print("bounds (score units): screen %.3e, per zero segment %.3e, list pass %.3e"
          % K.classify_screen_eps(63, MULTI, R, 2))


if __name__ == "__main__":
    main()
