"""Time hrf_kmeans_1d (k=2, k=3) on a 2048x2048 log-intensity image like segment_ecoli's, both
paths (sorted: one sort + step searches; stream: one pass per Lloyd iteration), and the
shared-sort pair segment_ecoli runs."""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        r = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, r


def main():
    stack, _, _, _ = S.tile(2048, 2048)
    img = K.channel_sum(stack, mode=1)
    for path in ("stream", "sorted"):
        for k in (2, 3):
            ms, (_, _, cen, it) = timed(lambda: K.kmeans_1d(img, k, want_labels=False, path=path))
            print("%-6s k=%d  %.3f ms  iters %d  centres %s" % (path, k, ms, it, cen))

    def pair():
        share = {}
        K.kmeans_1d(img, 2, want_labels=False, share=share)
        return K.kmeans_1d(img, 3, want_labels=False, share=share)
    ms, _ = timed(pair)
    print("sorted k=2 + k=3 sharing one sort: %.3f ms" % ms)


if __name__ == "__main__":
    main()
