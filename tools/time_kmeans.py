"""Time hrf_kmeans_1d (k=2, k=3) on a 2048x2048 log-intensity image like segment_ecoli's."""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    stack, _, _, _ = S.tile(2048, 2048)
    img = K.channel_sum(stack, mode=1)
    for k in (2, 3):
        K.kmeans_1d(img, k, want_labels=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            _, _, cen, it = K.kmeans_1d(img, k, want_labels=False)
        e1.record()
        torch.cuda.synchronize()
        print("k=%d  %.3f ms  iters %d  centres %s" % (k, e0.elapsed_time(e1) / 5, it, cen))


if __name__ == "__main__":
    main()
