"""Time hrf_classify_cells (per-cell segmented-cosine argmin, f64) for N cells against the
1023-barcode library: python tools/time_cells.py [N]"""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 700
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    x = torch.rand((N, 95), generator=g, device="cuda", dtype=torch.float64)
    ref = torch.rand((1023, 95), generator=g, device="cuda", dtype=torch.float64)
    for variant in (0,):
        K.classify_cells(x, ref, S.ECOLI_BOUNDS, variant)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            K.classify_cells(x, ref, S.ECOLI_BOUNDS, variant)
        e1.record()
        torch.cuda.synchronize()
        print("classify_cells N=%d R=1023 C=95 variant %d: %.3f ms" % (N, variant, e0.elapsed_time(e1) / 10))


if __name__ == "__main__":
    main()
