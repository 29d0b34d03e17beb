"""Wall time of the device pipeline per tile against tile size: at small tiles the GPU work
is negligible and what remains is host overhead (Python, launches, synchronisations)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    for hw in (128, 512, 2048):
        stack, _, _, ref = S.tile(hw, hw, seed=3)
        lib = P.Library(torch.tensor(ref, dtype=torch.float64, device="cuda"), S.ECOLI_BOUNDS, 10)
        lib.refx()
        for per_pixel in (False, True):
            P.process_tile(stack, lib, per_pixel=per_pixel)
            torch.cuda.synchronize()
            n = 10
            t = time.perf_counter()
            c = time.process_time()
            for _ in range(n):
                P.process_tile(stack, lib, per_pixel=per_pixel)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t) / n * 1e3
            cpu = (time.process_time() - c) / n * 1e3
            print("%4d^2 per_pixel=%d: %.3f ms wall, %.3f ms host CPU per tile" % (hw, per_pixel, wall, cpu))


if __name__ == "__main__":
    main()
