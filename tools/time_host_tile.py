"""Host CPU time per bench tile job (register_stack + process_tile with the flat field), at a
small tile where the GPU work is negligible and at the bench size.  Dev tool."""
import sys
import time

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    for hw in (128, 2048):
        stack, _, _, ref = S.tile(hw, hw, seed=3)
        lasers = S.laser_split(stack)
        cal = S.flat_field(hw, hw, device="cuda")
        lib = P.Library(torch.tensor(ref, dtype=torch.float64, device="cuda"), S.ECOLI_BOUNDS, 10)
        lib.refx()

        def job():
            st, cn = P.register_stack(lasers, want_cn=True)
            return P.process_tile(st, lib, calibration=cal, image_cn=cn)
        job()
        torch.cuda.synchronize()
        n = 10
        t = time.perf_counter()
        c = time.process_time()
        for _ in range(n):
            job()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / n * 1e3
        cpu = (time.process_time() - c) / n * 1e3
        print("%4d^2: %.3f ms wall, %.3f ms host CPU per tile job" % (hw, wall, cpu), flush=True)


if __name__ == "__main__":
    main()
