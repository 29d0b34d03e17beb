"""bench.py's extras.cfg3.preassembled_uncalibrated alone (six concurrent 2048^2 tiles through the
composed path pipeline.process_tile on a pre-assembled, uncalibrated stack), for A/B runs.
usage: python tools/time_preassembled.py [steps]"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    H = W = 2048
    T = 6
    dev = torch.device("cuda", 0)
    ref = S.reference_library(B.NBIT, S.ECOLI_BOUNDS)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).to(dev), S.ECOLI_BOUNDS, B.NBIT)
    lib.refx()
    lib.presence_flags()
    pre = []
    for t in range(2 * T):
        seed = 20190101 + t
        lay = S.cell_layout(H, W, S.default_ncells(H, W), lib.R, seed)
        truth, prof = S.render_truth(H, W, lay, with_profile=True)
        stack = S.render_stack(truth, lay, ref, seed=seed, device=dev, profile=prof)
        pre.append((P.register_stack(S.laser_split(stack), apply_mask=False),))
        del stack
    torch.cuda.synchronize()
    prio = torch.cuda.Stream.priority_range()[1]
    streams = [torch.cuda.Stream(device=dev, priority=prio) for _ in range(T)]
    pool = ThreadPoolExecutor(T)
    sec = B._timed_tiles(lambda t: P.process_tile(t[0], lib, variant=1), pre, T, streams, pool, steps, 2)
    print("preassembled_uncalibrated %.1f Mpix/s  %.3f ms per step" % (H * W * steps * T / sec / 1e6,
                                                                        sec / steps * 1e3))


if __name__ == "__main__":
    main()
