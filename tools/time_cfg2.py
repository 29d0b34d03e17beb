"""bench.py's extras.cfg2 alone (six concurrent 2048^2 synthetic-community tiles: registration on
channel sums, calibrated sum, NL-means, enhancement, segmentation, per-cell and per-pixel
classification), for kernel traces and A/B runs.  usage: python tools/time_cfg2.py [steps]"""
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
    b = S.MULTI_BOUNDS
    ref = S.reference_library(7, b)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).to(dev), b, 7)
    lib.refx()
    ccal = S.calibration_stack(H, W, 63, device=dev)
    tiles = []
    for t in range(2 * T):
        st = S.tile(H, W, nbit=7, bounds=b, seed=20190201 + t, device=dev)[0]
        tiles.append(S.laser_split(st, b, S.COMMUNITY_SHIFTS))
        del st
    torch.cuda.synchronize()

    def job(lasers):
        reg = P.register_multispecies(lasers)
        return P.process_tile(reg, lib, calibration=ccal, measure=P.measure_multispecies, variant=2)
    prio = torch.cuda.Stream.priority_range()[1]
    streams = [torch.cuda.Stream(device=dev, priority=prio) for _ in range(T)]
    sec = B._timed_tiles(job, tiles, T, streams, ThreadPoolExecutor(T), steps, 2)
    print("cfg2 %.1f Mpix/s  %.3f ms per tile" % (H * W * steps * T / sec / 1e6, sec / (steps * T) * 1e3))


if __name__ == "__main__":
    main()
