"""Upper bound on batching the segmentation chain across tiles: the native tile
path (hrf_tile_ecoli) over one tall image of K bench tiles stacked along H -- one launch per stage
for K tiles' pixels, the chain's host synchronisations shared -- against K concurrent 2048^2 tiles
(bench.py's schedule).  Same pixels, same cells per pixel; the tall image's registration is one
(2048 K) x 2048 estimate instead of K 2048^2 ones.  usage: python tools/time_tall.py [steps]"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    H = W = 2048
    dev = torch.device("cuda", 0)
    ref = S.reference_library(B.NBIT, S.ECOLI_BOUNDS)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).to(dev), S.ECOLI_BOUNDS, B.NBIT)
    lib.refx()
    lib.presence_flags()
    stacks = []
    for t in range(8):
        seed = 20190101 + t
        lay = S.cell_layout(H, W, S.default_ncells(H, W), lib.R, seed)
        truth, prof = S.render_truth(H, W, lay, with_profile=True)
        stacks.append(S.render_stack(truth, lay, ref, seed=seed, device=dev, profile=prof))
    small = [(S.laser_split(s), S.flat_field(H, W, device=dev)) for s in stacks]
    tall = {}
    for k in (4, 8):
        tiles = []
        for first in range(0, 8, k):
            tiles.append((S.laser_split(torch.cat(stacks[first:first + k], 0)), S.flat_field(k * H, W, device=dev)))
        tall[k] = tiles
    del stacks
    torch.cuda.synchronize()
    prio = torch.cuda.Stream.priority_range()[1]

    def job(per_pixel):
        def f(t):
            P.process_tile_native(t[0], lib, calibration=t[1], per_pixel=per_pixel, variant=1)
        return f

    def timed(tiles, T, per_pixel, px_per_tile):
        streams = [torch.cuda.Stream(device=dev, priority=prio) for _ in range(T)]
        pool = ThreadPoolExecutor(T) if T > 1 else None
        sec = B._timed_tiles(job(per_pixel), tiles, T, streams, pool, steps, 1)
        if pool:
            pool.shutdown()
        return px_per_tile * steps * T / sec / 1e6, sec / steps * 1e3

    rows = []
    for rnd in range(3):      # interleaved
        for per_pixel in (True, False):
            for name, tiles, T, px in (("8 x 2048^2, 8 concurrent", small, 8, H * W),
                                       ("6 x 2048^2, 6 concurrent", small, 6, H * W),
                                       ("16384 x 2048 (8 tiles), 1 stream", tall[8], 1, 8 * H * W),
                                       ("8192 x 2048 (4 tiles), 2 concurrent", tall[4], 2, 4 * H * W)):
                v, ms = timed(tiles, T, per_pixel, px)
                line = "round %d  per_pixel %-5s  %-38s %8.1f Mpix/s  %8.2f ms per step" % (rnd, per_pixel, name, v, ms)
                print(line, flush=True)
                rows.append(line)
    print("\n".join(rows))


if __name__ == "__main__":
    t0 = time.time()
    main()
    print("%.0f s" % (time.time() - t0))
