"""The watershed's heap replay (hrf_watershed_heap) alone on bench.py's adversarial plateau image
(n x n, default 1024), timed with HIP events and checked against the oracle's heap flood.  Dev tool
for the replay kernel (watershed.hip ws_heap_flood_kernel).  usage: python tools/time_heap_replay.py [n] [ramp]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
import oracle as orc  # noqa: E402   (the checker)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    ramp = len(sys.argv) > 2 and sys.argv[2] == "ramp"
    orc.build()
    rng = np.random.default_rng(7)
    if ramp:  # one marker at a corner of a ramp: the heap holds one anti-diagonal (< 2n items)
        f = np.add.outer(np.arange(n), np.arange(n)).astype(np.float64)
        markers = np.zeros((n, n), np.int32)
        markers[0, 0] = 1
        mask = np.ones((n, n), bool)
    else:
        f = np.kron(rng.integers(0, 4, (n // 4, n // 4)), np.ones((4, 4))).astype(np.float64)
        markers = np.zeros((n, n), np.int32)
        for lab in range(1, n * n // 300 + 1):
            r, c = rng.integers(1, n - 1), rng.integers(1, n - 1)
            markers[r - 1:r + 2, c - 1:c + 2] = lab
        f = f + 1e-3 * markers
        mask = rng.random((n, n)) < 0.9
    x, mk, mm = (torch.from_numpy(a).cuda() for a in (f, markers, mask))
    K.watershed_heap(x, mk, mm)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    got = K.watershed_heap(x, mk, mm)
    b.record()
    torch.cuda.synchronize()
    t = time.time()
    ref = orc.watershed(f, markers, mask)
    tc = time.time() - t
    ok = np.array_equal(got.cpu().numpy(), ref)
    print("heap replay %dx%d%s: %.1f ms on the device (oracle %.2f s on one host core), equal to the oracle: %s"
          % (n, n, " ramp" if ramp else "", a.elapsed_time(b), tc, ok))
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
