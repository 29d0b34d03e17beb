"""Kernel time of one whole cfg3 tile (registration with image_cn, calibrated measurement,
per-cell and per-pixel classification, counts) run serially on one stream, from a rocprofv3
--kernel-trace database, grouped by kernel.  Run:
  rocprofv3 --kernel-trace -d OUT -o run -- python3 tools/tile_timeline.py run
  python tools/tile_timeline.py OUT/run_results.db"""
import os
import re
import sys

if len(sys.argv) > 1 and sys.argv[1].endswith(".db"):
    import collections
    import sqlite3
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select name, start, end from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if "channel_max_multi" in r[0]]   # a tile's first kernel
    seq = rows[idx[-1]:]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in seq:
        n = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:60]
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    span = (seq[-1][2] - seq[0][1]) / 1e3
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print("%9.1f us %4d  %5.1f%%  %s" % (t, k, 100 * t / tot, n))
    print("kernels %.3f ms, span %.3f ms, %d launches" % (tot / 1e3, span / 1e3, len(seq)))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import pipeline as P, synthetic as S  # noqa: E402

ref = S.reference_library(10, S.ECOLI_BOUNDS)
lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
lib.refx()
st, _, _, _ = S.tile(2048, 2048, seed=20190101)
lasers = S.laser_split(st)
cal = S.flat_field(2048, 2048)
for i in range(4):
    torch.cuda.synchronize()
    torch.zeros(1, device="cuda").fill_(1.0)
    torch.cuda.synchronize()
    rt = P.register_tile(lasers)                 # bench.py's path (pixel table, no stack)
    P.process_tile(rt, lib, calibration=cal, overlap=False)
    torch.cuda.synchronize()
