"""Kernel timeline of one native E. coli segmentation of a registered cfg3 tile (the last of
5 calls), from a rocprofv3 --kernel-trace database: per kernel start offset, duration and the
idle gap before it.  Run: rocprofv3 --kernel-trace -d OUT -o run -- python3 tools/seg_timeline.py run
then: python tools/seg_timeline.py OUT/run_results.db"""
import os
import sys

if len(sys.argv) > 1 and sys.argv[1].endswith(".db"):
    import re
    import sqlite3
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select name, start, end from kernels order by start"))
    # the last segmentation: after the last 'seg_marker' fill (torch.zeros launch below)
    idx = [i for i, r in enumerate(rows) if "FillFunctor" in r[0]]
    start = idx[-1] + 1 if idx else 0
    seq = rows[start:]
    t0 = seq[0][1]
    prev_end = t0
    busy = 0
    for n, s, e in seq:
        n = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:60]
        print("%8.1f us  %7.1f us  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, max(0, s - prev_end) / 1e3, n))
        busy += e - max(s, prev_end) if e > prev_end else 0
        prev_end = max(prev_end, e)
    print("span %.3f ms, kernels busy %.3f ms, %d launches" % ((prev_end - t0) / 1e6, busy / 1e6, len(seq)))
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiprfish_image_analysis_amd import pipeline as P, synthetic as S  # noqa: E402

st, _, _, _ = S.tile(2048, 2048, seed=20190101)
reg = P.register_stack(S.laser_split(st))
for i in range(5):
    torch.cuda.synchronize()
    torch.zeros(1, device="cuda").fill_(1.0)     # marker launch before each call
    torch.cuda.synchronize()
    P.segment_ecoli(reg)
    torch.cuda.synchronize()
