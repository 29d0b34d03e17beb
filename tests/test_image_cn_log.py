"""a3: image_cn = log(sum + 1e-2) (ecoli measurement.py:71-72) feeds the KMeans thresholds
(:73-94) and the watershed priorities (:113), so its last bit could matter.  libhrf and the
oracle compute the correctly rounded log (detmath.h hrf_cr_log); the reference's numpy 1.16
called the C library's log, which differs from it in the last ulp on ~1e-4 of the inputs.

This runs the E. coli segmentation restatement (oracle/pipeline.py segment_ecoli, :44-127) on the
bench's full-size 2048x2048x95 tile -- bench.py's generator and seed, rendered on the CPU (torch's
CPU generator, so the noise realisation is not the GPU's), misregistered into the five lasers,
shifts estimated and registered as :45-70 do -- continuous and bioformats-like k/4095 and k/255
samples, twice: once with image_cn from glibc's log, once from the correctly rounded log.  The
segmentations must be identical; the number of differing image_cn pixels is printed.
CPU only (no GPU, no libhrf)."""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _one(q):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, REPO)
    import torch

    import oracle as O
    import pipeline as OP
    from hiprfish_image_analysis_amd import synthetic as S
    torch.set_num_threads(2)
    H = W = 2048
    seed = 20190101                         # bench.py's first tile (rank 0, t 0)
    ref = S.reference_library(10, S.ECOLI_BOUNDS)
    lay = S.cell_layout(H, W, S.default_ncells(H, W), ref.shape[0], seed)
    truth, prof = S.render_truth(H, W, lay, with_profile=True)
    stack = S.render_stack(truth, lay, ref, seed=seed, device="cpu", profile=prof)
    lasers = S.laser_split(stack)
    del stack
    if q:
        lasers = [(torch.round(l.double() * float(q)) / float(q)).float().contiguous() for l in lasers]
    hl = [l.numpy() for l in lasers]
    del lasers
    shifts = OP.estimate_shifts(hl, "max", 15)
    # numpy's pairwise channel sum of the registered f32 stack in f64 (libhrf's image_cn input),
    # 256 rows at a time (each pixel's sum is independent of the others)
    ssum = np.empty((H, W))
    reg = OP.register_stacks(hl, shifts, True).astype(np.float32)
    del hl
    for r0 in range(0, H, 256):
        ssum[r0:r0 + 256] = np.sum(reg[r0:r0 + 256].astype(np.float64), axis=2)
    del reg
    ssum += 1e-2
    cn_cr = O.cr_log(ssum)
    cn_libm = O.libm_log(ssum)
    ndiff = int((cn_cr != cn_libm).sum())
    seg_cr, n_cr = OP.segment_ecoli(None, image_cn=cn_cr)
    seg_libm, n_libm = OP.segment_ecoli(None, image_cn=cn_libm) if ndiff else (seg_cr, n_cr)
    return q, ndiff, int(n_cr), int(seg_cr.max()), bool(np.array_equal(seg_cr, seg_libm)), int(n_cr == n_libm)


@pytest.mark.timeout(900)
def test_image_cn_libm_log_gives_the_same_segmentation():
    qs = [None, 4095, 255]
    with ProcessPoolExecutor(len(qs)) as ex:
        res = list(ex.map(_one, qs))
    for q, ndiff, nseeds, maxlab, same, same_n in res:
        print("tile q=%s: image_cn pixels where glibc's log differs from the correctly rounded log: %d of %d; "
              "seeds %d, segmentation identical: %s" % (q, ndiff, 2048 * 2048, nseeds, same))
    for q, ndiff, nseeds, maxlab, same, same_n in res:
        assert nseeds > 500
        assert same and same_n, q
    assert any(r[1] > 0 for r in res)       # the two logs do differ on these tiles
