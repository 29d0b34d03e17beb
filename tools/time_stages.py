"""Per-stage wall time of the E. coli segmentation chain on one resident 2048x2048x95 tile
(each stage synchronised, so host round trips inside a stage are included).

python tools/time_stages.py [reps]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import pipeline as P  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    stack, truth, lay, ref = S.tile(2048, 2048, seed=20190101)
    lib = P.Library(torch.tensor(ref, dtype=torch.float64, device="cuda"), S.ECOLI_BOUNDS, 10)
    lib.refx()
    torch.cuda.synchronize()
    acc = {}

    def st(name, fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        acc.setdefault(name, []).append((time.perf_counter() - t) * 1e3)
        return r

    for _ in range(reps):
        image_cn = st("channel_sum+log", lambda: K.channel_sum(stack, mode=1))
        _, rough, _, _ = st("kmeans k=2", lambda: K.kmeans_1d(image_cn, 2, want_labels=False))
        _, interior, _, _ = st("kmeans k=3", lambda: K.kmeans_1d(image_cn, 3, want_labels=False))
        opened = st("holes+opening", lambda: K.binary_opening(K.remove_small_holes(interior, 64, 1)))
        cell_sm = st("rso(50)", lambda: K.remove_small_objects(opened, 50, conn=1))
        be = st("erosion seeds", lambda: P.erosion_seeds(cell_sm))
        seeds_mask = st("rso(10)", lambda: K.remove_small_objects(be, 10, conn=2))
        seeds, nseeds = st("label seeds", lambda: K.label(seeds_mask, conn=2))
        seg = st("watershed", lambda: K.watershed(image_cn, seeds, rough, negate=True))
        seg = st("rso labels(100)", lambda: K.remove_small_objects(seg, 100, maxlab=nseeds))
        seg = st("clear_border", lambda: K.clear_border(seg))
        props = st("region_props", lambda: K.region_props(seg, nseeds))
        final = st("shape_filter", lambda: K.shape_filter(seg, props, nseeds, 15.0, 35.0))
        sums, counts = st("label_sums", lambda: K.label_sums(stack, final, nseeds))
        tab = st("cell_table", lambda: K.cell_table(sums, counts, nseeds))
        idx, dist = st("classify_cells", lambda: P.classify_cells(tab[3], lib))
        st("counts+paint", lambda: (K.barcode_counts(idx, lib.R), K.paint_ids(final, idx + 1)))
        st("classify_pixels", lambda: P.classify_pixels(stack, lib))
        st("process_tile (no per-pixel)", lambda: P.process_tile(stack, lib, per_pixel=False))
        st("process_tile (overlapped per-pixel)", lambda: P.process_tile(stack, lib, per_pixel=True))
    tot = 0.0
    for k, v in acc.items():
        m = sorted(v)[len(v) // 2]
        if not k.startswith("process_tile") and k != "classify_pixels":
            tot += m
        print("%-40s %8.3f ms" % (k, m))
    print("%-40s %8.3f ms" % ("sum of segmentation stages", tot))


if __name__ == "__main__":
    main()
