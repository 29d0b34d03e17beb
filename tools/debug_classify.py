"""Compare classifier modes 1 and 2 on a synthetic tile pixel by pixel (debug aid)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def main():
    stack, truth, lay, ref = S.tile(512, 512, seed=5)
    R = ref.shape[0]
    out = {}
    for mode in (1, 2):
        refx = K.classify_prepare(torch.from_numpy(ref).cuda(), S.ECOLI_BOUNDS, mode)
        out[mode] = [t.cpu().numpy().ravel() for t in K.classify_pixels(stack, refx, R, S.ECOLI_BOUNDS)]
    d = np.abs(out[1][1] - out[2][1])
    bad = np.nonzero(d > 1e-4)[0]
    print("bad pixels:", len(bad), "of", d.size)
    for p in bad[:20]:
        print(p, "wg", p // 256, "lane-pixel", p % 64, "idx", out[1][0][p], out[2][0][p], "dist", out[1][1][p],
              out[2][1][p])
    if len(bad):
        print("workgroups:", np.unique(bad // 256)[:50])


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def in_process_tile():
    from hiprfish_image_analysis_amd import pipeline as P
    stack, truth, lay, ref = S.tile(512, 512, seed=5)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    alone = [t.cpu().numpy().ravel() for t in P.classify_pixels(stack, lib)]
    for overlap in (False, True):
        res = P.process_tile(stack, lib, per_pixel=True, overlap=overlap)
        got = [res.pixel_idx.cpu().numpy().ravel(), res.pixel_dist.cpu().numpy().ravel()]
        bad = np.nonzero(np.abs(got[1] - alone[1]) > 1e-6)[0]
        print("overlap", overlap, "bad", len(bad), "wgs", np.unique(bad // 256)[:40])
        for p in bad[:8]:
            print("  ", p, got[0][p], alone[0][p], got[1][p], alone[1][p])


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pt":
    in_process_tile()


def vs_oracle():
    sys.path.insert(0, "oracle")
    import oracle as O
    stack, truth, lay, ref = S.tile(512, 512, seed=5)
    R = ref.shape[0]
    st = stack.cpu().numpy().reshape(-1, 95)
    sel = np.random.default_rng(0).choice(512 * 512, 400, replace=False)
    x = st[sel].astype(np.float64)
    ri, rd = O.classify(x, ref.astype(np.float64), S.ECOLI_BOUNDS, 0)
    for mode in (1, 2):
        refx = K.classify_prepare(torch.from_numpy(ref).cuda(), S.ECOLI_BOUNDS, mode)
        gi, gd = [t.cpu().numpy().ravel()[sel] for t in K.classify_pixels(stack, refx, R, S.ECOLI_BOUNDS)]
        bad = np.nonzero(np.abs(gd - rd) > 1e-4)[0]
        print("mode", mode, "bad", len(bad))
        for b in bad[:6]:
            print("  pixel", sel[b], "gpu", gi[b], gd[b], "oracle", ri[b], rd[b], "x min/max/sum", x[b].min(), x[b].max(),
                  x[b].sum(), "segsums", [x[b][lo:hi].sum() for lo, hi in zip(S.ECOLI_BOUNDS[:-1], S.ECOLI_BOUNDS[1:])])


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "oracle":
    vs_oracle()


def like_test():
    sys.path.insert(0, "oracle")
    import oracle as O
    from hiprfish_image_analysis_amd import pipeline as P
    stack, truth, lay, ref = S.tile(512, 512, seed=5)
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    res = P.process_tile(stack, lib, per_pixel=True)
    sel = np.random.default_rng(0).choice(512 * 512, 400, replace=False)
    x = stack.cpu().numpy().reshape(512 * 512, -1)[sel].astype(np.float64)
    ri, rd = O.classify(x, ref.astype(np.float64), S.ECOLI_BOUNDS, 0)
    pi, pd = res.pixel_idx.cpu().numpy().ravel()[sel], res.pixel_dist.cpu().numpy().ravel()[sel]
    bad = np.nonzero(np.abs(pd - rd) > 1e-4)[0]
    print("like_test bad", len(bad), [(sel[b], pi[b], ri[b], pd[b], rd[b]) for b in bad[:6]])
    alone = [t.cpu().numpy().ravel()[sel] for t in P.classify_pixels(stack, lib)]
    print("alone bad", np.count_nonzero(np.abs(alone[1] - rd) > 1e-4))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "test":
    like_test()


def after_measure():
    if len(sys.argv) > 2:
        K.CLASSIFY_MODE = int(sys.argv[2])
    sys.path.insert(0, "oracle")
    import oracle as O
    from hiprfish_image_analysis_amd import pipeline as P
    st0, _, _, _ = S.tile(384, 640, seed=3)
    P.measure_ecoli(st0)
    del st0
    stack, truth, lay, ref = S.tile(512, 512, seed=5)
    stack_copy = stack.clone()
    lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, 10)
    res = P.process_tile(stack, lib, per_pixel=True)
    torch.cuda.synchronize()
    print("stack changed:", bool((stack != stack_copy).any()))
    fresh, _, _, _ = S.tile(512, 512, seed=5)
    print("stack == regenerated:", bool((stack == fresh).all()))
    alone = [t.cpu().numpy().ravel() for t in P.classify_pixels(fresh, lib)]
    got = [res.pixel_idx.cpu().numpy().ravel(), res.pixel_dist.cpu().numpy().ravel()]
    bad = np.nonzero(np.abs(got[1] - alone[1]) > 1e-6)[0]
    print("bad vs alone", len(bad), "wgs", np.unique(bad // 256)[:30], "rows", np.unique(bad // 512)[:30])
    for p in bad[:6]:
        print("  ", p, got[0][p], alone[0][p], got[1][p], alone[1][p])


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "after":
    after_measure()
