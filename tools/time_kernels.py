"""Time individual libhrf kernels on resident 2048x2048 inputs (HIP events, mean of 5).

python tools/time_kernels.py [nlmeans] [enhance3d] [classify] [stream] [path] [pathcal]
"""
import sys

import torch

sys.path.insert(0, ".")
from hiprfish_image_analysis_amd import kernels as K  # noqa: E402
from hiprfish_image_analysis_amd import synthetic as S  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    what = sys.argv[1:] or ["nlmeans", "classify"]
    H = W = 2048
    if "nlmeans" in what:
        stack, _, _, _ = S.tile(H, W, nbit=7, bounds=S.MULTI_BOUNDS, seed=1)
        s = K.channel_sum(stack)
        s = K.div_scalar(s, K.max_f64(s))
        ms = timed(lambda: K.nl_means_2d(s, h=0.02))
        print("nl_means_2d 2048^2: %.3f ms  (%.1f Mpix/s, %.2f G pixel-shifts/s)" % (ms, H * W / ms / 1e3,
                                                                                  H * W * 528 / ms / 1e6))
    if "enhance3d" in what:
        # the cfg4 volume: 1024 x 1024 x 64, edge-padded by 5 (biofilm :810-817)
        g = torch.Generator(device="cuda")
        g.manual_seed(4)
        vol = torch.rand((1024, 1024, 64), dtype=torch.float64, device="cuda", generator=g)
        pad = K.pad_edge_3d(vol, 5)
        ms = timed(lambda: K.enhance_3d(pad), 3)
        print("enhance_3d 1024x1024x64: %.3f ms  (%.1f Mvoxel/s)" % (ms, 1024 * 1024 * 64 / ms / 1e3))
    if "classify" in what:
        g = torch.Generator(device="cuda")
        g.manual_seed(0)
        for C, bounds, R in [(95, S.ECOLI_BOUNDS, 1023), (63, S.MULTI_BOUNDS, 127)]:
            stack = torch.rand((H, W, C), generator=g, device="cuda")
            ref = torch.rand((R, C), generator=g, device="cuda")
            for mode in K.classify_modes(bounds):
                refx = K.classify_prepare(ref, bounds, mode)
                ms = timed(lambda: K.classify_pixels(stack, refx, R, bounds, mode))
                tf = 2.0 * H * W * R * C / ms / 1e9
                print("classify C=%d R=%d mode %d: %.3f ms  %.1f TF/s algorithmic" % (C, R, mode, ms, tf))

    if "path" in what or "pathcal" in what:
        # the timed path's streaming kernels (bench.py path_kernel_rows) on one bench tile;
        # "pathcal": label_sums_lasers over a map with every pixel labelled (16x16 blocks), whose
        # algorithmic read is known exactly -- the FETCH_SIZE calibration of its 4-byte lane reads
        sys.path.insert(0, ".")
        import numpy as np
        import bench as B
        from hiprfish_image_analysis_amd import pipeline as P
        ref = S.reference_library(B.NBIT, S.ECOLI_BOUNDS)
        lib = P.Library(torch.from_numpy(ref.astype(np.float64)).cuda(), S.ECOLI_BOUNDS, B.NBIT)
        seed = 20190101
        lay = S.cell_layout(H, W, S.default_ncells(H, W), lib.R, seed)
        truth, prof = S.render_truth(H, W, lay, with_profile=True)
        stack = S.render_stack(truth, lay, ref, seed=seed, device="cuda", profile=prof)
        lasers = S.laser_split(stack)
        del stack
        cal = S.flat_field(H, W, device="cuda")
        rows, info = B.path_kernel_rows(lasers, cal, lib)
        if "path" in what:
            for name, (fn, nb) in rows.items():
                ms = timed(fn, 10)
                print("%s: %.4f ms  %.0f GB/s algorithmic (%.3f of 8 TB/s), %d bytes" % (name, ms, nb / ms / 1e6,
                                                                                       nb / ms / 8e9, nb))
            print(info)
        else:
            rr = torch.arange(H, device="cuda", dtype=torch.int32)[:, None] // 16
            cc = torch.arange(W, device="cuda", dtype=torch.int32)[None, :] // 16
            dense = (1 + rr * (W // 16) + cc).contiguous()
            shifts = P.estimate_shifts(lasers, device=True)
            ms = timed(lambda: K.label_sums_lasers(lasers, shifts, dense, int(dense.max()), True, cal=cal,
                                                   cal_range=(0, 32)), 10)
            nbd = H * W * (4 + 4 * 95 + 4)
            print("label_sums_lasers dense calibration map: %.4f ms, %d algorithmic read bytes" % (ms, nbd))

    if "stream" in what:
        from hiprfish_image_analysis_amd import pipeline as P
        stack, truth, _, _ = S.tile(H, W, seed=3)
        C = stack.shape[2]
        nb = H * W * (4 * C + 8)
        ms = timed(lambda: K.channel_sum(stack, mode=1))
        print("channel_sum (log) 2048^2x95: %.3f ms  %.0f GB/s (%.1f %% of 8 TB/s)" % (ms, nb / ms / 1e6, nb / ms / 8e7))
        lasers, c0 = [], 0
        for c1 in S.ECOLI_BOUNDS[1:]:
            lasers.append(stack[:, :, c0:c1].contiguous())
            c0 = c1
        shifts = [(0, 0), (2, -1), (0, 3), (-1, 0), (1, 1)]
        ms = timed(lambda: K.register_assemble(lasers, shifts, apply_mask=True))
        nb3 = H * W * 8 * C
        print("register_assemble 2048^2x95: %.3f ms  %.0f GB/s (%.1f %% of 8 TB/s)" % (ms, nb3 / ms / 1e6,
                                                                                   nb3 / ms / 8e7))
        cal = torch.rand(C, device="cuda") + 0.5
        ms = timed(lambda: K.channel_sum(stack, cal=cal))
        print("channel_sum cal(C) 2048^2x95: %.3f ms  %.0f GB/s" % (ms, nb / ms / 1e6))
        seg, maxlab = P.segment_ecoli(stack)
        fg = int(K.count_nonzero(seg))
        nb2 = fg * 4 * C + H * W * 4
        ms = timed(lambda: K.label_sums(stack, seg, maxlab))
        print("label_sums (%d labels, %.0f %% fg): %.3f ms  %.0f GB/s algorithmic" % (maxlab, 100.0 * fg / H / W, ms,
                                                                                      nb2 / ms / 1e6))
        # counter calibration for this access width (MI355X_MICROARCH.md: widths other than 16 B
        # per lane are uncalibrated): every pixel labelled (16x16 blocks), so the algorithmic
        # bytes are the whole stack + the label map and FETCH_SIZE / them is the width's factor
        rr = torch.arange(H, device="cuda", dtype=torch.int32)[:, None] // 16
        cc = torch.arange(W, device="cuda", dtype=torch.int32)[None, :] // 16
        dense = (1 + rr * (W // 16) + cc).contiguous()
        nbd = H * W * (4 * C + 4)
        ms = timed(lambda: K.label_sums(stack, dense, int(dense.max())))
        print("label_sums dense calibration map: %.3f ms  %.0f GB/s (%.0f bytes)" % (ms, nbd / ms / 1e6, nbd))
        calp = (0.5 + torch.rand((H, W), device="cuda"))
        ms = timed(lambda: K.label_sums(stack, seg, maxlab, cal=calp, cal_range=(0, 32)))
        print("label_sums plane cal: %.3f ms  %.0f GB/s algorithmic" % (ms, nb2 / ms / 1e6))


if __name__ == "__main__":
    main()
