"""Registration shift estimate: hipFFT cross-correlation argmax against
the numpy restatement of skimage.feature.register_translation (oracle.register_translation),
plus the channel projections it runs on and the calibrated stack (multispecies :104)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from hiprfish_image_analysis_amd import kernels
    return kernels


def smooth_image(H, W, seed):
    rng = np.random.default_rng(seed)
    x = rng.random((H, W))
    for _ in range(3):  # a few box blurs: a single dominant correlation peak
        x = (x + np.roll(x, 1, 0) + np.roll(x, -1, 0) + np.roll(x, 1, 1) + np.roll(x, -1, 1)) / 5
    return x


@pytest.mark.parametrize("H,W,dr,dc", [(64, 64, 3, -5), (128, 96, -7, 11), (200, 256, 0, 0), (255, 129, 12, -1),
                                       (512, 512, -15, 15)])
def test_register_translation_known_shift(K, orc, H, W, dr, dc):
    src = smooth_image(H, W, H + W)
    tgt = np.roll(src, (-dr, -dc), axis=(0, 1))    # src = tgt shifted by (dr, dc)
    want = tuple(int(v) for v in orc.register_translation(src, tgt))
    assert want == (dr, dc)
    got = K.register_translation(torch.from_numpy(src).cuda(), torch.from_numpy(tgt).cuda())
    assert got == want


@pytest.mark.parametrize("seed", range(4))
def test_register_translation_matches_restatement(K, orc, seed):
    rng = np.random.default_rng(seed)
    H, W = int(rng.integers(16, 300)), int(rng.integers(16, 300))
    a, b = rng.random((H, W)), rng.random((H, W))
    b[: H // 2] += 0.3 * a[: H // 2]
    got = K.register_translation(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda())
    assert got == tuple(int(v) for v in orc.register_translation(a, b))


def test_channel_projections_and_calibrate(K):
    rng = np.random.default_rng(5)
    x = rng.random((96, 80, 23)).astype(np.float32)
    x[3, 4, 7] = np.nan
    d = torch.from_numpy(x).cuda()
    got = K.channel_max(d).cpu().numpy()
    np.testing.assert_array_equal(got, np.max(x, axis=2).astype(np.float64))
    for cal in ((0.5 + rng.random(23)).astype(np.float32), (0.5 + rng.random((96, 80, 23))).astype(np.float32),
                (0.5 + rng.random((96, 80))).astype(np.float32)):
        want = x.astype(np.float64) / (cal.astype(np.float64)[..., None] if cal.ndim == 2 else cal.astype(np.float64))
        np.testing.assert_array_equal(K.calibrate(d, torch.from_numpy(cal).cuda()).cpu().numpy(), want)
        np.testing.assert_array_equal(K.channel_sum(d, cal=torch.from_numpy(cal).cuda()).cpu().numpy(),
                                      np.sum(want, axis=2))


def test_estimate_shifts_pipeline(K, orc):
    import pipeline as OP

    from hiprfish_image_analysis_amd import pipeline as P
    base = smooth_image(160, 160, 9)
    rng = np.random.default_rng(9)
    shifts = [(0, 0), (4, -3), (-20, 2), (1, 17)]
    lasers = []
    for i, (dr, dc) in enumerate(shifts):
        img = np.roll(base, (-dr, -dc), axis=(0, 1))
        lasers.append((img[..., None] * (0.5 + rng.random(5 + i))).astype(np.float32))
    dl = [torch.from_numpy(l).cuda() for l in lasers]
    for reduce, clamp in (("max", 15), ("sum", None)):
        got = P.estimate_shifts(dl, reduce, clamp)
        assert got == OP.estimate_shifts(lasers, reduce, clamp)
    assert P.estimate_shifts(dl, "max", 15) == [(0, 0), (4, -3), (0, 2), (1, 0)]
    assert P.estimate_shifts(dl, "sum", None) == shifts
    # registered stack as the reference assembles it (no frame mask in multispecies :100-102)
    reg = K.register_assemble(dl, shifts, apply_mask=False).cpu().numpy()
    np.testing.assert_array_equal(reg, OP.register_stacks(lasers, shifts, False).astype(np.float32))


def test_estimate_shifts_on_device_equals_host(K):
    """estimate_shifts(device=True) + register_assemble on the device shifts (no host round
    trip) == the host path: lasers cut from one smooth stack with known misregistrations"""
    from hiprfish_image_analysis_amd import pipeline as P
    rng = np.random.default_rng(9)
    H, W = 160, 144
    img = smooth_image(H, W, 40)                      # every channel a scaled copy: correlated projections
    base = (img[:, :, None] * (0.5 + np.arange(20) / 40.0) + 0.01 * rng.random((H, W, 20))).astype(np.float32)
    want_sh = [(0, 0), (3, -2), (0, 4), (-20, 1)]   # the last one beyond the clamp (15): -> (0, 1)
    lasers = []
    c0 = 0
    for (dr, dc), cl in zip(want_sh, (6, 5, 5, 4)):
        lasers.append(torch.from_numpy(np.ascontiguousarray(np.roll(base[:, :, c0:c0 + cl], (-dr, -dc), (0, 1)))).cuda())
        c0 += cl
    host = P.estimate_shifts(lasers)
    dev = P.estimate_shifts(lasers, device=True)
    assert dev.dtype == torch.int32 and dev.shape == (4, 2)
    assert [tuple(r) for r in dev.cpu().tolist()] == host
    assert host[1] == (3, -2) and host[2] == (0, 4) and host[3] == (0, 1)
    for m in (True, False):
        a = K.register_assemble(lasers, host, apply_mask=m)
        b = K.register_assemble(lasers, dev, apply_mask=m)
        assert torch.equal(a, b)
    assert torch.equal(P.register_stack(lasers), K.register_assemble(lasers, host, apply_mask=True))
    unclamped = P.estimate_shifts(lasers, clamp=None, device=True).cpu().tolist()
    assert tuple(unclamped[3]) == (-20, 1) and [tuple(r) for r in unclamped] == P.estimate_shifts(lasers, clamp=None)


@pytest.mark.parametrize("n,H,W", [(2, 64, 80), (5, 160, 144), (5, 257, 96)])
def test_batched_registration_equals_per_target(K, orc, n, H, W):
    """the batched estimate (one batched D2Z / Z2D) == one transform pair per target, and the
    numpy restatement, clamped and unclamped, odd sizes included"""
    rng = np.random.default_rng(n * 1000 + H)
    base = smooth_image(H, W, 30)
    imgs = [np.roll(base, (int(rng.integers(-20, 21)), int(rng.integers(-20, 21))), (0, 1))
            + 0.05 * rng.random((H, W)) for _ in range(n)]
    stackd = torch.from_numpy(np.stack(imgs)).cuda()
    for clamp in (15, None):
        got = K.register_translations_batch_dev(stackd, clamp).cpu().tolist()
        want = K.register_translations_dev(stackd[0], list(stackd[1:]), clamp).cpu().tolist()
        assert got == want
        assert tuple(got[0]) == (0, 0)
    for i in range(1, n):
        assert tuple(got[i]) == tuple(int(v) for v in orc.register_translation(imgs[0], imgs[i]))


def test_pad_edge_3d(K):
    rng = np.random.default_rng(2)
    a = rng.random((7, 5, 9))
    for w in (0, 1, 5):
        got = K.pad_edge_3d(torch.from_numpy(a).cuda(), w).cpu().numpy()
        assert np.array_equal(got, np.pad(a, w, mode="edge"))


@pytest.mark.parametrize("mask", [True, False])
def test_assembly_with_image_cn(K, mask):
    """register_assemble(cn_mode=...) writes the registered stack and, from the same pass, its
    channel sum in numpy's order: bit-equal to channel_sum on the written stack; the native
    E. coli chain from that image_cn equals the chain from the stack"""
    from hiprfish_image_analysis_amd import pipeline as P
    from hiprfish_image_analysis_amd import synthetic as S
    st, _, _, _ = S.tile(320, 352, seed=77)
    lasers = S.laser_split(st)
    sh = P.estimate_shifts(lasers, device=True)
    plain = K.register_assemble(lasers, sh, apply_mask=mask)
    for mode in (0, 1, 2):
        stack, cn = K.register_assemble(lasers, sh, apply_mask=mask, cn_mode=mode)
        assert torch.equal(stack, plain)
        assert torch.equal(cn, K.channel_sum(plain, mode=mode))
    stack, cn = P.register_stack(lasers, want_cn=True)
    a = P.segment_ecoli(stack)
    b = P.segment_ecoli(stack, image_cn=cn)
    assert a[1] == b[1] and torch.equal(a[0], b[0])
    # odd channel counts (C < 8 and a ragged tail) through the fused sum
    few = [l[:, :, :3].contiguous() for l in lasers[:2]]
    sh2 = P.estimate_shifts(few, device=True)
    st2, cn2 = K.register_assemble(few, sh2, apply_mask=mask, cn_mode=1)
    assert torch.equal(cn2, K.channel_sum(st2, mode=1))


def test_channel_max_multi_equals_per_laser(K):
    from hiprfish_image_analysis_amd import synthetic as S
    st, _, _, _ = S.tile(200, 264, seed=78)
    lasers = S.laser_split(st)
    lasers[2][5, 7, 3] = float("nan")            # numpy's max propagates NaN
    outs = K.channel_max_multi(lasers)
    for l, o in zip(lasers, outs):
        want = K.channel_max(l)
        assert torch.equal(torch.isnan(o), torch.isnan(want))
        assert torch.equal(torch.nan_to_num(o), torch.nan_to_num(want))
    assert torch.isnan(outs[2][5, 7])
    # the tile path's workgroup budget (hrf_channel_max_multi_grid): the same projections on any grid
    for budget in (512, 7, 1):
        got = K.channel_max_multi(lasers, max_workgroups=budget)
        for o, g in zip(outs, got):
            assert torch.equal(torch.isnan(o), torch.isnan(g)) and torch.equal(torch.nan_to_num(o), torch.nan_to_num(g))
    with pytest.raises(ValueError):
        K.channel_max_multi(lasers, max_workgroups=-1)


def test_concurrent_registrations_equal_serial(K):
    """four tiles registered at once on four streams from four host threads (as bench.py runs
    them): the FFT plans are shared, their work areas come from each call's own workspace, so
    the shifts and assembled stacks equal serial runs"""
    import threading

    from hiprfish_image_analysis_amd import pipeline as P
    from hiprfish_image_analysis_amd import synthetic as S
    shifts = [((0, 0), (2, -1), (0, 3), (-1, 0), (1, 1)), ((0, 0), (-3, 2), (1, -1), (2, 2), (0, -2)),
              ((0, 0), (1, 1), (-2, 0), (0, 4), (3, -3)), ((0, 0), (0, -4), (4, 0), (-1, -1), (2, 0))]
    tiles = [S.laser_split(S.tile(512, 512, seed=90 + i)[0], shifts=shifts[i]) for i in range(4)]
    want = [P.register_stack(t, want_cn=True) for t in tiles]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in tiles]
    got = [None] * 4

    def run(i):
        with torch.cuda.stream(streams[i]):
            for _ in range(3):
                got[i] = P.register_stack(tiles[i], want_cn=True)

    th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    for i in range(4):
        assert torch.equal(got[i][0], want[i][0]) and torch.equal(got[i][1], want[i][1])
        sh = P.estimate_shifts(tiles[i], device=True).cpu().tolist()
        assert [tuple(v) for v in sh] == list(shifts[i])
