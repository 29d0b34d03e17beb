"""Registration shifts through the hand-written f64 FFT pipeline (xcorr.hip, row f1): the
correlation surfaces against numpy's FFT (ecoli measurement.py:45-57 via
skimage.feature.register_translation; numpy is the reference's own FFT), the shifts against the
numpy restatement (oracle.register_translation) on random, correlated and known-shift images, and
against the hipFFT path on the bench's 2048 x 2048 laser projections."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from hiprfish_image_analysis_amd import kernels
    return kernels


def smooth(H, W, rng):
    x = rng.random((H, W))
    for _ in range(3):
        x = (x + np.roll(x, 1, 0) + np.roll(x, -1, 0) + np.roll(x, 1, 1) + np.roll(x, -1, 1)) / 5
    return x


@pytest.mark.parametrize("n,H,W", [(2, 16, 4), (3, 16, 16), (5, 64, 32), (4, 32, 128), (5, 128, 256), (2, 256, 64),
                                   (5, 512, 512), (3, 1024, 2048), (2, 4096, 64)])
def test_surfaces_equal_numpy(K, n, H, W):
    rng = np.random.default_rng(H * 7 + W + n)
    imgs = rng.random((n, H, W))
    imgs[1:] += 0.5 * imgs[:1]
    got = K.xcorr_surfaces(torch.from_numpy(imgs).cuda()).cpu().numpy()
    F = np.fft.fft2(imgs)
    for t in range(1, n):
        want = np.fft.ifft2(F[0] * F[t].conj()).real * (H * W // 2)
        scale = np.abs(want).max()
        np.testing.assert_allclose(got[t - 1], want, rtol=0, atol=scale * 1e-13)


@pytest.mark.parametrize("H,W", [(16, 16), (64, 128), (256, 256), (2048, 2048)])
def test_shifts_known_and_clamped(K, orc, H, W):
    rng = np.random.default_rng(H + W)
    ref = smooth(H, W, rng)
    sh = [(0, 0), (3, -5), (-7, 2), (min(H // 2, 40) - 1, -(min(W // 2, 40) - 1)), (0, 1)]
    imgs = np.stack([np.roll(ref, (-dr, -dc), axis=(0, 1)) for dr, dc in sh])
    got = K.xcorr_shifts_dev(torch.from_numpy(imgs).cuda()).cpu().numpy()
    assert [tuple(r) for r in got] == sh
    for t in range(1, len(sh)):
        assert tuple(int(v) for v in orc.register_translation(imgs[0], imgs[t])) == sh[t]
    cl = K.xcorr_shifts_dev(torch.from_numpy(imgs).cuda(), clamp=15).cpu().numpy()
    want = [(0 if abs(a) > 15 else a, 0 if abs(b) > 15 else b) for a, b in sh]
    assert [tuple(r) for r in cl] == want


@pytest.mark.parametrize("seed", range(6))
def test_shifts_random_match_restatement(K, orc, seed):
    rng = np.random.default_rng(100 + seed)
    H, W = 2 ** int(rng.integers(4, 10)), 2 ** int(rng.integers(3, 10))
    n = int(rng.integers(2, 7))
    imgs = rng.random((n, H, W))
    imgs[1:, : H // 2] += 0.3 * imgs[:1, : H // 2]
    got = K.xcorr_shifts_dev(torch.from_numpy(imgs).cuda()).cpu().numpy()
    for t in range(1, n):
        assert tuple(got[t]) == tuple(int(v) for v in orc.register_translation(imgs[0], imgs[t]))


def test_bench_projections_equal_hipfft_path(K):
    """the bench's five laser acquisitions: max projections -> shifts through both pipelines"""
    from hiprfish_image_analysis_amd import synthetic as S
    stack, _, _, _ = S.tile(2048, 2048, seed=20190101)
    lasers = S.laser_split(stack)
    proj = K.channel_max_multi(lasers, stacked=True)
    a = K.xcorr_shifts_dev(proj, clamp=15).cpu().numpy()
    b = K.register_translations_dev(proj[0], list(proj[1:]), clamp=15).cpu().numpy()
    assert np.array_equal(a, b)
    assert [tuple(r) for r in a] == [(0, 0)] + [tuple(s) for s in S.LASER_SHIFTS[1:]]
