"""a4 non-local means (skimage.restoration.denoise_nl_means, multispecies measurement.py:108)
on the device against the oracle restatement in the kernel's summation order and arithmetic
(same exp polynomial: bit-identical), and against the integral-image algorithm itself (rtol
1e-9).  skimage is not installed here: parity against
skimage proper is unpinned."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from hiprfish_image_analysis_amd import kernels
    return kernels


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def smooth(shape, seed, noise=0.01):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:shape[0], 0:shape[1]]
    return 0.5 + 0.3 * np.sin(yy / 6.0) * np.cos(xx / 5.0) + noise * rng.standard_normal(shape)


@pytest.mark.parametrize("shape", [(1, 1), (1, 9), (7, 5), (64, 64), (70, 130), (131, 67)])
def test_nl_means_vs_oracle(K, orc, shape):
    img = smooth(shape, sum(shape))
    got = K.nl_means_2d(dev(img), h=0.02).cpu().numpy()
    ref = orc.nl_means(img, 7, 11, 0.02)
    assert np.array_equal(got, ref)


def test_nl_means_random_and_sigma(K, orc):
    rng = np.random.default_rng(4)
    img = rng.random((45, 77))
    for h, sigma in [(0.1, 0.0), (0.3, 0.05)]:
        got = K.nl_means_2d(dev(img), h=h, sigma=sigma).cpu().numpy()
        assert np.array_equal(got, orc.nl_means(img, 7, 11, h, sigma))


def test_nl_means_vs_integral_image_algorithm(K, orc):
    img = smooth((48, 52), 9)
    got = K.nl_means_2d(dev(img), h=0.02).cpu().numpy()
    np.testing.assert_allclose(got, orc.nl_means_skimage(img, 7, 11, 0.02), rtol=1e-9, atol=0)


def test_nl_means_tile_sized(K, orc):
    """a synthetic-community sum image at 512^2: GPU vs oracle on a strip of rows"""
    from hiprfish_image_analysis_amd import synthetic as S
    stack, truth, lay, ref = S.tile(512, 512, nbit=7, bounds=S.MULTI_BOUNDS, seed=3)
    s = stack.double().sum(dim=2)
    s = (s / s.max()).cpu().numpy()
    got = K.nl_means_2d(dev(s), h=0.02).cpu().numpy()
    sub = orc.nl_means(s[200:260], 7, 11, 0.02)          # rows 200..259 with their own reflect
    assert np.array_equal(got[214:246], sub[14:46])


def test_nl_means_bad_parameters(K):
    with pytest.raises(ValueError):
        K.nl_means_2d(torch.zeros((8, 8), dtype=torch.float64, device="cuda"), patch_size=5)
    with pytest.raises(ValueError):
        K.nl_means_2d(torch.zeros((8, 8), dtype=torch.float32, device="cuda"))
