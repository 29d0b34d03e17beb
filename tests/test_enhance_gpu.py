"""Parity of the line-profile enhancement kernels (a5-a7) against the reference-derived
golden fixtures and the oracle.  Bit-exact (f64)."""
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


def same(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape
    assert np.array_equal(np.isnan(a), np.isnan(b))
    m = ~np.isnan(a)
    assert np.array_equal(a[m], b[m]), np.max(np.abs(a[m] - b[m]))


@pytest.mark.parametrize("case", ["a", "d"])
def test_line_profile_2d_golden(K, golden, case):
    g = golden("neighbor2d")
    same(K.line_profile_2d(dev(g["pad_" + case])).cpu().numpy(), g["lp_" + case])


@pytest.mark.parametrize("case", ["a", "b", "c", "d"])
def test_enhance_2d_golden(K, golden, case):
    g = golden("neighbor2d")
    same(K.enhance_2d(dev(g["pad_" + case])).cpu().numpy(), g["final_" + case])


@pytest.mark.parametrize("shape", [(1, 1), (63, 65), (130, 77), (257, 300)])
def test_enhance_2d_vs_oracle(K, orc, shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.random(shape) ** 2
    pad = np.pad(img, 5, mode="edge")
    same(K.enhance_2d(dev(pad)).cpu().numpy(), orc.enhance_2d(pad))


def test_enhance_2d_nonfinite_inputs(K, orc):
    rng = np.random.default_rng(3)
    pad = np.pad(rng.random((40, 50)), 5, mode="edge")
    pad[10, 10] = np.nan
    pad[20, 30] = np.inf
    pad[25:30, 5:9] = 0.5  # flat patch
    same(K.enhance_2d(dev(pad)).cpu().numpy(), orc.enhance_2d(pad))


def test_line_profile_2d_other_params(K, orc):
    rng = np.random.default_rng(5)
    pad = rng.random((30, 41))
    for patch, nphi in [(7, 5), (11, 12)]:
        same(K.line_profile_2d(dev(pad), patch, nphi).cpu().numpy(), orc.line_profile_2d(pad, patch, nphi))


def test_line_profile_3d_golden(K, golden):
    g = golden("neighbor3d")
    same(K.line_profile_3d(dev(g["pad_small"])).cpu().numpy(), g["lp_small"])
    same(K.line_profile_3d_norm(dev(g["pad"])).cpu().numpy(), g["lp_norm"])


def test_enhance_3d_golden(K, golden):
    g = golden("neighbor3d")
    same(K.enhance_3d(dev(g["pad"])).cpu().numpy(), g["final"])


@pytest.mark.parametrize("shape", [(5, 9, 37), (12, 10, 64), (9, 17, 70)])
def test_enhance_3d_vs_oracle(K, orc, shape):
    rng = np.random.default_rng(sum(shape))
    vol = rng.random(shape)
    pad = np.pad(vol, 5, mode="edge")
    same(K.enhance_3d(dev(pad)).cpu().numpy(), orc.enhance_3d(pad))
    same(K.line_profile_3d_norm(dev(pad)).cpu().numpy(), orc.line_profile_3d_norm(pad))


def test_enhance_3d_special_values(K, orc):
    """tiles with NaN, infinities, negative zeros and finite values whose window ranges overflow
    (max - min > DBL_MAX: inf / inf = NaN taps) take the reference's compare-select arithmetic;
    equal to the restatement, NaNs in place"""
    rng = np.random.default_rng(21)
    pad = rng.random((24, 22, 50))
    pad[3, 4, 5] = np.nan
    pad[12, 7, 40] = np.inf
    pad[14, 15, 20] = -np.inf
    pad[2:6, 2:6, 30:34] = -0.0
    pad[18, 17, 8] = 1.5e308                # finite, span with the next value > DBL_MAX
    pad[18, 18, 8] = -1.5e308
    pad[20, 3, 45] = 1e308                  # finite, span within DBL_MAX but above 2^1023
    pad[6, 20, 12] = 2.0 ** 1023            # exactly +-2^1023 side by side: span 2^1024 = inf
    pad[6, 20, 13] = -(2.0 ** 1023)
    same(K.enhance_3d(dev(pad)).cpu().numpy(), orc.enhance_3d(pad))


def test_enhance_3d_flat_volume(K, orc):
    pad = np.full((13, 12, 14), 0.3)
    same(K.enhance_3d(dev(pad)).cpu().numpy(), orc.enhance_3d(pad))


@pytest.mark.parametrize("case", ["a", "b", "c"])
def test_memory_efficient_v3(K, orc, golden, case):
    g = golden("neighbor3d_v3")
    pad = g["pad_" + case]
    got = K.enhance_3d_v3(dev(pad)).cpu().numpy()
    same(got, orc.enhance_3d_v3(pad))                  # everywhere, incl. the flat-address tail
    ok = orc.v3_defined(pad.shape)
    same(got[ok], g["final_" + case][ok])              # the reference itself where defined


def test_memory_efficient_v3_dropin(K, orc):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "hiprfish_image_analysis_amd", "scripts"))
    import neighbor
    pad = np.random.default_rng(3).random((22, 13, 17))
    same(neighbor.line_profile_memory_efficient_v3(pad, 11, 9, 9), orc.enhance_3d_v3(pad))
    with pytest.raises(ValueError):
        neighbor.line_profile_memory_efficient_v3(pad.astype(np.float32), 11, 9, 9)


def test_empty_and_too_small(K):
    pad = torch.zeros((10, 12), dtype=torch.float64, device="cuda")
    assert K.enhance_2d(pad).shape == (0, 2)
    with pytest.raises(ValueError):
        K.enhance_2d(torch.zeros((9, 12), dtype=torch.float64, device="cuda"))
    with pytest.raises(ValueError):
        K.enhance_2d(torch.zeros((20, 20), dtype=torch.float32, device="cuda"))


def test_enhance_volume_chain(K, orc):
    """biofilm :808-817 from the (X, Y, Z, C) volume: channel sum / max / edge pad / fused
    line-profile enhancement, against numpy's sum, max and pad plus the restated enhancement"""
    from hiprfish_image_analysis_amd import pipeline as P
    rng = np.random.default_rng(12)
    vol = rng.random((14, 12, 9, 63)).astype(np.float32)
    vol[:, :, :, :10] *= rng.random((14, 12, 9, 1)).astype(np.float32)
    s = np.sum(vol.astype(np.float64), axis=3)       # the stack as f64 (bioformats hands over f64)
    pad = np.pad(s / np.max(s), 5, mode="edge")
    same(P.enhance_volume(dev(vol)).cpu().numpy(), orc.enhance_3d(pad))
    same(P.enhance_volume(dev(vol), v3=True).cpu().numpy(), orc.enhance_3d_v3(pad))
