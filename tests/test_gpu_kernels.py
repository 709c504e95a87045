"""HIP kernels vs the golden path, bit-exact (MFMA conv: within 1 LSB)."""
import numpy as np
import pytest

import np_ref

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def m():
    import mpi_cuda_imagemanipulation_amd as m

    assert torch.cuda.is_available()
    return m


def _run(m, img, chain, border="reflect101"):
    x = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    y = m.ops.apply(x, chain, border)
    torch.cuda.synchronize()
    return y.cpu().numpy()


# (5, 2048): gray rows of exactly two 1 KiB sobel tiles (the right edge pixel is the margin)
SHAPES = [(1, 1), (3, 2), (17, 15), (64, 65), (37, 1365), (130, 4100), (9, 5000), (5, 2048)]
STENCILS = ["gaussian3", "gaussian5", "gaussian7", "box3", "box5", "emboss3", "emboss5", "sharpen", "laplace",
            "sobel", "sobel_l2"]


@pytest.mark.parametrize("name", STENCILS)
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("C", [1, 3])
def test_stencil_exact(m, rng, name, shape, C):
    h, w = shape
    img = rng.integers(0, 256, size=(h, w, C) if C == 3 else (h, w), dtype=np.uint8)
    for border in ("reflect101", "replicate", "constant"):
        got = _run(m, img, name, border)
        ref = m._C.golden_apply(img, name, border, True)
        assert got.shape == ref.shape
        bad = np.argwhere(got != ref)
        assert bad.size == 0, f"{name} {border} {img.shape}: {len(bad)} mismatches, first {bad[:5].tolist()}"


@pytest.mark.parametrize("name", STENCILS)
@pytest.mark.parametrize("shape", [(1, 1), (17, 15), (37, 1365), (9, 5000)])
def test_stencil_expand_epilogue(m, rng, name, shape):
    # gray prologue + 1-channel stencil + fused expand epilogue (48-byte stores,
    # 3-channel x-margins) vs the golden path
    img = rng.integers(0, 256, size=shape + (3,), dtype=np.uint8)
    chain = f"gray,{name},expand"
    assert m._C.plan_info(chain, 3)["passes"][0]["epi_expand"]
    for border in ("reflect101", "replicate", "constant"):
        got = _run(m, img, chain, border)
        ref = m._C.golden_apply(img, chain, border, True)
        assert got.shape == ref.shape == shape + (3,)
        bad = np.argwhere(got != ref)
        assert bad.size == 0, f"{chain} {border} {img.shape}: {len(bad)} mismatches, first {bad[:5].tolist()}"


@pytest.mark.parametrize("name", ["emboss3", "emboss5", "gaussian5", "sobel", "sobel_l2"])
def test_skip_border(m, rng, name):
    img = rng.integers(0, 256, size=(45, 77), dtype=np.uint8)
    got = _run(m, img, f"{name}@skip")
    assert (got == np_ref.stencil(img, name, "skip")).all()


@pytest.mark.parametrize("chain", [
    "gray", "gray:ref", "invert", "brightness:-40", "contrast:3.5", "contrast:3:cv", "threshold:77",
    "gray,expand", "gray:ref,contrast:3.5,emboss3", "ref-gpu", "ref-cpu,expand",
    "invert,gray,brightness:20,gaussian5,invert", "gaussian5,gaussian5,sobel", "gray,sobel,threshold:60",
    "brightness:10,gaussian3,contrast:1.5,sharpen,invert", "gaussian5@replicate,gaussian5@constant",
    "gray:ref,contrast:3.5,emboss3@skip,expand", "gray,gaussian5,expand,invert", "gray,sobel_l2,invert,expand",
    "gray:ref,emboss5@skip,expand,gaussian3",
])
@pytest.mark.parametrize("shape", [(33, 47), (128, 1000)])
def test_chains_exact(m, rng, chain, shape):
    img = rng.integers(0, 256, size=shape + (3,), dtype=np.uint8)
    got = _run(m, img, chain)
    ref = m._C.golden_apply(img, chain, "reflect101", True)
    assert got.shape == ref.shape and (got == ref).all(), chain


@pytest.mark.parametrize("K", [3, 5, 9, 15, 25, 31, 33])
@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("shape", [(70, 97), (1, 1), (3, 40), (161, 700), (40, 2100)])
def test_mfma_conv_blur(m, rng, K, C, shape):
    # blur:K takes the separable MFMA path (rank-one window)
    img = rng.integers(0, 256, size=shape + (C,) if C == 3 else shape, dtype=np.uint8)
    for border in ("reflect101", "replicate", "constant"):
        got = _run(m, img, f"blur:{K}", border)
        ref = m._C.golden_apply(img, f"blur:{K}", border, True)
        d = np.abs(got.astype(int) - ref.astype(int))
        # ties only: round 3 measured <= 1 in 2000 (tests/test_oracle_conv.py checks where)
        assert d.max() <= 1 and (d != 0).sum() <= max(2, d.size // 2000), (K, C, shape, border, d.max(), (d != 0).sum())


@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("K", [5, 17, 33])
def test_mfma_sepconv_asymmetric(m, rng, C, K):
    # distinct, asymmetric h and v catch transposed / mirrored fragment maps
    h = rng.uniform(-0.5, 1.0, K)
    v = rng.uniform(-0.25, 1.0, K)
    h /= h.sum()
    v /= v.sum()
    img = rng.integers(0, 256, size=(90, 333, C) if C == 3 else (90, 333), dtype=np.uint8)
    got = m.ops.sep_conv2d(torch.from_numpy(img).cuda(), h, v).cpu().numpy()
    ref = m.ops.sep_conv2d(img, h, v)
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() <= 1 and (d != 0).sum() <= max(2, d.size // 2000), (d.max(), (d != 0).sum())


@pytest.mark.parametrize("scale", [8.0, 16.0])
def test_mfma_sepconv_large_weights(m, rng, scale):
    # the separable kernel stages bytes as f16 subnormals and scales the
    # weights by powers of two (h x 2^k, v x 2^(24-k)): max|h| * max|v| <= 64
    # stays on it (scale 8), larger products run on the general conv kernel
    # (scale 16); both must match the golden path
    K = 5
    h = rng.uniform(0.25, 1.0, K) * scale
    v = rng.uniform(0.25, 1.0, K) * scale
    h[K // 2] = v[K // 2] = scale
    chain = f"sepconv:{K}:" + ";".join(repr(float(x)) for x in h) + ":" + ";".join(repr(float(x)) for x in v)
    img = (rng.integers(0, 256, size=(48, 200, 3), dtype=np.uint8) % 3 == 0).astype(np.uint8)
    got = _run(m, img, chain, "reflect101")
    ref = m._C.golden_apply(img, chain, "reflect101", True)
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() <= 1 and (d != 0).sum() <= max(2, d.size // 2000), (scale, d.max(), (d != 0).sum())


def test_mfma_sep_matches_general_conv(m, rng):
    # the same rank-one window through the separable and the general (Toeplitz) MFMA kernels
    K = 9
    g = np.exp(-np.linspace(-2, 2, K) ** 2)
    g /= g.sum()
    img = rng.integers(0, 256, size=(64, 300, 3), dtype=np.uint8)
    x = torch.from_numpy(img).cuda()
    a = m.ops.sep_conv2d(x, g, g).cpu().numpy()
    b = m.ops.conv2d(x, np.outer(g, g).astype(np.float32).astype(np.float64)).cpu().numpy()
    assert np.abs(a.astype(int) - b.astype(int)).max() <= 1


@pytest.mark.parametrize("K", [7, 9, 15, 31, 33])
@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("shape", [(1, 1), (37, 61), (150, 333), (70, 1100)])
def test_mfma_general_conv(m, rng, K, C, shape):
    # non-separable random weights through the Toeplitz MFMA kernel (paired
    # kernel rows in the K dimension); asymmetric, so a transposed or mirrored
    # fragment map, a wrong row pairing or a wrong channel plane shows up
    w = rng.uniform(-0.5, 1.0, (K, K))
    w /= w.sum()
    img = rng.integers(0, 256, size=shape + (C,) if C == 3 else shape, dtype=np.uint8)
    for border in ("reflect101", "constant"):
        got = m.ops.conv2d(torch.from_numpy(img).cuda(), w, border).cpu().numpy()
        ref = m.ops.conv2d(img, w, border)
        d = np.abs(got.astype(int) - ref.astype(int))
        assert d.max() <= 1 and (d != 0).sum() <= max(2, d.size // 2000), (K, C, shape, border, d.max(), (d != 0).sum())


def test_mfma_conv_asymmetric_weights(m, rng):
    # asymmetric kernel catches transposed fragment layouts
    K = 5
    w = np.arange(K * K, dtype=np.float64).reshape(K, K) / 300.0
    img = rng.integers(0, 256, size=(40, 50), dtype=np.uint8)
    got = m.ops.conv2d(torch.from_numpy(img).cuda(), w).cpu().numpy()
    ref = m.ops.conv2d(img, w)
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1


def test_determinism(m, rng):
    img = rng.integers(0, 256, size=(300, 700, 3), dtype=np.uint8)
    a = _run(m, img, "gray:ref,contrast:3.5,emboss3")
    b = _run(m, img, "gray:ref,contrast:3.5,emboss3")
    assert (a == b).all()


def test_large_frame_gaussian5(m):
    img = m.utils.synthetic_image(5, 4096, 512, 3)
    got = _run(m, img, "gaussian5")
    ref = m._C.golden_apply(img, "gaussian5", "reflect101", True)
    assert (got == ref).all()


def test_batched_frames(m, rng):
    # BxHxWxC runs frame by frame through one cached engine; equals per-frame results
    imgs = rng.integers(0, 256, size=(4, 37, 91, 3), dtype=np.uint8)
    x = torch.from_numpy(imgs).cuda()
    for chain in ("gaussian5", "gray:ref,contrast:3.5,emboss3"):
        got = m.ops.apply(x, chain).cpu().numpy()
        for b in range(4):
            assert (got[b] == m._C.golden_apply(imgs[b], chain, "reflect101", True)).all(), (chain, b)

