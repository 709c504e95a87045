"""conv:K / blur:K against third-party float64 oracles (scipy.ndimage,
torch.nn.functional.conv2d), not only against this repo's own golden path.

CPU: the C++ golden path vs scipy and torch (exact except exact-tie sums).
GPU: the HIP kernels (Toeplitz MFMA conv, separable MFMA blur, VALU small conv)
vs torch fp64 on asymmetric signed weights, K = 9, 31, 33, C = 1 and 3,
reflect101 (torch 'reflect' padding) and constant borders.  A kernel may round
a sum within `GPU_BAND` of k + 1/2 either way (f32 accumulation of up to 1089
terms); every other pixel must be exact.
"""
import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")

GOLDEN_BAND = 1e-9   # f64 vs f64 in a different summation order
GPU_BAND = 4e-3      # f32 accumulation (|sum| <= ~600 for these weights)


@pytest.fixture(scope="module")
def C():
    from mpi_cuda_imagemanipulation_amd._native import C

    return C


def _img(rng, shape, Cc):
    return rng.integers(0, 256, size=shape + (Cc,) if Cc == 3 else shape, dtype=np.uint8)


def _weights(rng, K):
    w = rng.uniform(-0.5, 1.0, (K, K))
    w[0, -1] = 0.9   # asymmetric on purpose: transposes / mirrors show up
    w /= w.sum()
    return oracle.f32_weights(w)


def _conv_chain(w):
    K = w.shape[0]
    return f"conv:{K}:" + ";".join(repr(float(v)) for v in w.reshape(-1))


@pytest.mark.parametrize("K", [3, 9, 31, 33])
@pytest.mark.parametrize("Cc", [1, 3])
@pytest.mark.parametrize("border", ["reflect101", "constant", "replicate"])
def test_golden_conv_vs_scipy_and_torch(C, rng, K, Cc, border):
    img = _img(rng, (41, 67), Cc)
    w = _weights(rng, K)
    got = C.golden_apply(img, _conv_chain(w), border, True)
    for sums in (oracle.scipy_sums(img, w, border), oracle.torch_sums(img, w, border)):
        r = oracle.compare(got, sums, GOLDEN_BAND)
        assert r["mismatch_outside_ties"] == 0 and r["max_diff"] <= 1, r


@pytest.mark.parametrize("K", [3, 15, 31])
@pytest.mark.parametrize("border", ["reflect101", "constant"])
def test_golden_blur_vs_torch(C, rng, K, border):
    img = _img(rng, (37, 53), 3)
    got = C.golden_apply(img, f"blur:{K}", border, True)
    r = oracle.compare(got, oracle.torch_sums(img, oracle.blur_weights(C, K), border), GOLDEN_BAND)
    assert r["mismatch_outside_ties"] == 0 and r["max_diff"] <= 1, r


def test_oracles_agree(rng):
    # the two third-party oracles agree with each other to f64 rounding
    img = _img(rng, (20, 31), 3)
    w = oracle.f32_weights(rng.uniform(-1, 1, (7, 7)))
    for border in ("reflect101", "constant", "replicate"):
        a = oracle.scipy_sums(img, w, border)
        b = oracle.torch_sums(img, w, border)
        assert np.abs(a - b).max() < 1e-9


def test_reflect101_pad_small_frames(rng):
    # frames shorter than the radius: torch's reflect pad cannot, the oracle's
    # periodic index map can; checked against scipy's 'mirror'
    img = _img(rng, (3, 5), 1)
    w = oracle.f32_weights(rng.uniform(-1, 1, (9, 9)))
    assert np.abs(oracle.scipy_sums(img, w, "reflect101") - oracle.torch_sums(img, w, "reflect101")).max() < 1e-9


# ---------------------------------------------------------------- GPU kernels
def _gpu(m, img, chain, border):
    x = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    y = m.ops.apply(x, chain, border)
    torch.cuda.synchronize()
    return y.cpu().numpy()


@pytest.fixture(scope="module")
def m():
    import mpi_cuda_imagemanipulation_amd as m

    assert torch.cuda.is_available()
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("K", [5, 9, 31, 33])
@pytest.mark.parametrize("Cc", [1, 3])
@pytest.mark.parametrize("border", ["reflect101", "constant"])
def test_gpu_conv_vs_torch(m, rng, K, Cc, border):
    img = _img(rng, (150, 333), Cc)
    w = _weights(rng, K)
    got = _gpu(m, img, _conv_chain(w), border)
    sums = oracle.torch_sums(img, w, border, device="cuda")
    r = oracle.compare(got, sums, GPU_BAND)
    assert r["mismatch_outside_ties"] == 0 and r["max_diff"] <= 1, r
    # measured on MI355X: the hi+lo split kernels round like f64 except a few
    # ties; bound the rate well below the round-2 0.5-1 % allowances
    assert r["mismatch"] <= max(2, r["n"] // 2000), r


@pytest.mark.gpu
@pytest.mark.parametrize("K", [9, 31, 33])
@pytest.mark.parametrize("Cc", [1, 3])
@pytest.mark.parametrize("border", ["reflect101", "constant"])
def test_gpu_blur_vs_torch(m, rng, K, Cc, border):
    img = _img(rng, (130, 1100), Cc)
    got = _gpu(m, img, f"blur:{K}", border)
    sums = oracle.torch_sums(img, oracle.blur_weights(m._C, K), border, device="cuda")
    r = oracle.compare(got, sums, GPU_BAND)
    assert r["mismatch_outside_ties"] == 0 and r["max_diff"] <= 1, r
    assert r["mismatch"] <= max(2, r["n"] // 2000), r


# ------------------------------------------------------------------ lsb mode
# conv:K:w..:lsb: 16-bit weight digits on the i8 MFMA path (2/3 of the MFMAs);
# every output within 1 LSB of the correctly rounded f64 result (the host
# checks the quantisation bound per weight set and falls back to 24-bit
# digits when it cannot promise that).
def test_conv_lsb_spec(C, rng):
    w = _weights(rng, 9)
    info = C.plan_info(_conv_chain(w) + ":lsb", 3)
    assert info["passes"][0]["desc"].endswith("lsb")
    assert "lsb" not in C.plan_info(_conv_chain(w) + ":exact", 3)["passes"][0]["desc"]
    with pytest.raises(Exception):
        C.plan_info(_conv_chain(w) + ":fast", 3)
    img = _img(rng, (23, 31), 3)
    # the golden path is exact whatever the requested precision
    assert (C.golden_apply(img, _conv_chain(w) + ":lsb", "reflect101", True) ==
            C.golden_apply(img, _conv_chain(w), "reflect101", True)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("K", [9, 31, 33])
@pytest.mark.parametrize("Cc", [1, 3])
def test_gpu_conv_lsb_vs_torch(m, rng, K, Cc):
    img = _img(rng, (150, 333), Cc)
    w = _weights(rng, K)
    got = _gpu(m, img, _conv_chain(w) + ":lsb", "reflect101")
    sums = oracle.torch_sums(img, w, "reflect101", device="cuda")
    r = oracle.compare(got, sums, GPU_BAND)
    print(f"conv:{K} lsb C={Cc}: {r['mismatch']} of {r['n']} outputs off by one")
    assert r["max_diff"] <= 1, r
    assert r["mismatch"] <= r["n"] // 50, r  # measured rate recorded in profiles/r3/conv/


@pytest.mark.gpu
@pytest.mark.parametrize("lsb", [False, True])
@pytest.mark.parametrize("Cc", [1, 3])
def test_gpu_conv33_uniform_box_saturated(m, rng, lsb, Cc):
    # K = 33 goes to the i8 digit kernel, where a top-digit sum over a uniform
    # box on saturated pixels reaches 1089 * 128 * 127 > 2^24: the
    # epilogue converts each sum in two exact parts, so the result stays the
    # correctly rounded one
    K = 33
    w = oracle.f32_weights(np.full((K, K), 1.0 / (K * K)))
    img = np.where(rng.random((120, 260)) < 0.5, 0, 255).astype(np.uint8)
    img[:, :130] = 0
    img[:60, 130:] = 255
    if Cc == 3:
        img = np.stack([img, 255 - img, img], axis=-1)
    chain = _conv_chain(w) + (":lsb" if lsb else "")
    got = _gpu(m, img, chain, "reflect101")
    r = oracle.compare(got, oracle.torch_sums(img, w, "reflect101", device="cuda"), GPU_BAND)
    assert r["max_diff"] <= 1, r
    if not lsb:
        assert r["mismatch_outside_ties"] == 0, r


@pytest.mark.gpu
def test_gpu_conv_lsb_falls_back_when_unsafe(m, rng):
    # one dominant tap: 16-bit digits of the small ones could miss by >= 0.45
    # LSB, so the pass runs on 24-bit digits and stays exact except ties
    K = 31
    w = rng.uniform(-1, 1, (K, K)) * 1e-3
    w[15, 15] = 1.5
    w = oracle.f32_weights(w)
    img = _img(rng, (90, 200), 3)
    got = _gpu(m, img, _conv_chain(w) + ":lsb", "reflect101")
    r = oracle.compare(got, oracle.torch_sums(img, w, "reflect101", device="cuda"), GPU_BAND)
    assert r["mismatch_outside_ties"] == 0 and r["mismatch"] <= max(2, r["n"] // 2000), r


# ------------------------------------------------------------- blur lsb mode
# blur:K:lsb / sepconv:..:lsb: the separable MFMA kernel on the centred input
# (x - 128, exact in f16) with single f16 weights and a single f16 X, the
# shift added back exactly: 8 MFMAs per tile instead of 20.  Every output
# within 1 LSB of the f64 result; the host bounds the error per weight set and
# keeps the hi + lo kernel above 0.45 LSB.
def test_blur_lsb_spec(C, rng):
    assert C.plan_info("blur:31:lsb", 3)["passes"][0]["desc"].endswith("lsb")
    assert C.plan_info("blur:31:4.5:lsb", 1)["passes"][0]["desc"].endswith("lsb")
    assert "lsb" not in C.plan_info("blur:31:exact", 3)["passes"][0]["desc"]
    assert "lsb" not in C.plan_info("blur:31", 3)["passes"][0]["desc"]
    h = ";".join(["0.2"] * 5)
    assert C.plan_info(f"sepconv:5:{h}:{h}:lsb", 3)["passes"][0]["desc"].endswith("lsb")
    with pytest.raises(Exception):
        C.plan_info("blur:31:4.5:lsb:exact", 3)
    img = _img(rng, (23, 40), 3)
    assert (C.golden_apply(img, "blur:15:lsb", "reflect101", True) ==
            C.golden_apply(img, "blur:15", "reflect101", True)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("K", [9, 31, 33])
@pytest.mark.parametrize("Cc", [1, 3])
@pytest.mark.parametrize("W", [1100, 1101])
def test_gpu_blur_lsb_vs_torch(m, rng, K, Cc, W):
    img = _img(rng, (130, W), Cc)
    got = _gpu(m, img, f"blur:{K}:lsb", "reflect101")
    sums = oracle.torch_sums(img, oracle.blur_weights(m._C, K), "reflect101", device="cuda")
    r = oracle.compare(got, sums, GPU_BAND)
    print(f"blur:{K} lsb C={Cc} W={W}: {r['mismatch']} of {r['n']} outputs off by one")
    assert r["max_diff"] <= 1, r
    # numpy model of the mode (31x31, random pixels): 0.09 % off by one
    assert r["mismatch"] <= r["n"] // 200, r


@pytest.mark.gpu
def test_gpu_sepconv_lsb_falls_back_when_unsafe(m, rng):
    # horizontal taps summing to ~20 (X of the centred input up to ~2600,
    # where an f16 step is 2), vertical taps summing to 1: the single-part mode
    # could miss by > 1 LSB, so the pass keeps the hi + lo kernel
    K = 9
    h = rng.uniform(1.5, 3.0, K).astype(np.float32)
    v = rng.uniform(0.5, 1.0, K)
    v = (v / v.sum()).astype(np.float32)
    chain = f"sepconv:{K}:" + ";".join(repr(float(x)) for x in h) + ":" + ";".join(repr(float(x)) for x in v)
    img = (_img(rng, (90, 300), 3) % 12).astype(np.uint8)  # outputs ~20 * 6, unsaturated
    w = np.outer(v.astype(np.float64), h.astype(np.float64)).astype(np.float32)
    sums = oracle.torch_sums(img, w, "reflect101", device="cuda")
    r = oracle.compare(_gpu(m, img, chain + ":lsb", "reflect101"), sums, GPU_BAND)
    assert r["mismatch_outside_ties"] == 0 and r["mismatch"] <= max(2, r["n"] // 2000), r
