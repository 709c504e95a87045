"""CPU golden path vs the independent numpy mirror (exact u8 equality)."""
import numpy as np
import pytest

import np_ref
from mpi_cuda_imagemanipulation_amd import ops

SHAPES = [(1, 1), (2, 3), (5, 4), (17, 15), (33, 64)]


def img3(rng, h, w):
    return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def img1(rng, h, w):
    return rng.integers(0, 256, size=(h, w), dtype=np.uint8)


def test_gray_modes_all_values(C):
    # exhaustively over one channel at a time (the terms are separable)
    v = np.arange(256, dtype=np.uint8)
    z = np.zeros_like(v)
    for ch in range(3):
        rgb = np.stack([v if c == ch else z for c in range(3)], -1)[None]
        assert (ops.apply(rgb, "gray:ref") == np_ref.gray_ref(rgb)).all()
        assert (ops.apply(rgb, "gray:bt601") == np_ref.gray_bt601(rgb)).all()


def test_gray_random(rng):
    x = img3(rng, 31, 29)
    assert (ops.apply(x, "gray:ref") == np_ref.gray_ref(x)).all()
    assert (ops.apply(x, "gray") == np_ref.gray_bt601(x)).all()
    assert np_ref.gray_ref(x).max() <= 254


def test_reference_gray_weights_by_semantic_channel():
    # kernel.cu:40-42 weights B*.11 G*.59 R*.3 (BGR memory); PPM is RGB: R is first
    px = np.array([[[200, 0, 0]]], np.uint8)
    assert ops.apply(px, "gray:ref")[0, 0] == int(200 * 0.3)


@pytest.mark.parametrize("f", [3.5, 1.0, 0.5, 2.25, -1.0])
def test_contrast_ref(f):
    v = np.arange(256, dtype=np.uint8).reshape(16, 16)
    assert (ops.apply(v, f"contrast:{f}") == np_ref.contrast_ref(v, f)).all()


def test_contrast_ref_known_points():
    v = np.arange(256, dtype=np.uint8).reshape(1, 256)
    out = ops.apply(v, "contrast:3.5")[0]
    assert (out[:92] == 0).all() and (out[165:] == 255).all()


@pytest.mark.parametrize("f", [3.0, 1.5, 0.7])
def test_contrast_cv(f):
    v = np.arange(256, dtype=np.uint8).reshape(16, 16)
    assert (ops.apply(v, f"contrast:{f}:cv") == np_ref.contrast_cv(v, f)).all()


def test_contrast_ref_vs_cv_differ_on_83_inputs():
    v = np.arange(256, dtype=np.uint8).reshape(1, 256)
    a = ops.apply(v, "contrast:3.5")
    b = ops.apply(v, "contrast:3:cv")
    assert int((a != b).sum()) == 83


def test_invert_brightness_threshold(rng):
    x = img3(rng, 9, 11)
    assert (ops.apply(x, "invert") == np_ref.invert(x)).all()
    for d in (-300, -40, 0, 77, 300):
        assert (ops.apply(x, f"brightness:{d}") == np_ref.brightness(x, d)).all()
    assert (ops.apply(x, "threshold:100") == np.where(x >= 100, 255, 0)).all()


@pytest.mark.parametrize("name", sorted(np_ref.STENCILS) + ["sobel", "sobel_l2"])
@pytest.mark.parametrize("border", ["reflect101", "replicate", "constant", "skip"])
@pytest.mark.parametrize("shape", SHAPES)
def test_stencils(rng, name, border, shape):
    h, w = shape
    R = 1 if name.startswith("sobel") else np_ref.STENCILS[name][0].shape[0] // 2
    if border == "reflect101" and (h < 2 or w < 2):
        pytest.skip("numpy reflect needs >= 2 samples")
    if border == "reflect101" and (h <= R or w <= R):
        pytest.skip("numpy reflect does not repeat; golden reflects repeatedly")
    for x in (img1(rng, h, w), img3(rng, h, w)):
        got = ops.apply(x, f"{name}@{border}")
        ref = np_ref.stencil(x, name, border)
        assert got.shape == ref.shape
        assert (got == ref).all(), f"{name} {border} {x.shape}"


def test_reflect101_tiny_images_repeat(C):
    # golden reflects repeatedly (OpenCV borderInterpolate); check the index map
    assert [C.border_index(i, 3, C.Border.reflect101) for i in range(-5, 8)] == [1, 0, 1, 2, 1, 0, 1, 2, 1, 0, 1, 2, 1]
    assert C.border_index(-1, 1, C.Border.reflect101) == 0
    assert C.border_index(-3, 4, C.Border.replicate) == 0
    assert C.border_index(9, 4, C.Border.replicate) == 3
    assert C.border_index(-1, 4, C.Border.constant) == -1


@pytest.mark.parametrize("K", [3, 5, 9])
def test_float_blur(rng, K):
    x = img3(rng, 19, 23)
    got = ops.apply(x, f"blur:{K}")
    ref = np_ref.blur(x, K)
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1
    assert (got == ref).mean() > 0.99


def test_conv_generic_equals_integer_stencil(rng):
    x = img1(rng, 12, 14)
    w = np_ref.STENCILS["gaussian5"][0] / 256.0
    spec = ";".join(str(v) for v in w.reshape(-1))
    got = ops.apply(x, f"conv:5:{spec}")
    ref = np_ref.stencil(x, "gaussian5")
    # float rint (half-even) vs integer (s+128)>>8 (half-up) differ only on exact ties
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1


def test_sepconv_equals_outer_product_conv(rng):
    x = img3(rng, 21, 18)
    h = np.array([0.1, -0.2, 0.5, 0.3, 0.05])
    v = np.array([0.25, 0.5, 0.125, 0.0625, 0.0625])
    got = ops.sep_conv2d(x, h, v)
    ref = ops.conv2d(x, np.outer(v, h).astype(np.float32).astype(np.float64))
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1


@pytest.mark.parametrize("bad", ["sepconv:3:1;2;3", "sepconv:3:1;2:1;2;3", "sepconv:4:1;2;3;4:1;2;3;4"])
def test_sepconv_parse_errors(bad):
    with pytest.raises(Exception):
        C.parse_chain(bad)


def test_reference_chains(rng):
    x = img3(rng, 24, 20)
    g = np_ref.gray_ref(x)
    c = np_ref.contrast_ref(g, 3.5)
    e = np_ref.stencil(c, "emboss3", "skip")
    assert (ops.apply(x, "gray:ref,contrast:3.5,emboss3@skip") == e).all()
    assert (ops.apply(x, "ref-gpu") == e).all()
    g2 = np_ref.gray_bt601(x)
    c2 = np_ref.contrast_cv(g2, 3.0)
    e2 = np_ref.stencil(c2, "emboss3", "reflect101")
    assert (ops.apply(x, "ref-cpu") == e2).all()
    assert (ops.apply(x, "ref-cpu,expand") == np_ref.expand(e2)).all()


@pytest.mark.parametrize("chain", [
    "gray:ref,contrast:3.5,emboss3",
    "invert,gray,brightness:20,gaussian5,invert",
    "brightness:-30,sobel,threshold:90",
    "gray,expand,gaussian3,contrast:1.5,sharpen",
    "gaussian5,gaussian5,emboss5",
    "contrast:2:cv,invert,box3",
    "gray:ref,invert,expand,invert",
])
def test_fusion_is_exact(rng, chain, C):
    x = img3(rng, 21, 26)
    fused = C.golden_apply(x, chain, "reflect101", True)
    unfused = C.golden_apply_unfused(x, chain, "reflect101")
    assert (fused == unfused).all()
