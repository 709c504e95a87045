"""Chain parser / compiler (fusion, halo and margin contracts)."""
import pytest

from mpi_cuda_imagemanipulation_amd import models


def test_parse_canonical(C):
    assert C.parse_chain("grayscale, contrast:3.5 ,emboss") == "gray:bt601,contrast:3.5,emboss3"
    assert C.parse_chain("ref-gpu") == "gray:ref,contrast:3.5,emboss3@skip"
    assert C.parse_chain("ref-cpu") == "gray:bt601,contrast:3:cv,emboss3"
    assert C.parse_chain("gaussian5@replicate") == "gaussian5@replicate"


@pytest.mark.parametrize("bad", ["", "blurp", "brightness", "gray:xyz", "contrast:abc", "conv:3:1;2",
                                 "blur:4", "gaussian5@nowhere", "gray,expand,expand", "a,,b"])
def test_parse_errors(C, bad):
    with pytest.raises(RuntimeError):
        C.plan_info(bad, 3)


def test_reference_chain_is_one_pass(C):
    info = C.plan_info("gray:ref,contrast:3.5,emboss3", 3)
    assert len(info["passes"]) == 1
    p = info["passes"][0]
    assert p["cin"] == 3 and p["cout"] == 1 and p["R"] == 1
    assert "prologue[gray:ref,lut]" in p["desc"]


def test_epilogue_and_pointwise_passes(C):
    info = C.plan_info("gaussian5,invert", 3)
    assert len(info["passes"]) == 1 and "epilogue[lut]" in info["passes"][0]["desc"]
    info = C.plan_info("invert,brightness:3", 3)
    assert len(info["passes"]) == 1 and info["passes"][0]["kind"] == 0
    info = C.plan_info("gaussian5,gray,sobel", 3)
    assert [p["kind"] for p in info["passes"]] == [1, 1]  # sobel runs as a separable pair
    assert "separable sobel" in info["passes"][1]["desc"]
    assert info["passes"][0]["out_margin_px"] == 0 or info["passes"][0]["out_margin_px"] == 1
    info = C.plan_info("gaussian5,expand", 1)
    assert [p["kind"] for p in info["passes"]] == [1] and info["passes"][0]["epi_expand"]
    info = C.plan_info("blur:31", 3)
    assert info["passes"][0]["kind"] == 3 and info["max_radius"] == 15


def test_expand_epilogue(C):
    # the reference's whole GPU chain (gray -> contrast -> emboss -> expand back
    # to RGB, kernel.cu:192-196) is one pass: gray prologue, expand epilogue
    info = C.plan_info("gray:ref,contrast:3.5,emboss3@skip,expand", 3)
    assert len(info["passes"]) == 1
    p = info["passes"][0]
    assert p["cin"] == 3 and p["cmid"] == 1 and p["cout"] == 3 and p["epi_expand"] and not p["epi_lut"]
    # 3 -> 3: iterable, so the fused pass keeps its own input's margin contract
    assert info["in_margin_px"] == 1 and p["out_margin_px"] == 1
    # a LUT on either side of the expand rides along (channels are copies)
    for chain in ("gray,gaussian5,expand,invert", "gray,gaussian5,invert,expand"):
        p = C.plan_info(chain, 3)["passes"]
        assert len(p) == 1 and p[0]["epi_expand"] and p[0]["epi_lut"], chain
    # a 3-channel stencil cannot expand; conv passes take no pointwise work
    assert [p["kind"] for p in C.plan_info("gray,blur:9,expand", 3)["passes"]] == [0, 3, 0]
    assert [p["kind"] for p in C.plan_info("gaussian5,gray,expand", 3)["passes"]] == [1, 0]
    assert len(C.plan_info("gray,gaussian5,expand", 3, "reflect101", False)["passes"]) == 3


def test_expand_epilogue_golden_matches_unfused(C, rng):
    import numpy as np

    img = rng.integers(0, 256, size=(23, 41, 3), dtype=np.uint8)
    for chain in ("gray:ref,contrast:3.5,emboss3@skip,expand", "gray,sobel,invert,expand",
                  "gray,gaussian5,expand,brightness:30"):
        a = C.golden_apply(img, chain, "reflect101", True)
        b = C.golden_apply(img, chain, "reflect101", False)
        assert a.shape == (23, 41, 3) and (a == b).all(), chain


def test_margin_contracts(C):
    info = C.plan_info("gaussian5,invert,sobel,gaussian7", 3)
    r = [p["R"] for p in info["passes"]]
    m = [p["out_margin_px"] for p in info["passes"]]
    assert info["in_margin_px"] == r[0]
    assert m[-1] == r[0] and m[0] == r[1]  # cyclic: iterating feeds pass 0 again
    info = C.plan_info("gray,gaussian5", 3)
    assert info["passes"][-1]["out_margin_px"] == 0  # 3 -> 1 channels cannot iterate


def test_unfused_plan(C):
    info = C.plan_info("gray:ref,contrast:3.5,emboss3", 3, "reflect101", False)
    assert len(info["passes"]) == 3


def test_presets_exist():
    for name in ["ref-gpu", "ref-cpu", "config1-gray", "config4-gauss5", "config5-blur31"]:
        p = models.Pipeline.preset(name)
        assert p.plan()
    with pytest.raises(KeyError):
        models.Pipeline.preset("nope")


# ---- affine post maps: a gray:ref prologue's post LUT as clamp((a v + b) >> k)
import re as _re

import numpy as np

_AFF = _re.compile(r"post=clamp\(\((-?\d+)v\+?(-?\d+)\)>>(\d+)\)")


@pytest.mark.parametrize("pw,affine", [("contrast:3.5", True), ("contrast:3", True), ("contrast:3:cv", True),
                                       ("contrast:0.25", True), ("brightness:40", True), ("brightness:-17", True),
                                       ("invert", True), ("contrast:0.25,invert", True), ("contrast:1.7", False),
                                       ("threshold:100", False),
                                       ("contrast:3.5,brightness:-30", False)])  # saturates at 225: not one clamp
def test_post_lut_affine_exact(C, pw, affine):
    desc = C.plan_info(f"gray:ref,{pw},emboss3", 3)["passes"][0]["desc"]
    m = _AFF.search(desc)
    assert (m is not None) == affine, desc
    if m:
        a, b, k = (int(x) for x in m.groups())
        v = np.arange(256, dtype=np.uint8).reshape(1, 256)
        lut = C.golden_apply(v, pw, "reflect101", True).reshape(-1).astype(np.int64)
        got = np.clip((a * np.arange(256) + b) >> k, 0, 255)
        assert (got == lut).all()
        assert abs(a) * 255 + abs(b) < 32768  # packed i16 arithmetic in the kernel


def test_post_affine_only_on_gray_ref(C):
    # the bt601 / plain-LUT prologues keep their tables (desc carries no post map)
    for ch in ("gray:bt601,contrast:3.5,emboss3", "contrast:3.5,gaussian5"):
        assert "post=" not in C.plan_info(ch, 3)["passes"][0]["desc"]
