"""Static resource checks of every compiled gfx950 kernel (SURVEY §5 "race
detection / sanitizers": `-Rpass-analysis=kernel-resource-usage` checks).

tools/build.py compiles each HIP file with the kernel-resource-usage remarks
and writes build/kernel_resources.json.  No kernel may touch scratch memory
(register spills to scratch are a silent 2-10x slowdown on a streaming kernel).
"""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPORT = os.path.join(ROOT, "build", "kernel_resources.json")


@pytest.fixture(scope="module")
def report():
    if not os.path.exists(REPORT):
        pytest.skip("build/kernel_resources.json missing (run python tools/build.py)")
    with open(REPORT) as f:
        rep = json.load(f)
    assert rep, "empty kernel resource report"
    return rep


def test_every_kernel_family_reported(report):
    names = " ".join(report)
    for fam in ["k_pointwise", "k_fill_margins", "k_synth", "k_copy_rows", "k_sep", "k_direct", "k_blur_sep",
                "k_conv_mfma"]:
        assert fam in names, fam


def test_no_scratch_no_vgpr_spills(report):
    bad = {k: v for k, v in report.items()
           if v.get("ScratchSize [bytes/lane]", 0) != 0 or v.get("VGPRs Spill", 0) != 0
           or v.get("Dynamic Stack", "False") != "False"}
    assert not bad, json.dumps(bad, indent=1)[:2000]


def test_hot_kernels_have_occupancy(report):
    # streaming stencils need >= 4 waves/SIMD to keep rows in flight; the MFMA
    # blur runs 2 waves/SIMD by design (one computes while the other loads)
    for k, v in report.items():
        occ = v.get("Occupancy [waves/SIMD]", 0)
        if "k_sep" in k or "k_direct" in k:
            assert occ >= 3, (k, occ)
        elif "k_blur_sep" in k:
            assert occ >= 2, (k, occ)


def test_headline_kernel_clean(report):
    # gaussian5 on RGB without prologue: the BASELINE headline kernel
    # (k_sep<C=3, Gaussian5, PRO_NONE, SKIP=false, any store policy>)
    hits = [v for k, v in report.items() if "k_sepILi3ENS_4sdef9Gaussian5ELi0ELb0E" in k]
    assert hits
    for v in hits:
        assert v["SGPRs Spill"] == 0 and v["VGPRs Spill"] == 0 and v["VGPRs"] <= 128
