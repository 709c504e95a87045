"""Fast host executor (csrc/core/cpu_exec.cpp: table-driven prologue, vectorised
tap sweeps, row-block threads) vs the per-pixel golden oracle: bit-identical."""
import numpy as np
import pytest



STENCILS = ["gaussian3", "gaussian5", "gaussian7", "box3", "box5", "emboss3", "emboss5", "sharpen", "laplace",
            "sobel", "sobel_l2"]


@pytest.mark.parametrize("name", STENCILS)
@pytest.mark.parametrize("ch", [1, 3])
def test_stencils_equal_golden(C, rng, name, ch):
    for shape in [(1, 1), (2, 3), (17, 15), (40, 203)]:
        img = rng.integers(0, 256, size=shape + ((3,) if ch == 3 else ()), dtype=np.uint8)
        for border in ("reflect101", "replicate", "constant", "skip"):
            chain = f"{name}@{border}"
            for threads in (1, 3):
                got = C.cpu_apply(img, chain, "reflect101", True, threads)
                ref = C.golden_apply(img, chain, "reflect101", True)
                assert got.shape == ref.shape and (got == ref).all(), (name, ch, shape, border, threads)


@pytest.mark.parametrize("chain", [
    "gray", "gray:ref", "invert", "brightness:-40", "contrast:3.5", "contrast:3:cv", "threshold:77",
    "gray,expand", "gray:ref,contrast:3.5,emboss3", "ref-gpu", "ref-cpu,expand",
    "gray:ref,contrast:3.5,emboss3@skip,expand", "gray,gaussian5,expand,invert", "gray,sobel_l2,invert,expand",
    "invert,gray,brightness:20,gaussian5,invert", "gaussian5,gaussian5,sobel", "gray,sobel,threshold:60",
    "brightness:10,gaussian3,contrast:1.5,sharpen,invert", "gaussian5@replicate,gaussian5@constant",
    "blur:9", "conv:3:1;2;1;2;4;2;1;2;1", "gray,blur:5,expand",
])
@pytest.mark.parametrize("fuse", [True, False])
def test_chains_equal_golden(C, rng, chain, fuse):
    img = rng.integers(0, 256, size=(61, 97, 3), dtype=np.uint8)
    got = C.cpu_apply(img, chain, "reflect101", fuse, 4)
    ref = C.golden_apply(img, chain, "reflect101", fuse)
    assert got.shape == ref.shape and (got == ref).all(), chain


def test_threads_split_rows_exactly(C, rng):
    # many threads over few rows: every row block rebuilds its own halo rows
    img = rng.integers(0, 256, size=(600, 700, 3), dtype=np.uint8)
    ref = C.golden_apply(img, "gaussian7,emboss5", "reflect101", True)
    for threads in (1, 2, 5, 16):
        assert (C.cpu_apply(img, "gaussian7,emboss5", "reflect101", True, threads) == ref).all(), threads


def test_ops_apply_numpy_uses_host_executor(rng):
    import mpi_cuda_imagemanipulation_amd as m

    img = rng.integers(0, 256, size=(50, 80, 3), dtype=np.uint8)
    assert (m.ops.apply(img, "gray:ref,contrast:3.5,emboss3@skip,expand") ==
            m._C.golden_apply(img, "gray:ref,contrast:3.5,emboss3@skip,expand", "reflect101", True)).all()


def test_batched_frames_numpy(C, rng):
    import mpi_cuda_imagemanipulation_amd as m

    imgs = rng.integers(0, 256, size=(3, 20, 33, 3), dtype=np.uint8)
    got = m.ops.apply(imgs, "gray,sobel")
    assert got.shape == (3, 20, 33)
    for b in range(3):
        assert (got[b] == C.golden_apply(imgs[b], "gray,sobel", "reflect101", True)).all()
