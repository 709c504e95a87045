"""Distributed engine on the GPU: N logical ranks on one device (local comm)
must reproduce the 1-rank result bit-for-bit (halo exchange correctness)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def m():
    import mpi_cuda_imagemanipulation_amd as m

    return m


@pytest.mark.parametrize("chain", ["gaussian5", "gray:ref,contrast:3.5,emboss3", "sobel,gaussian7", "blur:9",
                                   "gaussian3,invert,emboss5"])
@pytest.mark.parametrize("ranks", [2, 3, 4, 8])
def test_local_ranks_equal_golden(m, chain, ranks):
    img = m.utils.synthetic_image(11, 301, 97, 3)
    pipe = m.Pipeline(chain)
    got = pipe.run_distributed(img, ranks, backend="local")
    ref = m._C.golden_apply(img, chain, "reflect101", True)
    if chain.startswith("blur"):
        assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1
    else:
        assert (got == ref).all()


@pytest.mark.parametrize("overlap", [True, False])
def test_iterations_match_host(m, overlap):
    img = m.utils.synthetic_image(2, 130, 64, 3)
    pipe = m.Pipeline("gaussian5", overlap=overlap)
    dev = pipe.run_distributed(img, 4, backend="local", iterations=5)
    host = pipe.run_distributed(img, 1, backend="host", iterations=5)
    assert (dev == host).all()


def test_no_halo_shows_seams(m):
    img = m.utils.synthetic_image(4, 120, 64, 1)
    with_halo = m.Pipeline("gaussian5").run_distributed(img, 4, backend="local")
    no_halo = m.Pipeline("gaussian5", halo=False).run_distributed(img, 4, backend="local")
    diff_rows = np.nonzero((with_halo != no_halo).any(axis=1))[0]
    assert len(diff_rows) > 0
    assert set(diff_rows.tolist()) <= {14, 15, 16, 17, 30, 31, 32, 33, 46, 47, 48, 49}


def test_ref_gpu_preset_matches_per_stripe_reference(m):
    import np_ref

    img = m.utils.synthetic_image(9, 64, 42, 3)
    out = m.Pipeline.preset("ref-gpu").run_distributed(img, 4, backend="local")
    rows = 42 // 4
    for r in range(4):
        s = img[r * rows:(r + 1) * rows]
        e = np_ref.stencil(np_ref.contrast_ref(np_ref.gray_ref(s), 3.5), "emboss3", "skip")
        assert (out[r * rows:(r + 1) * rows] == np_ref.expand(e)).all()
    assert (out[4 * rows:] == 0).all()  # legacy split: remainder rows not processed (Q7)


def test_synthetic_on_device_matches_host(m):
    C = m._C
    cfg = m.Pipeline("gaussian5").config(257, 33, 3, "device", device=0)
    e = C.Engine(cfg)
    e.load_synthetic(5)
    e.run(1)
    out = e.store_packed()
    ref = C.golden_apply(m.utils.synthetic_image(5, 257, 33, 3), "gaussian5", "reflect101", True)
    assert (out == ref).all()


def test_rccl_single_rank(m):
    C = m._C
    uid = C.rccl_unique_id()
    comm = C.make_rccl_comm(uid, 0, 1, 0)
    cfg = m.Pipeline("gaussian5").config(300, 40, 3, "device", device=0)
    cfg.root_buffers = True
    e = C.Engine(cfg, comm)
    img = m.utils.synthetic_image(1, 300, 40, 3)
    e.load_root(img)
    e.scatter()
    e.run(2)
    e.gather()
    out = e.store_root()
    ref = C.golden_apply(C.golden_apply(img, "gaussian5", "reflect101", True), "gaussian5", "reflect101", True)
    assert (out == ref).all()


@pytest.mark.parametrize("chain,chunks", [("gaussian5", 1), ("gaussian5", 7), ("gray:ref,contrast:3.5,emboss3", 5),
                                          ("gaussian5,sobel", 4), ("blur:9", 3)])
def test_e2e_pinned_pipeline(m, chain, chunks):
    C = m._C
    W, H = 333, 97
    img = m.utils.synthetic_image(8, W, H, 3)
    cfg = m.Pipeline(chain).config(W, H, 3, "device", device=0)
    e = C.Engine(cfg)
    e.alloc_host_io()
    hin = e.host_input()
    hin[...] = img
    for _ in range(2):  # second step reuses the buffers (WAR ordering across steps)
        e.run_e2e(chunks)
        e.synchronize()
        out = np.array(e.host_output())
        ref = C.golden_apply(img, chain, "reflect101", True)
        if chain.startswith("blur"):
            assert np.abs(out.astype(int) - ref.astype(int)).max() <= 1
        else:
            assert (out == ref).all()


@pytest.mark.parametrize("chain", ["gaussian5", "gaussian5,sobel", "invert,gaussian3,emboss3", "blur:9"])
@pytest.mark.parametrize("iters", [2, 5, 8])
def test_graph_replay_matches_eager(m, chain, iters):
    """Iterated chains replay a captured hipGraph (one cycle of 1 or 2
    iterations); results equal the eager launches bit-for-bit."""
    C = m._C
    outs = []
    for graphs in (True, False):
        cfg = m.Pipeline(chain).config(257, 131, 3, "device", device=0)
        cfg.graphs = graphs
        e = C.Engine(cfg, None)
        e.load_synthetic(3)
        e.run(iters)
        e.run(iters)  # second call replays the already-captured graph
        e.synchronize()
        outs.append(e.store_packed())
        cycle = 1 if len(C.plan_info(chain, 3)["passes"]) % 2 == 0 else 2
        expect = graphs and iters >= 2 * cycle
        assert (e.graph_launches > 0) == expect, (chain, iters, e.graph_launches)
    assert (outs[0] == outs[1]).all()


@pytest.mark.parametrize("chain", ["gaussian5", "sobel", "emboss3", "blur:9", "gaussian7"])
@pytest.mark.parametrize("ranks,H", [(2, 96), (4, 130), (8, 97), (5, 40)])
def test_pipelined_halo_schedule(m, chain, ranks, H):
    """Iterated single-pass chains over several ranks run the core / rim /
    boundary schedule on two streams; it must equal the plain schedule and the
    1-rank result (H=40 with 5 ranks: stripes too short to pipeline mix with
    pipelined ones)."""
    img = m.utils.synthetic_image(7, 203, H, 3)
    C = m._C
    res = []
    for pipeline, nr in ((True, ranks), (False, ranks), (True, 1)):
        pipe = m.Pipeline(chain)
        cfg = pipe.config(203, H, 3, "device", device=0)
        cfg.pipeline = pipeline
        cfg.halo_depth = 1  # exchange every iteration (the deep-halo schedule is tested below)
        res.append(C.run_local_group(cfg, nr, img, 4))
    assert (res[0] == res[1]).all()
    assert (res[0] == res[2]).all()


@pytest.mark.parametrize("chain", ["gaussian5", "sobel", "emboss3", "gaussian7", "gray:ref,contrast:3.5,emboss5",
                                   "gray:ref,contrast:3.5,emboss3@skip,expand", "gray,gaussian7,expand"])
@pytest.mark.parametrize("ranks,H,depth", [(2, 96, 2), (4, 130, 3), (8, 233, 4), (3, 300, 8)])
@pytest.mark.parametrize("iters", [1, 6, 7])
def test_deep_halo_schedule(m, chain, ranks, H, depth, iters):
    """Deep halo on the GPU: the stencil kernels write output rows inside the
    halo (negative / past-the-end local rows); N ranks at depth k equal the
    1-rank result and the per-iteration exchange bit-for-bit."""
    C = m._C
    W = 203
    img = m.utils.synthetic_image(13, W, H, 3)
    if C.plan_info(chain, 3)["cin"] != C.plan_info(chain, 3)["cout"] and iters > 1:
        pytest.skip("chain changes the channel count: not iterable")
    res = []
    for d, nr in ((depth, ranks), (1, ranks), (1, 1)):
        pipe = m.Pipeline(chain, halo_depth=d)
        res.append(C.run_local_group(pipe.config(W, H, 3, "device", device=0), nr, img, iters))
    assert (res[0] == res[1]).all()
    assert (res[0] == res[2]).all()


@pytest.mark.parametrize("chain", ["gaussian5,sobel", "gaussian3,invert,emboss3", "gray,gaussian5,expand,box3",
                                   "invert,gaussian5,brightness:9,sharpen"])
@pytest.mark.parametrize("ranks,depth", [(2, 0), (4, 2), (8, 3)])
@pytest.mark.parametrize("iters", [1, 4])
def test_multipass_chain_level_exchange_gpu(m, chain, ranks, depth, iters):
    """Multi-pass chains on the GPU: one exchange of the summed radius per
    chain (per block of `depth` iterations), every pass (pointwise ones too)
    writing rows inside the halo; equals the 1-rank result bit-for-bit."""
    C = m._C
    W, H = 203, 211
    info = C.plan_info(chain, 3)
    if info["cin"] != info["cout"] and iters > 1:
        pytest.skip("chain changes the channel count: not iterable")
    img = m.utils.synthetic_image(19, W, H, 3)
    res = []
    for nr in (ranks, 1):
        pipe = m.Pipeline(chain, halo_depth=depth)
        res.append(C.run_local_group(pipe.config(W, H, 3, "device", device=0), nr, img, iters))
    assert (res[0] == res[1]).all()


@pytest.mark.parametrize("chain", ["gaussian5", "sobel,emboss3", "gray:ref,contrast:3.5,emboss3"])
def test_autotune_bands_keep_output_exact(m, chain):
    """The band autotuner (engine_tune.cpp autotune_bands: bursts of back-to-back
    launches into the scratch buffer) picks a band per stencil pass from its
    candidate set and leaves the run's result bit-exact vs the golden path."""
    C = m._C
    img = m.utils.synthetic_image(5, 640, 200, 3)
    cfg = m.Pipeline(chain).config(640, 200, 3, "device", device=0, autotune=True)
    e = C.Engine(cfg)
    e.load_packed(np.ascontiguousarray(img))
    e.run(1)
    e.synchronize()
    bands = e.bands
    assert len(bands) == len(C.plan_info(chain, 3)["passes"])
    assert all(b in (0, 4, 8, 12, 16, 24, 32) for b in bands), bands
    assert any(b > 0 for b in bands)
    got = e.store_packed()
    ref = C.golden_apply(img, chain, "reflect101", True)
    assert (got == ref).all()


@pytest.mark.parametrize("chain", ["gaussian5", "emboss5", "sobel", "gaussian7", "sharpen",
                                   "gray:ref,contrast:3.5,emboss3@skip,expand", "gray,gaussian5"])
@pytest.mark.parametrize("band", [4, 8, 20])
def test_explicit_band_heights_exact(m, chain, band):
    """Every band height the autotuner may pick (4-row bands included: shorter
    than k_direct's K-row steps for emboss5) leaves the stencil output exact."""
    C = m._C
    img = m.utils.synthetic_image(6, 333, 101, 3)
    cfg = m.Pipeline(chain).config(333, 101, 3, "device", device=0)
    cfg.band = band
    e = C.Engine(cfg)
    e.load_packed(np.ascontiguousarray(img))
    e.run(1)
    e.synchronize()
    assert (e.store_packed() == C.golden_apply(img, chain, "reflect101", True)).all()
