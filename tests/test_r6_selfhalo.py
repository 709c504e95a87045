"""Self-halo: one rank on a one-rank RCCL
communicator exchanges its boundary rows with itself every pass -- the two
grouped ncclSend / ncclRecv pairs an interior rank of an N > 1 run posts --
so the transfers that decide the 1 -> 8 curve run, and are timed, on one GPU.

The frame is then vertically periodic: the rows above row 0 are the last
rows (what the "upper neighbour" sends down) and the rows below the last row
are the first rows.  Every result is compared bit-exactly with the golden
path on that periodic frame, for every halo schedule, one and two streams.

Reference: the per-rank transfers RCCL replaces (kernel.cu:137,223); the
reference has no halo exchange at all.
"""
import numpy as np
import pytest

import mpi_cuda_imagemanipulation_amd as m
from mpi_cuda_imagemanipulation_amd import parallel
from mpi_cuda_imagemanipulation_amd.models import Pipeline

C = m._C


def torus_golden(img, chain, n_it):
    """golden path on a vertically periodic frame: pad with the other edge's
    rows (n_it x reach each side), filter n_it times, crop"""
    R = max(1, C.plan_info(chain, img.shape[2] if img.ndim == 3 else 1)["max_radius"])
    k = n_it * R
    ext = np.concatenate([img[-k:], img, img[:k]], axis=0)
    for _ in range(n_it):
        ext = C.golden_apply(ext, chain, "reflect101", True)
    return ext[k:-k]


def _clear_env(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)


@pytest.fixture(scope="module")
def rccl_ctx():
    """one one-rank RCCL communicator for the module (each init costs RCCL
    setup and device resources)"""
    import os

    saved = {k: os.environ.pop(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK") if k in os.environ}
    try:
        yield parallel.init("rccl")
    finally:
        os.environ.update(saved)


def test_torus_golden_is_periodic():
    # the oracle itself: shifting the periodic frame by s rows shifts the result
    img = C.synth_rows(3, 61, 3, 0, 40)
    a = torus_golden(img, "gaussian5", 2)
    b = torus_golden(np.roll(img, 7, axis=0), "gaussian5", 2)
    assert (np.roll(a, 7, axis=0) == b).all()


def test_self_halo_needs_a_one_rank_rccl_comm(monkeypatch):
    # host engines (no communicator) refuse the mode with a message
    _clear_env(monkeypatch)
    ctx = parallel.init("gloo")
    with pytest.raises(Exception, match="self_halo"):
        parallel.DistributedPipeline(ctx, Pipeline("gaussian5", self_halo=True), 64, 32, 3)


def test_config_carries_self_halo():
    cfg = Pipeline("gaussian5", self_halo=True).config(64, 32, 3)
    assert cfg.self_halo is True
    assert Pipeline("gaussian5").config(64, 32, 3).self_halo is False


CASES = [("gaussian5", 3), ("emboss3", 1), ("sharpen", 3), ("blur:9", 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("chain,cc", CASES)
@pytest.mark.parametrize("schedule", ["serial", "overlap", "pipeline", "batched", "ahead"])
@pytest.mark.parametrize("streams", [1, 2])
def test_self_halo_frame_stream_exact_gpu(rccl_ctx, chain, cc, schedule, streams):
    ctx = rccl_ctx
    W, H, F, n_it = 517, 96, 3, 2
    pipe = Pipeline(chain, halo_depth=1, self_halo=True)
    fs = parallel.FrameStream(ctx, pipe, W, H, cc, frames=F, streams=streams, autotune=False)
    assert all(f.engine.self_halo for f in fs.frames)
    fs.set_schedule(schedule)
    # every schedule applies to the self-halo rank (the MFMA blur keeps the
    # overlap schedule for a pipeline request, as at N > 1)
    assert fs.schedule == ("overlap" if (schedule == "pipeline" and chain.startswith("blur")) else schedule)
    fs.load_synthetic(11)
    before = ctx.comm.identity()["groups"]
    for i in range(n_it * F):
        fs.step(i)
    fs.synchronize()
    passes = len(C.plan_info(chain, cc)["passes"])
    groups = ctx.comm.identity()["groups"] - before
    if schedule == "batched":  # one group per stream and round: the frames sharing a stream post together
        assert groups == n_it * min(streams, F)
    elif schedule == "ahead":  # the first round's own exchanges, then one post after every step
        assert groups == F + n_it * F
    else:
        assert groups == n_it * F * passes  # one grouped exchange per pass and step
    tol = 1 if any(p["kind"] == 3 for p in C.plan_info(chain, cc)["passes"]) else 0
    for f, fr in enumerate(fs.frames):
        img = C.synth_rows(11 + f, W, cc, 0, H)
        ref = torus_golden(img, chain, n_it)
        got = fr.result_stripe()
        diff = np.abs(got.astype(np.int16) - ref.astype(np.int16))
        assert diff.max() <= tol, (chain, schedule, streams, f, int(diff.max()), np.argwhere(diff > tol)[:4])


@pytest.mark.gpu
def test_self_halo_bench_shape_exact_gpu(rccl_ctx):
    # the N=8 share's width (16384 RGB) and 4 cold frames, bench.py's frame
    # stream rule, the schedule the probe picks; both frame edges checked
    ctx = rccl_ctx
    W, H = 16384, 64
    fs = parallel.FrameStream(ctx, Pipeline("gaussian5", halo_depth=1, self_halo=True), W, H, 3, frames=4,
                              autotune=False)
    fs.load_synthetic(5)
    got = fs.pick_schedule(steps=8, rounds=1)
    assert got["chosen"] in fs.SCHEDULES and len(got["ms"]) >= 3
    fs.load_synthetic(5)
    for i in range(4):
        fs.step(i)
    fs.synchronize()
    for f, fr in enumerate(fs.frames):
        ref = torus_golden(C.synth_rows(5 + f, W, 3, 0, H), "gaussian5", 1)
        assert (fr.result_stripe() == ref).all(), f


@pytest.mark.gpu
def test_self_halo_engine_timings_gpu(rccl_ctx):
    # stage timing sees the exchange (device events on the comm stream)
    ctx = rccl_ctx
    d = parallel.DistributedPipeline(ctx, Pipeline("gaussian5", halo_depth=1, self_halo=True), 1024, 64, 3)
    d.load_synthetic(1)
    d.run(3)
    d.synchronize()
    t = d.stage_times()
    assert t["halo"] > 0 and t["compute"] > 0
    ref = torus_golden(C.synth_rows(1, 1024, 3, 0, 64), "gaussian5", 3)
    assert (d.result_stripe() == ref).all()


@pytest.mark.gpu
def test_batched_posts_survive_partial_rounds_gpu(rccl_ctx):
    # a loop that stops mid-round leaves a posted exchange behind; the next
    # loop (and a plain run, a reload) must neither skip nor double-apply it
    ctx = rccl_ctx
    W, H, F = 300, 64, 4
    fs = parallel.FrameStream(ctx, Pipeline("gaussian5", halo_depth=1, self_halo=True), W, H, 3, frames=F, streams=2,
                              autotune=False)
    fs.set_schedule("batched")
    fs.load_synthetic(3)
    steps = [0, 1, 2, 0, 1, 2, 3, 0, 1]  # frame 3 posted at step 1, never run in the first loop; loops restart at 0
    for i in steps:
        fs.step(i)
    fs.synchronize()
    for f, fr in enumerate(fs.frames):  # frame f stepped once per i == f in the sequence
        ref = torus_golden(C.synth_rows(3 + f, W, 3, 0, H), "gaussian5", steps.count(f))
        assert (fr.result_stripe() == ref).all(), f
    # a reload invalidates the post: the next step makes its own exchange
    # (posts go inside a group the caller opens -- a lone send to self has no
    # matching receive)
    ctx.comm.group_start()
    fs.frames[2].engine.post_halo()
    ctx.comm.group_end()
    fs.frames[2].load_synthetic(9)
    fs.frames[2].engine.run_posted()
    fs.synchronize()
    assert (fs.frames[2].result_stripe() == torus_golden(C.synth_rows(9, W, 3, 0, H), "gaussian5", 1)).all()


@pytest.mark.gpu
def test_ahead_posts_survive_partial_rounds_gpu(rccl_ctx):
    # ahead posts (next exchange on the communication stream right after each
    # step): loops that stop mid-round, a plain run and a reload between a post
    # and its step must neither skip nor double-apply an exchange
    ctx = rccl_ctx
    W, H, F = 300, 64, 4
    fs = parallel.FrameStream(ctx, Pipeline("gaussian5", halo_depth=1, self_halo=True), W, H, 3, frames=F, streams=2,
                              autotune=False)
    fs.set_schedule("ahead")
    assert fs.schedule == "ahead"
    fs.load_synthetic(3)
    steps = [0, 1, 2, 0, 1, 2, 3, 0, 1]
    for i in steps:
        fs.step(i)
    fs.synchronize()
    for f, fr in enumerate(fs.frames):
        ref = torus_golden(C.synth_rows(3 + f, W, 3, 0, H), "gaussian5", steps.count(f))
        assert (fr.result_stripe() == ref).all(), f
    # a plain run after a post: it waits for the posted exchange, then makes its own
    e1 = fs.frames[1].engine
    e1.post_halo_ahead(fs._comm_streams.handles[0])
    fs.frames[1].run(1)
    # a reload after a post: the pending exchange lands first, the reload wins
    e2 = fs.frames[2].engine
    e2.post_halo_ahead(fs._comm_streams.handles[0])
    fs.frames[2].load_synthetic(9)
    e2.run_posted()
    fs.synchronize()
    assert (fs.frames[1].result_stripe() ==
            torus_golden(C.synth_rows(4, W, 3, 0, H), "gaussian5", steps.count(1) + 1)).all()
    assert (fs.frames[2].result_stripe() == torus_golden(C.synth_rows(9, W, 3, 0, H), "gaussian5", 1)).all()
