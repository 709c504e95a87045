"""Deep frames: a frame stream whose frames exchange k*S halo rows every k-th
step (Engine.deep_steps, FrameStream "+deep" schedules).

Each step is still one step of the next frame, so the stream keeps reading
cold stripes.  A frame's first step of a block exchanges depth * S rows, and
the following steps recompute a shrinking band of the neighbours' rows
instead of exchanging (the per-step form of Engine::run_deep).  Every result
must equal the golden iterated path bit for bit:

* for block lengths that do not divide the step count;
* for multi-pass chains;
* on host engines over gloo (CPU);
* on the self-halo RCCL rank and on device engines in separate processes
  (GPU).

The reference exchanges no halo at all (kernel.cu:131-137).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import mpi_cuda_imagemanipulation_amd as m
from mpi_cuda_imagemanipulation_amd import parallel
from mpi_cuda_imagemanipulation_amd.models import Pipeline

C = m._C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


WORKER = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["STRIPE_ROOT"])
from mpi_cuda_imagemanipulation_amd import parallel, models
from mpi_cuda_imagemanipulation_amd._native import C
ctx = parallel.init(os.environ["BACKEND"])
W, H, Cc, F = 61, 90, 3, 2
res = []
for chain, depth, sched, n_it in json.loads(os.environ["CASES"]):
    fs = parallel.FrameStream(ctx, models.Pipeline(chain, halo_depth=depth), W, H, Cc, frames=F, autotune=False)
    fs.set_schedule(sched)
    fs.load_synthetic(5)
    for i in range(n_it * F):
        fs.step(i)
    fs.synchronize()
    row0, rows = fs.head.stripe
    worst = 0
    for f in range(F):
        ref = C.synth_image(5 + f, W, H, Cc)
        for _ in range(n_it):
            ref = C.golden_apply(ref, chain, "reflect101", True)
        got = fs.frames[f].result_stripe()
        worst = max(worst, int(np.abs(got.astype(int) - ref[row0:row0 + rows].astype(int)).max()) if rows else 0)
    res.append({"chain": chain, "depth": fs.depth, "sched": fs.schedule, "deep": fs.deep, "worst": worst})
with open(f"result_{ctx.rank}.json", "w") as fh:
    json.dump(res, fh)
# explicit teardown: engines before the process group, every rank together
import gc, torch.distributed as dist
del fs
gc.collect()
if ctx.device:
    import torch
    torch.cuda.synchronize()
dist.barrier()
dist.destroy_process_group()
'''


def _run_workers(tmp_path, n, backend, cases, env_extra=None):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script)]
    env = dict(os.environ, STRIPE_ROOT=ROOT, OMP_NUM_THREADS="1", BACKEND=backend, CASES=json.dumps(cases),
               **(env_extra or {}))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    out = []
    for rank in range(n):
        f = tmp_path / f"result_{rank}.json"
        assert f.exists(), (rank, r.stdout[-2000:])
        out.append(json.loads(f.read_text()))
    return out


def test_deep_frames_host_gloo_exact(tmp_path):
    # 3 processes (30-row stripes: depth <= 30 / (2 S)); 7 steps per frame,
    # not a multiple of the block; a multi-pass chain (its own exchange
    # inside each deep step) and the per-step schedule beside it
    cases = [["gaussian5", 3, "serial+deep", 7], ["gaussian5", 4, "serial+deep", 7],
             ["gaussian5,sobel", 2, "serial+deep", 5], ["emboss3", 5, "serial+deep", 6],
             ["gaussian5", 3, "serial", 7]]
    out = _run_workers(tmp_path, 3, "gloo", cases, {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    for rank_res in out:
        for case, r in zip(cases, rank_res):
            assert r["worst"] == 0, (case, r)
            assert r["depth"] == case[1]
            assert r["deep"] == case[2].endswith("+deep")


def test_schedule_names():
    # "+deep" parses on any base schedule; depth 1 frames ignore it
    ctx = parallel.DistContext(0, 1, 0, False, None, -1, "gloo")
    fs = parallel.FrameStream(ctx, Pipeline("gaussian5"), 64, 32, 3, frames=1, autotune=False)
    assert fs.depth == 1
    fs.set_schedule("serial+deep")
    assert fs.deep is False and fs.schedule == "serial"
    with pytest.raises(ValueError):
        fs.set_schedule("serial+shallow")


# ---- GPU: the self-halo rank (one-rank RCCL loopback) ----

def torus_golden(img, chain, n_it):
    R = max(1, C.plan_info(chain, img.shape[2] if img.ndim == 3 else 1)["max_radius"])
    k = n_it * R
    ext = np.concatenate([img[-k:], img, img[:k]], axis=0)
    for _ in range(n_it):
        ext = C.golden_apply(ext, chain, "reflect101", True)
    return ext[k:-k]


@pytest.fixture(scope="module")
def rccl_ctx():
    saved = {k: os.environ.pop(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK") if k in os.environ}
    try:
        yield parallel.init("rccl")
    finally:
        os.environ.update(saved)


@pytest.mark.gpu
@pytest.mark.parametrize("chain,cc", [("gaussian5", 3), ("sobel", 1), ("gaussian3", 3)])
@pytest.mark.parametrize("schedule", ["serial+deep", "batched+deep", "ahead+deep"])
@pytest.mark.parametrize("streams", [1, 2])
def test_deep_frames_self_halo_exact_gpu(rccl_ctx, chain, cc, schedule, streams):
    ctx = rccl_ctx
    W, H, F, depth, n_it = 517, 96, 3, 3, 7
    fs = parallel.FrameStream(ctx, Pipeline(chain, halo_depth=depth, self_halo=True), W, H, cc, frames=F,
                              streams=streams, autotune=False)
    assert fs.depth == depth
    fs.set_schedule(schedule)
    assert fs.schedule == schedule and fs.deep
    fs.load_synthetic(11)
    before = ctx.comm.identity()["groups"]
    for i in range(n_it * F):
        fs.step(i)
    fs.synchronize()
    groups = ctx.comm.identity()["groups"] - before
    blocks = -(-n_it // depth)  # exchanges per frame: steps 0, 3, 6
    if schedule.startswith("batched"):  # one group per stream and exchanging round
        assert groups == blocks * min(streams, F)
    else:  # serial: each frame's own; ahead: the first round's own, then one post before each later block
        assert groups == blocks * F
    for f, fr in enumerate(fs.frames):
        ref = torus_golden(C.synth_rows(11 + f, W, cc, 0, H), chain, n_it)
        got = fr.result_stripe()
        assert (got == ref).all(), (chain, schedule, streams, f, np.argwhere(got != ref)[:4])


@pytest.mark.gpu
def test_deep_frames_probe_and_engine_gpu(rccl_ctx):
    # auto depth on the self-halo rank: the probe times the deep schedules
    # beside the per-step ones; the chosen one stays exact.  A reload mid-block
    # restarts the block; run(n) on a deep-stepping engine is exact too.
    ctx = rccl_ctx
    W, H = 4096, 256
    fs = parallel.FrameStream(ctx, Pipeline("gaussian5", self_halo=True), W, H, 3, frames=4, autotune=False)
    assert fs.depth > 1
    got = fs.pick_schedule(steps=8, rounds=1)
    assert any("+deep" in k for k in got["ms"]) and any("+deep" not in k for k in got["ms"])
    fs.load_synthetic(2)
    for i in range(12):
        fs.step(i)
    fs.synchronize()
    for f, fr in enumerate(fs.frames):
        assert (fr.result_stripe() == torus_golden(C.synth_rows(2 + f, W, 3, 0, H), "gaussian5", 3)).all(), f
    fs.set_schedule("serial+deep")
    e = fs.frames[1]
    e.load_synthetic(7)
    e.run(1)
    e.load_synthetic(8)  # mid-block reload: the next step exchanges again
    e.run(4)
    e.synchronize()
    assert (e.result_stripe() == torus_golden(C.synth_rows(8, W, 3, 0, H), "gaussian5", 4)).all()


@pytest.mark.gpu
def test_deep_frames_gloo_gpu_processes(tmp_path):
    # device engines in 2 processes (gloo through pinned host memory): every
    # deep schedule, the transport an N > 1 run's deep steps use
    import torch

    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    cases = [["gaussian5", 3, s, 7] for s in ("serial+deep", "batched+deep", "ahead+deep")] + \
            [["gaussian5,sobel", 2, "serial+deep", 5]]
    out = _run_workers(tmp_path, 2, "gloo-gpu", cases)
    for rank_res in out:
        for case, r in zip(cases, rank_res):
            assert r["worst"] == 0, (case, r)
