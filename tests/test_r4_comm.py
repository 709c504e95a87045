"""Bounded communicator progress, pre-connect topology, runtime identity and
the benchmark's hang-proofing.

The reference's failure path is a hang: a rank that errors returns 1 without
MPI_Abort and its peers wait in MPI forever (kernel.cu:111-114).
Here every wait of a non-blocking communicator runs through one state
machine, await_progress (RCCL init / group end / pre-connect; the gloo
callback comm's posted groups), tested below through its Python hook, through
a callback communicator driven by an engine, and across processes.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seq(states):
    it = iter(states)
    last = [states[-1]]

    def probe():
        try:
            last[0] = next(it)
        except StopIteration:
            pass
        return last[0]

    return probe


def test_await_progress_done_after_pending(C):
    ms = C.await_progress("op", 5.0, _seq([1, 1, 1, 0]))
    assert ms >= 0


def test_await_progress_failure_raises(C):
    with pytest.raises(Exception, match="op failed"):
        C.await_progress("op", 5.0, _seq([1, 2]))


def test_await_progress_timeout_is_bounded(C):
    t0 = time.time()
    with pytest.raises(Exception, match="did not complete within"):
        C.await_progress("stuck op", 0.3, lambda: 1)
    took = time.time() - t0
    assert 0.3 <= took < 5


def test_await_progress_sees_abort_flag(C):
    calls = []

    def aborted():
        calls.append(1)
        return len(calls) > 3

    with pytest.raises(Exception, match="aborted while waiting"):
        C.await_progress("op", 30.0, lambda: 1, aborted)


@pytest.mark.parametrize("world", range(1, 10))
def test_preconnect_peers_symmetric(C, world):
    peers = [set(C.preconnect_peers(r, world)) for r in range(world)]
    for r in range(world):
        assert r not in peers[r]
        for q in peers[r]:
            assert r in peers[q], (r, q)
        # neighbours +-1 (halo exchange) and the root (scatter / gather)
        need = {q for q in (r - 1, r + 1, 0) if 0 <= q < world and q != r}
        assert need <= peers[r]
    assert peers[0] == set(range(1, world))


def _callback_engine(C, poll, world=2, rank=0):
    """rank `rank` of a `world`-rank host engine over a callback comm whose
    groups never complete (poll) -- nobody answers the halo exchange"""
    import mpi_cuda_imagemanipulation_amd as m

    noop = lambda *a: None  # noqa: E731
    comm = C.make_callback_comm(rank, world, noop, noop, noop, noop, noop, poll)
    cfg = m.models.Pipeline("gaussian5", halo_depth=1).config(64, 40, 3, "host")
    e = C.Engine(cfg, comm)
    e.load_synthetic(1)
    return e, comm


def test_callback_comm_posted_group_times_out(C, monkeypatch):
    monkeypatch.setenv("STRIPE_COMM_TIMEOUT_S", "0.5")
    e, _ = _callback_engine(C, lambda: 1)
    t0 = time.time()
    with pytest.raises(Exception, match="callback comm group on rank 0 did not complete"):
        e.run(1)
    assert time.time() - t0 < 10


def test_callback_comm_failed_group_raises(C):
    e, _ = _callback_engine(C, lambda: 2)
    with pytest.raises(Exception, match="transport reported failure"):
        e.run(1)


def test_callback_comm_abort_flag(C):
    e, comm = _callback_engine(C, lambda: 0)
    e.run(1)  # completes (poll: done)
    comm.abort("peer 1 failed")
    with pytest.raises(Exception, match="was aborted: peer 1 failed"):
        e.run(1)


def test_callback_comm_identity_default(C):
    noop = lambda *a: None  # noqa: E731
    comm = C.make_callback_comm(1, 3, noop, noop, noop, noop, noop)
    assert comm.identity() == {"rank": 1.0, "size": 3.0}


def test_one_runtime_copy_per_process(C):
    # torch (imported by the loader first) and the extension share one HIP
    # runtime, one RCCL and one HSA runtime: the extension resolves to the
    # copies torch mapped (same SONAMEs), never to a second stack
    libs = C.runtime_libs()
    for stem in ("libamdhip64", "librccl", "libhsa-runtime64"):
        assert len(libs[stem]) == 1, (stem, libs[stem])
    import torch

    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    assert libs["librccl"][0].startswith(tlib), libs
    assert libs["libamdhip64"][0].startswith(tlib), libs


def test_cli_binds_the_same_rccl_as_python(C):
    # `stripe info` reports the libraries it mapped: the CLI runs the same
    # HIP runtime / RCCL build as the Python path (RUNPATH: torch's lib first)
    exe = os.path.join(ROOT, "bin", "stripe")
    if not os.path.exists(exe):
        pytest.skip("CLI not built")
    r = subprocess.run([exe, "info", "--format", "json"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    libs = C.runtime_libs()
    assert info["libs"]["librccl"] == libs["librccl"]
    assert info["libs"]["libamdhip64"] == libs["libamdhip64"]
    assert info["rccl_version"] == C.rccl_version()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


STALL_WORKER = r'''
import os, sys, time
sys.path.insert(0, os.environ["STRIPE_ROOT"])
from mpi_cuda_imagemanipulation_amd import parallel, models
ctx = parallel.init("gloo")
dp = parallel.DistributedPipeline(ctx, models.Pipeline("gaussian5", halo_depth=1), 64, 48, 3)
dp.load_synthetic(1)
t0 = time.time()
try:
    dp.run(1)
    print("RANK", ctx.rank, "FINISHED", flush=True)
except Exception as e:
    print("RANK", ctx.rank, "ERROR after %.1fs:" % (time.time() - t0), str(e)[:300], flush=True)
    os._exit(7)
'''


def test_stalled_peer_bounded_by_comm_timeout(tmp_path):
    """Rank 1 is alive but never answers its halo exchange (STRIPE_FAULT
    halo@1:stall); rank 0's posted gloo group must fail at the comm bound
    with a message naming the wait, not block."""
    script = tmp_path / "w.py"
    script.write_text(STALL_WORKER)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), STRIPE_ROOT=ROOT, STRIPE_FAULT="halo@1:stall", STRIPE_COMM_TIMEOUT_S="4",
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    try:
        o0, _ = procs[0].communicate(timeout=90)
    finally:
        procs[1].kill()
        procs[1].communicate()
    out = o0.decode(errors="replace")
    assert procs[0].returncode == 7, out
    assert "callback comm group on rank 0 did not complete within" in out, out


def _bench(tmp_path, n, extra, env_extra, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--backend", "host", "--width", "96", "--height", "64", "--steps", "3", "--warmup", "1",
           "--dist-steps", "2", *extra]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", **env_extra)
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=str(tmp_path))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines, time.time() - t0


def test_bench_peer_exit_still_reports_headline(tmp_path):
    """A peer dies in an extra scope (STRIPE_FAULT=scatter@1:exit, the dist
    scope's scatter): the headline line still prints, once."""
    r, lines, took = _bench(tmp_path, 2, ["--comm-timeout-s", "20", "--budget-s", "120"],
                            {"STRIPE_FAULT": "scatter@1:exit"})
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and rec["verified_vs_golden"] is True and rec["n_gpus"] == 2
    assert took < 120


def test_bench_stalled_peer_within_budget(tmp_path):
    """A live peer stalls in an extra scope: rank 0 reports the headline
    within the wall-time budget instead of running into the driver's limit."""
    r, lines, took = _bench(tmp_path, 2, ["--comm-timeout-s", "5", "--budget-s", "60"],
                            {"STRIPE_FAULT": "scatter@1:stall"})
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and rec["verified_vs_golden"] is True
    assert rec["elapsed_s"] < 60


def test_bench_budget_skips_extra_scopes(tmp_path):
    # a budget already spent before the extra scopes: they are skipped and
    # listed, the headline is complete, the run exits 0
    r, lines, _ = _bench(tmp_path, 2, ["--budget-s", "0.01"], {})
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert set(rec["budget"]["skipped"]) >= {"dist", "resident_deep"}
    assert "partial" not in rec
    # host engines have one halo schedule: nothing to time, the choice is recorded
    assert rec["halo_schedule"]["chosen"] == "serial" and rec["halo_schedule"]["requested"] == "auto"


# ------------------------------------------------------------------ GPU box
@pytest.mark.gpu
def test_rccl_comm_identity_and_nonblocking_gpu(C):
    # a one-rank RCCL communicator goes through the same non-blocking init,
    # pre-connect and bounded waits as the multi-rank path
    import torch

    torch.cuda.set_device(0)
    comm = C.make_rccl_comm(C.rccl_unique_id(), 0, 1, 0)
    ident = comm.identity()
    assert ident["nccl_count"] == 1 and ident["nccl_device"] == 0 and ident["nccl_user_rank"] == 0
    assert ident["nonblocking"] == 1 and ident["init_ms"] >= 0
    comm.barrier()  # an all-reduce through the bounded enqueue + stream wait


@pytest.mark.gpu
def test_gpu_process_maps_one_runtime(C):
    import torch

    import mpi_cuda_imagemanipulation_amd as m

    x = torch.randint(0, 256, (64, 96, 3), dtype=torch.uint8, device="cuda")
    m.ops.apply(x, "gaussian5")
    torch.cuda.synchronize()
    libs = C.runtime_libs()
    for stem in ("libamdhip64", "librccl", "libhsa-runtime64"):
        assert len(libs[stem]) == 1, libs
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    assert libs["libamdhip64"][0].startswith(tlib) and libs["librccl"][0].startswith(tlib), libs


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["gaussian5", "sobel", "emboss3"])
def test_cold_engine_autotune_exact_gpu(C, chain):
    # EngineConfig.cold: the autotuner times candidates on a rotation of cold
    # scratch stripes and tunes the memory policy; the output stays exact
    import mpi_cuda_imagemanipulation_amd as m

    W, H, Cc = 2048, 512, (1 if chain == "sobel" else 3)
    cfg = m.models.Pipeline(chain).config(W, H, Cc, "device", device=0, autotune=True)
    cfg.cold = True
    e = C.Engine(cfg)
    e.load_synthetic(7)
    e.run(1)
    out = e.store_packed()
    assert e.policies[0] in (0, 1) and e.bands[0] > 0
    ref = C.golden_apply(C.synth_rows(7, W, Cc, 0, H), chain, "reflect101", True)
    assert (out == ref).all()


@pytest.mark.gpu
def test_stage_timing_switch_gpu(C):
    import mpi_cuda_imagemanipulation_amd as m

    e = C.Engine(m.models.Pipeline("gaussian5").config(1024, 256, 3, "device", device=0))
    e.load_synthetic(3)
    e.run(1)
    e.synchronize()
    assert e.times.as_dict()["compute"] > 0
    e.stage_timing = False
    e.load_synthetic(3)
    e.run(2)
    e.synchronize()
    ref = C.synth_rows(3, 1024, 3, 0, 256)
    for _ in range(2):
        ref = C.golden_apply(ref, "gaussian5", "reflect101", True)
    assert (e.store_packed() == ref).all()


def test_frame_stream_host_each_frame_exact(C, monkeypatch):
    # FrameStream: frames stepped round-robin, each an independent iterated
    # stripe (frame f = seed + f); after 2 rounds every frame equals 2 golden
    # passes of its own input
    import mpi_cuda_imagemanipulation_amd as m
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("gloo")
    fs = parallel.FrameStream(ctx, m.models.Pipeline("gaussian5", halo_depth=1), 70, 33, 3, frames=3)
    assert len(fs) == 3 and fs.nstreams == 1 and not fs.streams  # host engines: no streams
    fs.load_synthetic(5)
    fs.tune()
    for _ in range(6):
        fs.step()
    fs.synchronize()
    for f in range(3):
        ref = C.synth_image(5 + f, 70, 33, 3)
        for _ in range(2):
            ref = C.golden_apply(ref, "gaussian5", "reflect101", True)
        assert (fs.frames[f].result_stripe() == ref).all(), f


def test_halo_schedule_property(C):
    # request vs effective schedule: a one-rank (or host) engine exchanges
    # nothing, so every request runs as the serial schedule
    import mpi_cuda_imagemanipulation_amd as m

    e = C.Engine(m.models.Pipeline("gaussian5").config(64, 32, 3, "host"))
    for s in ("pipeline", "overlap", "serial"):
        e.halo_schedule = s
        assert e.halo_schedule == "serial"
    with pytest.raises(Exception, match="halo schedule"):
        e.halo_schedule = "fastest"


def test_frame_stream_pick_schedule_single_candidate(C, monkeypatch):
    # only schedules that differ on this engine are timed; one candidate -> no timing
    import mpi_cuda_imagemanipulation_amd as m
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("gloo")
    fs = parallel.FrameStream(ctx, m.models.Pipeline("gaussian5", halo_depth=1), 64, 40, 3)
    calls = []
    got = fs.pick_schedule(lambda v: calls.append(v) or v)
    assert got == {"chosen": "serial", "streams": 1, "queues": "none", "ms": {}} and not calls
    assert fs.schedule == "serial"


def test_frame_stream_pick_schedule_takes_fastest_max_over_ranks(monkeypatch):
    # device engines: all three schedules are timed `rounds` times (the same
    # list on every rank, whatever each rank's stripe runs), the per-rank
    # time goes through reduce_max (every rank must agree), the fastest wins
    # and stays set on every frame
    from types import SimpleNamespace

    from mpi_cuda_imagemanipulation_amd import parallel

    class _Clock:  # the stand-in steps advance a fake clock: exact timings on a loaded host
        t = 0.0

        def perf_counter(self):
            return self.t

        def sleep(self, dt):
            self.t += dt

    _t = _Clock()
    monkeypatch.setattr(parallel, "time", _t)

    cost = {"pipeline": 0.004, "overlap": 0.001, "serial": 0.002}
    frames = [SimpleNamespace(engine=SimpleNamespace(halo_schedule="pipeline")) for _ in range(2)]
    fs = parallel.FrameStream.__new__(parallel.FrameStream)
    fs.frames = frames
    fs.streams, fs.stream_options, fs.nstreams = [object()], [1], 1  # a device stream stand-in
    fs.set_streams = lambda n: None
    fs.step = lambda i=None: _t.sleep(cost[frames[0].engine.halo_schedule])
    fs.synchronize = lambda: None
    seen = []
    got = fs.pick_schedule(lambda v: seen.append(v) or v, steps=3, rounds=2)
    # (two frames on device streams at N > 1: the batched and ahead exchanges
    # are candidates too; their engines step the serial schedule)
    assert got["chosen"] == "overlap" and set(got["ms"]) == set(cost) | {"batched", "ahead"}
    assert len(seen) == 10 and all(f.engine.halo_schedule == "overlap" for f in frames)
    assert got["ms"]["overlap"] < got["ms"]["serial"] < got["ms"]["pipeline"]


def test_frame_stream_auto_frames_rule(C, monkeypatch):
    # auto frame count: 1 on the host or when one stripe exceeds the cache
    import mpi_cuda_imagemanipulation_amd as m
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("gloo")
    fs = parallel.FrameStream(ctx, m.models.Pipeline("gaussian5"), 64, 40, 3)
    assert len(fs) == 1 and fs.fits_mall and not fs.cold and fs.cache == "warm"  # host engines never rotate


@pytest.mark.parametrize("ws,iterable,device,frames,want", [
    # the headline's per-GPU step bytes (16384^2 RGB gaussian5) at N = 1 / 2 / 8
    (16384 * 16384 * 6, True, True, 0, (2, False, False, "exceeds the Infinity Cache")),
    (8192 * 16384 * 6, True, True, 0, (2, False, False, "exceeds the Infinity Cache")),
    (2048 * 16384 * 6, True, True, 0, (4, True, True, "cold")),
    # a small share: the 8-frame cap leaves the rotation inside 2 x the cache
    (16 << 20, True, True, 0, (8, True, False, "partially warm")),
    (16 << 20, True, True, 1, (1, False, False, "warm")),
    (16 << 20, True, False, 0, (1, False, False, "warm")),      # host engines never rotate
    (16 << 20, False, True, 0, (1, False, False, "warm")),      # channel-changing chain
])
def test_frame_stream_plan_same_rule_every_n(ws, iterable, device, frames, want):
    # one frames rule at every N (N = 1 too: two frames), and the
    # cache label says what the rotation achieves
    from mpi_cuda_imagemanipulation_amd import parallel

    assert parallel.FrameStream.plan(ws, iterable, device, frames) == want


@pytest.mark.gpu
@pytest.mark.parametrize("chain,Cc", [("gaussian5", 3), ("sobel", 1), ("gaussian5,sobel", 3)])
def test_frame_stream_gpu_each_frame_exact(C, monkeypatch, chain, Cc):
    # device FrameStream: frames on two alternating streams, cold autotune;
    # after 3 rounds each frame equals 3 golden passes of its own input
    import mpi_cuda_imagemanipulation_amd as m
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("rccl")
    W, H = 1030, 200
    fs = parallel.FrameStream(ctx, m.models.Pipeline(chain, halo_depth=1), W, H, Cc, frames=3)
    # (3 small frames fit the cache together: streaming policy, honestly not "cold")
    assert len(fs) == 3 and fs.nstreams == 2 and fs.streaming and not fs.cold and fs.cache == "partially warm"
    fs.load_synthetic(9)
    fs.tune()
    rounds = 3 if fs.iterable else 1
    for _ in range(3 * rounds):
        fs.step()
    fs.synchronize()
    for f in range(3):
        ref = C.synth_rows(9 + f, W, Cc, 0, H)
        for _ in range(rounds):
            ref = C.golden_apply(ref, chain, "reflect101", True)
        assert (fs.frames[f].result_stripe() == ref).all(), f


def test_bench_fixed_halo_schedule_recorded(tmp_path):
    # --halo-schedule fixes the request (no probe); a host engine runs it as
    # its one schedule and the record says both
    r, lines, _ = _bench(tmp_path, 2, ["--halo-schedule", "pipeline", "--budget-s", "0.01"], {})
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(lines[0])
    assert rec["halo_schedule"] == {"chosen": "serial", "ms": {}, "requested": "pipeline"}
