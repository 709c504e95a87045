#!/usr/bin/env python3
"""Headline benchmark: 5x5 Gaussian blur on a 16384x16384 RGB frame,
row-partitioned over N MI355X (one process per GPU, RCCL over xGMI).

    python bench.py --gpus N --steps K --warmup W
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

One step = one full-frame gaussian5 pass over the distributed frame: every rank
filters its stripe with the halo rows its neighbours sent (ncclSend/ncclRecv).
How the exchange meets the filter is measured, not assumed.  At N > 1 the
probe times every halo schedule on the real transport before the timed region
and keeps the fastest (max over ranks; `halo_schedule` in the record):
  * exchange then filter;
  * interior rows beside the exchange, boundary rows after it;
  * core / rim / edge on three streams;
  * serial steps whose exchanges go out as one group per stream and round;
  * each frame's next exchange posted right after its step;
  * the "+deep" forms: a frame exchanges k*2 rows every k-th step and
    recomputes a shrinking band of its neighbours' rows in between
    (bit-identical; `halo_depth` in the record).
Each is timed with the frames on one stream or alternating over two.  Steps
are iterated (ping-pong), so each step's halo rows are required work.

Cache temperature of the headline.  A step's per-GPU working set is its stripe
in + out: 1.61 GB on one GPU, 201 MB on each of 8.  When it fits the 256 MiB
Infinity Cache (N=8), iterating one frame would read every step's input from
the cache, not HBM; the headline then steps round-robin over F independent
frames (F engines, each its own stripe pair; consecutive frames may alternate
over two streams) with F x working set > 2 x 256 MiB, so every step reads data
evicted long before -- a stream of distinct frames, the way a video-rate
workload sees the GPUs.  Stripes too big for the cache (N = 1, 2, 4) get two
frames, so one frame's kernel boundary (and exchange) can run beside the
other's filter.  The rule and the 1-vs-2-stream probe are the same at every N,
N = 1 included, so a 1 -> N curve compares one execution mode.  The
warm single-frame number (resident_warm) and the communication-avoiding deep
halo (resident_deep: k*2 rows exchanged once per k steps, bit-identical) are
reported beside it as named scopes, never as `value`.

Order of work (the timed region holds nothing but the K steps):
  identity (what RCCL and the runtime report, gathered to rank 0) -> autotune
  (band height x occupancy cap x memory policy, on cold data when the frames
  rotate, each stage's candidates timed round-robin; collective at N > 1:
  every candidate's time is the slowest rank's; also ramps the clock) -> halo-schedule probe (N > 1) -> W warmup steps -> K timed steps (barrier +
  device sync on both sides, max over ranks) -> per-step device events of
  max(K, 20) more steps -> golden verification -> copy roofline -> the other
  scopes, each skipped once the wall-time budget is spent.

Hang-proofing: STRIPE_COMM_TIMEOUT_S defaults to 120 s here (every RCCL and
gloo wait is bounded by it), and a native "last words" watchdog on every rank
writes rank 0's record so far (the complete headline once it exists) and ends
the process when --budget-s runs out or torchrun stops the group with SIGTERM
after a peer died -- so the one JSON line prints well inside the driver's
600 s even if an extra scope hangs.

Scopes reported beside the headline ("resident": the frame stays in HBM):
  resident_warm   one frame iterated in place (cache-warm when it fits)
  resident_deep   (N > 1) deep halo: one exchange per k steps, k auto
  dist_*          root GPU frame -> scatter -> filter -> gather -> root GPU
                  (the reference's window, kernel.cu:135-225, device-resident)
  ref_window      the reference's exact window end, kernel.cu:190-226:
                  filter + D2H + gather into rank 0's host memory
  e2e             pinned host stripe -> H2D -> filter -> D2H -> pinned host,
                  with the same-box host-link roofline (H2D alone, D2H alone,
                  both at once) that explains it
Data: seeded synthetic random pixels (no dataset).

Prints ONE JSON line on rank 0 (driver contract).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import sys
import time

import numpy as np

METRIC = "Mpixels/sec, 5x5 Gaussian blur on 16384x16384 RGB at 1/2/4/8 MI355X"
BASELINE_MPX = None  # the reference publishes no number
MALL_BYTES = 256 << 20  # MI355X Infinity Cache
T_START = time.monotonic()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--width", type=int, default=16384)
    ap.add_argument("--height", type=int, default=16384)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--chain", default="gaussian5")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--band", type=int, default=0)
    ap.add_argument("--halo-schedule", default="auto",
                    choices=["auto", "serial", "overlap", "pipeline", "batched", "ahead", "serial+deep", "batched+deep",
                             "ahead+deep"],
                    help="halo schedule of the headline steps at N>1 (auto: time each on the real transport before "
                         "the timed region and keep the fastest, max over ranks; batched: serial steps with the "
                         "exchanges of the frames sharing a stream in one group per round; ahead: each frame's next "
                         "exchange posted right after its step on a communication stream of its own; +deep: "
                         "a frame exchanges k*S rows every k-th step, --halo-depth)")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames the headline steps over (0: auto -- enough to defeat the Infinity Cache when a "
                         "stripe fits it, else 2 at N>1 so one frame's exchange runs beside the other's filter, "
                         "else 1; 1: one frame iterated in place)")
    ap.add_argument("--streams", type=int, default=0,
                    help="streams the headline frames alternate over (0: auto -- at N>1 the probe times 1 and 2, else 2 "
                         "when frames rotate, so one frame's "
                         "kernel boundary overlaps the next frame's step; 1: strictly serial steps)")
    ap.add_argument("--deep-steps", type=int, default=-1, help="steps of the deep-halo scope (-1: --steps; 0: skip)")
    ap.add_argument("--halo-depth", type=int, default=0,
                    help="steps per deep-halo exchange (0: auto; 1: every step): the headline's deep schedules "
                         "(serial+deep, batched+deep, ahead+deep: a frame exchanges k*S rows every k-th step) and the "
                         "resident_deep scope")
    ap.add_argument("--dist-steps", type=int, default=5, help="steps of each dist-scope measurement (0: skip)")
    ap.add_argument("--ref-steps", type=int, default=3, help="steps of the ref-window measurement (0: skip)")
    ap.add_argument("--e2e-steps", type=int, default=3, help="steps of the e2e-scope measurement (0: skip)")
    ap.add_argument("--ref-shm", action="store_true",
                    help="ref-window host frame in POSIX shared memory even on one rank (tests the multi-rank path)")
    ap.add_argument("--self-halo", action="store_true",
                    help="N=1 only: the rank exchanges its boundary rows with itself through the one-rank RCCL "
                         "communicator (loopback) every step, the transfers an interior rank of an N>1 run makes; "
                         "the frame is then vertically periodic (verified against a periodic golden frame)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-autotune", action="store_true", help="skip the per-shape band / occupancy autotune")
    ap.add_argument("--budget-s", type=float, default=420.0,
                    help="wall-time budget: extra scopes are skipped after 60 %% of it, and the watchdog writes the "
                         "record and exits at 100 %%")
    ap.add_argument("--comm-timeout-s", type=float, default=120.0,
                    help="default of STRIPE_COMM_TIMEOUT_S (bound of every collective wait) for this run")
    ap.add_argument("--backend", default="rccl", choices=["rccl", "host", "gloo-gpu"],
                    help="rccl: GPU engine + RCCL (the benchmark); host: CPU golden engine + gloo (plumbing "
                         "tests); gloo-gpu: GPU engine, gloo transport through pinned host memory, processes may "
                         "share GPUs (the multi-rank device path on a one-GPU box)")
    return ap.parse_args()


def stats(ms):
    v = sorted(ms)
    if not v:
        return None
    return {"median": round(v[len(v) // 2], 5), "min": round(v[0], 5),
            "p90": round(v[min(len(v) - 1, int(math.ceil(0.9 * len(v))) - 1)], 5),
            "mean": round(sum(v) / len(v), 5), "n": len(v)}


def build_info(root):
    """What the in-tree native build was made from (the GPU box has no .git)."""
    info = {}
    try:
        with open(os.path.join(root, "mpi_cuda_imagemanipulation_amd", "_build_info.json")) as f:
            info = json.load(f)
        sys.path.insert(0, os.path.join(root, "tools"))
        import build as _b  # tools/build.py

        info["source_matches_build"] = _b.source_hash() == info.get("source_hash")
    except Exception as e:  # noqa: BLE001
        info["error"] = str(e)
    return info


def comm_counters(ctx) -> dict:
    """The communicator's host-side group counters (RCCL: groups, summed
    microseconds per grouped call); {} for transports without them."""
    if ctx.comm is None:
        return {}
    try:
        return {k: float(v) for k, v in ctx.comm.identity().items() if k.startswith("group")}
    except Exception:  # noqa: BLE001 - a transport without an identity
        return {}


def exchange_cost(before: dict, after: dict, steps: int) -> dict | None:
    """Host microseconds per grouped exchange over a timed region (the
    enqueue, ncclGroupEnd and the non-blocking progress poll), from two
    comm_counters snapshots."""
    n = after.get("groups", 0) - before.get("groups", 0)
    if n <= 0:
        return None
    us = after["group_us"] - before["group_us"]
    end = after.get("group_end_us", 0) - before.get("group_end_us", 0)
    return {"exchanges": int(n), "per_step": round(n / max(1, steps), 3), "host_us_per_exchange": round(us / n, 2),
            "group_end_us_per_exchange": round(end / n, 2), "host_us_per_step": round(us / max(1, steps), 2),
            "in_progress_ends": int(after.get("groups_in_progress", 0) - before.get("groups_in_progress", 0))}


def elapsed_s() -> float:
    return time.monotonic() - T_START


def main():
    a = parse()
    os.environ.setdefault("STRIPE_COMM_TIMEOUT_S", str(a.comm_timeout_s))
    # libraries (RCCL's init banner, HIP warnings) print to stdout; keep stdout for
    # the one JSON line of the driver contract and send everything else to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, root)
    from mpi_cuda_imagemanipulation_amd import parallel
    from mpi_cuda_imagemanipulation_amd._native import C
    from mpi_cuda_imagemanipulation_amd.models import Pipeline
    from mpi_cuda_imagemanipulation_amd.utils.log import get_logger

    rank_env = int(os.environ.get("RANK", "0"))
    # every rank: the watchdog ends a rank that outlives the budget; rank 0's
    # also writes the record (non-zero exit until the headline exists)
    C.last_words_arm(json_fd if rank_env == 0 else -1, max(30.0, a.budget_s - elapsed_s()) + (0 if rank_env == 0 else 15),
                     3)
    ctx = parallel.init({"rccl": "rccl", "host": "gloo", "gloo-gpu": "gloo-gpu"}[a.backend])
    log = get_logger("bench", ctx.rank)
    dev = ctx.device
    tdev = "cuda" if a.backend == "rccl" else "cpu"  # the process group's tensors

    def sync():
        if dev:
            torch.cuda.synchronize()
    world, rank = ctx.world, ctx.rank
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    W, H, Cc = a.width, a.height, a.channels

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_ok(ok: bool) -> bool:
        t = torch.tensor([1.0 if ok else 0.0], device=tdev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item() == 1.0)

    def from_root(vals):
        """rank 0's floats on every rank (so every rank plans the same split)"""
        t = torch.tensor(vals, dtype=torch.float64, device=tdev)
        if world > 1:
            dist.broadcast(t, 0)
        return [float(x) for x in t.tolist()]

    # ---- who is running: the transport's and the runtime's own view ----
    ids = parallel.world_identity(ctx)

    pinfo = C.plan_info(a.chain, Cc)
    iterable = pinfo["cin"] == pinfo["cout"]
    R = max(1, pinfo["max_radius"])
    # float conv passes (blur:K, conv:K) match the f64 golden within 1 LSB (ties)
    tol = 1 if any(p["kind"] == 3 for p in pinfo["passes"]) else 0

    def gold(band, n=1):
        for _ in range(n):
            band = C.golden_apply(band, a.chain, "reflect101", True)
        return band

    def same(x, y):
        return x.shape == y.shape and bool((np.abs(x.astype(np.int16) - y.astype(np.int16)) <= tol).all())

    def check_frame_rows(get_rows, cuts, n_it=1):
        """golden check of an assembled frame region: frame edges and the rows
        around every stripe boundary in `cuts` (get_rows(lo, hi) -> rows)"""
        reach = n_it * R
        crop = max(48, 4 * reach)
        ok = True
        for lo in (0, H - crop):
            if lo < 0:
                continue
            ref = gold(C.synth_rows(a.seed, W, Cc, lo, crop), n_it)
            sel = slice(0, crop - reach) if lo == 0 else slice(reach, crop)
            ok &= same(get_rows(lo, lo + crop)[sel], ref[sel])
        for c in cuts:
            lo = c - 2 * reach
            if 0 < c < H and lo >= 0 and c + 2 * reach <= H:
                ref = gold(C.synth_rows(a.seed, W, Cc, lo, 4 * reach), n_it)
                ok &= same(get_rows(lo, lo + 4 * reach)[reach:3 * reach], ref[reach:3 * reach])
        return ok

    part, active = C.plan_rows(H, world, R)
    max_rows = max(r for _, r in part)

    # ---- transport check (untimed): the headline's halo messages (R rows of
    # a stripe each way) around the ring through this run's communicator, in
    # the frame-stream pattern (4 frames over 2 streams), every word verified;
    # at N = 1 the RCCL communicator sends to and receives from itself ----
    transport = None
    if ctx.comm is not None and ctx.device:
        transport = dict(parallel.ring_check(ctx, 4 * (-(-R * W * Cc // 4)), frames=4, streams=2, iters=200),
                         peers="self (loopback)" if world == 1 else "ring r -> r+1")
        transport["errors"] = int(max_over_ranks(float(transport["errors"])))
        if transport["errors"]:
            log.error("transport check: %d corrupted words", transport["errors"])

    # ---- headline: a FrameStream (halo exchanged every step; when a stripe
    # fits the Infinity Cache, round-robin over enough frames that every step
    # reads HBM-cold data; consecutive frames on alternating streams) ----
    if a.self_halo and (world != 1 or a.backend != "rccl"):
        raise SystemExit("--self-halo needs one rank on the rccl backend (the communicator sends to itself)")
    if a.self_halo:
        # the ref-window and e2e scopes verify a non-periodic frame: not run here
        a.ref_steps = a.e2e_steps = 0
    # the frames' engines hold a deep halo (a.halo_depth, auto by default) so the
    # probe can time the deep schedules; the others exchange every step
    pipe1 = Pipeline(a.chain, overlap=not a.no_overlap, halo_depth=a.halo_depth, self_halo=a.self_halo)
    fs = parallel.FrameStream(ctx, pipe1, W, H, Cc, frames=a.frames, streams=a.streams, autotune=not a.no_autotune)
    ws_max, fits_mall, cold = fs.ws_max, fs.fits_mall, fs.cold
    nframes, nstreams = len(fs), fs.nstreams
    frames, streams = fs.frames, fs.streams
    stream = streams[0] if streams else None
    dp = fs.head
    if a.band > 0:
        dp.engine.set_tuning([a.band] * len(dp.engine.bands), [-1] * len(dp.engine.bands))
    row0, rows = dp.stripe
    fs.load_synthetic(a.seed)
    fs.tune(max_over_ranks)  # collective at N > 1: every rank decides on the slowest rank's timings
    # which halo schedule is fastest depends on the link and the transport's
    # per-exchange cost: at N>1 measure them here, untimed, on every rank
    # (N = 1 exchanges nothing, but runs the same frames x streams probe, so
    # every N of a scaling curve is measured in the same execution mode)
    if a.no_overlap and world > 1:
        fs.set_schedule("serial")
        sched = {"chosen": fs.schedule, "ms": {}, "requested": "serial"}
    elif a.halo_schedule != "auto" and (world > 1 or a.self_halo):
        fs.set_schedule(a.halo_schedule)
        sched = {"chosen": fs.schedule, "ms": {}, "requested": a.halo_schedule}
    else:
        sched = dict(fs.pick_schedule(max_over_ranks, barrier), requested="auto")
        if world == 1 and not a.self_halo:
            sched["chosen"] = "none (one rank: no exchange)"
    nstreams = fs.nstreams  # the probe may have settled on one stream (and picked the stream set)
    streams = fs.streams
    stream = streams[0] if streams else None
    log.info("halo schedule: %s on %d stream(s) %s", sched["chosen"], nstreams, sched["ms"])
    step = fs.step
    sync_frames = fs.synchronize
    frame_stream = fs.stream_of

    for i in range(a.warmup):
        step(i)
    sync_frames()
    sync()
    barrier()
    sync()
    comm_before = comm_counters(ctx)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    t_issue = time.perf_counter()  # the host's issue time (no sync yet): near t1 - t0 means host-bound steps
    sync_frames()
    sync()
    barrier()
    t1 = time.perf_counter()
    comm_after = comm_counters(ctx)
    ms = max_over_ranks((t1 - t0) * 1e3)
    ms_per_step = ms / a.steps
    mpx = W * H / (ms_per_step * 1e-3) / 1e6
    log.info("resident: %.5f ms/step over %d steps (%d frame(s), %d stream(s))", ms_per_step, a.steps, nframes,
             nstreams)

    # per-step device time distribution: an event on the step's stream after
    # each step, max(K, 20) steps, untimed by the host clock above (the events
    # themselves add a few us a step)
    step_ms = None
    if dev and rows > 0:
        n_ev = max(a.steps, 20)
        sync()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev + 1)]
        ev[0].record(stream)
        for st in streams[1:]:
            st.wait_event(ev[0])
        for i in range(n_ev):
            step(i)
            ev[i + 1].record(frame_stream(i))
        sync_frames()
        sync()
        # with s streams consecutive steps overlap: a step's time is the span
        # between two events on the SAME stream divided by the steps between
        # them.  Step i runs on stream (i mod F) mod s, so i and i + s share a
        # stream when s divides the frame count F; otherwise i and i + F do
        # (s = 1: the plain delta)
        w = nstreams if nframes % nstreams == 0 else nframes
        assert all(frame_stream(i) is frame_stream(i + w) for i in range(n_ev - w + 1))
        step_ms = stats([ev[i].elapsed_time(ev[i + w]) / w for i in range(n_ev - w + 1)])
    # device-event stage times of one step of frame 0 on rank 0
    dp.engine.stage_timing = True
    step(0)
    dp.synchronize()
    stages = {"resident": {k: round(v, 4) for k, v in dp.stage_times().items() if k in ("compute", "halo")}}

    def ramp(ms_target=30.0):
        """GPU clock ramp before a timed scope: the host-side checks between
        scopes leave the GPU idle long enough to drop its clock"""
        if not dev or rows == 0:
            return
        n = max(1, int(ms_target / max(1e-3, ms_per_step)))
        for i in range(min(n, 2000)):
            step(i)
        sync_frames()

    # ---- correctness of the timed engine (untimed, after the timed region):
    # n_it iterated steps through the same schedule vs the golden path on edge
    # crops and on this stripe's upper seam ----
    def torus_rows(lo, n):
        """frame rows lo .. lo + n - 1 modulo H (the self-halo frame is vertically periodic)"""
        parts, y = [], lo
        while y < lo + n:
            r = y % H
            k = min(H - r, lo + n - y)
            parts.append(C.synth_rows(a.seed, W, Cc, r, k))
            y += k
        return np.concatenate(parts, axis=0)

    verify = None
    if not a.no_verify and a.self_halo:
        n_it = 2 if iterable else 1
        dp.load_synthetic(a.seed)
        dp.run(n_it)
        out = dp.result_stripe()
        reach = n_it * R
        crop = max(48, 4 * reach)
        ok = True
        for lo in (0, H - crop):  # both frame edges read the other edge's rows through the exchange
            ref = gold(torus_rows(lo - reach, crop + 2 * reach), n_it)[reach:reach + crop]
            ok &= same(out[lo:lo + crop], ref)
        verify = all_ok(ok)
    elif not a.no_verify:
        n_it = 2 if iterable else 1
        dp.load_synthetic(a.seed)
        dp.run(n_it)
        out = dp.result_stripe()
        ok = True
        reach = n_it * R
        crop = max(48, 4 * reach)
        edges = ([0] if row0 == 0 else []) + ([H - crop] if row0 + rows == H else [])
        for lo in [e for e in edges if row0 <= e and e + crop <= row0 + rows]:  # crops inside this stripe
            # golden on a band of full rows; rows far enough from the band edge are exact
            ref = gold(C.synth_rows(a.seed, W, Cc, lo, crop), n_it)
            sel = slice(0, crop - reach) if lo == 0 else slice(reach, crop)
            ok &= same(out[lo - row0:lo - row0 + crop][sel], ref[sel])
        if rows >= reach and row0 >= 2 * reach and row0 + 2 * reach <= H:
            # interior stripe seam: the first rows depend on the neighbour's halo
            ref = gold(C.synth_rows(a.seed, W, Cc, row0 - 2 * reach, 4 * reach), n_it)
            ok &= same(out[0:reach], ref[2 * reach:3 * reach])
        verify = all_ok(ok)

    # the other scopes run one step per input (or their own schedule): the
    # head engine leaves the deep block here
    head_depth = fs.depth if fs.deep else 1
    fs.set_deep(False)

    # ---- same-box roofline: the framework's hand-written linear copy of the
    # same bytes per step (csrc/hip/pointwise.hip k_copy_linear: one 16-byte
    # chunk per lane, the faster of two store policies), rotating over enough
    # buffer pairs that every copy reads cache-cold data, like the headline ----
    bytes_in = rows * W * pinfo["cin"]
    bytes_out = rows * W * pinfo["cout"]
    step_bytes = bytes_in + bytes_out
    copy = None
    if dev and rows > 0:
        n = step_bytes // 2
        copy = C.copy_roofline(ctx.gpu, n, max(1, -(-3 * MALL_BYTES // (2 * n))), 20)
        torch.cuda.empty_cache()
    copy_ms = copy["event_ms"] if copy else None

    scopes = {"resident": {"mpx_s": round(mpx, 1), "ms": round(ms_per_step, 5), "verified": verify,
                           "frames": nframes, "streams": nstreams, "halo_depth": head_depth, "cache": fs.cache}}
    med = step_ms["median"] if step_ms else None
    rec = {
        "metric": METRIC,
        "value": round(mpx, 1),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None if BASELINE_MPX is None else round(mpx / BASELINE_MPX, 3),
        "dtype": "uint8 (int32 accumulate, exact)",
        "backend": a.backend,
        "data": "synthetic (seeded random pixels)",
        "config": {
            "model": a.chain,
            "image": f"{W}x{H}x{Cc}",
            "global_batch": 1,
            "seq_len": H,
            "parallelism": f"rowpart{world}+halo",
            "scope": (("resident: halo exchange every step + full-frame filter per step" if world > 1 else
                       "resident: self-halo -- the rank exchanges its boundary rows with itself through the one-rank "
                       "RCCL communicator every step (vertically periodic frame) + full-frame filter per step"
                       if a.self_halo else "resident: full-frame filter per step (one rank: no halo exchange)")
                      + (f", round-robin over {nframes} frames so every step reads HBM-cold data" if cold else
                         (f", round-robin over {nframes} independent frames" if nframes > 1 else ""))
                      + (f", consecutive frames on {nstreams} alternating streams" if nstreams > 1 else "")),
        },
        "verified_vs_golden": verify,
        # rank 0's per-step device time (HIP events between steps) and the
        # same-box hand-written copy of the same per-GPU bytes (read + write):
        # per copy (events between copies, vs step_ms_device) and back to back
        # (burst, vs the host-clock ms_per_step)
        "step_ms_device": step_ms,
        # rank 0's host time to issue the K timed steps, per step (the GPU
        # time is ms_per_step: a host issue time close to it means the host
        # loop, not the GPU, sets the step)
        "host_issue_ms_per_step": round((t_issue - t0) * 1e3 / a.steps, 5),
        "bytes_per_step_per_gpu": step_bytes,
        "copy_roofline_ms": None if copy_ms is None else round(copy_ms, 5),
        "frac_of_copy_roofline": None if not (copy_ms and med) else round(copy_ms / med, 4),
        "copy_burst_ms": None if not copy else round(copy["burst_ms"], 5),
        "frac_of_copy_burst": None if not copy else round(copy["burst_ms"] / ms_per_step, 4),
        "copy_roofline": copy,
        "hbm_tb_s": None if not med else round(step_bytes / (med * 1e-3) / 1e12, 3),
        "working_set_fits_mall": fits_mall,
        "frames": nframes,
        "streams": nstreams,
        "scopes": scopes,
        "tuned": {"band_rows": dp.engine.bands, "occupancy_caps": dp.engine.caps, "policies": dp.engine.policies,
                  "task_orders": dp.engine.orders,
                  "cold": cold, "streaming_policy": fs.streaming},
        "cache": fs.cache,
        "halo_depth": head_depth,
        "halo_schedule": sched,
        "self_halo": bool(a.self_halo),
        "exchange_cost": exchange_cost(comm_before, comm_after, a.steps),
        "transport_check": transport,
        "stripe_rows": [r for _, r in part],
        "stage_ms_rank0": stages,
        "world": {"summary": parallel.identity_summary(ids), "ranks": ids},
        "device": C.device_info(ctx.gpu) if dev else {},
        "build": build_info(root),
        "host": socket.gethostname(),
        "torch": torch.__version__,
        "budget": {"budget_s": a.budget_s, "comm_timeout_s": float(os.environ["STRIPE_COMM_TIMEOUT_S"]),
                   "skipped": []},
    }

    def publish(final=False):
        """rank 0: the record so far becomes the watchdog's last words (exit 0:
        the headline is complete)"""
        if rank == 0:
            rec["elapsed_s"] = round(elapsed_s(), 1)
            if not final:
                rec["partial"] = "the wall-time budget ran out or the group was stopped during the extra scopes"
            else:
                rec.pop("partial", None)
            C.last_words_set(json.dumps(rec), 0)

    publish()

    def guarded(name, fn):
        """run one extra scope unless the budget is spent; an exception is
        reported in the record (after every rank agrees the scope failed)
        instead of ending the run without the headline line"""
        # every rank takes the same decision (rank 0's clock)
        if from_root([1.0 if elapsed_s() > 0.6 * a.budget_s else 0.0])[0] > 0:
            rec["budget"]["skipped"].append(name)
            return
        ok, err = True, None
        try:
            fn()
        except Exception as e:  # noqa: BLE001
            ok, err = False, f"{type(e).__name__}: {e}"
            log.error("scope %s failed: %s", name, err)
        if not all_ok(ok):
            scopes.setdefault(name, {})["error"] = err or "failed on another rank"
        publish()

    def scope_warm():
        # ---- one frame iterated in place, halo every step (cache-warm when
        # the working set fits the Infinity Cache) ----
        if nframes == 1 or not iterable:
            return
        ramp()
        we = dp
        if dp.engine.halo_depth > 1:  # run(n) would run a deep block: this scope exchanges every step
            we = parallel.DistributedPipeline(ctx, Pipeline(a.chain, overlap=not a.no_overlap, halo_depth=1), W, H, Cc)
            we.engine.set_tuning(dp.engine.bands, dp.engine.caps, dp.engine.policies, dp.engine.orders)
            we.load_synthetic(a.seed)
            we.run(2)
            we.synchronize()
        sync()
        barrier()
        t0 = time.perf_counter()
        we.run(a.steps)
        we.synchronize()
        sync()
        barrier()
        wms = max_over_ranks((time.perf_counter() - t0) * 1e3) / a.steps
        del we
        scopes["resident_warm"] = {"mpx_s": round(W * H / (wms * 1e-3) / 1e6, 1), "ms": round(wms, 5),
                                   "frames": 1, "halo_depth": 1}

    def scope_deep():
        # ---- communication-avoiding deep halo: one exchange of k*S rows per
        # k steps (bit-identical), one frame ----
        deep_steps = a.steps if a.deep_steps < 0 else a.deep_steps
        if world == 1 or not iterable or deep_steps <= 0:
            return
        dd = parallel.DistributedPipeline(ctx, Pipeline(a.chain, overlap=not a.no_overlap, halo_depth=a.halo_depth),
                                          W, H, Cc)
        k = dd.engine.halo_depth
        if k <= 1:
            scopes["resident_deep"] = {"same_as": "resident_warm", "halo_depth": k}
            return
        dd.engine.set_tuning(dp.engine.bands, dp.engine.caps, dp.engine.policies, dp.engine.orders)
        n = k * int(math.ceil(deep_steps / k))  # whole exchange blocks
        dd.load_synthetic(a.seed)
        dd.run(2 * k)
        dd.synchronize()
        sync()
        barrier()
        t0 = time.perf_counter()
        dd.run(n)
        dd.synchronize()
        sync()
        barrier()
        dms = max_over_ranks((time.perf_counter() - t0) * 1e3) / n
        calls = dd.engine.run_timed(max(n, 20 * k), k, False) if dev and rows > 0 else []
        scopes["resident_deep"] = {"mpx_s": round(W * H / (dms * 1e-3) / 1e6, 1), "ms": round(dms, 5),
                                   "halo_depth": k, "steps": n, "frames": 1,
                                   "step_ms_device": stats([c / k for c in calls])}
        del dd

    def scope_dist():
        # ---- dist scopes (root frame -> scatter -> filter -> gather -> root) ----
        dist_chunks = 0
        if a.dist_steps > 0:
            pipe = Pipeline(a.chain, overlap=not a.no_overlap)
            dd = parallel.DistributedPipeline(ctx, pipe, W, H, Cc, root_buffers=True)
            dd.engine.set_tuning(dp.engine.bands, dp.engine.caps)
            if rank == 0:
                dd.engine.load_root_synthetic(a.seed)
            dd.synchronize()

            def verify_root(d, cuts):
                if rank != 0:
                    return all_ok(True)
                full = d.engine.store_root()
                return all_ok(check_frame_rows(lambda lo, hi: full[lo:hi], cuts))

            def time_dist(d, step_fn):
                ramp()
                for _ in range(2):
                    step_fn()
                d.synchronize()
                sync()
                barrier()
                t0 = time.perf_counter()
                for _ in range(a.dist_steps):
                    step_fn()
                d.synchronize()
                sync()
                barrier()
                return max_over_ranks((time.perf_counter() - t0) * 1e3) / a.dist_steps

            def seq_step():
                dd.scatter()
                dd.run(1)
                dd.gather()

            cuts = [r0 for r0, r in part[1:active]]
            seq_step()
            dd.synchronize()
            ok = verify_root(dd, cuts) if not a.no_verify else None
            dms = time_dist(dd, seq_step)
            scopes["dist_sequential"] = {"mpx_s": round(W * H / (dms * 1e-3) / 1e6, 1), "ms": round(dms, 5),
                                         "verified": ok}
            stages["dist_sequential"] = {k: round(v, 4) for k, v in dd.stage_times().items()
                                         if k in ("scatter", "compute", "halo", "gather")}
            # (device ranks only: host comms run each grouped call synchronously)
            dist_chunks = dd.engine.dist_chunks(8) if dev else 0
            direct = dev and world == 1 and dd.engine.dist_direct
            if dist_chunks > 0 or direct:
                name = "dist_direct" if direct else "dist_pipelined"
                dd.engine.run_dist(8)
                dd.synchronize()
                ok = verify_root(dd, cuts) if not a.no_verify else None
                dms = time_dist(dd, lambda: dd.engine.run_dist(8))
                scopes[name] = {"mpx_s": round(W * H / (dms * 1e-3) / 1e6, 1), "ms": round(dms, 5), "verified": ok,
                                "chunks": dist_chunks, "rows": [r for _, r in part]}
                stages[name] = {k: round(v, 4) for k, v in dd.stage_times().items()
                                if k in ("scatter", "compute", "gather")}
            del dd
            # link-aware weighted split: the root keeps the share that balances its
            # in-place filter against each peer link's transfer time
            if world > 1 and dev and pinfo["passes"] and len(pinfo["passes"]) == 1:
                link = C.probe_link_rate(ctx.comm, ctx.gpu, 64 << 20, 3)  # bytes/ms per link, one way
                rows_per_ms = rows / step_ms["median"] if step_ms else 1.0
                # bytes / ms the root's HBM sustains: the faster of a copy and this filter
                hbm = step_bytes / min(copy_ms, step_ms["median"]) if copy_ms and step_ms else 1.0
                rows_per_ms, link, hbm = from_root([rows_per_ms, link, hbm])
                plan = C.plan_dist_split(H, world, W * pinfo["cin"], W * pinfo["cout"], rows_per_ms, rows_per_ms,
                                         link, hbm, 8, R)
                dw = parallel.DistributedPipeline(ctx, pipe, W, H, Cc, root_buffers=True, row_weights=plan["weights"])
                if dw.engine.dist_chunks(8) > 0:
                    dw.engine.set_tuning(dp.engine.bands, dp.engine.caps)
                    if rank == 0:
                        dw.engine.load_root_synthetic(a.seed)
                    dw.engine.run_dist(8)
                    dw.synchronize()
                    wcuts = list(np.cumsum(plan["rows"])[:-1])
                    ok = verify_root(dw, [int(c) for c in wcuts]) if not a.no_verify else None
                    dms = time_dist(dw, lambda: dw.engine.run_dist(8))
                    scopes["dist_weighted"] = {
                        "mpx_s": round(W * H / (dms * 1e-3) / 1e6, 1), "ms": round(dms, 5), "verified": ok,
                        "rows": plan["rows"], "link_gb_s": round(link * 1e3 / 1e9, 2),
                        "model": {k: round(plan[k], 5) for k in ("root_ms", "peer_ms", "floor_ms", "predicted_ms",
                                                                 "even_ms")}}
                    stages["dist_weighted"] = {k: round(v, 4) for k, v in dw.stage_times().items()
                                               if k in ("scatter", "compute", "gather")}
                del dw

    def scope_ref():
        # ---- reference window: filter + D2H + gather into rank 0's host memory
        # (kernel.cu:190-226).  Every rank downloads its stripe, chunk by chunk as
        # it is filtered, into its slice of one host frame shared with rank 0
        # (POSIX shared memory, page-locked in every process: each GPU's own PCIe
        # link carries its stripe, and no host copy follows). ----
        if a.ref_steps > 0 and dev:
            from multiprocessing import shared_memory

            nbytes = H * W * pinfo["cout"]
            shm = None
            if world > 1 or a.ref_shm:
                # the frame lives in /dev/shm: a tmpfs smaller than the frame
                # would SIGBUS on first touch (no exception to guard), so rank 0
                # checks the free space and every rank follows its decision
                try:
                    st = os.statvfs("/dev/shm")
                    free = st.f_bavail * st.f_frsize
                except OSError:
                    free = 0
                if from_root([1.0 if free >= nbytes + (64 << 20) else 0.0])[0] < 1.0:
                    scopes["ref_window"] = {"skipped": f"/dev/shm has {free} B free, the host frame needs {nbytes} B"}
                    return
                names = [f"stripe_refwin_{os.getpid()}" if rank == 0 else None]
                if world > 1:
                    dist.broadcast_object_list(names, src=0)
                if rank == 0:
                    shm = shared_memory.SharedMemory(name=names[0], create=True, size=nbytes)
                barrier()
                if rank != 0:
                    shm = shared_memory.SharedMemory(name=names[0])
                frame = np.ndarray((nbytes,), dtype=np.uint8, buffer=shm.buf)
            else:
                frame_t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)  # keeps the pages alive
                frame = frame_t.numpy()
            base = frame.ctypes.data
            pinned = shm is None or C.host_register(base, nbytes)
            mine = base + row0 * W * pinfo["cout"]
            try:
                dp.load_synthetic(a.seed)
                dp.synchronize()
                dp.engine.run_to_host_ptr(mine, 8)
                dp.synchronize()
                barrier()
                ok = None
                full = None
                if not a.no_verify:
                    full = frame.reshape(H, W, -1) if pinfo["cout"] > 1 else frame.reshape(H, W)
                    ok = all_ok(rank != 0 or check_frame_rows(lambda lo, hi: full[lo:hi],
                                                              [r0 for r0, _ in part[1:active]]))
                ramp()
                dp.engine.run_to_host_ptr(mine, 8)
                dp.synchronize()
                sync()
                barrier()
                t0 = time.perf_counter()
                for _ in range(a.ref_steps):
                    dp.engine.run_to_host_ptr(mine, 8)
                    dp.synchronize()
                    barrier()  # rank 0's window ends when every stripe is in its memory
                rms = max_over_ranks((time.perf_counter() - t0) * 1e3) / a.ref_steps
                scopes["ref_window"] = {"mpx_s": round(W * H / (rms * 1e-3) / 1e6, 1), "ms": round(rms, 5),
                                        "verified": ok, "host_frame": "shared memory" if shm is not None else "pinned",
                                        "pinned": bool(pinned)}
                stages["ref_window"] = {k: round(v, 4) for k, v in dp.stage_times().items()
                                        if k in ("compute", "d2h", "e2e")}
            finally:
                if shm is not None:
                    if pinned:
                        C.host_unregister(base)
                    del frame
                    full = None
                    barrier()
                    shm.close()
                    if rank == 0:
                        shm.unlink()

    def host_link(nbytes: int) -> dict:
        """Same-box pinned host <-> device rates on this rank's stripe bytes,
        the way run_e2e moves them (8 row chunks per direction on the copy
        engines): H2D alone, D2H alone, and both directions at once (two
        streams, chunks interleaved), GB/s per direction, median of 3.  The e2e
        scope cannot beat the concurrent time of its bytes."""
        h_src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        h_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        d_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        d_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        s_up, s_down = torch.cuda.Stream(), torch.cuda.Stream()
        cuts = [nbytes * i // 8 for i in range(9)]

        def timed(up, down):
            res = []
            for _ in range(4):
                sync()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                e[0].record(s_up)
                e[2].record(s_down)
                for i in range(8):
                    lo, hi = cuts[i], cuts[i + 1]
                    if up:
                        with torch.cuda.stream(s_up):
                            d_a[lo:hi].copy_(h_src[lo:hi], non_blocking=True)
                    if down:
                        with torch.cuda.stream(s_down):
                            h_dst[lo:hi].copy_(d_b[lo:hi], non_blocking=True)
                e[1].record(s_up)
                e[3].record(s_down)
                sync()
                res.append((e[0].elapsed_time(e[1]) if up else 0.0, e[2].elapsed_time(e[3]) if down else 0.0))
            res = res[1:]
            return [sorted(r[i] for r in res)[len(res) // 2] for i in (0, 1)]

        h2d_ms, _ = timed(True, False)
        _, d2h_ms = timed(False, True)
        both_up, both_down = timed(True, True)
        gbs = lambda ms: round(nbytes / (ms * 1e-3) / 1e9, 2) if ms > 0 else None  # noqa: E731
        both = max(both_up, both_down)
        out = {"bytes": nbytes, "chunks": 8, "h2d_gb_s": gbs(h2d_ms), "d2h_gb_s": gbs(d2h_ms),
               "both_h2d_gb_s": gbs(both_up), "both_d2h_gb_s": gbs(both_down),
               "h2d_ms": round(h2d_ms, 3), "d2h_ms": round(d2h_ms, 3), "both_ms": round(both, 3),
               # 1.0: the directions overlap fully; 2.0: they take turns
               "both_over_one_way": round(both / max(h2d_ms, d2h_ms), 3)}
        del h_src, h_dst, d_a, d_b
        torch.cuda.empty_cache()
        return out

    def scope_e2e():
        # ---- e2e scope (pinned host stripe -> H2D -> filter -> D2H -> pinned host) ----
        if a.e2e_steps > 0 and dev:
            ramp()
            eng = dp.engine
            eng.alloc_host_io()
            if rows > 0:
                eng.host_input()[...] = C.synth_rows(a.seed, W, Cc, row0, rows)
            eng.run_e2e(8)
            eng.synchronize()
            # row chunks of the upload / filter / download pipeline: its fill
            # and drain cost about one chunk each way, so more chunks pay where
            # the link overlaps the two directions and cost per-chunk overhead
            # where it does not (profiles/r5/e2e/): time 8, 16 and 32 (max
            # over ranks), keep the fastest
            chunk_ms = {}
            for ch in (8, 16, 32):
                barrier()
                t0 = time.perf_counter()
                for _ in range(2):
                    eng.run_e2e(ch)
                eng.synchronize()
                chunk_ms[ch] = max_over_ranks((time.perf_counter() - t0) * 1e3 / 2)
            chunks = min(chunk_ms, key=chunk_ms.get)
            barrier()
            t0 = time.perf_counter()
            for _ in range(a.e2e_steps):
                eng.run_e2e(chunks)
            eng.synchronize()
            barrier()
            ems = max_over_ranks((time.perf_counter() - t0) * 1e3) / a.e2e_steps
            scopes["e2e"] = {"mpx_s": round(W * H / (ems * 1e-3) / 1e6, 1), "ms": round(ems, 5), "chunks": chunks,
                             "chunk_probe_ms": {str(k): round(v, 3) for k, v in chunk_ms.items()}}
            stages["e2e"] = {k: round(v, 4) for k, v in dp.stage_times().items()
                             if k in ("h2d", "compute", "halo", "d2h", "e2e")}
            if rows > 0:
                hl = host_link(max(bytes_in, bytes_out))
                # the floor the link allows this scope: both directions' bytes in flight together
                hl["e2e_floor_ms"] = hl["both_ms"]
                hl["e2e_frac_of_floor"] = round(hl["both_ms"] / ems, 3) if ems > 0 else None
                scopes["e2e"]["host_link_rank0"] = hl

    try:
        for name, fn in (("resident_warm", scope_warm), ("resident_deep", scope_deep), ("dist", scope_dist),
                         ("ref_window", scope_ref), ("e2e", scope_e2e)):
            guarded(name, fn)
    except Exception as e:  # noqa: BLE001 - a collective between scopes failed (a peer died or stalled)
        log.error("extra scopes abandoned: %s: %s", type(e).__name__, e)
        rec["budget"]["abandoned"] = f"{type(e).__name__}: {e}"[:300]
        if rank == 0:
            publish()
            C.last_words_emit()  # the headline is complete: report it, then leave
            C.last_words_disarm()
            sys.stderr.flush()
            os._exit(0)
        raise

    publish(final=True)
    if rank == 0:
        C.last_words_emit()
    C.last_words_disarm()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
