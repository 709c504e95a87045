"""Row-partitioned distributed execution (one process per GPU).

Reference: MPI_Init / Comm_rank / Comm_size, Barrier, Bcast of 4 ints,
Scatter, Gather, Finalize on MPI_COMM_WORLD over host buffers
(kernel.cu:104-137,223-225,250), all ranks on GPU 0 (kernel.cu:147), no halo
exchange (seams, Q6), remainder rows dropped (Q7).

Here: torch.distributed provides the process group/rendezvous (torchrun env),
the native engine owns an RCCL communicator (ncclCommInitRank; the unique id is
broadcast through torch.distributed) and moves stripes device-to-device over
xGMI: grouped ncclSend/ncclRecv scatter/gather and a neighbour halo exchange
overlapped with the interior compute.  On CPU-only hosts the same engine runs
the golden path and moves halos through gloo (callback communicator).
"""
from __future__ import annotations

import ctypes
import datetime
import json
import os
import socket
import threading
import time
from dataclasses import dataclass

import numpy as np

from .._native import C
from ..utils.log import get_logger

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None


@dataclass
class DistContext:
    rank: int
    world: int
    local_rank: int
    device: bool          # True: GPU engine (RCCL, or gloo staged through host); False: host engine + gloo
    comm: object          # native Comm handle (None when world == 1)
    gpu: int = -1         # device index of this rank's engine (-1: host engine)
    transport: str = ""   # rccl | gloo | gloo-gpu


def plan_rows(H: int, world: int, min_rows: int = 1, legacy: bool = False):
    """[(row0, rows)] per rank and the number of active ranks (uneven split by default)."""
    return C.plan_rows(H, world, min_rows, legacy)


def _host_view(ptr: int, n: int) -> "torch.Tensor":
    buf = (ctypes.c_uint8 * n).from_address(ptr)
    return torch.from_numpy(np.frombuffer(buf, dtype=np.uint8, count=n))


class GlooComm:
    """Callback communicator: the engine's grouped send/recv on host buffers,
    executed as torch.distributed P2P ops (gloo).

    group_end only posts the batch; the native side polls `poll` under
    STRIPE_COMM_TIMEOUT_S (the same bounded state machine as the non-blocking
    RCCL communicator), so a peer that never posts its half fails the group
    with a message instead of blocking it."""

    def __init__(self, group=None):
        self.group = group
        self.ops = []
        # state of the latest group_end: [done Event, error]; each group gets
        # its own pair, bound into its waiter thread, so a waiter left over from
        # a group the native side abandoned (timeout) can never mark a later
        # group done
        done = threading.Event()
        done.set()
        self._state = [done, None]

    def group_start(self):
        self.ops = []

    def send(self, ptr, n, peer):
        self.ops.append(dist.P2POp(dist.isend, _host_view(ptr, n), peer, self.group))

    def recv(self, ptr, n, peer):
        self.ops.append(dist.P2POp(dist.irecv, _host_view(ptr, n), peer, self.group))

    def group_end(self):
        works = dist.batch_isend_irecv(self.ops) if self.ops else []
        self.ops = []
        state = [threading.Event(), None]  # this group's own done flag and error slot
        self._state = state
        if not works:
            state[0].set()
            return
        # gloo p2p works only progress inside wait(): a helper thread waits on
        # them and `poll` reads its state (a stalled peer leaves the helper
        # blocked until the process group's own timeout; the native side has
        # given up and raised by then)

        def waiter(works=works, state=state):
            try:
                for w in works:
                    w.wait()
            except Exception as e:  # noqa: BLE001 - reported to the native side as a failed group
                state[1] = e
            finally:
                state[0].set()

        threading.Thread(target=waiter, daemon=True).start()

    @property
    def done(self) -> threading.Event:
        return self._state[0]

    @property
    def err(self):
        return self._state[1]

    def poll(self) -> int:
        """0: every posted op of the latest group completed, 1: pending, 2: an op failed."""
        done, err = self._state
        if not done.is_set():
            return 1
        return 2 if err is not None else 0

    def barrier(self):
        dist.barrier(group=self.group)

    def native(self, rank: int, world: int):
        return C.make_callback_comm(rank, world, self.group_start, self.send, self.recv, self.group_end,
                                    self.barrier, self.poll)


def init(backend: str = "auto") -> DistContext:
    """Initialise from torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    backend: 'rccl' (GPU engine, RCCL comm), 'gloo' (host engine),
    'gloo-gpu' (GPU engine, gloo transport staged through pinned host memory:
    processes may share GPUs -- rank r on GPU r mod count -- like the
    reference's MPI ranks all on GPU 0, kernel.cu:147), or 'auto'.
    """
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if backend == "auto":
        backend = "rccl" if (torch is not None and torch.cuda.is_available()) else "gloo"
    if backend not in ("rccl", "gloo", "gloo-gpu"):
        raise ValueError(f"unknown backend {backend!r} (rccl | gloo | gloo-gpu | auto)")
    device = backend != "gloo"
    gpu = -1
    if device:
        gpu = local_rank if backend == "rccl" else local_rank % max(1, torch.cuda.device_count())
    log = get_logger("parallel", rank)
    log.info("init: rank %d of %d, local rank %d, backend %s", rank, world, local_rank, backend)
    if device:
        torch.cuda.set_device(gpu)
    comm = None
    if device and world == 1:
        # a one-rank RCCL communicator: no traffic, but the same comm object,
        # bounded waits and barrier as the multi-rank path (exercised on 1-GPU boxes)
        comm = C.make_rccl_comm(C.rccl_unique_id(), 0, 1, gpu)
    if world > 1:
        if not dist.is_initialized():
            # the process-group timeout follows the native collective bound
            # (STRIPE_COMM_TIMEOUT_S): a dead peer surfaces as an error, not a hang
            dist.init_process_group("nccl" if backend == "rccl" else "gloo", rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=C.comm_timeout_s()))
        if backend == "rccl":
            uid = [C.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = C.make_rccl_comm(uid[0], rank, world, gpu)
        elif backend == "gloo-gpu":
            comm = C.make_staged_comm(GlooComm().native(rank, world), gpu)
        else:
            comm = GlooComm().native(rank, world)
    log.info("communicator ready (%s)", backend if world > 1 else ("rccl" if device else "none"))
    return DistContext(rank, world, local_rank, device, comm, gpu, backend)


def rank_identity(ctx: DistContext) -> dict:
    """What this rank's transport and runtime say about it: the communicator's
    own view (RCCL: ncclCommCount / ncclCommCuDevice / ncclCommUserRank and the
    bounded init / pre-connect times), the GPU's PCI address, and the HIP
    runtime / RCCL libraries actually mapped into the process."""
    d = {"rank": ctx.rank, "world": ctx.world, "transport": ctx.transport, "gpu": ctx.gpu,
         "host": socket.gethostname(), "pid": os.getpid()}
    if ctx.comm is not None:
        d["comm"] = {k: (int(v) if float(v).is_integer() else round(float(v), 3)) for k, v in ctx.comm.identity().items()}
    if ctx.device:
        info = C.device_info(ctx.gpu)
        d["pci"] = info.get("pci")
        d["hip_runtime"] = info.get("hip_runtime")
    d["rccl_version"] = C.rccl_version()
    d["libs"] = C.runtime_libs()
    return d


def world_identity(ctx: DistContext) -> list:
    """rank_identity of every rank, gathered on every rank (rank order)."""
    mine = rank_identity(ctx)
    if ctx.world == 1:
        return [mine]
    out = [None] * ctx.world
    dist.all_gather_object(out, mine)
    return out


def identity_summary(ids: list) -> dict:
    """Checks over world_identity(): one distinct GPU per rank, the
    communicator's rank count equal to the world size on every rank, and one
    copy of each runtime library per process, the same everywhere."""
    pcis = [(i.get("host"), i.get("pci")) for i in ids]
    counts = {i.get("comm", {}).get("nccl_count") for i in ids}
    libsets = {json.dumps(i.get("libs"), sort_keys=True) for i in ids}
    one_copy = all(len(v) <= 1 for i in ids for v in (i.get("libs") or {}).values())
    return {"ranks": len(ids), "distinct_gpus": len(set(pcis)), "nccl_count": sorted(c for c in counts if c is not None),
            "devices": [i.get("comm", {}).get("nccl_device", i.get("gpu")) for i in ids],
            "same_libs_everywhere": len(libsets) == 1, "one_copy_per_lib": one_copy}


class DistributedPipeline:
    """Per-rank handle on the native engine for one image geometry."""

    def __init__(self, ctx: DistContext, pipeline, W: int, H: int, Cc: int = 3, root_buffers: bool = False,
                 autotune: bool = False, row_weights=None, cold: bool = False):
        self.ctx = ctx
        cfg = pipeline.config(W, H, Cc, "device" if ctx.device else "host",
                              device=ctx.gpu if ctx.device else -1, autotune=autotune, row_weights=row_weights)
        cfg.root_buffers = root_buffers
        cfg.cold = bool(cold)  # stream of cache-cold frames: streaming policy, cold autotune
        self.engine = C.Engine(cfg, ctx.comm)
        self.W, self.H, self.C = W, H, Cc

    @property
    def stripe(self):
        return self.engine.stripe

    def stage_times(self) -> dict:
        """Milliseconds of the last call of each stage (device events / host clock)."""
        return self.engine.times.as_dict()

    def load_synthetic(self, seed: int):
        self.engine.load_synthetic(seed)

    def load_stripe(self, stripe: np.ndarray):
        self.engine.load_packed(np.ascontiguousarray(stripe, dtype=np.uint8))

    def load_root(self, full: np.ndarray):
        if self.ctx.rank == 0:
            self.engine.load_root(np.ascontiguousarray(full, dtype=np.uint8))

    def scatter(self):
        self.engine.scatter()

    def run(self, iterations: int = 1):
        self.engine.run(iterations)

    def gather(self):
        self.engine.gather()

    def result_root(self):
        return self.engine.store_root() if self.ctx.rank == 0 else None

    def result_stripe(self):
        return self.engine.store_packed()

    def synchronize(self):
        self.engine.synchronize()

    def use_stream(self, stream_handle: int):
        """Queue this engine's work on an external HIP stream (e.g. a torch
        stream shared by several engines, which then run in issue order)."""
        self.engine.use_external_stream(int(stream_handle))


MALL_BYTES = 256 << 20  # MI355X Infinity Cache


class _PlainStreams:
    """Plain (non-blocking) HIP streams owned by a frame stream's frames."""

    def __init__(self, gpu: int, n: int):
        self.handles = [C.stream_create(gpu, False) for _ in range(n)]

    def __del__(self):
        for h in self.handles:
            try:
                C.stream_destroy(h)
            except Exception:  # noqa: BLE001 - teardown of a failed device: nothing left to free
                pass


class FrameStream:
    """A stream of independent frames through one distributed pipeline: the
    video-rate workload (each frame filtered, halo exchanged every step).

    `frames` engines (each with its own stripe pair) are stepped round-robin;
    frame f's work is queued on stream f mod `streams`.  Frames are
    independent, so with two streams one frame's kernel boundary and tail
    overlap the next frame's step (measured on MI355X, one N=8 share of a
    16384^2 RGB gaussian5: 41.0 -> 35.6 us a step, profiles/r4/cold/).  With
    `frames=0` the rule is the same at every world size (N = 1 included, so a
    1 -> N scaling curve compares one execution mode): at least two frames,
    and when one stripe fits the 256 MiB Infinity Cache, enough that
    F x (stripe in + out) exceeds twice it -- every step then reads data
    evicted long before (cache-cold), never a warm re-read.  `cache` says
    what the rotation achieves: "cold" (F x working set > 2 x the cache),
    "exceeds the Infinity Cache" (one stripe alone does), "partially warm"
    (the frame cap left the rotation inside 2 x the cache) or "warm" (one
    frame that fits).

    The reference has one frame, one pass (kernel.cu:190-226); a frame stream
    is this framework's throughput mode on top of the same engine."""

    MAX_FRAMES = 8

    def __init__(self, ctx: DistContext, pipeline, W: int, H: int, Cc: int = 3, frames: int = 0, streams: int = 0,
                 autotune: bool = True, stage_timing: bool = False):
        info = C.plan_info(pipeline.spec.chain, Cc, pipeline.spec.border, pipeline.fuse)
        part, _ = C.plan_rows(H, ctx.world, max(1, info["max_radius"]))
        self.world = ctx.world
        self.every_rank_has_rows = all(r > 0 for _, r in part)
        self.iterable = info["cin"] == info["cout"]
        self.ws_max = max(r for _, r in part) * W * (info["cin"] + info["cout"])  # per-GPU bytes of one step
        self.fits_mall = self.ws_max <= MALL_BYTES
        frames, self.streaming, self.cold, self.cache = self.plan(self.ws_max, self.iterable, ctx.device, frames)
        nmax = max(1, min(streams if streams > 0 else 2, frames)) if ctx.device else 1
        # stream counts pick_schedule may choose between (a fixed --streams: that one)
        self.stream_options = [nmax] if (streams > 0 or nmax == 1) else [1, nmax]
        self.frames = [DistributedPipeline(ctx, pipeline, W, H, Cc, autotune=autotune and i == 0, cold=self.streaming)
                       for i in range(frames)]
        self.streams = []
        self.nstreams = 1
        self.queues = "none"
        self._sets = {}
        if ctx.device:
            # two stream sets: plain streams, which share GPU_MAX_HW_QUEUES
            # hardware queues round-robin (two of torch's pool streams landed
            # on one queue after the RCCL check: cold N=8 share 41.4 us a
            # step), and streams with hardware queues of their own
            # (process-wide, C.dedicated_stream: 35.6 us), which in turn made
            # cross-stream event schedules slower on some boxes
            # (profiles/r5/streams/).  pick_schedule measures both;
            # STRIPE_FRAME_QUEUES=plain|dedicated pins one.
            # Processes that share one GPU (gloo-gpu with more local ranks than
            # GPUs) get no dedicated queues: each one's extra HSA queues
            # oversubscribe the GPU's hardware queue slots, and the time-sliced
            # queues made a 4-process 16384^2 step 3x slower
            # (profiles/r5/shared/)
            pin = os.environ.get("STRIPE_FRAME_QUEUES", "")
            if pin == "dedicated" or not self.shares_gpu(ctx):
                self._sets["dedicated"] = [torch.cuda.ExternalStream(C.dedicated_stream(ctx.gpu, k), device=ctx.gpu)
                                           for k in range(nmax)]
            # plain HIP streams created back to back here, so they take
            # consecutive hardware queues of the round-robin: two of torch's
            # pool streams could share one after other code took pool streams
            # (4 processes on one GPU: 0.52 -> 0.39 ms a step,
            # profiles/r5/shared/); freed with the last frame that uses them
            holder = _PlainStreams(ctx.gpu, nmax)
            self._sets["plain"] = [torch.cuda.ExternalStream(h, device=ctx.gpu) for h in holder.handles]
            # the "ahead" schedule's exchanges run on a stream of their own
            self._comm_streams = _PlainStreams(ctx.gpu, 1)
            for f in self.frames:
                f._plain_streams = holder
                f._comm_streams = self._comm_streams
            if pin == "pool":  # the set's earlier name
                pin = "plain"
            kinds = [k for k in ("dedicated", "plain") if k in self._sets]
            self.queue_options = [pin] if pin in self._sets else (kinds if nmax > 1 else kinds[:1])
            self.queues = self.queue_options[0]
            self.streams = self._sets[self.queues]
            for f in self.frames:
                f.engine.stage_timing = stage_timing
        self.set_streams(nmax)
        self._i = 0
        # steps per deep-halo block the frames' engines allow (halo_depth of
        # the pipeline; 1: every step exchanges), and whether they use it
        self.depth = max(1, self.head.engine.halo_depth)
        self.deep = False

    @staticmethod
    def shares_gpu(ctx: DistContext) -> bool:
        """More processes of this node than GPUs (gloo-gpu places rank r on
        GPU r mod count; RCCL runs one rank per GPU)."""
        if ctx.transport != "gloo-gpu":
            return False
        local = int(os.environ.get("LOCAL_WORLD_SIZE", str(ctx.world)))
        return local > max(1, torch.cuda.device_count())

    @classmethod
    def plan(cls, ws_max: int, iterable: bool, device: bool, frames: int = 0):
        """(frames, streaming, cold, cache) for a stripe whose step touches
        ws_max bytes per GPU: the frame count (frames <= 0: the auto rule of
        the class docstring), the engine's streaming policy (a rotated stripe
        that fits the cache: nt stores, cold autotune), whether the rotation
        really defeats the cache, and the record's label for it."""
        fits = ws_max <= MALL_BYTES
        if frames <= 0:
            if fits and iterable and device:
                frames = min(cls.MAX_FRAMES, -(-2 * MALL_BYTES // max(1, ws_max)) + 1)
            elif device and iterable:
                # one frame's kernel boundary (and at N > 1 its halo exchange)
                # can run beside the other's filter -- at every N, N = 1 included
                frames = 2
            else:
                frames = 1
        streaming = frames > 1 and fits
        # bytes the rotation touches between two visits of one frame
        cold = streaming and frames * ws_max > 2 * MALL_BYTES
        if not fits:
            cache = "exceeds the Infinity Cache"
        elif cold:
            cache = "cold"
        elif frames > 1:
            cache = "partially warm"
        else:
            cache = "warm"
        return frames, streaming, cold, cache

    def set_queues(self, kind: str):
        """Use the "dedicated" or the "plain" stream set (same stream count)."""
        if not getattr(self, "_sets", {}):
            return
        self.queues = kind
        self.streams = self._sets[kind]
        self.set_streams(self.nstreams)

    def set_streams(self, n: int):
        """Queue frame f on stream f mod n (n <= the streams created)."""
        if not self.streams:
            return
        n = max(1, min(n, len(self.streams)))
        for i, f in enumerate(self.frames):
            f.use_stream(self.streams[i % n].cuda_stream)
        self.nstreams = n

    def __len__(self):
        return len(self.frames)

    @property
    def head(self) -> DistributedPipeline:
        return self.frames[0]

    def load_synthetic(self, seed: int):
        """Frame f holds seeded synthetic pixels of seed + f."""
        for i, f in enumerate(self.frames):
            f.load_synthetic(seed + i)

    def tune(self, reduce_max=None):
        """Autotune frame 0 (on cold scratch stripes when the frames rotate to
        defeat the cache) and give every frame its tuning.  With reduce_max
        (max over the ranks of the job) on device engines at N > 1, the tune
        is collective: each candidate's time is the slowest rank's, so every
        rank runs the configuration that is best for the job's step (the max
        over ranks), not one its own timing noise picked.  Every rank calls
        tune() together."""
        e0 = self.head.engine
        # a frame stream held to one stream tunes on one (cold tunes otherwise
        # alternate two, the probe's usual pick)
        e0.set_tune_streams(max(self.stream_options) if self.streams else 1)
        collective = (reduce_max is not None and getattr(self, "world", 1) > 1 and bool(self.streams)
                      and getattr(self, "every_rank_has_rows", False))
        if collective:
            e0.set_tune_reduce(reduce_max)
        try:
            e0.tune()
        finally:
            if collective:
                e0.set_tune_reduce(None)
        for f in self.frames[1:]:
            f.engine.set_tuning(e0.bands, e0.caps, e0.policies, e0.orders)

    SCHEDULES = ("pipeline", "overlap", "serial", "batched", "ahead")
    # with a deep halo (depth > 1): these schedules, each frame exchanging
    # depth * S rows every depth-th step (Engine.deep_steps)
    DEEP_SCHEDULES = ("serial+deep", "batched+deep", "ahead+deep")

    def set_deep(self, on: bool):
        """Deep steps for every frame: a frame exchanges depth * S rows on
        every depth-th step and none on the others, bit-exact
        (Engine.deep_steps).  Each step is still one step of the next frame, so
        every step reads a cold stripe.  No-op at depth 1."""
        self.deep = bool(on) and getattr(self, "depth", 1) > 1
        for f in self.frames:
            f.engine.deep_steps = self.deep

    def set_schedule(self, name: str):
        """Halo schedule of every frame ("serial" | "overlap" | "pipeline" |
        "batched" | "ahead").  "batched" is the serial schedule with the
        exchanges of all frames that share a stream posted as ONE communicator
        group, ahead of the first of those frames' steps in each round: one
        RCCL launch per stream and round instead of one per frame and step
        (the frames' own order on their stream already puts each frame's
        previous step before it).  "ahead" posts each frame's next exchange
        right after its step, on a communication stream of its own
        (Engine.post_halo_ahead): the rows are needed a whole round later, so
        the exchange runs beside the other frames' filters and the frame's
        next step only waits for an event that has long fired.
        A "+deep" suffix (DEEP_SCHEDULES) adds deep steps (set_deep)."""
        base, _, deep = name.partition("+")
        if deep not in ("", "deep"):
            raise ValueError(f"unknown halo schedule {name!r}")
        self.set_deep(deep == "deep")
        self.batched = base == "batched"
        self.ahead = base == "ahead"
        for f in self.frames:
            f.engine.halo_schedule = "serial" if (self.batched or self.ahead) else base

    def _batch_candidate(self) -> bool:
        """Whether the probe times "batched" and "ahead": frames of device engines that
        exchange halo rows (N > 1, or the self-halo rank).  Decided on what
        every rank shares -- never on a rank's own stripe -- so every rank
        times the same candidate list."""
        if not self.streams or len(self.frames) < 2:
            return False
        world = getattr(getattr(self.head, "ctx", None), "world", 2)
        return world > 1 or bool(getattr(self.head.engine, "self_halo", False))

    def _batches(self) -> bool:
        """Batched posts apply: device engines that exchange halo rows."""
        return bool(getattr(self, "batched", False) and self.streams and self.head.engine.posts_halo)

    def _aheads(self) -> bool:
        """Ahead posts apply: device engines that exchange halo rows."""
        return bool(getattr(self, "ahead", False) and self.streams and self.head.engine.posts_halo)

    def _deep_candidate(self) -> bool:
        """Whether the probe times the DEEP_SCHEDULES: frames that exchange
        halo rows (as _batch_candidate) with a halo depth above 1 (the same on
        every rank: the engines derive it from the whole partition)."""
        return getattr(self, "depth", 1) > 1 and self._batch_candidate()

    @property
    def schedule(self) -> str:
        if self._batches():
            base = "batched"
        elif self._aheads():
            base = "ahead"
        else:
            base = self.head.engine.halo_schedule
        return base + ("+deep" if getattr(self, "deep", False) and self.head.engine.posts_halo else "")

    def pick_schedule(self, reduce_max=None, barrier=None, steps: int = 0, rounds: int = 2) -> dict:
        """Time every halo schedule (interior / boundary overlap, the
        three-stream pipeline, the plain serial one),
        with the frames on one stream or alternating over two, on the real
        transport, and keep the fastest; two streams come from either stream
        set (dedicated hardware queues or plain streams, set_queues); returns
        {"chosen", "streams", "queues", "ms"} ("ms" keys: schedule, or
        schedule@streams[/queues] when several are tried).
        Which one wins depends on the link and RCCL's per-exchange cost, which
        one GPU cannot show, so the job measures it where it runs.
        reduce_max(ms) -> max over ranks and barrier() keep every rank on the
        same choice (each rank times the same steps; collective order holds)."""
        reduce_max = reduce_max or (lambda v: v)
        barrier = barrier or (lambda: None)
        # the candidate list must be the same on every rank (each timing is a
        # collective reduce_max): device engines try every schedule, even one a
        # rank's own stripe runs another way (e.g. a thin stripe without the
        # pipeline); host engines have one schedule and time nothing
        scheds = ([s for s in self.SCHEDULES if s not in ("batched", "ahead") or self._batch_candidate()]
                  if self.streams else ["serial"])
        if self.streams and self._deep_candidate():
            scheds += list(self.DEEP_SCHEDULES)
        if getattr(getattr(self.head, "ctx", None), "world", 2) == 1:
            # one rank exchanges nothing: only schedules that differ on it (none)
            eff = []
            for s in scheds:
                self.set_schedule(s)
                if self.schedule not in eff:
                    eff.append(self.schedule)
            scheds = eff
        opts = list(self.stream_options)
        sets = getattr(self, "_sets", {})
        qopts = list(getattr(self, "queue_options", ["dedicated"])) if sets else ["none"]
        # one stream: the queue kind makes no difference (the dedicated set)
        cands = [(s, ns, q) for ns in opts for s in scheds for q in (qopts if ns > 1 else qopts[:1])]

        def key(c):
            k = c[0] if len(opts) == 1 else f"{c[0]}@{c[1]}"
            return k + (f"/{c[2]}" if c[1] > 1 and len(qopts) > 1 else "")

        if len(cands) == 1:
            self.set_schedule(scheds[0])
            if sets:
                self.set_queues(cands[0][2])
            self.set_streams(opts[0])
            return {"chosen": self.schedule, "streams": self.nstreams, "queues": getattr(self, "queues", "none"),
                    "ms": {}}
        n = steps if steps > 0 else max(60, 4 * len(self.frames))
        best = {}
        for _ in range(rounds):
            for c in cands:
                self.synchronize()
                self.set_schedule(c[0])
                if sets:
                    self.set_queues(c[2])
                self.set_streams(c[1])
                for i in range(2 * len(self.frames)):
                    self.step(i)
                self.synchronize()
                barrier()
                t0 = time.perf_counter()
                for i in range(n):
                    self.step(i)
                self.synchronize()
                ms = reduce_max((time.perf_counter() - t0) * 1e3 / n)
                best[c] = min(best.get(c, float("inf")), ms)
        chosen = min(cands, key=lambda c: best[c])
        self.synchronize()
        self.set_schedule(chosen[0])
        if sets:
            self.set_queues(chosen[2])
        self.set_streams(chosen[1])
        return {"chosen": chosen[0], "streams": self.nstreams, "queues": getattr(self, "queues", "none"),
                "ms": {key(c): round(v, 5) for c, v in best.items()}}

    def stream_of(self, i: int):
        return self.streams[(i % len(self.frames)) % self.nstreams] if self.streams else None

    def step(self, i: int | None = None):
        """One step of the next frame (or of step index i): its halo exchange
        and full stripe filter."""
        if i is None:
            i = self._i
            self._i += 1
        k = i % len(self.frames)
        f = self.frames[k]
        if not self.iterable:  # a chain that changes the channel count re-reads its (unchanged) input
            f.engine.rewind()
        if self._batches():
            if k < self.nstreams and f.engine.exchange_due:
                # the first frame of its stream this round: one group with the
                # exchanges of every frame on this stream (k, k + s, k + 2s, ...)
                comm = f.ctx.comm
                comm.group_start()
                try:
                    for g in range(k, len(self.frames), self.nstreams):
                        self.frames[g].engine.post_halo()
                finally:
                    comm.group_end()
            f.engine.run_posted()  # (a frame whose exchange was not posted makes its own)
        elif self._aheads():
            # this step's exchange was posted a round ago (the first round makes
            # its own); the next one is posted now, on the communication stream
            f.engine.run_posted()
            f.engine.post_halo_ahead(self._comm_streams.handles[0])
        else:
            f.run(1)

    def synchronize(self):
        for f in self.frames:
            f.synchronize()


def run_local_group(pipeline, image: np.ndarray, ranks: int, backend: str = "host", iterations: int = 1):
    """N in-process ranks (threads): 'local' shares this process's GPU, 'host' uses the CPU."""
    return pipeline.run_distributed(image, ranks, backend, iterations)


def plan_rows_weighted(H: int, weights, min_rows: int = 1):
    """[(row0, rows)] per rank for per-rank shares `weights` and the number of active ranks."""
    return C.plan_rows_weighted(H, [float(w) for w in weights], min_rows)


def dist_split(H: int, world: int, row_in_bytes: int, row_out_bytes: int, root_rows_per_ms: float,
               link_bytes_per_ms: float, hbm_bytes_per_ms: float, chunks: int = 8, min_rows: int = 1,
               peer_rows_per_ms: float | None = None) -> dict:
    """Link-aware split of the root-resident dist step (the root filters its
    share in place, every peer's share crosses its own link): weights, rows and
    the modelled times (root, peer, root-HBM floor, predicted, even split)."""
    return C.plan_dist_split(H, world, row_in_bytes, row_out_bytes, root_rows_per_ms,
                             peer_rows_per_ms or root_rows_per_ms, link_bytes_per_ms, hbm_bytes_per_ms, chunks,
                             min_rows)


def probe_link_rate(ctx: DistContext, nbytes: int = 64 << 20, reps: int = 3) -> float:
    """Bytes per ms per root<->peer link, one direction, all links busy both ways
    (every rank must call it; 0 on one rank)."""
    if ctx.comm is None or ctx.world == 1:
        return 0.0
    return C.probe_link_rate(ctx.comm, ctx.gpu if ctx.device else -1, nbytes, reps)


def ring_check(ctx: DistContext, nbytes: int = 1 << 20, frames: int = 4, streams: int = 2, iters: int = 500) -> dict:
    """Transport check of this context's communicator in the FrameStream
    pattern: `iters` grouped send/recv exchanges around the ring (one rank:
    the RCCL communicator sends to and receives from itself), consecutive
    frames alternating over `streams` streams on the one communicator, every
    received word checked against its sender's (iteration, rank) pattern.
    Returns {"errors", "bytes_checked", "ms"} (every rank must call it)."""
    if ctx.comm is None:
        raise ValueError("ring_check needs a communicator (a device context, or world > 1)")
    return C.comm_ring_check(ctx.comm, ctx.gpu if ctx.device else -1, int(nbytes), frames, streams, iters)


__all__ = ["DistContext", "GlooComm", "init", "DistributedPipeline", "plan_rows", "plan_rows_weighted", "dist_split",
           "probe_link_rate", "ring_check", "run_local_group", "rank_identity", "world_identity", "identity_summary",
           "FrameStream"]
