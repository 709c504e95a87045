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
import os
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
    executed as torch.distributed P2P ops (gloo)."""

    def __init__(self, group=None):
        self.group = group
        self.ops = []

    def group_start(self):
        self.ops = []

    def send(self, ptr, n, peer):
        self.ops.append(dist.P2POp(dist.isend, _host_view(ptr, n), peer, self.group))

    def recv(self, ptr, n, peer):
        self.ops.append(dist.P2POp(dist.irecv, _host_view(ptr, n), peer, self.group))

    def group_end(self):
        if self.ops:
            for r in dist.batch_isend_irecv(self.ops):
                r.wait()
        self.ops = []

    def barrier(self):
        dist.barrier(group=self.group)

    def native(self, rank: int, world: int):
        return C.make_callback_comm(rank, world, self.group_start, self.send, self.recv, self.group_end,
                                    self.barrier)


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


class DistributedPipeline:
    """Per-rank handle on the native engine for one image geometry."""

    def __init__(self, ctx: DistContext, pipeline, W: int, H: int, Cc: int = 3, root_buffers: bool = False,
                 autotune: bool = False, row_weights=None):
        self.ctx = ctx
        cfg = pipeline.config(W, H, Cc, "device" if ctx.device else "host",
                              device=ctx.gpu if ctx.device else -1, autotune=autotune, row_weights=row_weights)
        cfg.root_buffers = root_buffers
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


__all__ = ["DistContext", "GlooComm", "init", "DistributedPipeline", "plan_rows", "plan_rows_weighted", "dist_split",
           "probe_link_rate", "run_local_group"]
