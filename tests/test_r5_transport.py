"""Transport check: ring send/recv exchanges in
the FrameStream pattern through the framework's Comm interface, every received
word verified against its sender's (iteration, rank) pattern.

* GPU, one rank: the RCCL communicator sends to and receives from itself
  (ncclSend / ncclRecv with peer == rank inside one group) -- real transfers
  through the non-blocking communicator's bounded polling, >= 4 frames
  alternating over 2 streams on the one communicator, >= 500 exchanges.
* CPU, 2 and 3 processes: the same driver over gloo (callback communicator).

Reference: the MPI_Scatter / MPI_Gather transfers this transport replaces
(kernel.cu:137,223).
"""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json
sys.path.insert(0, os.environ["STRIPE_ROOT"])
import torch.distributed as dist
from mpi_cuda_imagemanipulation_amd import parallel
ctx = parallel.init("gloo")
r = parallel.ring_check(ctx, int(os.environ["NBYTES"]), frames=3, streams=2, iters=int(os.environ["ITERS"]))
out = [None] * ctx.world
dist.all_gather_object(out, r)
if ctx.rank == 0:
    print("RESULT " + json.dumps(out))
dist.barrier()
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_ring_check_gloo_processes(tmp_path, world):
    import json

    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), STRIPE_ROOT=ROOT, NBYTES=str(4 * 1031), ITERS="24",
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        o, _ = p.communicate(timeout=240)
        logs.append(o.decode(errors="replace"))
        assert p.returncode == 0, "\n".join(logs)
    line = [ln for ln in logs[0].splitlines() if ln.startswith("RESULT ")]
    res = json.loads(line[0][len("RESULT "):])
    assert len(res) == world
    for r in res:
        assert r["errors"] == 0 and r["bytes_checked"] == 24 * 4 * 1031


def test_ring_check_needs_a_communicator(monkeypatch):
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("gloo")  # one host rank: no communicator
    with pytest.raises(ValueError):
        parallel.ring_check(ctx)


def test_pattern_words_differ_by_tag(C):
    # the pattern of one (iteration, sender) tag never equals another's: a
    # stale or misrouted message cannot pass the check
    import numpy as np

    a = np.array([C.pattern_word(7, j) for j in range(64)], dtype=np.uint64)
    b = np.array([C.pattern_word(8, j) for j in range(64)], dtype=np.uint64)
    assert (a != b).mean() > 0.99 and len(set(a.tolist())) == 64


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [2 * 2 * 16384 * 3, 1 << 20])
def test_rccl_loopback_frame_stream_pattern_gpu(monkeypatch, nbytes):
    # one-rank RCCL communicator: grouped ncclSend / ncclRecv to itself, 4
    # frames alternating over 2 streams, 500 exchanges, every byte verified
    # (2 x 2 halo rows of a 16384-wide RGB stripe, and 1 MiB)
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("rccl")
    assert ctx.comm is not None and ctx.comm.backend == "rccl" and ctx.comm.size == 1
    r = parallel.ring_check(ctx, nbytes, frames=4, streams=2, iters=500)
    assert r["errors"] == 0 and r["bytes_checked"] == 500 * nbytes and r["ms"] > 0


@pytest.mark.gpu
def test_rccl_loopback_one_stream_gpu(monkeypatch):
    # the same on one stream (consecutive exchanges strictly ordered)
    from mpi_cuda_imagemanipulation_amd import parallel

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("rccl")
    r = parallel.ring_check(ctx, 4096, frames=2, streams=1, iters=64)
    assert r["errors"] == 0 and r["bytes_checked"] == 64 * 4096
