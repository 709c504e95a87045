"""Failure path, bounded waits and stage tracing.

The reference's failure mode (Q9): a rank that errors returns 1 without
MPI_Abort and its peers block forever.  Here a failure on one rank (injected
with STRIPE_FAULT) must surface as an error on every rank, quickly, in-process
(host group: shared abort flag) and across processes (gloo: the dead peer's
closed connection / the bounded process-group timeout).
"""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def host_cfg(C):
    import mpi_cuda_imagemanipulation_amd as m

    def make(W=40, H=36, chain="gaussian5"):
        return m.models.Pipeline(chain).config(W, H, 3, "host")

    return make


@pytest.mark.parametrize("stage", ["scatter", "halo", "compute", "gather"])
def test_injected_fault_aborts_whole_host_group(C, host_cfg, monkeypatch, stage):
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(2, 40, 36, 3)
    monkeypatch.setenv("STRIPE_FAULT", f"{stage}@1")
    t0 = time.time()
    with pytest.raises(Exception, match="injected fault"):
        C.run_local_group(host_cfg(), 3, img, 1)
    assert time.time() - t0 < 30, "peers of the failing rank must not wait for the full timeout"


def test_fault_spec_grammar(C, monkeypatch):
    monkeypatch.setenv("STRIPE_FAULT", "halo@2,compute@*")
    C.fault_point("halo", 1)  # other rank: no fault
    with pytest.raises(Exception, match="stage 'halo' on rank 2"):
        C.fault_point("halo", 2)
    with pytest.raises(Exception, match="stage 'compute' on rank 5"):
        C.fault_point("compute", 5)
    C.fault_point("gather", 2)
    monkeypatch.delenv("STRIPE_FAULT")
    C.fault_point("halo", 2)


def test_comm_timeout_env(C, monkeypatch):
    assert C.comm_timeout_s() == 600.0
    monkeypatch.setenv("STRIPE_COMM_TIMEOUT_S", "12.5")
    assert C.comm_timeout_s() == 12.5


def test_no_fault_group_still_exact(C, host_cfg, monkeypatch):
    import mpi_cuda_imagemanipulation_amd as m

    monkeypatch.delenv("STRIPE_FAULT", raising=False)
    img = m.utils.synthetic_image(2, 40, 36, 3)
    out = C.run_local_group(host_cfg(), 3, img, 1)
    assert (out == C.golden_apply(img, "gaussian5", "reflect101", True)).all()


def test_stage_times_host_engine(C):
    import mpi_cuda_imagemanipulation_amd as m

    pipe = m.models.Pipeline("gaussian5,sobel")
    e = C.Engine(pipe.config(300, 200, 3, "host"), None)
    e.load_synthetic(1)
    e.run(2)
    e.synchronize()
    t = e.times.as_dict()
    assert set(t) >= {"compute", "load", "halo", "scatter", "gather", "h2d", "d2h", "e2e"}
    assert t["compute"] > 0 and t["load"] > 0


def test_trace_mark_is_callable(C):
    C.trace_mark("test marker")  # no profiler attached: a no-op, must not raise


WORKER = r'''
import os, sys
sys.path.insert(0, os.environ["STRIPE_ROOT"])
from mpi_cuda_imagemanipulation_amd import parallel, models
ctx = parallel.init("gloo")
dp = parallel.DistributedPipeline(ctx, models.Pipeline("gaussian5"), 64, 48, 3)
dp.load_synthetic(1)
try:
    dp.run(1)
    print("RANK", ctx.rank, "FINISHED", flush=True)
except Exception as e:
    print("RANK", ctx.rank, "ERROR", type(e).__name__, str(e)[:200], flush=True)
    sys.exit(7)
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dead_peer_process_fails_fast(tmp_path):
    """Rank 1 dies (STRIPE_FAULT=halo@1:exit) before sending its halo rows;
    rank 0 must fail with an error well before the wait bound, not hang."""
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), STRIPE_ROOT=ROOT, STRIPE_FAULT="halo@1:exit", STRIPE_COMM_TIMEOUT_S="60",
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    t0 = time.time()
    outs = []
    for p in procs:
        o, _ = p.communicate(timeout=120)
        outs.append(o.decode(errors="replace"))
    took = time.time() - t0
    assert procs[1].returncode == 3, outs[1]           # the injected crash
    assert procs[0].returncode != 0, outs[0]           # the survivor reports failure...
    assert "FINISHED" not in outs[0]
    assert took < 90, f"survivor took {took:.0f}s"     # ...instead of hanging
