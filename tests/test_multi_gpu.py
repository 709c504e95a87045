"""Real multi-GPU runs (one process per GPU over RCCL), skipped on 1-GPU boxes.

bench.py under torchrun on N = 2, 4 and 8 GPUs when present: the iterated
deep-halo schedule and the dist scope must verify against the golden path on
the stripe seams.  The CPU (gloo) and single-GPU (local ranks) suites cover
the same partition/halo logic; this checks the RCCL transport itself.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ngpus() -> int:
    try:
        return torch.cuda.device_count()  # does not initialise the GPU
    except Exception:
        return 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("chain,depth", [("gaussian5", 0), ("gaussian5", 1), ("sobel", 0), ("blur:9", 0)])
def test_torchrun_bench_rccl(n, chain, depth):
    if _ngpus() < n:
        pytest.skip(f"needs {n} GPUs")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "9", "--warmup", "2", "--width", "2048", "--height", "1024",
           "--chain", chain, "--halo-depth", str(depth), "--dist-steps", "2", "--e2e-steps", "1"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["value"] > 0
    assert rec["verified_vs_golden"] is True
    # RCCL's own view: n ranks in the communicator, n distinct GPUs, one
    # runtime / RCCL copy per process, the same in every process
    summ = rec["world"]["summary"]
    assert summ["ranks"] == n and summ["distinct_gpus"] == n and summ["nccl_count"] == [n]
    assert sorted(summ["devices"]) == list(range(n))
    assert summ["one_copy_per_lib"] and summ["same_libs_everywhere"]
    for sc in rec["scopes"].values():
        assert "error" not in sc, sc


@pytest.mark.parametrize("n,chunks", [(1, 0), (2, 0), (4, 0), (2, 4), (4, 8)])
def test_python_cli_rccl_one_process_per_gpu(tmp_path, n, chunks):
    """`torchrun -m mpi_cuda_imagemanipulation_amd run --backend rccl`: the
    reference's mpiexec flow with one process per GPU (n = 1 runs on every
    box: a one-rank RCCL communicator through the same scatter/gather path)."""
    if _ngpus() < n:
        pytest.skip(f"needs {n} GPUs")
    import numpy as np

    sys.path.insert(0, ROOT)
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(9, 301, 157, 3)
    src, out = tmp_path / "in.ppm", tmp_path / "out.ppm"
    m.utils.write_image(str(src), img)
    chain = "gray:ref,contrast:3.5,emboss3,expand"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "mpi_cuda_imagemanipulation_amd",
           "run", "--input", str(src), "--output", str(out), "--backend", "rccl", "--chain", chain,
           "--dist-chunks", str(chunks)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = m.utils.read_image(str(out))
    ref = m._C.golden_apply(img, chain, "reflect101", True)
    assert got.shape == ref.shape and np.array_equal(got, ref)


@pytest.mark.parametrize("n,chunks,chain", [(1, 0, "gaussian5"), (1, 8, "gaussian5"), (1, 0, "gaussian5,sobel"),
                                            (2, 0, "gaussian5"), (2, 4, "gaussian5"), (4, 8, "emboss3"),
                                            (8, 8, "gaussian5"), (8, 0, "blur:9")])
def test_run_distributed_rccl_in_process(n, chunks, chain):
    """One process driving GPUs 0..n-1 (a thread per rank, ncclCommInitAll):
    Pipeline.run_distributed(backend='rccl') equals the golden path."""
    if _ngpus() < n:
        pytest.skip(f"needs {n} GPUs")
    import numpy as np

    sys.path.insert(0, ROOT)
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(11, 389, 263, 3)
    got = m.models.Pipeline(chain, dist_chunks=chunks).run_distributed(img, n, backend="rccl")
    ref = m._C.golden_apply(img, chain, "reflect101", True)
    if chain.startswith("blur"):
        assert got.shape == ref.shape and np.abs(got.astype(int) - ref).max() <= 1
    else:
        assert got.shape == ref.shape and np.array_equal(got, ref)


@pytest.mark.parametrize("n,chunks,stage", [(2, 4, "scatter"), (2, 0, "halo"), (4, 8, "dist"), (8, 0, "compute")])
def test_rccl_in_process_fault_aborts_group(monkeypatch, n, chunks, stage):
    """One rank of an in-process RCCL group fails (STRIPE_FAULT): every rank's
    thread must fail fast -- the failing thread raises the others' abort
    flags and each rank tears its non-blocking communicator down from its own
    thread, inside a bounded poll, instead of waiting in ncclGroupEnd or a
    stream for the dead rank."""
    if _ngpus() < n:
        pytest.skip(f"needs {n} GPUs")
    import time

    sys.path.insert(0, ROOT)
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(4, 611, 257, 3)
    monkeypatch.setenv("STRIPE_FAULT", f"{stage}@1")
    monkeypatch.setenv("STRIPE_COMM_TIMEOUT_S", "60")
    t0 = time.time()
    with pytest.raises(Exception, match="injected fault|aborted"):
        m.models.Pipeline("gaussian5", dist_chunks=chunks).run_distributed(img, n, backend="rccl")
    assert time.time() - t0 < 45, "peers of the failing rank must not wait for the comm timeout"
