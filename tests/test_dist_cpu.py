"""Multi-process distributed path on CPU: gloo process group + host engine.

The same Engine call sequence (scatter / halo exchange / gather) that runs over
RCCL on GPUs runs here through the callback communicator, so the partition and
halo logic of the multi-process path is covered without a GPU.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json
import numpy as np
sys.path.insert(0, os.environ["STRIPE_ROOT"])
import torch.distributed as dist
from mpi_cuda_imagemanipulation_amd import parallel, models, utils
from mpi_cuda_imagemanipulation_amd._native import C
ctx = parallel.init("gloo")
chain = os.environ["CHAIN"]; W, H = 61, 45
img = utils.synthetic_image(3, W, H, 3)
pipe = models.Pipeline(chain, halo=os.environ.get("HALO", "1") == "1")
dp = parallel.DistributedPipeline(ctx, pipe, W, H, 3, root_buffers=True)
dp.load_root(img)
dp.scatter()
dp.run(int(os.environ.get("ITERS", "1")))
dp.gather()
out = dp.result_root()
# resident path: every rank generates its own stripe
dp2 = parallel.DistributedPipeline(ctx, pipe, W, H, 3)
dp2.load_synthetic(3)
dp2.run(1)
stripe = dp2.result_stripe()
parts = [None] * ctx.world
dist.all_gather_object(parts, (dp2.stripe, stripe.tolist()))
if ctx.rank == 0:
    np.save(os.environ["OUT"], out)
    res = np.zeros_like(out)
    for (row0, rows), data in parts:
        if rows:
            res[row0:row0 + rows] = np.array(data, dtype=np.uint8)
    np.save(os.environ["OUT"] + ".res.npy", res)
dist.barrier()
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(tmp_path, world, chain, halo=True, iters=1):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    out = tmp_path / "out.npy"
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), STRIPE_ROOT=ROOT, CHAIN=chain, OUT=str(out), HALO="1" if halo else "0",
                   ITERS=str(iters), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        o, _ = p.communicate(timeout=240)
        logs.append(o.decode(errors="replace"))
        assert p.returncode == 0, "\n".join(logs)
    return np.load(out), np.load(str(out) + ".res.npy")


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("chain", ["gaussian5", "gray:ref,contrast:3.5,emboss3,expand", "sobel,gaussian7"])
def test_gloo_ranks_match_golden(tmp_path, C, world, chain):
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(3, 61, 45, 3)
    ref = C.golden_apply(img, chain, "reflect101", True)
    out, res = _launch(tmp_path, world, chain)
    assert (out == ref).all()
    assert (res == ref).all()


def test_gloo_iterated(tmp_path, C):
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(3, 61, 45, 3)
    ref = img
    for _ in range(3):
        ref = C.golden_apply(ref, "gaussian5", "reflect101", True)
    out, _ = _launch(tmp_path, 2, "gaussian5", iters=3)
    assert (out == ref).all()


@pytest.mark.parametrize("nproc,depth", [(2, 0), (3, 3)])
def test_bench_host_backend_multi_rank(tmp_path, nproc, depth):
    """bench.py under torchrun on the host engine + gloo; the headline exchanges
    every step, and depth 3 runs the resident_deep scope's schedule across
    processes (exchange every 3 steps, 7 steps rounded up to 9)."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus",
           str(nproc), "--steps", "7" if depth else "3", "--warmup", "1", "--width", "200", "--height", "96",
           "--backend", "host", "--dist-steps", "2", "--halo-depth", str(depth)]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"]:
        assert k in rec
    assert rec["n_gpus"] == nproc and rec["steps"] == (7 if depth else 3) and rec["value"] > 0
    assert rec["verified_vs_golden"] is True
    assert rec["halo_depth"] == 1  # the headline exchanges every step
    deep = rec["scopes"]["resident_deep"]
    if depth:
        assert deep["halo_depth"] == depth and deep["steps"] % depth == 0


@pytest.mark.parametrize("nproc,preset,chain,chunks", [(3, None, "gaussian5,sobel", 0), (2, "ref-cpu", None, 0),
                                                        (3, None, "gaussian5", 4), (2, "ref-cpu", None, 3)])
def test_python_cli_one_process_per_rank(tmp_path, C, nproc, preset, chain, chunks):
    """`torchrun -m mpi_cuda_imagemanipulation_amd run --backend gloo`: the
    reference's mpiexec flow (root load, metadata broadcast, scatter, filter,
    gather, root write), one process per rank; output equals the single-rank
    run of the same pipeline."""
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(5, 83, 47, 3)
    src, out = tmp_path / "in.ppm", tmp_path / "out.ppm"
    m.utils.write_image(str(src), img)
    sel = ["--preset", preset] if preset else ["--chain", chain]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "mpi_cuda_imagemanipulation_amd",
           "run", "--input", str(src), "--output", str(out), "--backend", "gloo", *sel, "--dist-chunks", str(chunks)]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["ranks"] == nproc and rec["backend"] == "gloo"
    got = m.utils.read_image(str(out))
    pipe = m.models.Pipeline.preset(preset) if preset else m.models.Pipeline(chain)
    ref = pipe.run_distributed(img, nproc, backend="host")
    assert got.shape == ref.shape and (got == ref).all()
    if not preset:
        assert (got == C.golden_apply(img, chain, "reflect101", True)).all()
