"""The target world size, 8, wherever it runs without 8 GPUs.

* torchrun --nproc-per-node 8 bench.py --backend host: 8 processes over gloo
  (auto deep-halo depth, the dist scopes), every scope verified against golden;
* the Python CLI at 8 gloo processes: --dist-chunks 8 (pipelined scatter /
  filter / gather), --preset ref-gpu (the reference's H/N split, dropped rows
  and per-stripe seams, kernel.cu:117,137,195) against the numpy mirror, and a
  weighted split;
* Pipeline.run_distributed(img, 8) for the config-4 (gaussian5) and config-5
  (31x31 blur, conv) chains on reduced frames: host ranks here, local ranks on
  one GPU under -m gpu.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import np_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 8


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    return dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
                STRIPE_CPU_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))


def _torchrun(args, tmp_path, timeout=420):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(N),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=timeout, cwd=str(tmp_path))
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_host_8_processes(tmp_path):
    recs = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", str(N), "--steps", "9", "--warmup", "1",
                      "--width", "96", "--height", "1600", "--backend", "host", "--dist-steps", "2"], tmp_path)
    assert len(recs) == 1
    rec = recs[0]
    assert rec["n_gpus"] == N and rec["steps"] == 9 and rec["value"] > 0
    assert rec["verified_vs_golden"] is True
    assert rec["halo_depth"] == 1  # the headline exchanges every step
    assert rec["scopes"]["resident_deep"]["halo_depth"] >= 2  # auto deep halo at 200-row stripes
    summ = rec["world"]["summary"]
    assert summ["ranks"] == N and summ["one_copy_per_lib"] and summ["same_libs_everywhere"]
    assert rec["stripe_rows"] == [200] * N
    assert rec["scopes"]["dist_sequential"]["verified"] is True


def _cli(tmp_path, img, extra):
    import mpi_cuda_imagemanipulation_amd as m

    src, out = tmp_path / "in.ppm", tmp_path / "out.ppm"
    m.utils.write_image(str(src), img)
    recs = _torchrun(["-m", "mpi_cuda_imagemanipulation_amd", "run", "--input", str(src), "--output", str(out),
                      "--backend", "gloo", *extra], tmp_path)
    assert len(recs) == 1 and recs[0]["ranks"] == N
    return m.utils.read_image(str(out))


@pytest.mark.parametrize("chain", ["gaussian5", "gray:ref,contrast:3.5,emboss3,expand"])
def test_cli_8_gloo_dist_chunks(tmp_path, C, chain):
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(7, 91, 203, 3)
    got = _cli(tmp_path, img, ["--chain", chain, "--dist-chunks", "8"])
    assert (got == C.golden_apply(img, chain, "reflect101", True)).all()


def test_cli_8_gloo_weighted(tmp_path, C):
    import mpi_cuda_imagemanipulation_amd as m

    img = m.utils.synthetic_image(8, 77, 250, 3)
    w = ",".join(["0.58"] + ["0.06"] * (N - 1))
    got = _cli(tmp_path, img, ["--chain", "gaussian5", "--dist-chunks", "4", "--row-weights", w])
    assert (got == C.golden_apply(img, "gaussian5", "reflect101", True)).all()


def test_cli_8_gloo_ref_gpu_preset(tmp_path):
    # the reference's own distributed output: H/N rows per rank (H mod N rows
    # dropped, kernel.cu:117), each stripe filtered as its own image with the
    # interior-only emboss bounds (seams, kernel.cu:83), gray -> 3 channels
    import mpi_cuda_imagemanipulation_amd as m

    H, W = 8 * 13 + 5, 66
    img = m.utils.synthetic_image(9, W, H, 3)
    got = _cli(tmp_path, img, ["--preset", "ref-gpu"])
    rows = H // N
    for r in range(N):
        s = img[r * rows:(r + 1) * rows]
        e = np_ref.stencil(np_ref.contrast_ref(np_ref.gray_ref(s), 3.5), "emboss3", "skip")
        assert (got[r * rows:(r + 1) * rows] == np_ref.expand(e)).all(), r


@pytest.mark.parametrize("chain,shape", [("gaussian5", (203, 97, 3)), ("blur:31", (180, 75, 3)),
                                         ("conv:9:" + ";".join(str((i % 7 - 2) / 60) for i in range(81)),
                                          (150, 64, 1))])
@pytest.mark.parametrize("chunks", [0, 8])
def test_run_distributed_8_host(C, rng, chain, shape, chunks):
    # config 4 (gaussian5) and config 5 (31x31 blur; a general conv) on 8 host ranks
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    if shape[2] == 1:
        img = img[..., 0]
    from mpi_cuda_imagemanipulation_amd import models

    got = models.Pipeline(chain, dist_chunks=chunks).run_distributed(img, N, "host")
    assert (got == C.golden_apply(img, chain, "reflect101", True)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("chain,shape", [("gaussian5", (1031, 1537, 3)), ("blur:31", (900, 1200, 3)),
                                         ("sobel", (1024, 2048, 1))])
@pytest.mark.parametrize("chunks", [0, 8])
def test_run_distributed_8_local_gpu(C, rng, chain, shape, chunks):
    # 8 logical ranks on one GPU (local comm: device copies between stripes)
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    if shape[2] == 1:
        img = img[..., 0]
    from mpi_cuda_imagemanipulation_amd import models

    got = models.Pipeline(chain, dist_chunks=chunks).run_distributed(img, N, "local")
    ref = C.golden_apply(img, chain, "reflect101", True)
    d = np.abs(got.astype(int) - ref.astype(int))
    tol = 1 if chain.startswith("blur") else 0
    assert d.max() <= tol and (d == 0).mean() > 0.9999


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["blur:31:lsb", "blur:31", "gray:ref,contrast:3.5,emboss3@skip,expand"])
def test_8_local_ranks_bit_identical_to_one(C, rng, chain):
    # the float blur kernels sum every output in an order fixed by global rows,
    # so 8 stripes (with halos) reproduce the 1-rank frame bit for bit, lsb
    # mode included; the reference pipeline (affine post map) likewise
    img = rng.integers(0, 256, size=(901, 1201, 3), dtype=np.uint8)
    from mpi_cuda_imagemanipulation_amd import models

    one = models.Pipeline(chain).run_distributed(img, 1, "local")
    eight = models.Pipeline(chain).run_distributed(img, N, "local")
    assert (one == eight).all()
    ref = C.golden_apply(img, chain, "reflect101", True)
    assert np.abs(one.astype(int) - ref.astype(int)).max() <= (1 if "blur" in chain else 0)
