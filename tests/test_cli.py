"""Native `stripe` CLI (bin/stripe) on the CPU host backend.

Config 1 of BASELINE.json (grayscale on a 512x512 PPM, CPU path, world_size=1)
plus the reference presets run as multi-rank in-process groups.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import np_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "bin", "stripe")

pytestmark = pytest.mark.skipif(not os.path.exists(EXE), reason="bin/stripe not built")


def run(*args, check=True):
    r = subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "")))
    if check:
        assert r.returncode == 0, r.stdout + r.stderr
    return r


def test_config1_gray_512(tmp_path):
    from mpi_cuda_imagemanipulation_amd import utils

    src = tmp_path / "in.ppm"
    run("gen", "--synthetic", "512x512x3", "--seed", "1", "--output", src)
    img = utils.read_image(src)
    assert img.shape == (512, 512, 3)
    out = tmp_path / "gray.pgm"
    r = run("run", "--input", src, "--output", out, "--chain", "gray", "--backend", "host", "--ranks", "1")
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["ranks"] == 1 and rec["backend"] == "host"
    # the file stages around the run are timed too
    assert rec["read_ms"] >= 0 and rec["write_ms"] >= 0 and rec["wall_ms"] > 0
    g = utils.read_image(out)
    assert g.shape == (512, 512) and (g == np_ref.gray_bt601(img)).all()
    assert out.read_bytes().startswith(b"P5\n512 512\n255\n")


@pytest.mark.parametrize("ranks", [1, 3, 4])
def test_presets_multi_rank(tmp_path, ranks):
    from mpi_cuda_imagemanipulation_amd import utils

    src = tmp_path / "in.ppm"
    run("gen", "--synthetic", "96x50x3", "--seed", "4", "--output", src)
    img = utils.read_image(src)
    rows = 50 // ranks
    out = tmp_path / "gpu.ppm"
    run("run", "--input", src, "--output", out, "--preset", "ref-gpu", "--ranks", ranks, "--backend", "host")
    got = utils.read_image(out)
    assert got.shape == img.shape  # 3-channel output like the reference's GRAY2BGR (kernel.cu:210)
    for r in range(ranks):
        s = img[r * rows:(r + 1) * rows]
        e = np_ref.stencil(np_ref.contrast_ref(np_ref.gray_ref(s), 3.5), "emboss3", "skip")
        assert (got[r * rows:(r + 1) * rows] == np_ref.expand(e)).all()
    assert (got[ranks * rows:] == 0).all()
    out2 = tmp_path / "cpu.ppm"
    run("run", "--input", src, "--output", out2, "--preset", "ref-cpu", "--ranks", ranks, "--backend", "host")
    got2 = utils.read_image(out2)
    for r in range(ranks):
        s = img[r * rows:(r + 1) * rows]
        e = np_ref.stencil(np_ref.contrast_cv(np_ref.gray_bt601(s), 3.0), "emboss3", "reflect101")
        assert (got2[r * rows:(r + 1) * rows] == np_ref.expand(e)).all()


def test_halo_run_equals_single_rank(tmp_path):
    src = tmp_path / "in.ppm"
    run("gen", "--synthetic", "77x64x3", "--seed", "2", "--output", src)
    a, b = tmp_path / "a.ppm", tmp_path / "b.ppm"
    run("run", "--input", src, "--output", a, "--chain", "gaussian5,sobel", "--ranks", "1", "--backend", "host")
    run("run", "--input", src, "--output", b, "--chain", "gaussian5,sobel", "--ranks", "5", "--backend", "host")
    r = run("cmp", a, b)
    assert json.loads(r.stdout)["max_abs"] == 0
    c = tmp_path / "c.ppm"
    run("run", "--input", src, "--output", c, "--chain", "gaussian5,sobel", "--ranks", "5", "--backend", "host",
        "--no-halo")
    r = run("cmp", a, c, check=False)
    assert r.returncode == 1 and json.loads(r.stdout)["n_diff"] > 0  # stripe seams (Q6)


def test_cmp_and_errors(tmp_path):
    src = tmp_path / "in.ppm"
    run("gen", "--synthetic", "10x10x3", "--output", src)
    assert run("cmp", src, src).returncode == 0
    r = run("run", "--input", tmp_path / "missing.ppm", "--output", tmp_path / "o.ppm", check=False)
    assert r.returncode != 0 and "cannot open" in r.stderr
    r = run("run", "--input", src, "--output", tmp_path / "o.ppm", "--chain", "nope", "--backend", "host",
            check=False)
    assert r.returncode != 0 and "unknown filter" in r.stderr
    r = run("info", "--chain", "gray:ref,contrast:3.5,emboss3")
    assert "prologue[gray:ref,lut]" in r.stdout


def test_bench_host(tmp_path):
    js = tmp_path / "b.json"
    r = run("bench", "--synthetic", "128x64x3", "--chain", "gaussian5", "--ranks", "1,2", "--iters", "2",
            "--warmup", "1", "--scope", "resident,dist", "--backend", "host", "--json", js)
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert [(x["n_ranks"], x["scope"]) for x in recs] == [(1, "resident"), (1, "dist"), (2, "resident"), (2, "dist")]
    assert all(x["value"] > 0 for x in recs)


def test_bench_frames_host(tmp_path):
    # --frames F: the resident scope steps a stream of F independent frames
    js = tmp_path / "f.json"
    run("bench", "--synthetic", "128x64x3", "--chain", "gaussian5", "--ranks", "1,2", "--iters", "4",
        "--warmup", "1", "--frames", "3", "--backend", "host", "--json", js)
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert [(x["n_ranks"], x["frames"]) for x in recs] == [(1, 3), (2, 3)] and all(x["value"] > 0 for x in recs)
    assert all("halo_schedule" not in x for x in recs)  # host engines: nothing to choose
    js2 = tmp_path / "f2.json"
    run("bench", "--synthetic", "128x64x3", "--chain", "gaussian5", "--ranks", "2", "--iters", "2", "--warmup", "1",
        "--frames", "2", "--backend", "host", "--halo-schedule", "overlap", "--json", js2)
    assert json.loads(js2.read_text().splitlines()[0])["value"] > 0
    # deep frames pinned (k*S rows every k-th step; 32-row stripes: depth 8)
    js3 = tmp_path / "f3.json"
    run("bench", "--synthetic", "128x64x3", "--chain", "gaussian5", "--ranks", "2", "--iters", "9", "--warmup", "1",
        "--frames", "2", "--backend", "host", "--halo-schedule", "serial+deep", "--json", js3)
    assert json.loads(js3.read_text().splitlines()[0])["value"] > 0


@pytest.mark.gpu
def test_gpu_bench_frames_local(tmp_path):
    js = tmp_path / "f.json"
    run("bench", "--synthetic", "2048x512x3", "--chain", "gaussian5", "--ranks", "1,2", "--iters", "8",
        "--warmup", "2", "--frames", "4", "--backend", "local", "--json", js)
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert [x["frames"] for x in recs] == [4, 4] and all(x["value"] > 0 for x in recs)
    # two ranks: the three halo schedules were timed (max over ranks), the fastest kept
    hs = recs[1]["halo_schedule"]
    assert "halo_schedule" not in recs[0] and hs["chosen"] == min(hs["ms"], key=hs["ms"].get)
    assert all(v > 0 for v in hs["ms"].values())


@pytest.mark.gpu
def test_gpu_backends_and_file_rendezvous(tmp_path):
    """local (4 logical ranks on one GPU), rccl (in-process) and the one-process-
    per-rank rccl path with a file rendezvous (world 1 on a 1-GPU box) all match
    the host golden run bit-for-bit."""
    src = tmp_path / "in.ppm"
    run("gen", "--synthetic", "700x333x3", "--seed", "4", "--output", src)
    chain = "gray:ref,contrast:3.5,emboss3,expand"
    ref = tmp_path / "ref.ppm"
    run("run", "--input", src, "--output", ref, "--chain", chain, "--backend", "host", "--ranks", "3")
    outs = []
    for extra in (["--backend", "local", "--ranks", "4"], ["--backend", "rccl", "--ranks", "1"],
                  ["--backend", "rccl", "--world", "1", "--rank", "0", "--rendezvous", tmp_path / "rv.id"]):
        o = tmp_path / f"o{len(outs)}.ppm"
        r = run("run", "--input", src, "--output", o, "--chain", chain, *extra)
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        assert rec["kernel_ms"] >= 0
        outs.append(o)
    for o in outs:
        assert run("cmp", ref, o, check=False).returncode == 0, o


def test_precision_suffixes_in_cli(tmp_path):
    # blur:K:lsb / conv:..:lsb parse through the native CLI; the host backend
    # runs the exact golden path whatever the requested precision
    r = run("info", "--chain", "blur:9:lsb")
    assert "lsb" in r.stdout
    r = run("info", "--chain", "gray:ref,contrast:3.5,emboss3@skip")
    assert "post=clamp((7v-640)>>1)" in r.stdout
    src = tmp_path / "in.ppm"
    run("gen", "--synthetic", "64x40x3", "--seed", "3", "--output", src)
    a, b = tmp_path / "a.ppm", tmp_path / "b.ppm"
    run("run", "--input", src, "--output", a, "--chain", "blur:9", "--ranks", "1", "--backend", "host")
    run("run", "--input", src, "--output", b, "--chain", "blur:9:lsb", "--ranks", "2", "--backend", "host")
    assert json.loads(run("cmp", a, b).stdout)["max_abs"] == 0
