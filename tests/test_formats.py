"""Image formats beyond PNM (Pillow, optional) and the Python front end
(`python -m mpi_cuda_imagemanipulation_amd`), host backend."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIL = pytest.importorskip("PIL")


def test_png_roundtrip_and_jpeg_read(tmp_path):
    from mpi_cuda_imagemanipulation_amd import utils

    img = utils.synthetic_image(5, 40, 30, 3)
    utils.write_image(tmp_path / "a.png", img)
    assert (utils.read_image(tmp_path / "a.png") == img).all()
    g = img[..., 0].copy()
    utils.write_image(tmp_path / "g.png", g)
    assert (utils.read_image(tmp_path / "g.png") == g).all()
    yy, xx = np.mgrid[0:30, 0:40]
    smooth = np.stack([xx * 6, yy * 8, (xx + yy) * 3], axis=-1).astype(np.uint8)  # JPEG-friendly content
    utils.write_image(tmp_path / "a.jpg", smooth, quality=100)
    j = utils.read_image(tmp_path / "a.jpg")
    assert j.shape == smooth.shape and np.abs(j.astype(int) - smooth.astype(int)).mean() < 3  # lossy


def test_python_cli_run_preset_and_convert(tmp_path):
    from mpi_cuda_imagemanipulation_amd import utils
    from mpi_cuda_imagemanipulation_amd._native import C

    img = utils.synthetic_image(6, 64, 48, 3)
    utils.write_image(tmp_path / "in.png", img)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "mpi_cuda_imagemanipulation_amd", "run", "--input",
                        str(tmp_path / "in.png"), "--output", str(tmp_path / "out.ppm"), "--chain",
                        "gray:ref,contrast:3.5,emboss3", "--ranks", "3", "--backend", "host"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["ranks"] == 3
    out = utils.read_image(tmp_path / "out.ppm")
    assert (out == C.golden_apply(img, "gray:ref,contrast:3.5,emboss3", "reflect101", True)).all()
    r = subprocess.run([sys.executable, "-m", "mpi_cuda_imagemanipulation_amd", "convert", str(tmp_path / "out.ppm"),
                        str(tmp_path / "out.png")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (utils.read_image(tmp_path / "out.png") == out).all()
    r = subprocess.run([sys.executable, "-m", "mpi_cuda_imagemanipulation_amd", "filters"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0 and "sepconv" in r.stdout
