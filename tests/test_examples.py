"""The examples/ scripts run as documented (host paths here; the GPU paths
are the same calls on device tensors, covered by tests/test_jpeg.py)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")


def _run(*args):
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, env=ENV, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    return r.stdout


def test_reference_flow_example(C, tmp_path):
    import mpi_cuda_imagemanipulation_amd as m

    y, x = np.mgrid[0:96, 0:130]
    img = np.stack([128 + 100 * np.sin(x / 17 + k) * np.cos(y / 23 - k) for k in range(3)], -1).astype(np.uint8)
    src = tmp_path / "in.jpg"
    m.utils.write_image(str(src), img, 92)
    dec = C.decode_jpeg(src.read_bytes())
    out = tmp_path / "out.ppm"
    assert "on host" in _run("examples/reference_flow.py", str(src), str(out))
    ref = C.golden_apply(dec, "gray:ref,contrast:3.5,emboss3@skip,expand", "reflect101", True)
    assert np.array_equal(m.utils.read_image(str(out)), ref)
    out3 = tmp_path / "out3.ppm"
    assert "3 ranks" in _run("examples/reference_flow.py", str(src), str(out3), "--ranks", "3")
    assert m.utils.read_image(str(out3)).shape == img.shape


def test_frame_stream_example():
    out = _run("examples/frame_stream.py", "--backend", "gloo", "--shape", "96x64x3", "--frames", "4")
    assert "frames/s" in out and "schedule serial" in out


def test_large_kernels_example():
    out = _run("examples/large_kernels.py", "--shape", "120x70x3", "--iters", "1")
    assert "on host" in out and out.count("max |diff| vs golden") == 4


def _run_gpu(*args):
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    return r.stdout


import pytest  # noqa: E402


@pytest.mark.gpu
def test_reference_flow_example_gpu(C, tmp_path):
    import mpi_cuda_imagemanipulation_amd as m

    y, x = np.mgrid[0:200, 0:260]
    img = np.stack([128 + 100 * np.sin(x / 17 + k) * np.cos(y / 23 - k) for k in range(3)], -1).astype(np.uint8)
    src = tmp_path / "in.jpg"
    m.utils.write_image(str(src), img, 92)
    out = tmp_path / "out.ppm"
    assert "on GPU" in _run_gpu("examples/reference_flow.py", str(src), str(out))
    dec = m.utils.read_image_device(str(src)).cpu().numpy()
    ref = C.golden_apply(dec, "gray:ref,contrast:3.5,emboss3@skip,expand", "reflect101", True)
    assert np.array_equal(m.utils.read_image(str(out)), ref)


@pytest.mark.gpu
def test_frame_stream_example_gpu():
    out = _run_gpu("examples/frame_stream.py", "--backend", "rccl", "--shape", "2048x1024x3", "--frames", "16")
    assert "frames/s" in out and "1 rank(s) (rccl)" in out


@pytest.mark.gpu
def test_large_kernels_example_gpu():
    out = _run_gpu("examples/large_kernels.py", "--shape", "1024x512x3", "--iters", "2")
    assert "on GPU" in out and out.count("max |diff| vs golden") == 4
