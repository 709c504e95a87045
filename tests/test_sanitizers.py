"""Host AddressSanitizer + UBSan run of the native CLI (host
ASan/UBSan build option).  tools/build.py --sanitize instruments host code only
(-Xarch_host); the runs use the host backend so no GPU is involved.  Malformed
PPM inputs must fail cleanly (error exit, no sanitizer report)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def asan_cli():
    import build  # tools/build.py

    try:
        exe = build.build_sanitized()
    except SystemExit as e:  # toolchain without sanitizer runtimes
        pytest.skip(f"sanitized build unavailable: {e}")
    return str(exe)


def _run(exe, *args, cwd=None):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env, cwd=cwd)


def test_asan_cli_pipeline(asan_cli, tmp_path):
    a, b, c = (str(tmp_path / n) for n in ("a.ppm", "b.ppm", "c.ppm"))
    assert _run(asan_cli, "gen", "--synthetic", "97x61x3", "--seed", "2", "--output", a).returncode == 0
    for chain, ranks in [("gray:ref,contrast:3.5,emboss3,expand", "3"), ("gaussian5,sobel,blur:9,sharpen", "4")]:
        r = _run(asan_cli, "run", "--input", a, "--output", b, "--chain", chain, "--ranks", ranks, "--backend", "host")
        assert r.returncode == 0, r.stderr[-3000:]
        r = _run(asan_cli, "run", "--input", a, "--output", c, "--chain", chain, "--ranks", "1", "--backend", "host")
        assert r.returncode == 0, r.stderr[-3000:]
        r = _run(asan_cli, "cmp", b, c)
        assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    r = _run(asan_cli, "run", "--input", a, "--output", b, "--preset", "ref-gpu", "--ranks", "3", "--backend", "host")
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("payload", [
    b"", b"P6", b"P6\n", b"P6\n10 10\n", b"P6\n10 10\n255\n\x00\x01", b"P6\n-3 4\n255\n", b"P6\n4 4\n65536\n",
    b"P5\n99999999 99999999\n255\n", b"P3\n2 2\n255\n1 2 3\n", b"P7\n1 1\n255\n\x00", b"P2\n2 1\n255\n300 1\n",
    b"P6\n#comment\n1 1\n255\n\x01\x02\x03",
])
def test_asan_malformed_ppm(asan_cli, tmp_path, payload):
    f = tmp_path / "bad.ppm"
    f.write_bytes(payload)
    r = _run(asan_cli, "run", "--input", str(f), "--output", str(tmp_path / "o.ppm"), "--chain", "gaussian5",
             "--backend", "host")
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.returncode in (0, 1), (r.returncode, r.stderr[-2000:])


def test_asan_jpeg_round_trip_and_mutations(asan_cli, tmp_path):
    # JPEG in / out through the instrumented CLI, then corrupted JPEGs: each
    # either decodes or fails with an error exit, never a sanitizer report
    import random

    src, out = str(tmp_path / "a.jpg"), str(tmp_path / "b.jpg")
    assert _run(asan_cli, "gen", "--synthetic", "45x29x3", "--seed", "4", "--output", src).returncode == 0
    r = _run(asan_cli, "run", "--input", src, "--output", out, "--chain", "gaussian5", "--backend", "host")
    assert r.returncode == 0, r.stderr[-3000:]
    good = open(src, "rb").read()
    rnd = random.Random(11)
    for k in range(24):
        b = bytearray(good)
        for _ in range(rnd.randint(1, 4)):
            b[rnd.randrange(2, len(b))] = rnd.randrange(256)
        if k % 4 == 3:
            b = b[:rnd.randrange(2, len(b))]
        f = tmp_path / f"bad{k}.jpg"
        f.write_bytes(bytes(b))
        r = _run(asan_cli, "run", "--input", str(f), "--output", str(tmp_path / "o.ppm"), "--chain", "gaussian5",
                 "--backend", "host")
        assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
        assert r.returncode in (0, 1), (r.returncode, r.stderr[-2000:])


def test_asan_jpeg_decoder_fuzz(tmp_path):
    # the decoder alone, host ASan + UBSan (g++), random and header-targeted
    # mutations: every input decodes or raises, no sanitizer report
    import shutil

    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = tmp_path / "jpeg_fuzz"
    src = [os.path.join(ROOT, "tests", "native", "jpeg_fuzz.cpp"), os.path.join(ROOT, "csrc", "core", "jpeg.cpp"),
           os.path.join(ROOT, "csrc", "core", "image.cpp")]
    b = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                        "-I" + os.path.join(ROOT, "csrc", "include"), *src, "-o", str(exe), "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitizer" in b.stderr.lower():
        pytest.skip("sanitizer runtimes unavailable: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-3000:]
    seeds = []
    try:  # progressive (SOF2) seeds from libjpeg, with and without restart intervals
        import numpy as np
        from PIL import Image

        rng = np.random.default_rng(5)
        for k, kw in enumerate(({}, {"restart_marker_rows": 1})):
            img = np.clip(128 + rng.normal(0, 30, (29, 37, 3)), 0, 255).astype(np.uint8)
            f = tmp_path / f"prog{k}.jpg"
            Image.fromarray(img).save(f, "JPEG", quality=85, progressive=True, **kw)
            seeds.append(str(f))
    except ImportError:
        pass
    r = _run(str(exe), "1000", *seeds)
    assert r.returncode == 0 and "jpeg fuzz:" in r.stdout, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    if seeds:
        # a frame of >= 4096 blocks: its scans run concurrently on the row
        # pipeline (threads + progress counters) -- fewer, slower iterations
        y, x = np.mgrid[0:520, 0:600]
        big = np.clip(np.stack([128 + 90 * np.sin(x / (9.0 + k)) * np.cos(y / 13.0) for k in range(3)], -1)
                      + rng.normal(0, 12, (520, 600, 3)), 0, 255).astype(np.uint8)
        f = tmp_path / "prog_big.jpg"
        Image.fromarray(big).save(f, "JPEG", quality=85, progressive=True)
        # > 1 MiB of sequential data without restart markers: the speculative
        # parallel decode (pieces, resynchronisation, stitching)
        noise = np.clip(128 + rng.normal(0, 50, (1200, 1400, 3)), 0, 255).astype(np.uint8)
        g = tmp_path / "seq_big.jpg"
        Image.fromarray(noise).save(g, "JPEG", quality=90)
        r = _run(str(exe), "40", str(f), str(g))
        assert r.returncode == 0 and "jpeg fuzz:" in r.stdout, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]


def test_tsan_jpeg_scan_pipeline(tmp_path):
    # the threaded paths of the JPEG decoder under ThreadSanitizer (host g++):
    # the row pipeline between progressive scans (progress counters, one thread
    # per scan), restart intervals decoded in parallel, the speculative pieces
    # of a long sequential scan, the parallel pixel stages; a few mutations too (a failing scan unwinds the ones waiting on it)
    import shutil

    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    np = pytest.importorskip("numpy")
    Image = pytest.importorskip("PIL.Image")
    exe = tmp_path / "jpeg_tsan"
    src = [os.path.join(ROOT, "tests", "native", "jpeg_fuzz.cpp"), os.path.join(ROOT, "csrc", "core", "jpeg.cpp"),
           os.path.join(ROOT, "csrc", "core", "image.cpp")]
    b = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I" + os.path.join(ROOT, "csrc", "include"),
                        *src, "-o", str(exe), "-lpthread"], capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitizer" in b.stderr.lower():
        pytest.skip("ThreadSanitizer runtime unavailable: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-3000:]
    rng = np.random.default_rng(2)
    y, x = np.mgrid[0:520, 0:600]
    img = np.clip(np.stack([128 + 90 * np.sin(x / (9.0 + k)) * np.cos(y / 13.0) for k in range(3)], -1)
                  + rng.normal(0, 12, (520, 600, 3)), 0, 255).astype(np.uint8)
    seeds = []
    for k, kw in enumerate(({}, {"restart_marker_rows": 1})):
        f = tmp_path / f"p{k}.jpg"
        Image.fromarray(img).save(f, "JPEG", quality=85, progressive=True, **kw)
        seeds.append(str(f))
    # and the speculative parallel decode of a long sequential scan
    noise = np.clip(128 + rng.normal(0, 50, (1200, 1400, 3)), 0, 255).astype(np.uint8)
    f = tmp_path / "seq.jpg"
    Image.fromarray(noise).save(f, "JPEG", quality=90)
    seeds.append(str(f))
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([str(exe), "6", *seeds], capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "jpeg fuzz:" in r.stdout, (r.returncode, (r.stdout + r.stderr)[-3000:])
