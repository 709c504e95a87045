"""Native JPEG codec (csrc/core/jpeg.cpp: sequential + progressive decode, baseline encode): the reference's own I/O
format (cv::imread of a JPEG, kernel.cu:110; imwrite JPEG, kernel.cu:236).

Oracle: Pillow (libjpeg-turbo) where it is importable.  Decoders may differ by
the IDCT's arithmetic and the colour conversion's fixed point: ours (float
IDCT, float YCbCr) stays within 3 levels of libjpeg-turbo's integer path, with
a mean difference well under 0.1 level.
"""
import io
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIL = pytest.importorskip("PIL.Image")


def _smooth(h, w, c, noise=6.0, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([128 + 100 * np.sin(x / 17.0 + k) * np.cos(y / 23.0 - k) for k in range(c)], -1)
    img = np.clip(base + rng.normal(0, noise, base.shape), 0, 255).astype(np.uint8)
    return img[..., 0] if c == 1 else img


def _pil_encode(img, **kw):
    b = io.BytesIO()
    PIL.fromarray(img).save(b, "JPEG", **kw)
    return b.getvalue()


def _pil_decode(data, gray):
    return np.asarray(PIL.open(io.BytesIO(data)).convert("L" if gray else "RGB"))


def _psnr(a, b):
    mse = ((a.astype(np.float64) - b.astype(np.float64)) ** 2).mean()
    return 10 * np.log10(255.0 ** 2 / max(mse, 1e-12))


@pytest.mark.parametrize("shape", [(64, 64, 3), (67, 93, 3), (200, 301, 3), (57, 41, 1), (1, 1, 3), (9, 300, 1)])
@pytest.mark.parametrize("subsampling", [0, 1, 2])  # Pillow: 4:4:4, 4:2:2, 4:2:0
def test_decode_matches_libjpeg(C, shape, subsampling):
    h, w, c = shape
    if c == 1 and subsampling:
        pytest.skip("gray has one sampling")
    img = _smooth(h, w, c)
    data = _pil_encode(img, quality=90, subsampling=subsampling)
    ours = C.decode_jpeg(data)
    ref = _pil_decode(data, c == 1)
    assert ours.shape == ref.shape
    d = np.abs(ours.astype(int) - ref.astype(int))
    assert d.max() <= 3 and d.mean() < 0.1, (d.max(), d.mean())


@pytest.mark.parametrize("quality", [10, 50, 95, 100])
def test_decode_across_quality(C, quality):
    img = _smooth(48, 80, 3, seed=quality)
    data = _pil_encode(img, quality=quality)
    d = np.abs(C.decode_jpeg(data).astype(int) - _pil_decode(data, False).astype(int))
    assert d.max() <= 3 and d.mean() < 0.15


@pytest.mark.parametrize("subsample", [True, False])
@pytest.mark.parametrize("shape", [(64, 64, 3), (67, 93, 3), (33, 17, 1)])
def test_encode_decodes_in_libjpeg(C, shape, subsample):
    # our files are valid JFIF: libjpeg-turbo decodes them to what we decode,
    # and the picture survives (a smooth frame at quality 95)
    h, w, c = shape
    img = _smooth(h, w, c, noise=0.0)
    enc = C.encode_jpeg(img, 95, subsample, 0)
    theirs = _pil_decode(enc, c == 1)
    ours = C.decode_jpeg(enc)
    assert np.abs(theirs.astype(int) - ours.astype(int)).max() <= 3
    assert _psnr(theirs, img) > (36.0 if (subsample and c == 3) else 40.0)


def test_encode_quality_orders_size_and_error(C):
    img = _smooth(96, 128, 3)
    sizes, errs = [], []
    for q in (20, 60, 95):
        enc = C.encode_jpeg(img, q)
        sizes.append(len(enc))
        errs.append(_psnr(C.decode_jpeg(enc), img))
    assert sizes[0] < sizes[1] < sizes[2] and errs[0] < errs[1] < errs[2]


def test_restart_interval_round_trip(C):
    img = _smooth(120, 170, 3)
    for ri in (1, 3, 7):
        enc = C.encode_jpeg(img, 90, True, ri)
        assert b"\xff\xdd" in enc and b"\xff\xd0" in enc
        ours = C.decode_jpeg(enc)
        assert np.abs(ours.astype(int) - _pil_decode(enc, False).astype(int)).max() <= 3
        assert np.array_equal(ours, C.decode_jpeg(C.encode_jpeg(img, 90, True, ri)))


def test_extreme_statistics_huffman_tables(C):
    # pure noise at quality 100 (every AC symbol class) and a flat frame (a
    # handful of symbols): the fitted Huffman tables stay valid JPEG (<= 16-bit
    # codes, no all-ones code)
    rng = np.random.default_rng(3)
    for img in (rng.integers(0, 256, (64, 96, 3), dtype=np.uint8), np.full((40, 40, 3), 77, np.uint8),
                np.zeros((16, 16), np.uint8)):
        enc = C.encode_jpeg(img, 100, False, 0)
        theirs = _pil_decode(enc, img.ndim == 2)
        assert np.abs(theirs.astype(int) - C.decode_jpeg(enc).astype(int)).max() <= 3


@pytest.mark.parametrize("shape", [(64, 64, 3), (67, 93, 3), (200, 301, 3), (57, 41, 1), (1, 1, 3), (9, 300, 1),
                                   (530, 610, 3)])
@pytest.mark.parametrize("subsampling", [0, 1, 2])
@pytest.mark.parametrize("restart", [{}, {"restart_marker_rows": 1}, {"restart_marker_blocks": 3}])
def test_progressive_decode_matches_libjpeg(C, shape, subsampling, restart):
    # SOF2 (libjpeg's default progression: interleaved DC first / refine,
    # spectral bands, successive approximation down to Al = 0), with and
    # without restart intervals
    h, w, c = shape
    if c == 1 and subsampling:
        pytest.skip("gray has one sampling")
    img = _smooth(h, w, c)
    data = _pil_encode(img, quality=90, subsampling=subsampling, progressive=True, **restart)
    assert b"\xff\xc2" in data
    ours = C.decode_jpeg(data)
    ref = _pil_decode(data, c == 1)
    assert ours.shape == ref.shape
    d = np.abs(ours.astype(int) - ref.astype(int))
    assert d.max() <= 3 and d.mean() < 0.1, (d.max(), d.mean())


@pytest.mark.parametrize("shape,subsampling", [((67, 93, 3), 2), ((200, 301, 3), 0), ((200, 301, 3), 1),
                                               ((57, 41, 1), 0), ((520, 600, 3), 2), ((600, 520, 1), 0)])
@pytest.mark.parametrize("quality", [50, 95])
def test_progressive_equals_sequential_exactly(C, shape, subsampling, quality):
    # (the two largest frames, >= 4096 blocks, take the threaded row pipeline
    # between scans; the small ones decode their scans in order)
    # the same frame saved sequential and progressive carries the same
    # quantised coefficients: the two decodes must agree bit for bit
    img = _smooth(*shape, noise=20.0, seed=quality)
    kw = {"subsampling": subsampling} if shape[2] == 3 else {}
    seq = C.decode_jpeg(_pil_encode(img, quality=quality, **kw))
    prog = C.decode_jpeg(_pil_encode(img, quality=quality, progressive=True, **kw))
    assert np.array_equal(seq, prog)


def test_truncated_progressive_decodes_what_arrived(C):
    # like libjpeg: the scans that arrived give a coarser picture, the missing
    # refinements stay zero (no error, same size, still the picture)
    img = _smooth(96, 128, 3, noise=10.0)
    data = _pil_encode(img, quality=90, progressive=True)
    full = C.decode_jpeg(data)
    part = C.decode_jpeg(data[: len(data) * 2 // 3])
    assert part.shape == full.shape and not np.array_equal(part, full)
    assert _psnr(part, img) > 20.0


def test_progressive_out_of_order_refinement_rejected_or_decoded(C):
    # a refinement scan whose Al is not Ah - 1 is malformed (T.81 G.1.1.1.1)
    data = bytearray(_pil_encode(_smooth(32, 32, 3), quality=80, progressive=True))
    k = data.index(b"\xff\xda", data.index(b"\xff\xda") + 2)  # second scan header
    ns = data[k + 4]
    data[k + 4 + 1 + 2 * ns + 2] = 0x31  # Ah 3, Al 1
    with pytest.raises(RuntimeError, match="progressive scan parameters"):
        C.decode_jpeg(bytes(data))


def test_corrupt_input_raises(C):
    with pytest.raises(RuntimeError, match="JPEG"):
        C.decode_jpeg(b"\xff\xd8\xff\xc0\x00")
    good = C.encode_jpeg(_smooth(16, 16, 3), 90)
    with pytest.raises(RuntimeError):
        C.decode_jpeg(good[: len(good) // 3])  # truncated: header fine, tables / scan cut


def _sof_file(W, H, pad):
    # SOI, a 3-component progressive SOF declaring W x H, then `pad` bytes
    sof = bytes([0xFF, 0xC2, 0x00, 17, 8, H >> 8, H & 255, W >> 8, W & 255, 3,
                 1, 0x11, 0, 2, 0x11, 0, 3, 0x11, 0])
    return b"\xff\xd8" + sof + b"\x00" * pad


def test_huge_frame_header_in_small_file_rejected(C):
    # a ~262 KB file declaring 65535 x 65535 4:4:4 passed the
    # pixels-per-byte guard and would allocate ~40 GB; the absolute pixel cap
    # (2^28 by default) rejects it before any allocation
    with pytest.raises(RuntimeError, match="pixel limit"):
        C.decode_jpeg(_sof_file(65535, 65535, 262144 + 1024))


def test_pixel_cap_env_override(tmp_path):
    # STRIPE_JPEG_MAX_PIXELS lowers (or raises) the cap; read once per process
    code = ("import sys; sys.path.insert(0, %r); from mpi_cuda_imagemanipulation_amd._native import C\n"
            "import numpy as np\n"
            "img = np.full((64, 64, 3), 90, np.uint8)\n"
            "data = C.encode_jpeg(img, 90)\n"
            "try:\n    C.decode_jpeg(data); print('DECODED')\n"
            "except RuntimeError as e:\n    print('REJECTED', 'pixel limit' in str(e))\n") % ROOT
    env = dict(os.environ, STRIPE_JPEG_MAX_PIXELS="1000")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert "REJECTED True" in r.stdout, r.stdout + r.stderr
    env["STRIPE_JPEG_MAX_PIXELS"] = "4096"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert "DECODED" in r.stdout, r.stdout + r.stderr


def test_read_image_sniffs_content_and_python_io(C, tmp_path):
    import mpi_cuda_imagemanipulation_amd as m

    img = _smooth(40, 50, 3)
    p = tmp_path / "x.jpg"
    m.utils.write_image(str(p), img, quality=92)
    assert open(p, "rb").read(2) == b"\xff\xd8"
    back = m.utils.read_image(str(p))
    assert back.shape == img.shape and _psnr(back, img) > 30
    # content, not extension, decides on read
    q = tmp_path / "y.ppm"
    q.write_bytes(p.read_bytes())
    assert np.array_equal(C.read_image(str(q)), back)


def test_cli_runs_on_jpeg_input_and_output(C, tmp_path):
    # the reference's flow: JPEG in, filtered, JPEG out (kernel.cu:110,236)
    import mpi_cuda_imagemanipulation_amd as m

    img = _smooth(70, 90, 3)
    src = tmp_path / "in.jpg"
    src.write_bytes(_pil_encode(img, quality=92))
    decoded = C.decode_jpeg(src.read_bytes())
    cli = os.path.join(ROOT, "bin", "stripe")
    if not os.path.exists(cli):
        pytest.skip("bin/stripe not built")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    out_ppm, out_jpg = tmp_path / "out.ppm", tmp_path / "out.jpg"
    for out in (out_ppm, out_jpg):
        r = subprocess.run([cli, "run", "--input", str(src), "--output", str(out), "--chain", "gaussian5",
                            "--backend", "host", "--quality", "97"], capture_output=True, text=True, env=env,
                           timeout=120)
        assert r.returncode == 0, r.stderr
    ref = C.golden_apply(decoded, "gaussian5", "reflect101", True)
    assert np.array_equal(m.utils.read_image(str(out_ppm)), ref)
    assert _psnr(C.read_image(str(out_jpg)), ref) > 38


@pytest.mark.gpu
def test_cli_jpeg_on_gpu_ref_preset(C, tmp_path):
    # the reference's whole flow on the GPU: JPEG in, gray -> contrast 3.5 ->
    # emboss3 on 3 ranks (legacy split, stripes independent), expand, JPEG and
    # PPM out; the PPM equals the golden path on the decoded frame
    import numpy as np_

    img = _smooth(211, 157, 3)
    src = tmp_path / "in.jpg"
    src.write_bytes(_pil_encode(img, quality=90))
    cli = os.path.join(ROOT, "bin", "stripe")
    out = tmp_path / "out.ppm"
    r = subprocess.run([cli, "run", "--input", str(src), "--output", str(out), "--preset", "ref-gpu", "--ranks", "3",
                        "--backend", "local"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    got = C.read_image(str(out))
    # a device run keeps the JPEG as coefficients and makes the pixels on the
    # GPU (jpeg_dev.hip): the reference frame is that same decode
    import mpi_cuda_imagemanipulation_amd as m

    dec = m.utils.read_image_device(str(src)).cpu().numpy()
    assert np.abs(dec.astype(int) - C.decode_jpeg(src.read_bytes()).astype(int)).max() <= 1
    rows = 211 // 3
    for k in range(3):
        ref = C.golden_apply(dec[k * rows:(k + 1) * rows], "gray:ref,contrast:3.5,emboss3@skip,expand", "skip", True)
        assert np_.array_equal(got[k * rows:(k + 1) * rows], ref), k


def test_parallel_restart_intervals_decode_identically(C):
    # the default encode puts a restart marker after every MCU row and both
    # sides code the intervals in parallel: the coefficients do not depend on
    # the intervals, so the decoded frames are bit-identical
    img = _smooth(250, 333, 3, seed=5)
    per_row, none, every3 = (C.encode_jpeg(img, 88, True, ri) for ri in (-1, 0, 3))
    assert b"\xff\xdd" in per_row and b"\xff\xdd" not in none
    ref = C.decode_jpeg(none)
    assert np.array_equal(C.decode_jpeg(per_row), ref) and np.array_equal(C.decode_jpeg(every3), ref)
    assert np.abs(_pil_decode(per_row, False).astype(int) - ref.astype(int)).max() <= 3
    # a lost marker: the parallel split no longer matches, the sequential
    # decoder resynchronises (no crash, same size)
    k = per_row.index(b"\xff\xd3")
    broken = per_row[:k] + per_row[k + 2:]
    assert C.decode_jpeg(broken).shape == img.shape


# ---- pixel stages on the GPU (csrc/hip/jpeg_dev.hip) ----
@pytest.mark.gpu
@pytest.mark.parametrize("shape,subsampling,progressive",
                         [((211, 157, 3), 0, False), ((211, 157, 3), 1, False), ((211, 157, 3), 2, False),
                          ((64, 99, 1), 0, False), ((1, 1, 3), 2, False), ((211, 157, 3), 2, True),
                          ((64, 99, 1), 0, True)])
def test_device_decode_matches_host(C, tmp_path, shape, subsampling, progressive):
    import mpi_cuda_imagemanipulation_amd as m

    h, w, c = shape
    img = _smooth(h, w, c)
    data = _pil_encode(img, quality=90, progressive=progressive, **({"subsampling": subsampling} if c == 3 else {}))
    p = tmp_path / "x.jpg"
    p.write_bytes(data)
    got = m.utils.read_image_device(str(p))
    assert got.is_cuda and tuple(got.shape) == img.shape
    d = np.abs(got.cpu().numpy().astype(int) - C.decode_jpeg(data).astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 0.01, (d.max(), (d > 0).mean())


@pytest.mark.gpu
def test_device_decode_restart_intervals_and_rgb_output_pitch(C):
    import torch

    img = _smooth(300, 401, 3, seed=2)
    data = C.encode_jpeg(img, 85, True, -1)
    jc = C.jpeg_entropy_decode(data)
    assert (jc.W, jc.H, jc.C) == (401, 300, 3)
    pitch = 401 * 3 + 64  # a padded destination (e.g. an engine stripe row)
    buf = torch.full((300, pitch), 7, dtype=torch.uint8, device="cuda")
    jc.to_device(buf.data_ptr(), pitch, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    assert (out[:, 401 * 3:] == 7).all()  # nothing written past the row
    d = np.abs(out[:, :401 * 3].reshape(300, 401, 3).astype(int) - jc.to_host().astype(int))
    assert d.max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("c", [3, 1])
def test_device_encode_matches_host(C, tmp_path, c):
    import torch

    import mpi_cuda_imagemanipulation_amd as m

    img = _smooth(250, 333, c, seed=4)
    p = tmp_path / "o.jpg"
    m.utils.write_image_device(str(p), torch.from_numpy(img).cuda(), quality=90)
    enc = p.read_bytes()
    ours = C.decode_jpeg(enc)
    ref = C.decode_jpeg(C.encode_jpeg(img, 90, True, -1))
    # a coefficient on a quantisation tie may round the other way: tiny differences only
    d = np.abs(ours.astype(int) - ref.astype(int))
    assert d.mean() < 0.05 and _psnr(ours, ref) > 45
    assert np.abs(_pil_decode(enc, c == 1).astype(int) - ours.astype(int)).max() <= 3
    assert _psnr(ours, img) > 30


@pytest.mark.gpu
def test_cli_jpeg_to_jpeg_on_gpu(C, tmp_path):
    # JPEG in and out of a device run: the input's pixels are made on the GPU
    # into the root buffer, the output is encoded from the root buffer on the
    # GPU (colour + DCT + quantisation) and Huffman-coded on the host
    import mpi_cuda_imagemanipulation_amd as m

    img = _smooth(301, 203, 3, seed=8)
    src = tmp_path / "in.jpg"
    src.write_bytes(_pil_encode(img, quality=92))
    out = tmp_path / "out.jpg"
    cli = os.path.join(ROOT, "bin", "stripe")
    r = subprocess.run([cli, "run", "--input", str(src), "--output", str(out), "--chain", "gaussian5", "--ranks", "2",
                        "--backend", "local", "--quality", "97"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    dec = m.utils.read_image_device(str(src)).cpu().numpy()
    ref = C.golden_apply(dec, "gaussian5", "reflect101", True)
    got = C.read_image(str(out))
    assert got.shape == ref.shape and _psnr(got, ref) > 40
    assert np.abs(_pil_decode(out.read_bytes(), False).astype(int) - got.astype(int)).max() <= 3


def test_cli_convert_and_cmp(C, tmp_path):
    cli = os.path.join(ROOT, "bin", "stripe")
    if not os.path.exists(cli):
        pytest.skip("bin/stripe not built")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    img = _smooth(50, 70, 3)
    src = tmp_path / "a.ppm"
    C.write_pnm(str(src), img)
    jpg, back = tmp_path / "b.jpg", tmp_path / "c.ppm"
    for a, b in ((src, jpg), (jpg, back)):
        r = subprocess.run([cli, "convert", "--input", str(a), "--output", str(b), "--quality", "93"],
                           capture_output=True, text=True, env=env, timeout=60)
        assert r.returncode == 0 and '"cmd":"convert"' in r.stdout, r.stderr
    assert jpg.read_bytes()[:2] == b"\xff\xd8"
    assert np.array_equal(C.read_image(str(back)), C.decode_jpeg(jpg.read_bytes()))
    r = subprocess.run([cli, "cmp", str(back), str(jpg)], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0 and '"max_abs":0' in r.stdout


@pytest.mark.parametrize("shape,subsampling", [((1200, 1400, 3), 2), ((1300, 1100, 3), 0), ((1500, 1600, 1), 0),
                                               ((1024, 1536, 3), 1)])
def test_long_scan_speculative_decode_is_exact(C, shape, subsampling):
    # > 1 MiB of entropy-coded data and no restart markers (libjpeg's default):
    # the scan is cut into pieces decoded speculatively in parallel and
    # stitched by one exact pass.  The same frame saved WITH restart markers
    # (the same coefficients, decoded interval by interval) must come out
    # bit-identical, and both agree with libjpeg
    rng = np.random.default_rng(shape[0])
    img = np.clip(128 + rng.normal(0, 50, shape), 0, 255).astype(np.uint8)
    if shape[2] == 1:
        img = img[..., 0]
    kw = {"subsampling": subsampling} if shape[2] == 3 else {}
    plain = _pil_encode(img, quality=90, **kw)
    marked = _pil_encode(img, quality=90, restart_marker_rows=1, **kw)
    assert len(plain) > (1 << 20) and b"\xff\xdd" not in plain and b"\xff\xdd" in marked
    ours = C.decode_jpeg(plain)
    assert np.array_equal(ours, C.decode_jpeg(marked))
    d = np.abs(ours.astype(int) - _pil_decode(plain, shape[2] == 1).astype(int))
    assert d.max() <= 3 and d.mean() < 0.1
    # truncated: the rows before the cut decode as in the whole file
    part = C.decode_jpeg(plain[: len(plain) * 3 // 5])
    rows = shape[0] // 3
    assert part.shape == ours.shape and np.array_equal(part[:rows], ours[:rows])


# ---- the device pixel stages (k_jpeg_idct8, k_jpeg_color16, k_jpeg_planes16)
# against the host codec, over 4:4:4 / 4:2:2 / 4:2:0 / gray, widths that are and
# are not multiples of 16, a 1x1 frame (the per-pixel / per-block kernels they
# replaced in round 5 were removed in round 6) ----
_COLOR_WORKER = r'''
import io, os, sys, json
import numpy as np
sys.path.insert(0, os.environ["STRIPE_ROOT"])
import torch
import mpi_cuda_imagemanipulation_amd as m
from mpi_cuda_imagemanipulation_amd._native import C
from PIL import Image
out = os.environ["OUT"]
def smooth(h, w, c, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([128 + 100 * np.sin(x / 17.0 + k) * np.cos(y / 23.0 - k) for k in range(c)], -1)
    img = np.clip(base + rng.normal(0, 6.0, base.shape), 0, 255).astype(np.uint8)
    return img[..., 0] if c == 1 else img
k = 0
worst = {"decode": 0, "encode": 0}
for (h, w, c) in [(211, 157, 3), (96, 512, 3), (61, 1000, 3), (64, 99, 1), (48, 256, 1), (1, 1, 3), (17, 33, 3)]:
    for sub in ([0, 1, 2] if c == 3 else [None]):
        img = smooth(h, w, c, k)
        b = io.BytesIO()
        Image.fromarray(img).save(b, "JPEG", quality=90, **({"subsampling": sub} if sub is not None else {}))
        p = os.path.join(out, f"in{k}.jpg")
        open(p, "wb").write(b.getvalue())
        dev = m.utils.read_image_device(p).cpu().numpy()
        host = C.decode_jpeg(b.getvalue())
        assert dev.shape == host.shape, (k, dev.shape, host.shape)
        worst["decode"] = max(worst["decode"], int(np.abs(dev.astype(int) - host.astype(int)).max()))
        q = os.path.join(out, f"enc{k}.jpg")
        m.utils.write_image_device(q, torch.from_numpy(img).cuda(), quality=90)
        back = C.decode_jpeg(open(q, "rb").read())
        ref = C.decode_jpeg(C.encode_jpeg(img, 90, True, -1))
        assert back.shape == ref.shape, k
        worst["encode"] = max(worst["encode"], int(np.abs(back.astype(int) - ref.astype(int)).max()))
        k += 1
print("RESULT", json.dumps(dict(worst, n=k)))
'''


@pytest.mark.gpu
def test_device_pixel_stages_match_host_codec(tmp_path):
    # device decode within one level of the host decode (float IDCT / colour
    # rounding of ties), device encode decoding within a few levels of the host
    # encoder's file
    script = tmp_path / "w.py"
    script.write_text(_COLOR_WORKER)
    env = dict(os.environ, STRIPE_ROOT=ROOT, OUT=str(tmp_path))
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "RESULT" in r.stdout, (r.stdout + r.stderr)[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][0][len("RESULT "):])
    assert res["n"] == 17 and res["decode"] <= 1 and res["encode"] <= 3, res
