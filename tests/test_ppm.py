"""PPM/PGM codec (replaces the reference's OpenCV imread/imwrite, kernel.cu:110,236)."""
import numpy as np
import pytest

from mpi_cuda_imagemanipulation_amd import utils


def test_roundtrip_rgb_gray(tmp_path, rng):
    for shape in [(7, 5, 3), (1, 1, 3), (13, 17), (2, 300)]:
        img = rng.integers(0, 256, size=shape, dtype=np.uint8)
        p = tmp_path / "x.pnm"
        utils.write_image(p, img)
        back = utils.read_image(p)
        assert back.shape == img.shape and (back == img).all()
        raw = p.read_bytes()
        assert raw.startswith(b"P6" if len(shape) == 3 else b"P5")


def test_header_comments_and_ascii(C):
    data = b"P6\n# a comment\n2 1\n# another\n255\n" + bytes([1, 2, 3, 4, 5, 6])
    img = utils.decode_pnm(data)
    assert img.shape == (1, 2, 3) and img.reshape(-1).tolist() == [1, 2, 3, 4, 5, 6]
    asc = b"P2\n3 2\n255\n0 1 2\n 250 251 255\n"
    g = utils.decode_pnm(asc)
    assert g.tolist() == [[0, 1, 2], [250, 251, 255]]
    asc3 = b"P3 1 1 255 9 8 7"
    assert utils.decode_pnm(asc3).reshape(-1).tolist() == [9, 8, 7]


@pytest.mark.parametrize("bad", [b"", b"P7\n1 1\n255\n\x00", b"P5\n2 2\n255\n\x00\x01", b"P5\n2 2\n65535\n" + b"\x00" * 8,
                                 b"P5\n0 2\n255\n", b"Q5\n1 1\n255\n\x00", b"P5\nx 1\n255\n\x00"])
def test_bad_headers(bad):
    with pytest.raises(RuntimeError):
        utils.decode_pnm(bad)


def test_encode_is_binary_pnm():
    img = np.arange(12, dtype=np.uint8).reshape(2, 2, 3)
    enc = utils.encode_pnm(img)
    assert enc == b"P6\n2 2\n255\n" + img.tobytes()


def test_synthetic_is_deterministic_and_row_addressable(C):
    a = utils.synthetic_image(7, 33, 20, 3)
    b = utils.synthetic_image(7, 33, 20, 3)
    assert (a == b).all()
    assert not (a == utils.synthetic_image(8, 33, 20, 3)).all()
    rows = utils.synthetic_rows(7, 33, 3, 5, 9)
    assert (rows == a[5:14]).all()
    # byte values are well spread
    assert 100 < a.mean() < 155 and len(np.unique(a)) > 200


def test_file_reads_direct_and_fallback_paths(C, tmp_path, rng):
    # binary files are read straight into the frame from a 4 KiB header
    # prefix; a header longer than the prefix (comments) and ASCII files take
    # the whole-file path; both agree with the in-memory decoder
    img = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    cases = {"plain.ppm": b"P6\n53 37\n255\n" + img.tobytes(),
             "long_comment.ppm": b"P6\n#" + b"c" * 5000 + b"\n53 37\n255\n" + img.tobytes(),
             "ascii.ppm": b"P3\n53 37\n255\n" + " ".join(map(str, img.reshape(-1).tolist())).encode()}
    for name, data in cases.items():
        p = tmp_path / name
        p.write_bytes(data)
        for reader in (C.read_pnm, C.read_image):
            assert np.array_equal(reader(str(p)), img), (name, reader)
    short = tmp_path / "short.ppm"
    short.write_bytes(cases["plain.ppm"][:-5])
    with pytest.raises(RuntimeError, match="truncated"):
        C.read_pnm(str(short))
    with pytest.raises(RuntimeError):
        C.read_pnm(str(tmp_path / "missing.ppm"))
