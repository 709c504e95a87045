"""Output x-margins when the row's last wave tile is short.

The stencil kernels (k_sep, k_direct, k_sobel_rp) keep each output
row's x-margins (the border extension the next pass reads) up to date after
every band: the row's edge tiles rewrite them.  Until round 6 a last tile
holding fewer than px + 1 pixels copied pixels the tile before it had stored:
another wave, unordered with the copying one.  A 333-pixel RGB row (999
bytes: tiles of 992 + 7) then read stale right-margin sources now and then --
1-LSB errors in the last columns, first seen in `test_r6_local.py` under the
pipelined schedule.  The last tile now starts early enough to hold them
(`tile_base`); it cannot hand the copy to the tile before it, because its own
last 16-byte store reaches past the row into the margin.  These shapes put the
short tile in every row and iterate, so a stale margin shows as a mismatch
against the golden path.

Reference: the interior-only bounds of embossKernel (kernel.cu:83)
are what the margins replace.
"""
import numpy as np
import pytest

import mpi_cuda_imagemanipulation_amd as m

C = m._C


def _golden(img, chain, n):
    ref = img
    for _ in range(n):
        ref = C.golden_apply(ref, chain, "reflect101", True)
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("chain,cc,W", [
    ("gaussian5", 3, 333),   # k_sep: 999-byte rows, last tile 7 bytes
    ("gaussian5", 3, 331),   # 993 bytes: last tile 1 byte
    ("gaussian7", 3, 665),   # 1995 bytes: last tile 11 bytes, px = 3
    ("sharpen", 3, 333),     # k_direct
    ("emboss5", 3, 333),
    ("sobel", 1, 993),       # k_sobel_rp: 993-byte gray rows
    ("sobel", 1, 1025),      # past a 1024-byte wide tile
    ("gaussian5", 1, 994),
])
@pytest.mark.parametrize("ranks,schedule", [(1, "serial"), (3, "pipeline"), (3, "overlap")])
def test_margins_straddling_tiles_gpu(monkeypatch, chain, cc, W, ranks, schedule):
    monkeypatch.setenv("STRIPE_HALO_SCHEDULE", schedule)
    H, it = 240, 8
    img = C.synth_rows(11, W, cc, 0, H)
    if cc == 1:
        img = img.reshape(H, W)
    out = np.asarray(m.models.Pipeline(chain, halo_depth=1).run_distributed(img, ranks, "local", it))
    ref = _golden(img, chain, it)
    d = np.abs(out.reshape(ref.shape).astype(np.int16) - ref.astype(np.int16))
    assert d.max() == 0, (chain, W, ranks, schedule, int(d.max()), np.argwhere(d > 0)[:4])
