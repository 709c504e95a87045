"""Images larger than one buffer-descriptor view (2 GiB): launch_pass splits
the stencil / conv launches into row chunks with re-based views (dispatch.cpp
launch_chunked).  A child process with a small STRIPE_DESC_LIMIT runs the
chunked path on small images for every kernel family and border; one real
> 2 GiB frame checks the production limit."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
import torch
import mpi_cuda_imagemanipulation_amd as m
rng = np.random.default_rng(5)
bad = []
chains = ["gaussian5", "gaussian7", "sobel_l2", "emboss5", "sharpen", "gray:ref,contrast:3.5,emboss3@skip,expand",
          "gray,gaussian5,expand,invert", "blur:9", "blur:31", "conv:3:1;2;1;2;4;2;1;2;1", "gaussian5,emboss3"]
for shape in [(300, 257, 3), (517, 123, 3), (400, 700)]:
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    for chain in chains:
        if chain.startswith("gray") and img.ndim == 2:
            continue
        for border in ("reflect101", "constant", "replicate"):
            got = m.ops.apply(torch.from_numpy(img).cuda(), chain, border).cpu().numpy()
            ref = m._C.golden_apply(img, chain, border, True)
            d = np.abs(got.astype(int) - ref.astype(int))
            tol = 1 if ("blur" in chain or "conv" in chain) else 0
            if got.shape != ref.shape or d.max() > tol:
                bad.append((shape, chain, border, int(d.max())))
print("BAD", bad)
sys.exit(1 if bad else 0)
"""


def test_chunked_descriptor_views_exact():
    env = dict(os.environ, STRIPE_DESC_LIMIT=str(256 * 1024), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_frame_larger_than_2gib():
    torch = pytest.importorskip("torch")
    import mpi_cuda_imagemanipulation_amd as m

    W, H = 16384, 45056  # 2.2 GB per RGB buffer: two descriptor chunks
    img = m.utils.synthetic_image(3, W, H, 3)
    x = torch.from_numpy(img).cuda()
    for chain in ("gaussian5", "emboss3@constant"):
        got = m.ops.apply(x, chain).cpu().numpy()
        ref = m._C.cpu_apply(img, chain, "reflect101", True, 0)
        assert (got == ref).all(), chain
