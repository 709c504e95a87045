"""Separable stencil task order (PassLaunch::order): one task per wave in
band-major order (0) or XCD-local runs of bands in alternating directions
(1, `k_sep` kRuns, csrc/hip/stencil_kernels.h runs_task).  Bottom-up bands
must give the same bits as top-down ones: every separable filter's vertical
taps are symmetric (sobel's difference taps only flip the sign under its
magnitude).  Reference parity: the reference's stencil is kernel.cu:64-94;
the order is a launch choice of this framework (profiles/r5/cold/README.md)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import mpi_cuda_imagemanipulation_amd as m

C = m._C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_set_tuning_orders_validated():
    e = C.Engine(m.models.Pipeline("gaussian5").config(64, 40, 3, "host"))
    assert e.orders == [0]
    e.set_tuning([12], [-1], [], [1])
    assert e.orders == [1] and e.bands == [12]
    with pytest.raises(Exception):
        e.set_tuning([12], [-1], [], [2])
    with pytest.raises(Exception):
        e.set_tuning([12], [-1], [], [0, 1])


@pytest.mark.gpu
@pytest.mark.parametrize("border", ["reflect101", "skip"])
@pytest.mark.parametrize("chain,Cc", [("gaussian5", 3), ("gaussian3", 3), ("gaussian7", 1), ("sobel", 1),
                                      ("box5", 3), ("gaussian5,sobel", 1), ("gray:ref,sobel", 3)])
def test_runs_order_exact_gpu(chain, Cc, border):
    # odd width / height, every band the tuner may pick, both memory policies,
    # two iterations (ping-pong): bit-exact against the golden path.  The skip
    # border (the reference's interior-only bounds) leaves rows near the frame
    # edges untouched by physical row, which bottom-up bands must respect; a
    # gray prologue takes no task order (the launch ignores the request)
    W, H = 4100, 301
    img = C.synth_rows(11, W, Cc, 0, H)
    ref = img
    n_it = 1 if Cc == 3 and chain.startswith("gray") else 2
    for _ in range(n_it):
        ref = C.golden_apply(ref, chain, border, True)
    pipe = m.models.Pipeline(chain, border=border)
    n = len(C.Engine(pipe.config(W, H, Cc, "device", device=0)).bands)
    for band in (4, 12, 16, 32):
        for nt in (0, 1):
            e = C.Engine(pipe.config(W, H, Cc, "device", device=0))
            e.set_tuning([band] * n, [-1] * n, [nt] * n, [1] * n)
            e.load_synthetic(11)
            e.run(n_it)
            assert (e.store_packed() == ref).all(), (chain, border, band, nt)


_GROUP = r"""
import sys
import numpy as np
import mpi_cuda_imagemanipulation_amd as m
C = m._C
chain, Cc, ranks = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
W, H = 2050, 999
img = C.synth_rows(5, W, Cc, 0, H)
cfg = m.models.Pipeline(chain).config(W, H, Cc, "device", device=0, autotune=True)
out = C.run_local_group(cfg, ranks, img, 3)
ref = img
for _ in range(3):
    ref = C.golden_apply(ref, chain, "reflect101", True)
print("RESULT", int((np.asarray(out).reshape(ref.shape) != ref).sum()))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("chain,Cc", [("gaussian5", 3), ("sobel", 1)])
def test_runs_order_local_ranks_gpu(chain, Cc):
    # STRIPE_SEP_ORDER=1 pins the tuned order to kRuns on every rank: the
    # interior launch and the two-range edge launch of the halo schedule, the
    # deep-halo blocks, all bit-exact after 3 iterations on 3 ranks
    env = dict(os.environ, STRIPE_SEP_ORDER="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _GROUP, chain, str(Cc), "3"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][-1]
    assert line.split()[1] == "0", r.stdout[-2000:]
