"""The `local` hub's halo rounds: every active
rank posts its halo exchange, the last to arrive issues all of it -- a wait
on every rank's rows, one multi-copy launch, one event every rank's stream
waits on -- instead of each of N rank threads issuing ~9 HIP calls per
exchange.  N in-process ranks sharing the GPU must still stitch bit-exactly
to the golden frame under every halo schedule, halo depth and rank count,
and the grouped send / receive path (STRIPE_LOCAL_ROUNDS=0) must agree.

Reference: the per-rank transfers of kernel.cu:137,223 (no halo exchange in
the reference).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import mpi_cuda_imagemanipulation_amd as m

C = m._C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _golden(img, chain, n):
    ref = img
    for _ in range(n):
        ref = C.golden_apply(ref, chain, "reflect101", True)
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("schedule", ["serial", "overlap", "pipeline"])
@pytest.mark.parametrize("ranks", [2, 3, 4, 8])
@pytest.mark.parametrize("chain,cc,depth", [("gaussian5", 3, 1), ("sobel", 1, 1), ("gaussian5,sobel", 1, 1),
                                            ("gaussian5", 3, 0), ("blur:9", 3, 1)])
def test_local_rounds_stitch_exact_gpu(monkeypatch, schedule, ranks, chain, cc, depth):
    monkeypatch.setenv("STRIPE_HALO_SCHEDULE", schedule)
    W, H, it = 333, 203, 3
    img = C.synth_rows(7, W, cc, 0, H)
    if cc == 1:
        img = img.reshape(H, W)
    out = np.asarray(m.models.Pipeline(chain, halo_depth=depth).run_distributed(img, ranks, "local", it))
    ref = _golden(img, chain, it)
    tol = 1 if chain.startswith("blur") else 0
    d = np.abs(out.reshape(ref.shape).astype(np.int16) - ref.astype(np.int16))
    assert d.max() <= tol, (chain, ranks, schedule, depth, int(d.max()), np.argwhere(d > tol)[:4])


_AB = r"""
import sys, numpy as np
import mpi_cuda_imagemanipulation_amd as m
C = m._C
img = C.synth_rows(3, 1000, 3, 0, 517)
out = m.models.Pipeline("gaussian5", halo_depth=1).run_distributed(img, 4, "local", 5)
np.save(sys.argv[1], np.asarray(out))
"""


@pytest.mark.gpu
def test_local_rounds_match_grouped_path_gpu(tmp_path):
    # the round path and the grouped send / receive path give the same bits
    outs = []
    for flag in ("1", "0"):
        p = tmp_path / f"o{flag}.npy"
        env = dict(os.environ, STRIPE_LOCAL_ROUNDS=flag, PYTHONPATH=ROOT)
        r = subprocess.run([sys.executable, "-c", _AB, str(p)], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(np.load(p))
    assert np.array_equal(outs[0], outs[1])


def test_host_local_group_unchanged():
    # host hubs keep the grouped path (no device rounds): N ranks == golden
    img = C.synth_rows(9, 120, 3, 0, 77)
    out = np.asarray(m.models.Pipeline("gaussian5", halo_depth=1).run_distributed(img, 3, "host", 2))
    assert np.array_equal(out.reshape(img.shape), _golden(img, "gaussian5", 2))


@pytest.mark.gpu
@pytest.mark.parametrize("chain,cc", [("gaussian5,invert,gaussian3", 3), ("sobel,brightness:10,gaussian3", 1),
                                      ("blur:9,invert", 3)])
@pytest.mark.parametrize("ranks", [2, 4])
def test_local_lazy_sends_mixed_passes_gpu(monkeypatch, chain, cc, ranks):
    # per-pass serial exchanges (STRIPE_DEEP=0; blur has no chain-level halo
    # anyway) complete their sends lazily, at the next pass's exchange; a
    # pointwise pass between two stencils has no exchange and writes the rows
    # the previous pass sent, so it must complete them first (flush_sends).
    # Stitched output == golden, iterated
    monkeypatch.setenv("STRIPE_DEEP", "0")
    monkeypatch.setenv("STRIPE_HALO_SCHEDULE", "serial")
    W, H, it = 333, 203, 3
    img = C.synth_rows(17, W, cc, 0, H)
    if cc == 1:
        img = img.reshape(H, W)
    out = np.asarray(m.models.Pipeline(chain, halo_depth=1).run_distributed(img, ranks, "local", it))
    ref = _golden(img, chain, it)
    tol = 1 if chain.startswith("blur") else 0
    d = np.abs(out.reshape(ref.shape).astype(np.int16) - ref.astype(np.int16))
    assert d.max() <= tol, (chain, ranks, int(d.max()), np.argwhere(d > tol)[:4])
