"""Pipelined scatter -> chain -> gather (Engine::run_dist) vs the three-call path
and the golden path: in-process host ranks (CPU) and local ranks on one GPU."""
import numpy as np
import pytest

from mpi_cuda_imagemanipulation_amd import models
from mpi_cuda_imagemanipulation_amd._native import C

CHAINS = ["gaussian5", "emboss3", "gray:ref,contrast:3.5,emboss3@skip,expand", "invert", "sobel", "gaussian7"]


def _img(rng, H, W, Cc):
    return rng.integers(0, 256, size=(H, W, Cc) if Cc > 1 else (H, W), dtype=np.uint8)


@pytest.mark.parametrize("chain", CHAINS)
@pytest.mark.parametrize("ranks,chunks", [(2, 2), (3, 4), (4, 8)])
def test_run_dist_host_matches_golden(rng, chain, ranks, chunks):
    img = _img(rng, 97, 41, 3)
    ref = C.golden_apply(img, chain, "reflect101", True)
    got = models.Pipeline(chain, dist_chunks=chunks).run_distributed(img, ranks, "host")
    assert got.shape == ref.shape
    assert (got == ref).all()


@pytest.mark.parametrize("halo,legacy", [(False, False), (False, True), (True, True)])
def test_run_dist_host_legacy_modes(rng, halo, legacy):
    # no-halo stripes (reference seams) and the legacy H/N split: same result as
    # the three-call path
    img = _img(rng, 101, 37, 3)
    chain = "gray:ref,contrast:3.5,emboss3@skip,expand"
    a = models.Pipeline(chain, halo=halo, legacy_partition=legacy).run_distributed(img, 4, "host")
    b = models.Pipeline(chain, halo=halo, legacy_partition=legacy, dist_chunks=4).run_distributed(img, 4, "host")
    assert (a == b).all()


class _Mailbox:
    """In-process transport for callback communicators (one per rank thread):
    sends post bytes, receives wait for them; group_end runs sends first."""

    def __init__(self, world):
        import threading

        self.cv = threading.Condition()
        self.box = {}
        self.groups = [0] * world

    def comm(self, rank, world):
        import ctypes

        ops = []
        seq = {}

        def group_start():
            ops.clear()

        def send(ptr, n, peer):
            ops.append(("s", ptr, n, peer))

        def recv(ptr, n, peer):
            ops.append(("r", ptr, n, peer))

        def group_end():
            self.groups[rank] += 1
            for kind, ptr, n, peer in [o for o in ops if o[0] == "s"] + [o for o in ops if o[0] == "r"]:
                key = (rank, peer) if kind == "s" else (peer, rank)
                k = seq.get((kind,) + key, 0)
                seq[(kind,) + key] = k + 1
                with self.cv:
                    if kind == "s":
                        self.box[key + (k,)] = ctypes.string_at(ptr, n)
                        self.cv.notify_all()
                    else:
                        assert self.cv.wait_for(lambda: key + (k,) in self.box, timeout=60), "recv timed out"
                        data = self.box.pop(key + (k,))
                        assert len(data) == n
                        ctypes.memmove(ptr, data, n)
            ops.clear()

        return C.make_callback_comm(rank, world, group_start, send, recv, group_end, lambda: None)


def _run_threads(img, chain, ranks, chunks, pipelined):
    import threading

    H, W, Cc = img.shape[0], img.shape[1], (1 if img.ndim == 2 else img.shape[2])
    mb = _Mailbox(ranks)
    out, errs, used = {}, [], {}

    def body(r):
        try:
            cfg = models.Pipeline(chain).config(W, H, Cc, "host")
            cfg.root_buffers = True
            e = C.Engine(cfg, mb.comm(r, ranks))
            if r == 0:
                e.load_root(img)
            used[r] = e.dist_chunks(chunks)
            if pipelined:
                e.run_dist(chunks)
            else:
                e.scatter()
                e.run(1)
                e.gather()
            if r == 0:
                out[0] = e.store_root()
        except Exception as ex:  # pragma: no cover - surfaced below
            errs.append(ex)

    th = [threading.Thread(target=body, args=(r,)) for r in range(ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    return out[0], used, mb.groups


@pytest.mark.parametrize("chain", ["gaussian5", "gray:ref,contrast:3.5,emboss3@skip,expand"])
def test_run_dist_callback_comm_pipelines(rng, chain):
    # the grouped calls match across ranks (n + 1 of them instead of scatter +
    # gather) and the gathered frame equals the three-call path and golden
    img = _img(rng, 64, 48, 3)
    a, used_a, groups_a = _run_threads(img, chain, 3, 4, pipelined=False)
    b, used_b, groups_b = _run_threads(img, chain, 3, 4, pipelined=True)
    assert set(used_b.values()) == {4}
    assert groups_b == [5, 5, 5] and groups_a[1] == groups_a[2]
    ref = C.golden_apply(img, chain, "reflect101", True)
    assert (a == ref).all() and (b == ref).all()


def test_run_dist_falls_back():
    # multi-pass chains and single ranks take scatter / run / gather
    cfg = models.Pipeline("gaussian5").config(32, 64, 3, "host")
    assert C.Engine(cfg).dist_chunks(8) == 0
    mb = _Mailbox(2)
    cfg2 = models.Pipeline("gaussian5,sobel").config(32, 64, 3, "host")
    assert C.Engine(cfg2, mb.comm(0, 2)).dist_chunks(8) == 0
    cfg3 = models.Pipeline("gaussian5").config(32, 64, 3, "host")
    assert C.Engine(cfg3, mb.comm(0, 2)).dist_chunks(8) == 8
    assert C.Engine(cfg3, mb.comm(0, 2)).dist_chunks(100) == 16  # chunks keep >= R rows


@pytest.mark.gpu
@pytest.mark.parametrize("chain", CHAINS + ["gaussian5@constant", "sobel_l2"])
@pytest.mark.parametrize("ranks,chunks", [(2, 2), (3, 5), (4, 8)])
def test_run_dist_local_gpu_matches_golden(rng, chain, ranks, chunks):
    # N logical ranks sharing one GPU (device copies between rank buffers on the
    # comm streams): the event choreography of run_dist on real HIP streams
    img = _img(rng, 203, 517, 3)
    ref = C.golden_apply(img, chain, "reflect101", True)
    got = models.Pipeline(chain, dist_chunks=chunks).run_distributed(img, ranks, "local")
    assert got.shape == ref.shape
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{chain} ranks={ranks} chunks={chunks}: {len(bad)} mismatches, first {bad[:5].tolist()}"


@pytest.mark.gpu
def test_run_dist_local_gpu_large(rng):
    # a 4096-wide RGB frame over 4 local ranks, 8 chunks, vs the three-call path
    img = _img(rng, 1024, 4096, 3)
    a = models.Pipeline("gaussian5").run_distributed(img, 4, "local")
    b = models.Pipeline("gaussian5", dist_chunks=8).run_distributed(img, 4, "local")
    assert (a == b).all()


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["gaussian5", "gaussian5@constant", "emboss3@constant", "sobel",
                                   "gray:ref,contrast:3.5,emboss3@skip,expand", "invert", "gaussian5,sobel"])
def test_run_dist_one_rank_direct(rng, chain):
    # one GPU rank: the pass reads the root frame and writes the root output
    # directly (no scatter / gather copies); multi-pass chains fall back
    img = _img(rng, 131, 1029, 3)
    cfg = models.Pipeline(chain).config(1029, 131, 3, "device", device=0)
    cfg.root_buffers = True
    e = C.Engine(cfg)
    assert e.dist_direct == (chain != "gaussian5,sobel")
    e.load_root(img)
    e.run_dist(8)
    got = e.store_root()
    ref = C.golden_apply(img, chain, "reflect101", True)
    assert got.shape == ref.shape
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{chain}: {len(bad)} mismatches, first {bad[:5].tolist()}"
