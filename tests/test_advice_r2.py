"""Regression tests for the round-1 advisor findings.

* iterated chains that end in separate pointwise passes keep the x-margins the
  first pass reads (chain.cpp margin contract walks back to the last stencil);
* a legacy split (Q7) with halo exchange treats the covered rows as the frame;
* ops.apply on a new torch stream waits for the previous stream's work.
"""
import threading

import numpy as np
import pytest


def _golden_iter(C, img, chain, n, fuse=True, border="reflect101"):
    out = img
    for _ in range(n):
        out = C.golden_apply(out, chain, border, fuse)
    return out


@pytest.mark.parametrize("chain,fuse", [("gaussian5,invert", False), ("gaussian5,sharpen,gray,expand", True),
                                        ("gaussian5,sharpen,gray,expand", False), ("emboss3,brightness:9", False),
                                        ("gaussian3,invert,threshold:100", False)])
def test_iterated_margin_contract(C, chain, fuse):
    info = C.plan_info(chain, 3, "reflect101", fuse)
    need = info["passes"][0]["R"]
    assert need > 0
    # every pass from the last stencil to the end maintains the first pass's margins
    passes = info["passes"]
    last_stencil = max(i for i, p in enumerate(passes) if p["kind"] != 0)
    for p in passes[last_stencil:]:
        assert p["out_margin_px"] >= need, (chain, fuse, passes)


def test_legacy_partition_with_halo_uses_covered_frame(m_host):
    m = m_host
    img = m.utils.synthetic_image(7, 64, 42, 3)
    pipe = m.Pipeline("gaussian5", halo=True, legacy_partition=True)
    out = pipe.run_distributed(img, 4, backend="host")
    covered = 40  # 42 // 4 * 4 rows are scattered (kernel.cu:117)
    ref = m._C.golden_apply(np.ascontiguousarray(img[:covered]), "gaussian5", "reflect101", True)
    assert (out[:covered] == ref).all()
    assert (out[covered:] == 0).all()  # dropped rows are never processed (Q7)


def test_legacy_partition_with_halo_matches_one_rank(m_host):
    m = m_host
    img = m.utils.synthetic_image(8, 50, 36, 1)
    one = m.Pipeline("sobel", legacy_partition=True).run_distributed(img[:36], 1, backend="host")
    four = m.Pipeline("sobel", legacy_partition=True).run_distributed(img, 4, backend="host")
    assert (four[:36] == one).all()


@pytest.fixture(scope="module")
def m_host():
    import mpi_cuda_imagemanipulation_amd as m

    return m


# ---------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("chain,fuse", [("gaussian5,invert", False), ("gaussian5,sharpen,gray,expand", True),
                                        ("gaussian5,sharpen,gray,expand", False), ("emboss3,brightness:9", False)])
@pytest.mark.parametrize("iters", [2, 3])
def test_iterated_chain_gpu_vs_golden(m_host, chain, fuse, iters):
    m = m_host
    img = m.utils.synthetic_image(21, 133, 47, 3)
    cfg = m.Pipeline(chain, fuse=fuse).config(133, 47, 3, "device", device=0)
    e = m._C.Engine(cfg)
    e.load_packed(img)
    e.run(iters)
    got = e.store_packed()
    ref = _golden_iter(m._C, img, chain, iters, fuse)
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{chain} fuse={fuse} x{iters}: first mismatches {bad[:5].tolist()}"


@pytest.mark.gpu
def test_iterated_chain_local_ranks_vs_golden(m_host):
    m = m_host
    img = m.utils.synthetic_image(22, 97, 64, 3)
    for chain, fuse in [("gaussian5,invert", False), ("gaussian5,sharpen,gray,expand", True)]:
        got = m.Pipeline(chain, fuse=fuse).run_distributed(img, 3, backend="local", iterations=3)
        assert (got == _golden_iter(m._C, img, chain, 3, fuse)).all(), chain


@pytest.mark.gpu
def test_apply_stream_switch_orders_work(m_host):
    import torch

    m = m_host
    m.ops.clear_cache()
    img = m.utils.synthetic_image(5, 1024, 512, 3)
    ref = m._C.golden_apply(img, "gaussian5", "reflect101", True)
    x = torch.from_numpy(img).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for i in range(6):
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            outs.append(m.ops.apply(x, "gaussian5"))
    torch.cuda.synchronize()
    for o in outs:
        assert (o.cpu().numpy() == ref).all()


@pytest.mark.gpu
def test_apply_threads_share_engine(m_host):
    import torch

    m = m_host
    imgs = [m.utils.synthetic_image(30 + i, 256, 128, 3) for i in range(4)]
    refs = [m._C.golden_apply(a, "sharpen", "reflect101", True) for a in imgs]
    errs = []

    def worker(k):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                x = torch.from_numpy(imgs[k]).cuda()
                for _ in range(5):
                    y = m.ops.apply(x, "sharpen")
                torch.cuda.current_stream().synchronize()
                if not (y.cpu().numpy() == refs[k]).all():
                    errs.append(k)
        except Exception as exc:  # pragma: no cover - reported below
            errs.append(repr(exc))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
