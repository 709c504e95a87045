"""Round-3 engine entry points on the GPU: the reference-window step
(run_to_host: filter + D2H into host memory, kernel.cu:190-226), per-step
device timing, the band x occupancy-cap tuning, and registered shared-memory
host frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def m():
    import mpi_cuda_imagemanipulation_amd as m

    assert torch.cuda.is_available()
    return m


def _engine(m, chain, W, H, Cc, autotune=False):
    cfg = m.models.Pipeline(chain).config(W, H, Cc, "device", device=0, autotune=autotune)
    return m._C.Engine(cfg)


@pytest.mark.parametrize("chain", ["gaussian5", "gray:ref,contrast:3.5,emboss3@skip,expand", "gaussian5,sobel",
                                   "invert", "blur:9"])
@pytest.mark.parametrize("chunks", [1, 8])
def test_run_to_host_matches_golden(m, chain, chunks):
    W, H, Cc = 1000, 301, 3
    e = _engine(m, chain, W, H, Cc)
    e.load_synthetic(4)
    info = m._C.plan_info(chain, Cc)
    shape = (H, W, info["cout"]) if info["cout"] > 1 else (H, W)
    host = torch.empty(int(np.prod(shape)), dtype=torch.uint8, pin_memory=True)
    ref = m._C.golden_apply(m._C.synth_rows(4, W, Cc, 0, H), chain, "reflect101", True)
    for _ in range(2):  # single-pass chains leave the input in place; multi-pass ones consume it
        if len(info["passes"]) > 1:
            e.load_synthetic(4)
        host.zero_()
        e.run_to_host_ptr(host.data_ptr(), chunks)
        e.synchronize()
        got = host.numpy().reshape(shape)
        d = np.abs(got.astype(int) - ref.astype(int))
        assert d.max() <= (1 if chain.startswith("blur") else 0), chain
    t = e.times.as_dict()
    assert t["d2h"] > 0 and t["e2e"] > 0


def test_run_to_host_shared_memory_frame(m):
    # the multi-rank reference window downloads into a POSIX shared-memory frame
    # page-locked with hipHostRegister (bench.py --ref-shm exercises it end to end)
    from multiprocessing import shared_memory

    W, H, Cc = 777, 128, 3
    shm = shared_memory.SharedMemory(create=True, size=W * H * Cc)
    try:
        frame = np.ndarray((W * H * Cc,), dtype=np.uint8, buffer=shm.buf)
        base = frame.ctypes.data
        assert m._C.host_register(base, W * H * Cc)
        e = _engine(m, "gaussian5", W, H, Cc)
        e.load_synthetic(2)
        e.run_to_host_ptr(base, 4)
        e.synchronize()
        ref = m._C.golden_apply(m._C.synth_rows(2, W, Cc, 0, H), "gaussian5", "reflect101", True)
        assert (frame.reshape(H, W, Cc) == ref).all()
        m._C.host_unregister(base)
        del frame
    finally:
        shm.close()
        shm.unlink()


def test_run_timed_per_step(m):
    e = _engine(m, "gaussian5", 2048, 512, 3)
    e.load_synthetic(1)
    ms = e.run_timed(12, 1, False)
    assert len(ms) == 12 and all(t > 0 for t in ms)
    ms3 = e.run_timed(12, 4, False)
    assert len(ms3) == 3
    e2 = _engine(m, "gray,gaussian5,expand", 2048, 512, 3)
    e2.load_synthetic(1)
    assert len(e2.run_timed(5, 1, True)) == 5  # channel-changing chain: same input each step


@pytest.mark.parametrize("chain", ["gaussian5", "emboss3", "gray:ref,contrast:3.5,emboss3@skip,expand", "sobel"])
def test_occupancy_caps_exact(m, chain):
    # every cap the autotuner may pick (LDS reservation: 0 / 2 / 3 / 4 workgroups
    # per CU, or the family default) leaves the output bit-exact
    W, H, Cc = 4100, 300, 3
    ref = m._C.golden_apply(m._C.synth_rows(6, W, Cc, 0, H), chain, "reflect101", True)
    for band in (4, 16):
        for cap in (-1, 0, 2, 3, 4):
            e = _engine(m, chain, W, H, Cc)
            e.set_tuning([band], [cap])
            e.load_synthetic(6)
            e.run(1)
            assert (e.store_packed() == ref).all(), (chain, band, cap)


def test_autotune_picks_band_and_cap(m):
    e = _engine(m, "gaussian5", 16384, 1024, 3, autotune=True)
    e.load_synthetic(1)
    e.tune()
    assert e.bands[0] in (4, 8, 12, 16, 24, 32)
    assert e.caps[0] in (-1, 0, 2, 3, 4)
    e.run(2)
    ref = m._C.synth_rows(1, 16384, 3, 0, 1024)
    for _ in range(2):
        ref = m._C.golden_apply(ref, "gaussian5", "reflect101", True)
    assert (e.store_packed() == ref).all()


def test_device_info(m):
    d = m._C.device_info(0)
    assert d["gcn_arch"].startswith("gfx950") and d["cu_count"] >= 1 and d["hbm_gib"] > 1


@pytest.mark.parametrize("pw", ["contrast:3.5", "contrast:0.25,invert", "brightness:-17", "contrast:1.7",
                                "threshold:100"])
@pytest.mark.parametrize("st", ["emboss3@skip", "gaussian5", "sharpen"])
@pytest.mark.parametrize("expand", [False, True])
def test_gray_ref_post_affine_matches_golden(m, pw, st, expand):
    # gray:ref prologue with the post map in packed i16 (affine) or the LDS table
    chain = f"gray:ref,{pw},{st}" + (",expand" if expand else "")
    W, H = 1037, 77
    img = m._C.synth_rows(9, W, 3, 0, H)
    x = torch.from_numpy(img).cuda()
    got = m.ops.apply(x, chain, "reflect101").cpu().numpy()
    ref = m._C.golden_apply(img, chain, "reflect101", True)
    assert (got == ref).all()
