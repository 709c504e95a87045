"""Round-5 advisor findings, fixed in round 6.

* copy_roofline (the bench record's same-box copy floor) copies > 2 GiB in
  launches under the buffer-descriptor limit instead of refusing them.
* The autotuner probes the separable task order only for passes whose launch
  honours it (no gray / LUT prologue, no expand epilogue).
* A failed `local` group leaves no pending sends / receives behind.
"""
import pytest

import mpi_cuda_imagemanipulation_amd as m

C = m._C


@pytest.mark.gpu
def test_copy_roofline_above_2gib_gpu():
    # a 32768^2 RGB frame moves 3 GiB per copy: 2.25 GiB here, one frame pair
    r = C.copy_roofline(0, (9 << 28), 1, 3)
    assert r["bytes"] == 9 << 28 and r["event_ms"] > 0 and r["burst_ms"] > 0
    # ~ 2 x 2.25 GiB at a few TB/s: well under 10 ms, well over 0.1 ms
    assert 0.1 < r["event_ms"] < 10.0


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["gray:ref,gaussian5", "contrast:3.5,gaussian5", "gray:ref,gaussian5,expand"])
def test_order_probe_skips_passes_without_task_order_gpu(chain):
    cfg = m.models.Pipeline(chain).config(2048, 256, 3, "device", device=0, autotune=True)
    e = C.Engine(cfg)
    e.tune()
    assert all(o == 0 for o in e.orders), (chain, e.orders)


def test_local_group_failure_leaves_no_pending_ops():
    # rank 1 receives a message of the wrong size: its group fails with the
    # mismatch, rank 0's send fails on the aborted hub, and a later group on
    # rank 1 fails on the aborted hub too -- not on the failed group's stale
    # receive or a group left open
    e_recv, e_send, e_next = C.local_comm_failure_probe()
    assert "size mismatch" in e_recv
    assert "aborted" in e_send
    assert "aborted" in e_next and "nested" not in e_next and "size mismatch" not in e_next.split("aborted")[0]
