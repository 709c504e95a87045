"""The autotune's round-robin stages and the collective tune
(Engine.set_tune_reduce, FrameStream.tune(reduce_max)): every candidate's
median goes through the reduce, so every rank of a job decides on the same
numbers (profiles/r6/tune/)."""
import os

import pytest

import mpi_cuda_imagemanipulation_amd as m
from mpi_cuda_imagemanipulation_amd import parallel
from mpi_cuda_imagemanipulation_amd.models import Pipeline

C = m._C


def test_set_tune_reduce_accepts_function_and_none():
    e = C.Engine(Pipeline("gaussian5").config(64, 32, 3, "host"))
    calls = []
    e.set_tune_reduce(lambda v: calls.append(v) or v)
    e.tune()  # host engines have nothing to tune: the reduce is never called
    e.set_tune_reduce(None)
    assert calls == []


def test_frame_stream_tune_is_local_on_host_engines(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = parallel.init("gloo")
    fs = parallel.FrameStream(ctx, Pipeline("gaussian5", halo_depth=1), 64, 40, 3)
    calls = []
    fs.tune(lambda v: calls.append(v) or v)
    assert calls == [] and fs.every_rank_has_rows


@pytest.mark.gpu
def test_engine_tune_reduce_sees_every_candidate_gpu():
    # a cold-tuned separable pass: 6 bands, the 2 fastest again, the cap
    # challenge (incumbent + 4 caps), the cold policy challenge (incumbent + 2)
    # and the task-order challenge (incumbent + 1 or 2): every median passes
    # through the reduce, and the tuning it picks is a valid one
    cfg = Pipeline("gaussian5").config(4096, 1024, 3)
    cfg.cold = True
    cfg.autotune = True
    e = C.Engine(cfg)
    e.load_synthetic(1)
    calls = []
    e.set_tune_reduce(lambda v: calls.append(v) or v)
    e.tune()
    e.set_tune_reduce(None)
    assert 6 + 2 + 5 + 3 + 2 <= len(calls) <= 6 + 2 + 5 + 3 + 3, len(calls)
    assert all(v > 0 for v in calls)
    assert e.bands[0] in (4, 8, 12, 16, 24, 32) and e.caps[0] in (-1, 0, 2, 3, 4) and e.orders[0] in (0, 1)


@pytest.mark.gpu
def test_engine_tune_reduce_decides_gpu():
    # the reduce's numbers, not the rank's own, decide: a reduce that makes
    # every median but the first (the 4-row band) look slow picks 4 rows, and
    # no cap or task order can beat an incumbent that ties it
    cfg = Pipeline("gaussian5").config(4096, 1024, 3)
    cfg.autotune = True
    e = C.Engine(cfg)
    e.load_synthetic(1)
    # the band sweep is round-robin over 6 bands: the first median is 4 rows'
    def reduce_first(v, seen=[]):
        seen.append(v)
        return 1.0 if len(seen) == 1 else 100.0

    e.set_tune_reduce(reduce_first)
    e.tune()
    e.set_tune_reduce(None)
    assert e.bands[0] == 4 and e.caps[0] == -1
