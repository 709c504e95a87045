"""Filter-chain "models": named pipelines and the Pipeline front end.

The reference's only "model" is its fixed chain: grayscale -> contrast ->
emboss on the GPU (kernel.cu:192-195) and the OpenCV equivalent on the CPU
(kern.cpp:73-75).  Both are presets here (bit-exact semantics, SURVEY
Appendix A), next to the BASELINE.json benchmark configurations.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, replace

import numpy as np

from .._native import C


@dataclass(frozen=True)
class PipelineSpec:
    chain: str
    border: str = "reflect101"
    halo: bool = True              # False: stripes filtered independently (reference seams, Q6)
    legacy_partition: bool = False  # True: H/N rows per rank, remainder dropped (Q7)
    description: str = ""
    extra: dict = field(default_factory=dict)


PRESETS: dict[str, PipelineSpec] = {
    # kernel.cu: gray (0.11/0.59/0.30, per-channel trunc) -> contrast 3.5 (trunc) ->
    # emboss3 with the reference's interior-only bounds; stripes independent;
    # output expanded to 3 channels (GRAY2BGR, kernel.cu:210).
    "ref-gpu": PipelineSpec("gray:ref,contrast:3.5,emboss3@skip,expand", halo=False, legacy_partition=True,
                            description="reference CUDA chain (kernel.cu:31-94,192-210)"),
    # kern.cpp: cvtColor BGR2GRAY -> 3*(x-128)+128 (saturating) -> filter2D emboss3
    # (BORDER_REFLECT_101) -> GRAY2BGR.
    "ref-cpu": PipelineSpec("gray:bt601,contrast:3:cv,emboss3,expand", halo=False, legacy_partition=True,
                            description="reference OpenCV CPU chain (kern.cpp:58-77)"),
    # BASELINE.json configs
    "config1-gray": PipelineSpec("gray", description="Grayscale 512x512 PPM, CPU path world_size=1",
                                 extra={"shape": (512, 512, 3), "ranks": 1, "backend": "host"}),
    "config2-gauss5": PipelineSpec("gaussian5", description="5x5 Gaussian 4096x4096 RGB, 1 GPU",
                                   extra={"shape": (4096, 4096, 3), "ranks": 1}),
    "config3-sobel": PipelineSpec("sobel", description="Sobel 8192x8192 gray, 4 GPUs",
                                  extra={"shape": (8192, 8192, 1), "ranks": 4}),
    "config4-gauss5": PipelineSpec("gaussian5", description="5x5 Gaussian 16384x16384 RGB, 8 GPUs, halo",
                                   extra={"shape": (16384, 16384, 3), "ranks": 8}),
    "config5-blur31": PipelineSpec("blur:31", description="31x31 blur 16384x16384 RGB (MFMA), 8 GPUs",
                                   extra={"shape": (16384, 16384, 3), "ranks": 8}),
}


def describe(chain: str, channels: int = 3, border: str = "reflect101", fuse: bool = True) -> str:
    """Human-readable compiled plan (fused passes, halo radius, margins)."""
    return C.describe_chain(chain, channels, border, fuse)


class Pipeline:
    """A filter chain bound to an execution backend.

    Pipeline("gaussian5")(img)                         # one device / golden CPU
    Pipeline.preset("ref-gpu").run_distributed(img, ranks=4, backend="local")
    """

    def __init__(self, chain: str = "gaussian5", border: str = "reflect101", halo: bool = True,
                 legacy_partition: bool = False, fuse: bool = True, overlap: bool = True, halo_depth: int = 0,
                 dist_chunks: int = 0, self_halo: bool = False):
        self.spec = PipelineSpec(chain, border, halo, legacy_partition)
        self.fuse = fuse
        self.overlap = overlap
        # iterations per halo exchange of iterated multi-rank runs (0 = auto, 1 = every step)
        self.halo_depth = int(halo_depth)
        # > 1: a one-iteration distributed run ships, filters and gathers single-pass
        # chains in this many overlapped row chunks (Engine::run_dist)
        self.dist_chunks = int(dist_chunks)
        # one rank on a one-rank RCCL communicator exchanges its boundary rows
        # with itself every pass (an interior rank's transfers, on one GPU;
        # the frame is then vertically periodic -- EngineConfig::self_halo)
        self.self_halo = bool(self_halo)
        C.parse_chain(chain)  # validate early

    @classmethod
    def preset(cls, name: str, **overrides) -> "Pipeline":
        if name not in PRESETS:
            raise KeyError(f"unknown preset {name!r}; known: {sorted(PRESETS)}")
        s = replace(PRESETS[name], **overrides) if overrides else PRESETS[name]
        return cls(s.chain, s.border, s.halo, s.legacy_partition)

    @property
    def chain(self) -> str:
        return self.spec.chain

    def plan(self, channels: int = 3) -> str:
        return describe(self.spec.chain, channels, self.spec.border, self.fuse)

    def __call__(self, image):
        from .. import ops

        return ops.apply(image, self.spec.chain, self.spec.border, self.fuse)

    def config(self, W: int, H: int, Cc: int, backend: str = "device", device: int = -1, autotune: bool = False,
               row_weights=None):
        cfg = C.EngineConfig()
        cfg.W, cfg.H, cfg.C = int(W), int(H), int(Cc)
        cfg.chain = self.spec.chain
        cfg.border = C.parse_border(self.spec.border)
        cfg.halo = self.spec.halo
        cfg.legacy_partition = self.spec.legacy_partition
        cfg.fuse = self.fuse
        cfg.overlap = self.overlap
        cfg.device = int(device)
        cfg.backend = C.Backend.host if backend == "host" else C.Backend.device
        cfg.autotune = bool(autotune)
        cfg.halo_depth = self.halo_depth
        cfg.dist_chunks = self.dist_chunks
        cfg.self_halo = self.self_halo
        if row_weights is not None:
            cfg.row_weights = [float(w) for w in row_weights]
        sched = os.environ.get("STRIPE_HALO_SCHEDULE")  # tuning: overlap | pipeline | serial
        if sched:
            cfg.pipeline = sched == "pipeline"
            cfg.overlap = sched != "serial"
        return cfg

    def run_distributed(self, image: np.ndarray, ranks: int, backend: str = "host", iterations: int = 1,
                        row_weights=None):
        """Root -> scatter -> per-rank chain with halo exchange -> gather, on `ranks`
        in-process ranks ('local' = N logical ranks sharing this process's GPU,
        'rccl' = one rank per GPU 0..N-1, one thread each, over an in-process
        RCCL communicator, 'host' = CPU golden path).  Returns the gathered
        output on the host.  row_weights: one share per rank (weighted split,
        e.g. plan_dist_split's link-aware root share); default even rows."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        H, W = img.shape[:2]
        Cc = 1 if img.ndim == 2 else img.shape[2]
        if backend not in ("local", "host", "rccl"):
            raise ValueError(f"backend must be local, host or rccl, got {backend!r}")
        cfg = self.config(W, H, Cc, "host" if backend == "host" else "device", device=0 if backend != "host" else -1,
                          row_weights=row_weights)
        if backend == "rccl":
            return C.run_rccl_group(cfg, list(range(int(ranks))), img, int(iterations))
        return C.run_local_group(cfg, int(ranks), img, int(iterations))


__all__ = ["PipelineSpec", "PRESETS", "Pipeline", "describe"]
