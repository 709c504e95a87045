"""MI355X-native distributed image filtering (the capabilities of
Dohruba/MPI-CUDA-ImageManipulation, rebuilt for gfx950 + RCCL over xGMI).

Layers:
  ops       - filters on torch tensors (HIP kernels) or numpy arrays (golden CPU path)
  models    - filter chains ("models"): presets ref-gpu / ref-cpu, north-star configs
  parallel  - row-partitioned distributed pipeline: RCCL / local / host / gloo comms,
              FrameStream (a stream of frames, halo schedule measured per job)
  utils     - PPM/PGM and baseline JPEG I/O (JPEG pixel stages on the GPU: read_image_device /
              write_image_device), synthetic frames, logging
The native core (C++/HIP, csrc/) is loaded from `_C`; the `stripe` CLI in bin/
drives the same core without Python.
"""
from ._native import C as _C  # noqa: F401  (loads torch first, then the extension)
from . import ops, models, parallel, utils  # noqa: E402
from .models import Pipeline, PRESETS  # noqa: E402
from .ops import apply  # noqa: E402

__version__ = "0.4.0"

__all__ = ["ops", "models", "parallel", "utils", "Pipeline", "PRESETS", "apply", "__version__"]
