"""Loader for the native core (`_C`, built in-tree by tools/build.py).

torch is imported first so that the HIP runtime and RCCL libraries the
extension links against resolve to the copies torch already loaded (same
SONAMEs), giving one HIP runtime per process.  A missing extension is a hard
error: there is no silent Python fallback for the HIP path.
"""
from __future__ import annotations

import importlib
import os

try:  # noqa: SIM105 - torch is optional for pure-CPU use of the golden path
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
    try:
        return importlib.import_module(__package__ + "._C")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise ImportError(
            "mpi_cuda_imagemanipulation_amd native extension (_C) is not built; run "
            "`python tools/build.py` (hipcc, gfx950) from the repository root"
        ) from e


C = _load()
