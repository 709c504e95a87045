#!/usr/bin/env python3
"""Build the native core for gfx950: the Python extension and the `stripe` CLI.

Everything is compiled in-tree with hipcc (no JIT cache) so the built `.so`
travels with the repository snapshot to the GPU box:

    mpi_cuda_imagemanipulation_amd/_C.cpython-*.so   (pybind11 module)
    bin/stripe                                        (native CLI, links RCCL)

Objects are cached under build/obj and rebuilt when their source or any header
under csrc/ is newer.  Usage: python tools/build.py [-j N] [--clean] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "obj"
PKG = ROOT / "mpi_cuda_imagemanipulation_amd"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("STRIPE_ARCH", "gfx950")

CORE_SOURCES = [
    "core/filters.cpp",
    "core/chain.cpp",
    "core/partition.cpp",
    "core/image.cpp",
    "core/golden.cpp",
    "hip/pointwise.hip",
    "hip/stencil.hip",
    "hip/conv.hip",
    "hip/blur_sep.hip",
    "hip/dispatch.cpp",
    "runtime/comm_rccl.cpp",
    "runtime/comm_local.cpp",
    "runtime/engine.cpp",
    "runtime/trace.cpp",
]
BINDING_SOURCES = ["python/bindings.cpp"]
CLI_SOURCES = ["cli/main.cpp"]


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def module_path() -> Path:
    return PKG / ("_C" + ext_suffix())


def cli_path() -> Path:
    return ROOT / "bin" / "stripe"


def common_flags() -> list[str]:
    return [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-Wall",
        "-Wno-unused-function",
        "-Wno-unused-variable",
        "-Wno-unused-result",
        f"-I{CSRC / 'include'}",
        f"-I{CSRC / 'hip'}",
        "-I/opt/rocm/include",
    ]


def python_flags() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def newest_header() -> float:
    m = 0.0
    for p in CSRC.rglob("*.h"):
        m = max(m, p.stat().st_mtime)
    return m


def obj_for(src: str) -> Path:
    return BUILD / (src.replace("/", "__") + ".o")


def compile_one(src: str, extra: list[str], hdr_mtime: float, verbose: bool) -> Path:
    s = CSRC / src
    o = obj_for(src)
    if o.exists() and o.stat().st_mtime >= max(s.stat().st_mtime, hdr_mtime):
        return o
    cmd = [HIPCC, *common_flags(), *extra]
    if src.endswith(".hip"):
        cmd += ["-x", "hip"]
    cmd += ["-c", str(s), "-o", str(o)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise SystemExit(f"compile failed: {src}")
    if r.stderr.strip() and verbose:
        sys.stderr.write(r.stderr)
    print(f"  compiled {src}", flush=True)
    return o


def link(objs: list[Path], out: Path, shared: bool, verbose: bool) -> None:
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_name(out.name + ".tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-fPIC"]
    if shared:
        cmd += ["-shared"]
    cmd += [str(o) for o in objs]
    cmd += ["-L/opt/rocm/lib", "-lrccl", "-lamdhip64", "-lrocprofiler-sdk-roctx", "-lpthread", "-Wl,-rpath,/opt/rocm/lib", "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise SystemExit(f"link failed: {out}")
    os.replace(tmp, out)
    print(f"  linked {out.relative_to(ROOT)}", flush=True)


def build(jobs: int | None = None, verbose: bool = False, clean: bool = False, cli: bool = True) -> None:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    hdr = newest_header()
    jobs = jobs or min(8, os.cpu_count() or 4)
    pyf = python_flags()
    tasks = [(s, []) for s in CORE_SOURCES] + [(s, pyf) for s in BINDING_SOURCES]
    if cli:
        tasks += [(s, []) for s in CLI_SOURCES]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {s: ex.submit(compile_one, s, e, hdr, verbose) for s, e in tasks}
        objs = {s: f.result() for s, f in futs.items()}
    core = [objs[s] for s in CORE_SOURCES]
    mod = module_path()
    if not mod.exists() or any(o.stat().st_mtime > mod.stat().st_mtime for o in core + [objs[BINDING_SOURCES[0]]]):
        link(core + [objs[s] for s in BINDING_SOURCES], mod, shared=True, verbose=verbose)
    if cli:
        exe = cli_path()
        if not exe.exists() or any(o.stat().st_mtime > exe.stat().st_mtime for o in core + [objs[CLI_SOURCES[0]]]):
            link(core + [objs[s] for s in CLI_SOURCES], exe, shared=False, verbose=verbose)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--verbose", "-v", action="store_true")
    ap.add_argument("--no-cli", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.verbose, a.clean, cli=not a.no_cli)


if __name__ == "__main__":
    main()
