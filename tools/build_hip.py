#!/usr/bin/env python3
"""Build the gfx950 HIP kernel library in-tree: csrc/*.hip -> distributedpytorch_amd/_C/libdpa_hip.so.

Each translation unit is compiled by ``hipcc --offload-arch=gfx950 -O3 -fPIC`` in parallel, then
linked into one shared object whose HIP runtime dependency is torch's bundled ``libamdhip64.so.7``
(rpath to torch/lib), so torch and our kernels share one runtime and one set of streams.
Incremental: an object is rebuilt only when its source or csrc/*.h changed.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OUT = ROOT / "distributedpytorch_amd" / "_C"
BUILD = ROOT / "build" / "hip"
ARCH = os.environ.get("DPA_ARCH", "gfx950")


def torch_lib_dir() -> Path:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return Path(spec.origin).parent / "lib"


def hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c
    return "hipcc"


def compile_one(src: Path, extra, verbose=False) -> Path:
    obj = BUILD / (src.stem + ".o")
    hdrs = list(CSRC.glob("*.h"))
    newest = max([src.stat().st_mtime] + [h.stat().st_mtime for h in hdrs])
    if obj.exists() and obj.stat().st_mtime >= newest and not extra.get("force"):
        return obj
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", str(src), "-o", str(obj),
           "-I", str(CSRC), "-ffp-contract=fast", "-munsafe-fp-atomics", "-Wno-unused-result"]
    cmd += extra.get("flags", [])
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    if r.stderr.strip() and verbose:
        print(r.stderr[-3000:])
    return obj


def build(force=False, verbose=False, jobs=None, flags=()):
    BUILD.mkdir(parents=True, exist_ok=True)
    OUT.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    extra = {"force": force, "flags": list(flags)}
    jobs = jobs or min(8, max(1, len(srcs)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: compile_one(s, extra, verbose), srcs))
    so = OUT / "libdpa_hip.so"
    newest = max(o.stat().st_mtime for o in objs)
    if so.exists() and so.stat().st_mtime >= newest and not force:
        build_comm(force, verbose)
        return so
    tl = torch_lib_dir()
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(so), *map(str, objs),
           f"-L{tl}", "-lamdhip64", f"-Wl,-rpath,{tl}", "-Wl,--enable-new-dtags"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    build_comm(force, verbose)
    return so


def build_comm(force=False, verbose=False) -> Path:
    """Host-only RCCL communicator library (csrc/dp_comm.cpp -> _C/libdpa_comm.so) for ``-t DP``.
    Linked against torch's bundled librccl.so (SONAME librccl.so.1), the copy torch itself loads."""
    src = CSRC / "dp_comm.cpp"
    so = OUT / "libdpa_comm.so"
    if so.exists() and so.stat().st_mtime >= src.stat().st_mtime and not force:
        return so
    tl = torch_lib_dir()
    cmd = [hipcc(), "-O2", "-fPIC", "-std=c++17", "-shared", str(src), "-o", str(so), "-I/opt/rocm/include",
           f"-L{tl}", "-l:librccl.so", "-lamdhip64", f"-Wl,-rpath,{tl}", "-Wl,--enable-new-dtags"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for dp_comm.cpp:\n{r.stderr[-4000:]}")
    return so


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--save-temps", action="store_true", help="keep .s files under build/hip")
    a = ap.parse_args()
    flags = ["-save-temps"] if a.save_temps else []
    if a.save_temps:
        os.chdir(BUILD if BUILD.exists() else ROOT)
    print(build(a.force, a.verbose, a.jobs, flags))
    sys.exit(0)
