"""Build libvs.so (the HIP/CDNA4 C-ABI library) in-tree with hipcc for gfx950.

Run: ``python -m photo_search_engine_amd.build`` (no GPU needed; hipcc cross-compiles).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvs.so")
SOURCES = ["vs_kernels.hip", "vs_api.hip", "vs_fullscan.hip", "vs_hnsw.hip", "vs_io.hip", "vs_ivf.hip", "vs_k1probe.hip",
           "vs_multi.hip"]
ARCH = os.environ.get("VS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "vs.h")]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


OBJ_DIR = os.path.join(HERE, "_obj")  # per-source objects, kept between builds (not shipped)


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every source for gfx950 and link libvs.so."""
    if not force and not needs_build():
        return LIB
    obj_dir = OBJ_DIR
    os.makedirs(obj_dir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(HERE, "..", "include", "vs.h"))
    objs, jobs = [], []
    for src in SOURCES:
        spath = os.path.join(CSRC, src)
        obj = os.path.join(obj_dir, src.replace(".hip", ".o"))
        if force or _stale(obj, [spath] + headers):
            cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result",
                   "-Wno-unused-value", "-Wno-inline-asm", "-c", spath, "-o", obj + ".tmp.o"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            jobs.append((cmd, obj))
        objs.append(obj)
    # the sources compile concurrently (vs_kernels.hip alone takes ~3 minutes)
    procs = [(subprocess.Popen(cmd), obj) for cmd, obj in jobs]
    failed = [obj for p, obj in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, "hipcc " + " ".join(os.path.basename(o) for o in failed))
    for _, obj in jobs:
        os.replace(obj + ".tmp.o", obj)
    tmp = os.path.join(HERE, "libvs.tmp.so")  # a .so suffix keeps hipcc from emitting bundle side files
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
