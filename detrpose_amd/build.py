"""Build libdetrpose_hip.so (gfx950) in-tree from detrpose_amd/csrc.

    python -m detrpose_amd.build            # incremental
    python -m detrpose_amd.build --force    # rebuild everything

Each translation unit is compiled by hipcc in parallel into build/*.o, then linked into
detrpose_amd/lib/libdetrpose_hip.so. The .so is git-ignored but travels to the GPU box
with the repo snapshot.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(REPO, "build", "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libdetrpose_hip.so")
ARCH = os.environ.get("DETRPOSE_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libdetrpose_hip.so)")


def _flags() -> list[str]:
    extra = os.environ.get("DETRPOSE_EXTRA_FLAGS", "").split()
    return ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
            "-I", os.path.join(REPO, "include")] + extra


def source_hash() -> str:
    """Content hash of everything that decides which kernels a plan launches and how they
    touch memory (kernel sources, the C-ABI header, the planner). Profiles committed under
    profiles/ record it, so bench.py only quotes measured HBM traffic for the exact code it
    is timing (the box receives no .git, so this is not a commit id)."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                   glob.glob(os.path.join(CSRC, "*.cpp")))
    files += [os.path.join(REPO, "include", "detrpose_hip.h"), os.path.join(PKG, "engine.py")]
    for f in files:
        h.update(os.path.relpath(f, REPO).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _stale(obj: str, src: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def build(force: bool = False, verbose: bool = False, variant: str = "") -> str:
    """variant != '': build into build/csrc-<variant> and lib/variants/<variant>/ (A/B experiments,
    with DETRPOSE_EXTRA_FLAGS) instead of the production library."""
    global BUILD, LIB
    if variant:
        BUILD = os.path.join(REPO, "build", "csrc-" + variant)
        LIB = os.path.join(LIBDIR, "variants", variant, "libdetrpose_hip.so")
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hipcc = _hipcc()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    deps = glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(REPO, "include", "detrpose_hip.h")]
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, s, deps):
            jobs.append([hipcc, *_flags(), "-c", s, "-o", o])
    if jobs:
        nproc = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
        with cf.ThreadPoolExecutor(nproc) as ex:
            for cmd, r in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
                if verbose or r.returncode:
                    sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
                if r.returncode:
                    raise RuntimeError(f"hipcc failed on {cmd[-3]}")
    if jobs or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", default="")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose, variant=a.variant))
