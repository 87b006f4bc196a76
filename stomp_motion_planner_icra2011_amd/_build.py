"""Builds the in-tree HIP engine library (libstomp_engine.so) for gfx950 with hipcc.

The library is written next to this file so it travels with the repository
snapshot to the GPU box; nothing is installed into site-packages.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libstomp_engine.so")
BUILD = os.path.join(ROOT, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["kernels.hip", "selftest.hip", "engine.cpp", "setup.cpp"]
HEADERS = ["kernels.h", "setup.h", "stomp_math.h"]

# One rounding per operation on host and device (parity with the oracle's FP contract).
COMMON = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-Wall",
          "-Wno-unused-result", "-Wno-unused-value", "-I" + INCLUDE, "-DSTOMP_WITH_RCCL"]
ARCH = ["--offload-arch=gfx950"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False, jobs: int = 4) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "stomp_engine.h")]
    objs, procs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, src + ".o")
        objs.append(obj)
        if not force and not _newer(obj, [path] + hdrs):
            continue
        cmd = [HIPCC] + COMMON + ARCH + ["-x", "hip", "-c", path, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        if len(procs) >= jobs:
            _wait(procs)
    _wait(procs)
    if force or _newer(LIB, objs):
        cmd = [HIPCC] + ARCH + ["-shared", "-fPIC", "-o", LIB] + objs + ["-L/opt/rocm/lib", "-lrccl",
                                                                         "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout)
    return LIB


def _wait(procs):
    errs = []
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            errs.append(" ".join(cmd) + "\n" + out.decode(errors="replace"))
    procs.clear()
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
