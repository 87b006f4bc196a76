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

SOURCES = ["k_noise.hip", "k_cost.hip", "k_terms.hip", "k_weights.hip", "k_misc.hip", "k_sdf.hip", "selftest.hip", "engine.cpp", "setup.cpp"]
HEADERS = ["kernels.h", "setup.h", "stomp_math.h", "device_fk.h", "stamps.h", "noise_device.h", "limits_device.h", "update_device.h"]

# One rounding per operation on host and device (parity with the oracle's FP contract).
COMMON = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-Wall",
          "-Wno-unused-result", "-Wno-unused-value", "-I" + INCLUDE, "-DSTOMP_WITH_RCCL"]
ARCH = ["--offload-arch=gfx950"]


def source_hash(defines=()) -> str:
    """sha256 (16 hex digits) of the engine library's sources and compile flags (with a variant's
    extra -D defines): identifies the build a profile was taken of (tools/pmc_traffic.py records it;
    bench.py reports PMC numbers only for a match).  Compiled into the library
    (stomp_engine_source_hash), so the binding can tell a stale library from a current one."""
    import hashlib
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "stomp_engine.h")]:
        with open(path, "rb") as f:
            h.update(os.path.basename(path).encode() + b"\0" + f.read())
    h.update(" ".join(f for f in COMMON + ARCH if not f.startswith("-I")).encode())   # no checkout paths
    if defines:
        h.update((" " + " ".join(defines)).encode())
    return h.hexdigest()[:16]


_MARKER = b"STOMP_SOURCE_HASH="


def embedded_hash(lib: str):
    """The source hash compiled into a built library (read from the file, not loaded), or None."""
    try:
        with open(lib, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(_MARKER)
    if i < 0:
        return None
    return data[i + len(_MARKER): i + len(_MARKER) + 16].decode(errors="replace")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _digest(paths, flags) -> str:
    import hashlib
    h = hashlib.sha256()
    for path in paths:
        with open(path, "rb") as f:
            h.update(os.path.basename(path).encode() + b"\0" + f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def build(verbose: bool = False, force: bool = False, jobs: int = 4, variant: str = "", defines=()) -> str:
    """variant "stamps": diagnostic library with in-kernel phase stamps (libstomp_engine_stamps.so);
    any other variant name builds libstomp_engine_<name>.so with the extra -D `defines`
    (experiments only: the product library is the plain build).  An object is rebuilt when the
    digest of its source, the headers and the flags differs from the one recorded beside it (not by
    modification times); the library always carries source_hash() in a generated object."""
    os.makedirs(BUILD, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "stomp_engine.h")]
    extra = (["-DSTOMP_STAMPS"] if variant == "stamps" else []) + list(defines)
    lib = LIB.replace(".so", "_" + variant + ".so") if variant else LIB
    suffix = ("." + variant) if variant else ""
    want = source_hash(extra)
    objs, procs, stamps = [], [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, src + suffix + ".o")
        objs.append(obj)
        cmd = [HIPCC] + COMMON + extra + ARCH + ["-x", "hip", "-c", path, "-o", obj]
        dig = _digest([path] + hdrs, [f for f in cmd if not f.startswith("-I") and not f.startswith("/")])
        try:
            with open(obj + ".digest") as f:
                same = f.read().strip() == dig
        except OSError:
            same = False
        if not force and same and os.path.exists(obj):
            continue
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        stamps.append((obj + ".digest", dig))
        if len(procs) >= jobs:
            _wait(procs)
    _wait(procs)
    for f, dig in stamps:
        with open(f, "w") as fh:
            fh.write(dig + "\n")
    # the hash object: stomp_engine_source_hash() and the marker embedded_hash reads
    hsrc = os.path.join(BUILD, "source_hash" + suffix + ".cpp")
    hobj = os.path.join(BUILD, "source_hash" + suffix + ".o")
    with open(hsrc, "w") as f:
        f.write('// generated by _build.py: the source hash of this library\n'
                'static const char kMarker[] = "STOMP_SOURCE_HASH=%s";\n'
                'extern "C" const char* stomp_engine_source_hash(void) { return kMarker + 18; }\n' % want)
    r = subprocess.run(["g++", "-O2", "-fPIC", "-c", hsrc, "-o", hobj], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("hash object failed:\n" + r.stdout)
    cmd = [HIPCC] + ARCH + ["-shared", "-fPIC", "-o", lib] + objs + [hobj, "-L/opt/rocm/lib", "-lrccl",
                                                                     "-Wl,-rpath,/opt/rocm/lib"]
    if force or embedded_hash(lib) != want or _newer(lib, objs):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout)
    return lib


FACADE_SRC = os.path.join(PKG, "facade", "stomp_facade.cpp")
FACADE_LIB = os.path.join(PKG, "libstomp_facade.so")
FACADE_HDR = os.path.join(INCLUDE, "stomp_motion_planner", "stomp_facade.h")


def build_facade(verbose: bool = False, force: bool = False) -> str:
    """libstomp_facade.so: the reference-shaped C++ classes over the C ABI (host code only)."""
    lib = build(verbose=verbose)
    # the host PolicyImprovement shares the engine's setup (R^-1, chol, projection) and noise
    # (stomp_math.h) code: compiled in, with the engine's one-rounding-per-operation contract
    setup = os.path.join(CSRC, "setup.cpp")
    deps = [FACADE_SRC, FACADE_HDR, os.path.join(INCLUDE, "stomp_engine.h"), lib, setup,
            os.path.join(CSRC, "setup.h"), os.path.join(CSRC, "stomp_math.h")]
    if force or _newer(FACADE_LIB, deps):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-ffp-contract=off", "-fno-fast-math",
               "-I" + INCLUDE, "-I" + CSRC, FACADE_SRC, setup, "-o", FACADE_LIB,
               "-L" + PKG, "-l:libstomp_engine.so", "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("facade build failed:\n" + r.stdout)
    return FACADE_LIB


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
    args = sys.argv[1:]
    variant = "stamps" if "--stamps" in args else ""
    if "--variant" in args:
        variant = args[args.index("--variant") + 1]
    defs = [a for a in args if a.startswith("-D")]
    print(build(verbose=True, force="--force" in args or bool(defs), variant=variant, defines=defs))
    if not variant:
        print(build_facade(verbose=True, force="--force" in args))
