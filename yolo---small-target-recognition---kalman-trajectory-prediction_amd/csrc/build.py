"""Build libyk.so (all HIP kernels + the C ABI of include/yk.h) for gfx950, in-tree.

Objects are compiled with hipcc --offload-arch=gfx950 and linked into one shared
library next to this package, so the built file travels with the repo snapshot to the
GPU box.  The library resolves libamdhip64.so.7 to torch's bundled HIP runtime when
torch is imported first (the package always imports torch before loading it), so torch
tensors and libyk share one HIP runtime / one device context.

Usage:  python csrc/build.py [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
# YK_DEFINES="-DNAME=1 ..." builds a diagnostic variant into YK_OUT (default libyk_diag.so) with
# its own object directory; the product library is never built with extra defines
DEFINES = os.environ.get("YK_DEFINES", "").split()
OUT = os.environ.get("YK_OUT") or os.path.join(PKG, "libyk_diag.so" if DEFINES else "libyk.so")
BUILD = os.path.join(HERE, ("_build_diag_" + hashlib.sha1(" ".join(DEFINES).encode()).hexdigest()[:8]) if DEFINES
                     else "_build")
ARCH = os.environ.get("YK_OFFLOAD_ARCH", "gfx950")

# (source, extra flags).  The tracker must not contract a*b+c into FMA: it reproduces
# numpy's separately rounded float64 arithmetic (see tracker.hip header).
SOURCES = [
    ("yk_host.cpp", []),
    ("yk_capi.cpp", []),
    ("program.cpp", []),
    ("tracker.hip", ["-ffp-contract=off"]),
    ("detector.hip", []),
    ("bytetrack.hip", ["-ffp-contract=off"]),
    ("gmd.hip", ["-ffp-contract=off"]),
]
HEADERS = ["yk_internal.h", "yk_host.h", os.path.join("..", "..", "include", "yk.h"), os.path.join("..", "..", "include", "yk_diag.h")]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libyk.so)")


def _torch_lib_dir() -> str | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            if os.path.isdir(d):
                return d
    except Exception:
        pass
    return None


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(src: str, extra: list[str], force: bool) -> str:
    hipcc = _hipcc()
    path = os.path.join(HERE, src)
    obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
    flags = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
             "-I", os.path.join(REPO, "include")] + DEFINES + extra
    hdrs = [os.path.join(HERE, h) for h in HEADERS]
    stamp = obj + ".sha"
    dig = _digest([path] + hdrs, flags)
    if not force and os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == dig:
        return obj
    cmd = [hipcc] + flags + ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(dig)
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(lambda s: _compile(s[0], s[1], force), SOURCES))
    tl = _torch_lib_dir()
    link = ["g++", "-shared", "-o", OUT + ".tmp"] + objs
    if tl:
        link += [f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"]
    else:
        link += ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    link += ["-Wl,--no-undefined", "-Wl,-z,defs", "-lstdc++"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
    os.replace(OUT + ".tmp", OUT)
    if verbose:
        print(f"[yk build] {OUT} ({len(objs)} objects, arch {ARCH})")
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    try:
        build(a.force, a.j)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
