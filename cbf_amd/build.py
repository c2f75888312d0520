"""Build libcbf_amd.so (hand-written HIP for gfx950) in-tree with hipcc.

No torch extension: the product boundary is a plain C ABI (include/cbf_amd.h) that Python
reaches through ctypes with device pointers from torch tensors.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libcbf_amd.so")
SOURCES = ["abi.cpp", "cells.hip", "filter.hip", "swarm.hip", "mc.hip", "hocbf.hip", "rps.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CBF_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
         f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"), "-I", CSRC]


def _compile(src: str) -> str:
    out = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
    path = os.path.join(CSRC, src)
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".hpp")] + \
        [os.path.join(ROOT, "include", "cbf_amd.h")]
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + FLAGS + lang + ["-c", path, "-o", out]
    subprocess.run(cmd, check=True)
    return out


def build(verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs
        subprocess.run(cmd, check=True)
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
