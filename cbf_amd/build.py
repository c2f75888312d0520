"""Build libcbf_amd.so (hand-written HIP for gfx950) in-tree with hipcc.

The product boundary is a plain C ABI (include/cbf_amd.h): non-torch callers bind it directly
(ctypes, cgo, ...); cbf_amd/_lib.py uses ctypes, and the thin PyTorch-ROCm extension
(csrc/torch_ops.cpp -> libcbf_amd_torch.so) registers torch.ops.cbf_amd.* over it.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libcbf_amd.so")
SOURCES = ["abi.cpp", "cells.hip", "filter.hip", "swarm.hip", "window.hip", "mc.hip", "hocbf.hip", "rps.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CBF_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
         f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"), "-I", CSRC]
# A/B builds only (tools/_ab): extra -D switches from the environment; the shipped build sets none
FLAGS += [f"-D{d}" for d in os.environ.get("CBF_EXTRA_DEFS", "").split()]


def _compile(src: str, variant: str = "", defines=()) -> str:
    bdir = os.path.join(BUILD, variant) if variant else BUILD
    os.makedirs(bdir, exist_ok=True)
    out = os.path.join(bdir, os.path.splitext(src)[0] + ".o")
    path = os.path.join(CSRC, src)
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + FLAGS + [f"-D{d}" for d in defines] + lang + ["-c", path, "-o", out]
    # the object is reused only if it is newer than its sources AND was built with this exact
    # command line (a stamp beside it): an A/B build with CBF_EXTRA_DEFS never leaks into a plain one
    stamp = out + ".cmd"
    key = hashlib.sha256("\0".join(cmd).encode()).hexdigest()
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".hpp")] + \
        [os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include")) if h.endswith(".h")]
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        try:
            with open(stamp) as f:
                if f.read() == key:
                    return out
        except OSError:
            pass
    subprocess.run(cmd, check=True)
    with open(stamp, "w") as f:
        f.write(key)
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


TORCH_SRC = os.path.join(CSRC, "torch_ops.cpp")
TORCH_LIB = os.path.join(PKG, "libcbf_amd_torch.so")


def build_torch_ops(verbose: bool = False) -> str:
    """The thin PyTorch-ROCm extension (torch.ops.cbf_amd.*, csrc/torch_ops.cpp): host C++ over the
    C ABI, linked against libcbf_amd.so (rpath $ORIGIN) and torch's own libraries, built in-tree."""
    import torch
    from torch.utils import cpp_extension as ce
    deps = [TORCH_SRC, os.path.join(ROOT, "include", "cbf_amd.h"), LIB]
    if os.path.exists(TORCH_LIB) and os.path.getmtime(TORCH_LIB) >= max(os.path.getmtime(d) for d in deps):
        return TORCH_LIB
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = (["g++", "-O2", "-std=c++17", "-fPIC", "-shared", TORCH_SRC, "-o", TORCH_LIB, "-I", os.path.join(ROOT, "include"),
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
            "-DTORCH_EXTENSION_NAME=cbf_amd_torch", "-Wno-deprecated-declarations"] +
           [f"-I{p}" for p in ce.include_paths("cuda")] +
           ["-L", tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch", f"-Wl,-rpath,{tlib}",
            "-L", PKG, "-lcbf_amd", "-Wl,-rpath,$ORIGIN"])
    subprocess.run(cmd, check=True)
    if verbose:
        print(f"built {TORCH_LIB}")
    return TORCH_LIB


# Test-only builds of the library with a compile switch flipped in some sources (never loaded by
# the package): name -> (sources, defines).  CBF_SCAN_TEST_TIMEOUT makes every scan look-back give
# up, so tests/test_gpu_parity.py can check that the failure is reported, not silent; hocbfnocert
# runs every HOCBF relaxation pass (no infeasibility certificate), for tests/test_gpu_hocbf.py.
TEST_VARIANTS = {"scantimeout": (["cells.hip", "swarm.hip", "hocbf.hip", "filter.hip"], ["CBF_SCAN_TEST_TIMEOUT=1"]),
                 "apwpe8": (["filter.hip"], ["CBF_AP_WPE=8"]),
                 "winnowait": (["window.hip"], ["CBF_WIN_SPIN_LIMIT=-1"]),
                 "evqueue": (["swarm.hip", "window.hip"], ["CBF_EVENT_IN_PLACE=64"]),
                 "hocbfnocert": (["hocbf.hip"], ["CBF_HOCBF_CERT=0"])}
TEST_LIB_DIR = os.path.join(ROOT, "tests", "_lib")


def build_test_variants(verbose: bool = False) -> None:
    os.makedirs(TEST_LIB_DIR, exist_ok=True)
    base = {src: _compile(src) for src in SOURCES}
    for name, (srcs, defines) in TEST_VARIANTS.items():
        objs = [(_compile(src, name, defines) if src in srcs else base[src]) for src in SOURCES]
        out = os.path.join(TEST_LIB_DIR, f"libcbf_{name}.so")
        if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
            subprocess.run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", out] + objs, check=True)
        if verbose:
            print(f"built {out}")


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
