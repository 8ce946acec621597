"""Build libdsocr.so (gfx950 HIP kernels + C++ host engine + C ABI) in-tree.

    python deepseek-ocr.rs_amd/build.py [--jobs N] [--force]

Objects go to deepseek-ocr.rs_amd/build/, the library to
deepseek-ocr.rs_amd/lib/libdsocr.so (git-ignored, shipped to the GPU box by the
gpurun snapshot).  hipcc cross-compiles for gfx950 without a GPU.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
LIBDIR = os.path.join(ROOT, "lib")
LIB = os.path.join(LIBDIR, "libdsocr.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CLANG = os.environ.get("DSOCR_CXX", "/opt/rocm/llvm/bin/clang++")
ARCH = "gfx950"

KERNELS = ["gemm", "gemm_bf16", "moe", "norm", "attention", "misc", "decode", "lmhead", "dsq", "preprocess", "sampling",
           "dots_ops", "attention_bf16", "decode_mm", "decode_persist"]
HOST = ["engine", "dots", "capi"]


def sources():
    out = []
    for k in KERNELS:
        out.append((os.path.join(CSRC, "kernels", k + ".hip"), os.path.join(BUILD, k + ".o"), True))
    for h in HOST:
        out.append((os.path.join(CSRC, "engine", h + ".cpp"), os.path.join(BUILD, h + ".o"), False))
    return out


def headers():
    hs = []
    for d in ("common", "kernels", "engine"):
        for f in os.listdir(os.path.join(CSRC, d)):
            if f.endswith((".hpp", ".h")):
                hs.append(os.path.join(CSRC, d, f))
    hs.append(os.path.join(ROOT, "..", "include", "dsocr.h"))
    return hs


def stale(obj, src, hdrs):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in hdrs)


def compile_one(src, obj, is_kernel):
    common = ["-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-unused-command-line-argument"]
    if is_kernel:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-x", "hip"] + common + ["-c", src, "-o", obj]
    else:
        # host code: strict IEEE (no FMA contraction) for the table resizes / RoPE tables
        cmd = [CLANG, "-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-ffp-contract=off",
               "-fopenmp", "-Wall", "-Wno-unused-function"] + common + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 8, force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hdrs = headers()
    todo = [(s, o, k) for (s, o, k) in sources() if force or stale(o, s, hdrs)]
    if todo:
        if verbose:
            print(f"[dsocr build] compiling {len(todo)} file(s) for {ARCH}", file=sys.stderr)
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(lambda a: compile_one(*a), todo))
    objs = [o for (_, o, _) in sources()]
    if force or todo or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fopenmp", "-Wl,-rpath,/opt/rocm/lib/llvm/lib",
               "-Wl,-rpath,/opt/rocm/lib", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.jobs, a.force))
