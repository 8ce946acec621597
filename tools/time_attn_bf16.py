"""Time the dots.ocr tower's attention launch (dsocr_k_attention_bf16) for two or more builds of libdsocr.so in ONE
process, alternating, on the 2048-px page's shape (one sequence of 146 x 146 = 21316 patch tokens, 12 heads of 128,
dots_vit.rs:433-498), and check the builds' outputs are bitwise equal.

    python tools/time_attn_bf16.py --lib new=deepseek-ocr.rs_amd/lib/libdsocr.so --lib old=deepseek-ocr.rs_amd/lib/libdsocr_ab_old.so
"""
import argparse
import ctypes as C
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", required=True, help="name=path")
    ap.add_argument("--L", type=int, default=21316)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    import torch
    hd = 128
    D = args.heads * hd
    libs = []
    for spec in args.lib:
        name, path = spec.split("=", 1)
        lib = C.CDLL(os.path.join(ROOT, path) if not os.path.isabs(path) else path)
        lib.dsocr_k_attention_bf16.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_void_p, C.c_long,
                                               C.c_void_p, C.c_long, C.c_int]
        lib.dsocr_k_attention_bf16.restype = C.c_int
        libs.append((name, lib))
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn(args.L, 3 * D, generator=g)
    qkv[:, :D] *= 0.6
    qkv = qkv.to(torch.bfloat16).cuda()
    outs = {n: torch.empty(args.L, D, dtype=torch.float32, device="cuda") for n, _ in libs}
    scale = 1.0 / math.sqrt(hd)
    flops = 4.0 * args.L * args.L * hd * args.heads

    def run(name, lib):
        rc = lib.dsocr_k_attention_bf16(1, args.L, args.heads, hd, scale, qkv.data_ptr(), 3 * D,
                                        outs[name].data_ptr(), D, 0)
        if rc != 0:
            raise RuntimeError(f"{name}: status {rc}")

    for name, lib in libs:  # warm
        run(name, lib)
    torch.cuda.synchronize()
    res = {n: [] for n, _ in libs}
    for r in range(args.rounds):
        for name, lib in libs:
            t0 = time.perf_counter()
            for _ in range(args.reps):
                run(name, lib)  # each call synchronises
            ms = (time.perf_counter() - t0) * 1e3 / args.reps
            res[name].append(ms)
            print(f"[attn] round {r} {name:8s} {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
    ref = outs[libs[0][0]].view(torch.int32)
    for name, _ in libs[1:]:
        same = bool(torch.equal(ref, outs[name].view(torch.int32)))
        print(f"[attn] {name} bitwise equal to {libs[0][0]}: {same}", flush=True)
    for name, _ in libs:
        print(f"[attn] {name:8s} median {float(np.median(res[name])):.3f} ms", flush=True)


if __name__ == "__main__":
    sys.exit(main())
