#!/usr/bin/env python3
"""Golden fixtures for the dots.ocr vision tower (tests/golden/dots_*.npz) from the CPU oracle
(oracle/dots.py, the bf16-semantics restatement of crates/infer-dots/src/vision/dots_vit.rs;
test infrastructure, run in the dev container only).

Full dots.ocr vision config (dsocr/configs/dots-ocr.json), seeded synthetic checkpoint (seed 3,
tensor names `vision_tower.*`), synthetic document pages whose smart_resize target is their own
size (multiples of 28: the reference resizes nothing):
  * dots_448.npz   448 x 448  -> grid 32 x 32, 1024 patch tokens, 256 output rows
  * dots_2044.npz  2044 x 2044 -> grid 146 x 146, 21316 tokens, 5329 rows (BASELINE configs[3], "2048px")
Stored (data only): grid, row sums of the output, a few full rows (first, middle, last, seeded
picks), the sum / abs-sum, and checksums of the patch tensor.

    python tests/golden/make_dots_golden.py [--sizes 448,2044]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))
CFG = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "dots-ocr.json")
SEED = 3


def page(size):
    from dsocr.synth import synthetic_page
    return synthetic_page(0, size, size)


def pick_rows(n):
    rng = np.random.default_rng(n)
    return np.unique(np.concatenate([[0, 1, n // 2, n - 1], rng.choice(n, 12, replace=False)])).astype(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="448,2044")
    a = ap.parse_args()
    from oracle.dots import DotsVision, preprocess
    from oracle.weights import Weights
    vcfg = json.load(open(CFG))["vision_config"]
    W = Weights(seed=SEED, dtype="f32")
    model = DotsVision(vcfg, W)
    for size in [int(s) for s in a.sizes.split(",")]:
        img = page(size)
        t0 = time.time()
        patches, grid = preprocess(img)
        out = model.forward(patches, grid)
        rows = pick_rows(out.shape[0])
        np.savez_compressed(os.path.join(HERE, f"dots_{size}.npz"), size=np.int64(size), grid=np.asarray(grid, np.int64),
                            patches_sha=np.bytes_(hashlib.sha256(patches.tobytes()).hexdigest()[:16]),
                            row_sum=out.astype(np.float64).sum(1), rows=rows, row_vals=out[rows],
                            total=np.float64(out.astype(np.float64).sum()),
                            abs_total=np.float64(np.abs(out).astype(np.float64).sum()), weights_seed=np.int64(SEED))
        print(f"dots {size}: grid {grid} out {out.shape} in {time.time() - t0:.0f}s", flush=True)


if __name__ == "__main__":
    main()
