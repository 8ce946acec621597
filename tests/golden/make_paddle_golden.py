"""Fixtures of the PaddleOCR-VL CPU plumbing path (BASELINE configs[0]) — tests/test_paddle.py checks them.

The reference's own PaddleOCR-VL parity fixtures (baselines/fixtures/paddleocr_vl/*.npz, crates/infer-paddleocr/
tests/model.rs:35-64) and its checkpoint are not in /root/reference, so these fixtures pin the numpy restatement
(dsocr/paddle.py) against itself: greedy ids of the seeded synthetic checkpoint on the reference's
assets/sample_1.png (full PaddleOCR-VL-0.9B architecture, image_size 640 as the CLI default) and on a seeded
synthetic page (tiny architecture), with the prompt ids, the grid and checksums of the projected image rows.
Parity against the reference itself is unpinned (no Rust toolchain, no checkpoint offline).

    python tests/golden/make_paddle_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deepseek-ocr.rs_amd")]

from dsocr import paddle  # noqa: E402

PROMPT = "<image>\nOCR:"
CASES = {
    # name: (config, image, image_size, max_new_tokens)
    "tiny": (paddle.PADDLE_TINY_CONFIG, "synthetic", 224, 24),
    "sample1": (paddle.PADDLE_CONFIG, "sample_1.png", 640, 16),
}


def image(name):
    if name == "synthetic":
        return np.random.default_rng(3).integers(0, 256, (300, 420, 3), dtype=np.uint8)
    from PIL import Image
    return np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", name)).convert("RGB"))


def run(name):
    cfg_path, img_name, image_size, n = CASES[name]
    eng = paddle.PaddleOcrEngine(cfg_path, synthetic_seed=0)
    tok = paddle.PaddleSyntheticTokenizer(eng.cfg)
    img = image(img_name)
    emb, grid = eng.encode_image(img, image_size)
    toks, mask = paddle.build_prompt_tokens(tok, PROMPT, [grid], eng.cfg)
    pos, delta = paddle.compute_position_ids(eng.cfg, toks, [grid])
    ids, plen = eng.generate(tok, PROMPT, [img], image_size=image_size, max_new_tokens=n, no_repeat_ngram_size=20)
    eng.close()
    return {"ids": np.array(ids, np.int64), "prompt_ids": np.array(toks, np.int64), "image_mask": np.array(mask, np.uint8),
            "grid": np.array(grid, np.int64), "positions": pos, "delta": np.int64(delta),
            "emb_sum": np.float64(emb.astype(np.float64).sum()), "emb_abs_sum": np.float64(np.abs(emb.astype(np.float64)).sum()),
            "emb_row0": emb[0, :16].astype(np.float32), "image_size": np.int64(image_size), "max_new": np.int64(n)}


if __name__ == "__main__":
    for name in sys.argv[1:] or CASES:
        out = run(name)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", f"paddle_{name}.npz"), **out)
        print(name, out["ids"].tolist(), out["grid"].tolist(), len(out["prompt_ids"]))
