#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.json) from the CPU oracle.

The oracle is pinned independently (tests/test_oracle_crosscheck.py: decoder / SAM / CLIP against
HF transformers; tests/test_host_cpu.py: preprocessing against Pillow), the reference itself
cannot run here.  Fixtures are data only: inputs are seeds + shapes, outputs are
token ids, shapes and float checksums.  Regenerate with:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))

from oracle.model import OracleModel, build_prompt_tokens  # noqa: E402
from oracle.preprocess import prepare_vision_input  # noqa: E402
from oracle.weights import Weights  # noqa: E402

TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")
SEED = 7
PROMPT = "<image>\nConvert the document to markdown."
IMAGES = [(300, 420), (256, 256), (120, 500)]


def image(seed, h, w):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def encode(text, vocab=512):
    """The synthetic tokenizer of dsocr/synth.py, restated: FNV-1a of each word / punctuation /
    newline piece -> id in [16, vocab-1); `<image>` = vocab - 1."""
    import re
    ids = []
    for piece in re.findall(r"\w+|[^\w\s]|\n", text):
        h = 2166136261
        for ch in piece.encode():
            h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
        ids.append(16 + h % (vocab - 17))
    return ids


def main():
    cfg = json.load(open(TINY))
    orc = OracleModel(cfg, Weights(seed=SEED, dtype="f16"))
    out = {"config": "deepseek-ocr.rs_amd/dsocr/configs/tiny.json", "weights_seed": SEED, "prompt": PROMPT,
           "vision": {"base_size": 256, "image_size": 128, "crop_mode": True}, "pages": []}
    for i, (h, w) in enumerate(IMAGES):
        img = image(1000 + i, h, w)
        glob, tiles, _ = prepare_vision_input(img, 256, 128, True)
        emb, crop = orc.image_embeddings(img, 256, 128, True)
        ids, mask = build_prompt_tokens([encode(seg) for seg in PROMPT.split("<image>")], 511, [emb.shape[0]])
        gen, _ = orc.generate(ids, mask, emb, 24, eos_token_id=1, no_repeat_ngram_size=20)
        out["pages"].append({
            "image_seed": 1000 + i, "height": h, "width": w, "crop": list(crop),
            "global_pixels_sha": digest(glob), "tiles_sha": digest(tiles) if tiles is not None else None,
            "n_image_rows": int(emb.shape[0]), "embedding_sum": float(emb.astype(np.float64).sum()),
            "embedding_abs_sum": float(np.abs(emb).astype(np.float64).sum()),
            "embedding_row0_head": [float(v) for v in emb[0, :8]],
            "prompt_ids": [int(v) for v in ids], "image_mask": [int(v) for v in mask],
            "generated": [int(v) for v in gen]})
    json.dump(out, open(os.path.join(HERE, "tiny_pages.json"), "w"), indent=1)
    print("wrote tests/golden/tiny_pages.json")


if __name__ == "__main__":
    main()
