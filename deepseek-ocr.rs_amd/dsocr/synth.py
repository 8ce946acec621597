"""Synthetic inputs for benchmarks and tests (no network, no checkpoint here).

* ``synthetic_page``: 1024x1024 RGB8 "document" pages: white
  background, dark glyph boxes in text rows (8-24 px high), Gaussian noise sigma 8,
  seeded by the page index (numpy PCG64).
* ``SyntheticTokenizer``: a deterministic stand-in exposing the two calls
  build_prompt_tokens needs (`encode`, `token_to_id("<image>")`); a real
  `tokenizers.Tokenizer` works the same way.
"""
from __future__ import annotations

import numpy as np


def synthetic_page(index: int, width: int = 1024, height: int = 1024) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(1000 + index))
    img = np.full((height, width, 3), 255, np.uint8)
    y = int(rng.integers(24, 40))
    while y + 24 < height:
        line_h = int(rng.integers(8, 25))
        x = int(rng.integers(24, 48))
        while x + 16 < width - 24:
            gw = int(rng.integers(4, 16))
            gap = int(rng.integers(1, 5)) + (int(rng.integers(6, 16)) if rng.random() < 0.11 else 0)
            ink = int(rng.integers(0, 60))
            img[y:y + line_h, x:x + gw] = ink
            x += gw + gap
        y += line_h + int(rng.integers(6, 20))
    noise = rng.normal(0.0, 8.0, img.shape)
    return np.clip(img.astype(np.float32) + noise, 0, 255).astype(np.uint8)


class _Enc:
    def __init__(self, ids):
        self.ids = ids


class SyntheticTokenizer:
    """Whitespace/punctuation tokenizer with hashed ids in [16, vocab); `<image>` = vocab-1."""

    def __init__(self, vocab_size: int):
        self.vocab_size = vocab_size

    def token_to_id(self, tok: str):
        return self.vocab_size - 1 if tok == "<image>" else None

    def encode(self, text: str, add_special_tokens: bool = False):
        import re
        ids = []
        for piece in re.findall(r"\w+|[^\w\s]|\n", text):
            h = 2166136261
            for ch in piece.encode():
                h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
            ids.append(16 + h % (self.vocab_size - 17))
        return _Enc(ids)

    def decode(self, ids, skip_special_tokens: bool = True):
        return " ".join(f"<{i}>" for i in ids)


BENCH_PROMPT = "<image>\n<|grounding|>Convert the document to markdown."
