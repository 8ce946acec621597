"""Synthetic inputs for benchmarks and tests (no network, no checkpoint here).

* ``synthetic_page``: 1024x1024 RGB8 "document" pages: white
  background, dark glyph boxes in text rows (8-24 px high), Gaussian noise sigma 8,
  seeded by the page index (numpy PCG64).
* ``text_page_prompt``: a page's worth of text tokens (BOS + random ids, 706 by default: the prompt
  length of an image page) seeded by the page index; the decode streams of such prompts differ from
  page to page, so a batch of them routes its MoE layers like distinct real pages (the synthetic
  checkpoint decodes every synthetic image page into nearly the same stream).
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


def text_page_prompt(index: int, length: int = 706, vocab: int = 129280) -> list:
    """BOS (0) + length - 1 token ids uniform in [16, vocab - 280), numpy PCG64 seeded by 500 + index."""
    rng = np.random.default_rng(500 + index)
    return [0] + rng.integers(16, vocab - 280, length - 1).astype(np.int64).tolist()


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


# ------------------------------------------------------------------ synthetic DSQ snapshot (configs[4])
_DSQ_Q8_0, _DSQ_Q4K = 8, 12
_DSQ_BLOCK = {_DSQ_Q8_0: (32, 34), _DSQ_Q4K: (256, 144)}


def snapshot_linears(cfg: dict):
    """(name, out_dim, in_dim, has_bias) of every linear the reference's DeepSeek-OCR adapter puts in
    a snapshot (crates/dsq-models/src/adapters/deepseek_ocr.rs:41-140): q/k/v/o per layer, routed
    experts + fused shared experts on MoE layers (should_use_moe :164-172), the dense MLP otherwise,
    lm_head, the projector (with its bias)."""
    lang = cfg.get("language_config", cfg)
    H, nl, nh = lang["hidden_size"], lang["num_hidden_layers"], lang["num_attention_heads"]
    nkv = lang.get("num_key_value_heads") or nh
    hd = H // nh
    vhd = lang.get("v_head_dim") or hd
    inter = lang["intermediate_size"]
    moe_i = lang.get("moe_intermediate_size") or inter
    n_routed, n_shared = lang.get("n_routed_experts") or 0, lang.get("n_shared_experts") or 0
    freq, first_dense = lang.get("moe_layer_freq") or 1, lang.get("first_k_dense_replace") or 0
    out = []

    def mlp(p, inner):
        return [(f"{p}.gate_proj.weight", inner, H, False), (f"{p}.up_proj.weight", inner, H, False),
                (f"{p}.down_proj.weight", H, inner, False)]

    for l in range(nl):
        a = f"model.layers.{l}.self_attn"
        out += [(f"{a}.q_proj.weight", nh * hd, H, False), (f"{a}.k_proj.weight", nkv * hd, H, False),
                (f"{a}.v_proj.weight", nkv * vhd, H, False), (f"{a}.o_proj.weight", H, nh * vhd, False)]
        m = f"model.layers.{l}.mlp"
        if n_routed and l >= first_dense and freq and l % freq == 0:
            for e in range(n_routed):
                out += mlp(f"{m}.experts.{e}", moe_i)
            if n_shared:
                out += mlp(f"{m}.shared_experts", moe_i * n_shared)
        else:
            out += mlp(m, inter)
    if lang.get("lm_head", True):
        out.append(("lm_head.weight", lang["vocab_size"], H, False))
    p = cfg["projector_config"]
    out.append(("model.projector.layers.weight", p["n_embed"], p["input_dim"], True))
    return out


def snapshot_dtype(name: str, in_dim: int) -> int:
    """The reference quantizer's dtype choice for a Q4_K snapshot: lm_head and the projector Q8_0
    (adapter recommend_dtype, deepseek_ocr.rs:141-154), every other linear Q4_K, falling back to
    Q8_0 when in_dim is not a multiple of 256 (dsq-cli/src/main.rs:945-998: the expert and dense
    down projections, in_dim 896 / 6848)."""
    if name in ("lm_head.weight", "model.projector.layers.weight"):
        return _DSQ_Q8_0
    return _DSQ_Q4K if in_dim % 256 == 0 else _DSQ_Q8_0


def _q4k_blocks(rng, nb: int) -> np.ndarray:
    """nb valid Q4_K blocks whose values y = d*sc*q - dmin*m are roughly zero-mean, std ~0.02
    (the synthetic checkpoint's scale): sc in [40, 63], dmin = 8 d, m = round(7.5 sc / 8)."""
    b = rng.integers(0, 256, (nb, 144), dtype=np.uint8)
    d = (8.5e-5 * rng.uniform(0.8, 1.2, nb)).astype("<f2")
    sc = rng.integers(40, 64, (nb, 8)).astype(np.uint8)
    mc = np.rint(sc.astype(np.float32) * (7.5 / 8.0)).astype(np.uint8)
    b[:, 0:2] = d.view(np.uint8).reshape(-1, 2)
    b[:, 2:4] = (d.astype(np.float32) * 8).astype("<f2").view(np.uint8).reshape(-1, 2)
    b[:, 4:8] = sc[:, 0:4] | ((sc[:, 4:8] >> 4) << 6)
    b[:, 8:12] = mc[:, 0:4] | ((mc[:, 4:8] >> 4) << 6)
    b[:, 12:16] = (sc[:, 4:8] & 0xF) | ((mc[:, 4:8] & 0xF) << 4)
    return b


def _q8_0_blocks(rng, nb: int) -> np.ndarray:
    """nb valid Q8_0 blocks (d f16 ~ 2.7e-4, int8 codes uniform in [-127, 127]: std ~0.02)."""
    b = np.empty((nb, 34), np.uint8)
    b[:, 0:2] = (2.7e-4 * rng.uniform(0.8, 1.2, nb)).astype("<f2").view(np.uint8).reshape(-1, 2)
    b[:, 2:] = rng.integers(-127, 128, (nb, 32), dtype=np.int8).view(np.uint8)
    return b


def write_synthetic_snapshot(cfg: dict, path: str, seed: int = 0) -> dict:
    """Write a full-size Q4_K `.dsq` snapshot (crates/dsq/src/lib.rs container: magic DSQSNAP,
    version 1, header, records, payload) with random but valid blocks for every linear the
    adapter lists; payloads are streamed to the file record by record.  Returns a summary."""
    import struct
    rng = np.random.Generator(np.random.PCG64(seed))
    recs = []
    for name, out_dim, in_dim, has_bias in snapshot_linears(cfg):
        qt = snapshot_dtype(name, in_dim)
        bel, bby = _DSQ_BLOCK[qt]
        recs.append((name, out_dim, in_dim, qt, out_dim * (in_dim // bel) * bby, out_dim * 4 if has_bias else 0))

    def s(v):
        e = v.encode()
        return struct.pack("<I", len(e)) + e

    head = b"DSQSNAP" + struct.pack("<I", 1) + s("dsocr-synthetic") + s("deepseek-ocr") + s("HIP")
    head += struct.pack("<III", _DSQ_Q4K, 256, len(recs))
    meta = len(head) + sum(52 + len(r[0].encode()) for r in recs)
    table, off = bytearray(), meta
    for name, out_dim, in_dim, qt, qlen, blen in recs:
        table += s(name) + struct.pack("<IIIQQ", out_dim, in_dim, qt, off, qlen)
        off += qlen
        table += struct.pack("<QQI", off, blen, 4) if blen else struct.pack("<QQI", 0, 0, 0)  # bias f32
        off += blen
    counts = {}
    with open(path, "wb") as f:
        f.write(head)
        f.write(table)
        for name, out_dim, in_dim, qt, qlen, blen in recs:
            nb = qlen // _DSQ_BLOCK[qt][1]
            for i in range(0, nb, 1 << 20):  # bounded host memory per chunk
                n = min(1 << 20, nb - i)
                f.write((_q4k_blocks(rng, n) if qt == _DSQ_Q4K else _q8_0_blocks(rng, n)).tobytes())
            if blen:
                f.write(rng.normal(0.0, 0.02, out_dim).astype("<f4").tobytes())
            counts[qt] = counts.get(qt, 0) + 1
    return {"records": len(recs), "bytes": off, "q4k_records": counts.get(_DSQ_Q4K, 0),
            "q8_0_records": counts.get(_DSQ_Q8_0, 0)}
