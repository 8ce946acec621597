#!/usr/bin/env python3
"""Full-size, full-length golden fixtures (tests/golden/full_*.npz) from the CPU oracle.

BASELINE configs[1] workload through the oracle (numpy restatement of the reference path, SURVEY
§8c; test infrastructure only): the full DeepSeek-OCR config with the seeded synthetic checkpoint
(seed 7, the reference's `--dtype f16` rounding), 512 greedy tokens with the reference's default
20-gram ban, EOS ignored (the bench's budget).  Two pages:

* ``synthetic0``: the bench's synthetic 1024x1024 document page 0 (crop grid (2,2), 693 image rows);
  ``synthetic1`` .. ``synthetic7`` (64 tokens each, `--max-new 64`) complete the 8-page batch of the
  configs[2] shape (8 pages per GPU);
* ``text0`` .. ``text7`` (64 tokens): text-only prompts of an image page's length (706 tokens,
  ``dsocr.synth.text_page_prompt``): their decode streams differ from page to page, so the 8-page batch
  routes ~35 distinct experts per MoE layer and step (the image pages of the synthetic checkpoint
  decode into nearly the same stream and route 10-20);
* ``sample_1``: the reference's own asset ``assets/sample_1.png`` (2852x1756 RGBA; the reference
  drops alpha with ``to_rgb8``, model/mod.rs:2323 / preprocess.rs:115), committed here as
  tests/golden/sample_1.png (crop grid (3,2)).

Per page the fixture holds data only: prompt ids + mask, embedding checksums, the 512 greedy ids,
and per step the oracle's raw logits at its top-8 indices, at 64 fixed probe indices, plus the
top-1 / top-2 margin among the un-banned logits (what a divergence report needs).  The
reference's own bars this is read against: teacher-forcing logits <= 0.6
(crates/infer-deepseek/tests/baseline.rs:1108), exact greedy ids over a long generation
(tests/long_generation_baseline.rs:366-381).

    python tests/golden/make_full_golden.py [--pages synthetic0,sample_1] [--max-new 512]
    python tests/golden/make_full_golden.py --pages synthetic1,...,synthetic7 --max-new 64
    python tests/golden/make_full_golden.py --pages text0,...,text7 --max-new 64
    python tests/golden/make_full_golden.py --snapshot q4k --seed 0 --pages synthetic0 --max-new 64

``--snapshot q4k``: BASELINE configs[4] — the full-size synthetic Q4_K / Q8_0 DSQ snapshot
(dsocr.synth.write_synthetic_snapshot, seed 0, written to $TMPDIR) replaces every linear the reference's
DeepSeek-OCR adapter quantises, dequantised to fp16 as the engine's dequant-on-load does; the fixtures
are named full_q4k_<page>.npz.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))

FULL = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "deepseek-ocr.json")
SEED = 7
PROMPT = "<image>\n<|grounding|>Convert the document to markdown."
N_TOP, N_PROBE = 8, 64


def page_image(name):
    if name.startswith("synthetic"):
        from dsocr.synth import synthetic_page
        return synthetic_page(int(name[len("synthetic"):]))
    if name == "sample_1":
        from PIL import Image
        return np.asarray(Image.open(os.path.join(HERE, "sample_1.png")).convert("RGB"))
    raise KeyError(name)


def probe_indices(vocab):
    return np.sort(np.random.default_rng(12345).choice(vocab, N_PROBE, replace=False)).astype(np.int64)


def banned(ctx, n):
    from oracle.decoder import banned_ngram_tokens
    return banned_ngram_tokens(ctx, n)


def make(name, orc, tok, max_new, prefix="full", seed=SEED):
    from oracle.model import build_prompt_tokens
    t0 = time.time()
    if name.startswith("text"):
        from dsocr.synth import text_page_prompt
        ids = text_page_prompt(int(name[len("text"):]), vocab=tok.vocab_size)
        mask = [0] * len(ids)
        emb, crop = np.zeros((0, 1280), np.float32), (0, 0)
    else:
        img = page_image(name)
        emb, crop = orc.image_embeddings(img)
        segs = [tok.encode(s).ids for s in PROMPT.split("<image>")]
        ids, mask = build_prompt_tokens(segs, tok.token_to_id("<image>"), [emb.shape[0]])
    t1 = time.time()
    gen, logs = orc.generate(ids, mask, emb if len(emb) else None, max_new, eos_token_id=None, no_repeat_ngram_size=20, record_logits=True)
    t2 = time.time()
    V = logs[0].shape[0]
    probe = probe_indices(V)
    top_idx = np.zeros((max_new, N_TOP), np.int64)
    top_val = np.zeros((max_new, N_TOP), np.float32)
    probe_val = np.zeros((max_new, N_PROBE), np.float32)
    margin = np.zeros(max_new, np.float32)
    ctx = list(ids)
    for s, lg in enumerate(logs):
        o = np.argsort(-lg, kind="stable")[:N_TOP]
        top_idx[s], top_val[s] = o, lg[o]
        probe_val[s] = lg[probe]
        f = lg.copy()
        for t in banned(ctx, 20):
            f[t] = -np.inf
        o2 = np.argsort(-f, kind="stable")[:2]
        margin[s] = f[o2[0]] - f[o2[1]]
        assert int(o2[0]) == gen[s]
        ctx.append(gen[s])
    print(f"[{name}] crop {crop} rows {emb.shape[0]} vision {t1 - t0:.1f}s generate {t2 - t1:.1f}s "
          f"min margin {margin.min():.3g} distinct ids {len(set(gen))}", flush=True)
    np.savez_compressed(
        os.path.join(HERE, f"{prefix}_{name}.npz"),
        prompt_ids=np.asarray(ids, np.int64), image_mask=np.asarray(mask, np.uint8),
        crop=np.asarray(crop, np.int64), n_image_rows=np.int64(emb.shape[0]),
        emb_sum=np.float64(emb.astype(np.float64).sum()), emb_abs_sum=np.float64(np.abs(emb).astype(np.float64).sum()),
        emb_row0=emb[0, :16].astype(np.float32) if len(emb) else np.zeros(16, np.float32),
        emb_rowlast=emb[-1, :16].astype(np.float32) if len(emb) else np.zeros(16, np.float32),
        ids=np.asarray(gen, np.int64), top_idx=top_idx, top_val=top_val, probe_idx=probe, probe_val=probe_val,
        margin=margin, weights_seed=np.int64(seed), max_new=np.int64(max_new))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", default="synthetic0,sample_1")
    ap.add_argument("--max-new", type=int, default=512)
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--snapshot", choices=["q4k"], default=None)
    a = ap.parse_args()
    from dsocr.synth import SyntheticTokenizer
    from oracle.model import OracleModel
    from oracle.weights import Weights
    cfg = json.load(open(FULL))
    snap, prefix = None, "full"
    if a.snapshot == "q4k":
        import tempfile

        from dsocr.synth import write_synthetic_snapshot
        from oracle import dsq
        path = os.path.join(tempfile.gettempdir(), "dsocr_golden_q4k.dsq")
        write_synthetic_snapshot(cfg, path, seed=0)
        snap, prefix = dsq.Snapshot(path), "full_q4k"
    orc = OracleModel(cfg, Weights(seed=a.seed, dtype="f16", snapshot=snap))
    tok = SyntheticTokenizer(cfg.get("language_config", cfg).get("vocab_size", 129280))
    for name in a.pages.split(","):
        make(name, orc, tok, a.max_new, prefix=prefix, seed=a.seed)


if __name__ == "__main__":
    main()
