"""Oracle: whole DeepSeek-OCR page path (TEST INFRASTRUCTURE).

load -> prepare_vision_input -> image embeddings -> build_prompt_tokens ->
inject -> generate, restating model/mod.rs:1181-1251 (forward),
1760-1857 (inject_image_tokens), 1870-2048 (generate), 2370-2455 (decode),
2536-2689 (build_prompt_tokens / build_image_placeholders).
"""
from __future__ import annotations

import math

import numpy as np

from . import preprocess
from .config import resolved_language_config
from .decoder import Decoder, select_token_id
from .vision import Vision
from .weights import Weights

F32 = np.float32


def image_placeholder_count(base_size, image_size, crop_mode, crop_shape):
    """build_image_placeholders model/mod.rs:2605-2689 (Ocr1): number of <image> slots."""
    patch, down = 16, 4
    n = 0
    if crop_mode:
        ng = int(math.ceil((base_size // patch) / down))
        nl = int(math.ceil((image_size // patch) / down))
        wc, hc = crop_shape if crop_shape is not None else (1, 1)
        if wc > 1 or hc > 1:
            n += (nl * hc) * (nl * wc + 1)
        n += ng * (ng + 1) + 1
    else:
        nq = int(math.ceil((image_size // patch) / down))
        n += nq * (nq + 1) + 1
    return n


def build_prompt_tokens(segment_ids, image_token_id, placeholder_counts, bos_id=0):
    """build_prompt_tokens model/mod.rs:2536-2603 with pre-tokenised segments
    (segment_ids[i] = tokenizer.encode(segments[i], add_special_tokens=false))."""
    if len(segment_ids) - 1 != len(placeholder_counts):
        raise ValueError(f"prompt/image embedding mismatch: {len(segment_ids) - 1} slots vs {len(placeholder_counts)} embeddings")
    ids, mask = [bos_id], [0]
    for i, seg in enumerate(segment_ids):
        ids += list(seg)
        mask += [0] * len(seg)
        if i < len(placeholder_counts):
            ids += [image_token_id] * placeholder_counts[i]
            mask += [1] * placeholder_counts[i]
    return ids, mask


class OracleModel:
    def __init__(self, cfg: dict, weights: Weights):
        self.cfg = cfg
        self.W = weights
        self.vision = Vision(cfg, weights)
        self.dec = Decoder(cfg, weights)
        self.lang = resolved_language_config(cfg)

    def image_embeddings(self, rgb: np.ndarray, base=1024, image_size=640, crop_mode=True):
        glob, patches, crop = preprocess.prepare_vision_input(rgb, base, image_size, crop_mode)
        emb = self.vision.embeddings(glob, patches, crop)
        return emb, crop

    def prefill_embeddings(self, ids, mask, image_rows):
        """embed_tokens + inject_image_tokens (model/mod.rs:1208-1239)."""
        e = self.dec.embed(ids)
        m = np.asarray(mask, bool)
        if m.any():
            if image_rows is None or image_rows.shape[0] != int(m.sum()):
                raise ValueError("image embeddings provide {} tokens but mask requires {}".format(
                    0 if image_rows is None else image_rows.shape[0], int(m.sum())))
            e = e.copy()
            e[m] = image_rows
        return e.astype(F32)

    def generate_without_cache(self, ids, mask, image_rows, max_new_tokens, eos_token_id=None,
                               repetition_penalty=1.0, no_repeat_ngram_size=20):
        """DeepseekOcrModel::generate_without_cache model/mod.rs:2051-2283 (greedy): every step runs the
        whole forward on prompt + generated tokens (image mask extended with 0, rows re-injected) and
        selects from the last position's logits with the tokens so far as context."""
        tokens = [int(t) for t in ids]
        msk = list(mask) if mask is not None else [0] * len(tokens)
        if max_new_tokens == 0:
            return []

        def last_logits():
            self.dec.reset()
            return self.dec.forward(self.prefill_embeddings(tokens, msk, image_rows))[0]

        cur = select_token_id(last_logits(), tokens, repetition_penalty, no_repeat_ngram_size)
        if eos_token_id is not None and cur == eos_token_id:
            return []
        out = []
        for step in range(max_new_tokens):
            out.append(cur)
            if step + 1 == max_new_tokens:
                break
            tokens.append(cur)
            msk.append(0)
            cur = select_token_id(last_logits(), tokens, repetition_penalty, no_repeat_ngram_size)
            if eos_token_id is not None and cur == eos_token_id:
                break
        return out

    def generate(self, ids, mask, image_rows, max_new_tokens, eos_token_id=None,
                 repetition_penalty=1.0, no_repeat_ngram_size=20, record_logits=False, ignore_eos=False,
                 do_sample=False, temperature=0.0, top_k=None, top_p=None, seed=None):
        """DeepseekOcrModel::generate model/mod.rs:1870-2048 (use_cache; rng = init_rng(seed) per call,
        model/mod.rs:1917)."""
        from .sampling import StdRng
        rng = StdRng(seed) if (do_sample and temperature > 0.0 and seed is not None) else None
        if rng is None and do_sample and temperature > 0.0:
            raise ValueError("oracle sampling needs a seed")
        sel = dict(do_sample=do_sample, temperature=temperature, top_k=top_k, top_p=top_p, rng=rng)
        self.dec.reset()
        ctx = [int(t) for t in ids]
        logits_log = []
        if max_new_tokens == 0:
            return [], logits_log
        lg = self.dec.forward(self.prefill_embeddings(ids, mask, image_rows))[0]
        if record_logits:
            logits_log.append(lg)
        cur = select_token_id(lg, ctx, repetition_penalty, no_repeat_ngram_size, **sel)
        if eos_token_id is not None and cur == eos_token_id and not ignore_eos:
            return [], logits_log
        out = []
        for step in range(max_new_tokens):
            ctx.append(cur)
            out.append(cur)
            if step + 1 == max_new_tokens:
                break
            lg = self.dec.forward(self.dec.embed([cur]))[0]
            if record_logits:
                logits_log.append(lg)
            cur = select_token_id(lg, ctx, repetition_penalty, no_repeat_ngram_size, **sel)
            if eos_token_id is not None and cur == eos_token_id and not ignore_eos:
                break
        return out, logits_log
