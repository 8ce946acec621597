"""Oracle: DeepSeek-V2 MoE decoder + greedy generation (TEST INFRASTRUCTURE).

f32 numpy restatement of transformer/{block,decoder,model,rope}.rs,
core/src/{cache,sampling,tensor}.rs and DeepseekOcrModel::generate
(model/mod.rs:1870-2048).  The KV cache stores K and V per layer in f32
(block.rs:776-789); RoPE tables are built exactly as rope.rs:172-207.
"""
from __future__ import annotations

import math

import numpy as np

from .config import resolved_language_config, should_use_moe

F32 = np.float32


def rms_norm(x, w, eps):
    """candle_nn::ops::rms_norm_slow: x / sqrt(mean(x^2) + eps) * w (block.rs:24-29)."""
    x = x.astype(F32, copy=False)
    ms = (x * x).sum(axis=-1, keepdims=True, dtype=F32) / F32(x.shape[-1])
    return (x / np.sqrt(ms + F32(eps))) * w


def silu(x):
    return (x / (F32(1.0) + np.exp(-x))).astype(F32)


def softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(axis=axis, keepdims=True, dtype=F32)).astype(F32)


def rope_tables(lang, length, rope_dim):
    """rope.rs:172-207: inv_freq = 1/theta^(2i/d) (f32), angles = pos*inv_freq, [half|half]."""
    half = rope_dim // 2
    base = F32(lang.rope_theta)
    inv = np.array([F32(1.0) / (base ** (F32(i * 2.0) / F32(rope_dim))) for i in range(half)], F32)
    pos = np.arange(length, dtype=F32)[:, None]
    ang = (pos * inv[None, :]).astype(F32)
    cos = np.cos(ang).astype(F32)
    sin = np.sin(ang).astype(F32)
    return np.concatenate([cos, cos], 1), np.concatenate([sin, sin], 1)


def apply_rope(x, cos, sin, reorder):
    """block.rs:1403-1471 (reorder = use_mla even/odd regroup)."""
    if reorder:
        *lead, d = x.shape
        x = x.reshape(*lead, d // 2, 2).swapaxes(-1, -2).reshape(*lead, d)
    half = x.shape[-1] // 2
    rot = np.concatenate([-x[..., half:], x[..., :half]], -1)
    return (x * cos + rot * sin).astype(F32)


class Decoder:
    def __init__(self, cfg, W):
        self.lang = resolved_language_config(cfg)
        self.W = W
        L = self.lang
        if L.q_lora_rank is not None or L.kv_lora_rank is not None:
            raise NotImplementedError("LoRA attention path not yet implemented")  # block.rs:452-454
        self.H = L.hidden_size
        self.nh = L.num_attention_heads
        self.hd = self.H // self.nh
        self.nkv = L.num_key_value_heads or self.nh
        rd = L.qk_rope_head_dim if L.qk_rope_head_dim is not None else self.hd
        self.rope_dim = self.hd if rd == 0 else rd
        self.eps = L.rms_norm_eps
        self.cos = self.sin = None
        self.reset()

    def reset(self):
        self.k_cache = [None] * self.lang.num_hidden_layers
        self.v_cache = [None] * self.lang.num_hidden_layers
        self.past = 0

    def w(self, name, shape):
        return self.W.get(name, shape)

    def lin(self, x, pre, out_dim, in_dim):
        y = x @ self.w(pre + ".weight", (out_dim, in_dim)).T
        if self.W.has(pre + ".bias"):
            y = y + self.w(pre + ".bias", (out_dim,))
        return y.astype(F32)

    def embed(self, ids):
        """gather_token_embeddings core/src/tensor.rs:8-25."""
        tab = self.w("model.embed_tokens.weight", (self.lang.vocab_size, self.H))
        return tab[np.asarray(ids, dtype=np.int64)]

    def _ensure_rope(self, n):
        if self.cos is None or self.cos.shape[0] < n:
            cap = 1
            while cap < n:
                cap *= 2
            self.cos, self.sin = rope_tables(self.lang, cap, self.rope_dim)

    def attention(self, li, x):
        """attention_forward block.rs:446-804 (batch 1, f32 path, full KV cache)."""
        pre = f"model.layers.{li}.self_attn"
        s = x.shape[0]
        q = self.lin(x, pre + ".q_proj", self.nh * self.hd, self.H).reshape(s, self.nh, self.hd).transpose(1, 0, 2)
        k = self.lin(x, pre + ".k_proj", self.nkv * self.hd, self.H).reshape(s, self.nkv, self.hd).transpose(1, 0, 2)
        v = self.lin(x, pre + ".v_proj", self.nkv * self.hd, self.H).reshape(s, self.nkv, self.hd).transpose(1, 0, 2)
        pos = np.arange(self.past, self.past + s)
        self._ensure_rope(self.past + s)
        cos, sin = self.cos[pos], self.sin[pos]
        r = self.rope_dim
        use_mla = bool(self.lang.use_mla)
        q = np.concatenate([apply_rope(q[..., :r], cos, sin, use_mla), q[..., r:]], -1)
        k = np.concatenate([apply_rope(k[..., :r], cos, sin, use_mla), k[..., r:]], -1)
        rep = self.nh // self.nkv
        k = np.repeat(k, rep, axis=0)
        v = np.repeat(v, rep, axis=0)
        if self.k_cache[li] is None:
            kall, vall = k, v
        else:
            kall = np.concatenate([self.k_cache[li], k], 1)
            vall = np.concatenate([self.v_cache[li], v], 1)
        self.k_cache[li], self.v_cache[li] = kall, vall
        scores = (q @ kall.transpose(0, 2, 1)) / F32(math.sqrt(self.hd))
        if self.past == 0 and s > 1:                                  # build_attention_bias 1504-1526
            mask = np.triu(np.ones((s, s), bool), 1)
            scores = scores + np.where(mask, F32(-1e9), F32(0.0))[None]
        p = softmax(scores.astype(F32))
        o = (p @ vall).transpose(1, 0, 2).reshape(s, self.nh * self.hd)
        return self.lin(o, pre + ".o_proj", self.H, self.nh * self.hd)

    def dense_mlp(self, x, pre, inter):
        """run_dense_mlp block.rs:1179-1213 (silu)."""
        g = self.lin(x, pre + ".gate_proj", inter, self.H)
        u = self.lin(x, pre + ".up_proj", inter, self.H)
        return self.lin(silu(g) * u, pre + ".down_proj", self.H, inter)

    def moe(self, li, x):
        """run_moe block.rs:1215-1395: softmax router, greedy top-k, per-expert SwiGLU, shared experts."""
        L = self.lang
        pre = f"model.layers.{li}.mlp"
        ne, topk, inter = L.n_routed_experts, L.num_experts_per_tok, L.moe_intermediate_size
        if (L.topk_method or "greedy") != "greedy":
            raise NotImplementedError("greedy only")
        logits = x @ self.w(pre + ".gate.weight", (ne, self.H)).T
        if self.W.has(pre + ".gate.e_score_correction_bias"):
            logits = logits + self.w(pre + ".gate.e_score_correction_bias", (ne,))
        scoring = L.scoring_func or "softmax"
        scores = softmax(logits.astype(F32)) if scoring == "softmax" else (F32(1) / (F32(1) + np.exp(-logits))).astype(F32)
        order = np.argsort(-scores, axis=-1, kind="stable")[:, :topk]
        wts = np.take_along_axis(scores, order, -1)
        if topk > 1 and L.norm_topk_prob:
            wts = wts / (wts.sum(-1, keepdims=True) + F32(1e-20))
        if L.routed_scaling_factor != 1.0:
            wts = wts * F32(L.routed_scaling_factor)
        T = x.shape[0]
        outs = np.zeros((T, topk, self.H), F32)
        for e in np.unique(order):
            rows, slots = np.nonzero(order == e)
            y = self.dense_mlp(x[rows], f"{pre}.experts.{e}", inter)
            outs[rows, slots] = y
        comb = (outs * wts[:, :, None]).sum(1, dtype=F32)
        if (L.n_shared_experts or 0) > 0:
            comb = comb + self.dense_mlp(x, pre + ".shared_experts", inter * L.n_shared_experts)
        return comb.astype(F32)

    def layer(self, li, x):
        """TransformerBlock::forward_internal block.rs:124-191."""
        pre = f"model.layers.{li}"
        h = x + self.attention(li, rms_norm(x, self.w(pre + ".input_layernorm.weight", (self.H,)), self.eps))
        n = rms_norm(h, self.w(pre + ".post_attention_layernorm.weight", (self.H,)), self.eps)
        if should_use_moe(self.lang, li):
            m = self.moe(li, n)
        else:
            m = self.dense_mlp(n, pre + ".mlp", self.lang.intermediate_size)
        return (h + m).astype(F32)

    def forward(self, embeds, last_only=True):
        """DeepseekLanguageModel::forward transformer/model.rs:151-278 -> logits."""
        x = embeds.astype(F32)
        for li in range(self.lang.num_hidden_layers):
            x = self.layer(li, x)
        self.past += embeds.shape[0]
        if last_only:
            x = x[-1:]
        n = rms_norm(x, self.W.get("model.norm.weight", (self.H,)), self.eps)
        lm = self.W.get("lm_head.weight", (self.lang.vocab_size, self.H))
        return (n @ lm.T).astype(F32)


# ----------------------------------------------------------------------------- sampling
def banned_ngram_tokens(seq, n):
    """core/src/sampling.rs:141-158."""
    if n <= 1 or len(seq) < n - 1:
        return set()
    prefix = tuple(seq[len(seq) - (n - 1):])
    banned = set()
    for i in range(len(seq) - n + 1):
        if tuple(seq[i:i + n - 1]) == prefix:
            banned.add(seq[i + n - 1])
    return banned


def select_token_id(logits, context, repetition_penalty=1.0, no_repeat_ngram_size=None, do_sample=False,
                    temperature=0.0, top_k=None, top_p=None, rng=None):
    """select_token_id core/src/sampling.rs:34-96 (the sampling branch: oracle/sampling.py)."""
    logits = np.asarray(logits, F32)
    adjusted = logits.copy()
    if repetition_penalty > 0.0 and abs(repetition_penalty - 1.0) > np.finfo(np.float32).eps:
        pen = F32(max(repetition_penalty, np.finfo(np.float32).tiny))
        for t in dict.fromkeys(int(c) for c in context):
            if 0 <= t < len(adjusted):
                adjusted[t] = adjusted[t] / pen if adjusted[t] > 0 else adjusted[t] * pen
    filtered = adjusted.copy()
    if no_repeat_ngram_size is not None and no_repeat_ngram_size > 1:
        for t in banned_ngram_tokens([int(c) for c in context], no_repeat_ngram_size):
            if 0 <= t < len(filtered):
                filtered[t] = -np.inf
    if not np.any(np.isfinite(filtered)):
        filtered = adjusted
    if do_sample and temperature > 0.0:
        from .sampling import sample_token
        tok = sample_token(filtered, temperature, top_k, top_p, rng)
        if tok is not None:
            return tok
    for arr in (filtered, adjusted, logits):
        idx = argmax_first(arr)
        if idx is not None:
            return idx
    return 0


def argmax_first(values):
    """argmax_index sampling.rs:104-118: first max, skipping non-finite."""
    v = np.where(np.isfinite(values), values, -np.inf)
    if not np.any(np.isfinite(v)):
        return None
    return int(np.argmax(v))
