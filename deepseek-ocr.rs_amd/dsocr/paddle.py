"""PaddleOCR-VL on the host CPU (BASELINE configs[0]: "paddleocr-vl fp16 on Candle CPU backend, assets/sample_1.png
single page, greedy decode (plumbing, no GPU)").

The reference runs this model on Candle's CPU backend (crates/infer-paddleocr); this module is that plumbing path,
restated in numpy (f32 compute on fp16-rounded weights, the DeepSeek path's `--dtype f16` contract), behind the same
OcrEngine surface as the GPU engine (dsocr.engine.DeepseekOcrEngine), and reachable from the CLI as
`--model paddleocr-vl`.  Pieces and the reference they follow:

* preprocess_image (vision/preprocess.rs:91-300): smart_resize with factor patch x merge, min / max pixels (max
  capped by VisionSettings.image_size, with_max_image_size :44-50), fast_image_resize Catmull-Rom convolution
  (dsocr_resize_catmull_rom, the C++ restatement the dots.ocr path uses), x / 255 then (x - 0.5) / 0.5, patches
  [N][3][p][p] in row-major grid order, temporal patch 1 (:27-31);
* SiglipVisionModel (vision/encoder.rs): patch embedding + the bilinearly interpolated position table
  (resize_positional_grid :782-838), 27 pre-norm layers (PreciseLayerNorm :924-966, q/k/v/out with bias, 2-D rotary
  over (row, col) (build_rotary :459-481, SiglipRotaryEmbedding :488-525), softmax attention, fc1 ->
  gelu_pytorch_tanh :765-780 -> fc2), post_layernorm;
* SiglipProjector (vision/projector.rs): LayerNorm eps 1e-5, 2 x 2 merge (reshape_for_merge), linear_1 -> gelu (tanh
  form, candle's Tensor::gelu) -> linear_2;
* build_prompt_tokens / compute_position_ids / inject_image_embeddings (model.rs:411-818): bos, text segments,
  <vision_start> + image tokens + <|IMAGE_END|>, 3-axis positions (text: scalar on every axis, image: base + (0,
  row, col), the next text position = base + token count), decode positions prompt_len + delta + i;
* ErnieDecoder (transformer/): RMSNorm, GQA attention with the multimodal rotary (mrope sections doubled, section k
  from position axis k, rotate_half), causal prefill bias -1e9, f32 KV cache, SwiGLU MLP, final norm, lm_head;
* select_token_id (core/src/sampling.rs:34-158) greedy: repetition penalty once per distinct context token, the
  no-repeat n-gram ban, first-index argmax skipping non-finite, un-banned fallback.

Weights: no PaddleOCR-VL checkpoint exists offline, so the published architecture (dsocr/configs/paddleocr-vl.json)
is filled with seeded synthetic fp16-rounded weights (`synthetic_weights`); sampled decoding (ChaCha12 StdRng) is
not part of this plumbing path and raises.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import zlib
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

F32 = np.float32
HERE = os.path.dirname(os.path.abspath(__file__))
PADDLE_CONFIG = os.path.join(HERE, "configs", "paddleocr-vl.json")
PADDLE_TINY_CONFIG = os.path.join(HERE, "configs", "paddleocr-vl-tiny.json")

MIN_PIXELS, MAX_PIXELS = 147_384, 2_822_400   # vision/preprocess.rs:8-9
IMAGE_END_TOKEN = "<|IMAGE_END|>"


# ------------------------------------------------------------------ config
@dataclass
class VisionCfg:
    hidden_size: int
    intermediate_size: int
    num_hidden_layers: int
    num_attention_heads: int
    num_channels: int
    image_size: int
    patch_size: int
    layer_norm_eps: float = 1e-6
    spatial_merge_size: int = 2
    tokens_per_second: int = 2


@dataclass
class PaddleCfg:
    head_dim: int
    hidden_size: int
    intermediate_size: int
    vocab_size: int
    num_attention_heads: int
    num_hidden_layers: int
    num_key_value_heads: int
    image_token_id: int
    vision_start_token_id: int
    bos_token_id: Optional[int]
    eos_token_id: Optional[int]
    rms_norm_eps: float
    rope_theta: float
    mrope_section: Tuple[int, int, int]
    use_bias: bool
    use_3d_rope: bool
    hidden_act: str
    vision: VisionCfg

    @staticmethod
    def load(path: str) -> "PaddleCfg":
        with open(path) as f:
            c = json.load(f)
        v = c["vision_config"]
        rs = c.get("rope_scaling") or {}
        sec = tuple(rs.get("mrope_section") or ())
        if len(sec) != 3:
            raise ValueError("mrope_section missing from rope_scaling configuration")  # rope.rs:33-46
        if 2 * sum(sec) != c["head_dim"]:
            raise ValueError("sum of doubled mrope sections must equal head_dim")
        vc = VisionCfg(v["hidden_size"], v["intermediate_size"], v["num_hidden_layers"], v["num_attention_heads"],
                       v["num_channels"], v["image_size"], v["patch_size"], v.get("layer_norm_eps", 1e-6),
                       v.get("spatial_merge_size", 2), v.get("tokens_per_second", 2))
        return PaddleCfg(c["head_dim"], c["hidden_size"], c["intermediate_size"], c["vocab_size"],
                         c["num_attention_heads"], c["num_hidden_layers"],
                         c.get("num_key_value_heads") or c["num_attention_heads"], c["image_token_id"],
                         c["vision_start_token_id"], c.get("bos_token_id"), c.get("eos_token_id"),
                         c.get("rms_norm_eps", 1e-5), float(c.get("rope_theta", 10000.0)), sec,
                         bool(c.get("use_bias", False)), bool(c.get("use_3d_rope", False)),
                         c.get("hidden_act", "silu"), vc)


# ------------------------------------------------------------------ synthetic checkpoint
def tensor_specs(cfg: PaddleCfg) -> List[Tuple[str, Tuple[int, ...], str]]:
    """(name, shape, kind) of every tensor the reference loads (weights.rs / encoder.rs / projector.rs names);
    kind: w (linear / table), b (bias), n (norm weight), z (layer-norm bias)."""
    v = cfg.vision
    vh, vi = v.hidden_size, v.intermediate_size
    out = []
    vp = "visual.vision_model."
    out.append((vp + "embeddings.patch_embedding.weight", (vh, v.num_channels, v.patch_size, v.patch_size), "w"))
    out.append((vp + "embeddings.patch_embedding.bias", (vh,), "b"))
    out.append((vp + "embeddings.position_embedding.weight", ((v.image_size // v.patch_size) ** 2, vh), "w"))
    for i in range(v.num_hidden_layers):
        lp = f"{vp}encoder.layers.{i}."
        for n in ("layer_norm1", "layer_norm2"):
            out += [(lp + n + ".weight", (vh,), "n"), (lp + n + ".bias", (vh,), "z")]
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            out += [(lp + "self_attn." + n + ".weight", (vh, vh), "w"), (lp + "self_attn." + n + ".bias", (vh,), "b")]
        out += [(lp + "mlp.fc1.weight", (vi, vh), "w"), (lp + "mlp.fc1.bias", (vi,), "b"),
                (lp + "mlp.fc2.weight", (vh, vi), "w"), (lp + "mlp.fc2.bias", (vh,), "b")]
    out += [(vp + "post_layernorm.weight", (vh,), "n"), (vp + "post_layernorm.bias", (vh,), "z")]
    mh = vh * v.spatial_merge_size ** 2
    out += [("mlp_AR.pre_norm.weight", (vh,), "n"), ("mlp_AR.pre_norm.bias", (vh,), "z"),
            ("mlp_AR.linear_1.weight", (mh, mh), "w"), ("mlp_AR.linear_1.bias", (mh,), "b"),
            ("mlp_AR.linear_2.weight", (cfg.hidden_size, mh), "w"), ("mlp_AR.linear_2.bias", (cfg.hidden_size,), "b")]
    H, hd = cfg.hidden_size, cfg.head_dim
    out.append(("model.embed_tokens.weight", (cfg.vocab_size, H), "w"))
    for i in range(cfg.num_hidden_layers):
        lp = f"model.layers.{i}."
        for n, o, k in (("q_proj", cfg.num_attention_heads * hd, H), ("k_proj", cfg.num_key_value_heads * hd, H),
                        ("v_proj", cfg.num_key_value_heads * hd, H), ("o_proj", H, cfg.num_attention_heads * hd)):
            out.append((lp + "self_attn." + n + ".weight", (o, k), "w"))
            if cfg.use_bias:
                out.append((lp + "self_attn." + n + ".bias", (o,), "b"))
        for n, o, k in (("gate_proj", cfg.intermediate_size, H), ("up_proj", cfg.intermediate_size, H),
                        ("down_proj", H, cfg.intermediate_size)):
            out.append((lp + "mlp." + n + ".weight", (o, k), "w"))
            if cfg.use_bias:
                out.append((lp + "mlp." + n + ".bias", (o,), "b"))
        out += [(lp + "input_layernorm.weight", (H,), "n"), (lp + "post_attention_layernorm.weight", (H,), "n")]
    out += [("model.norm.weight", (H,), "n"), ("lm_head.weight", (cfg.vocab_size, H), "w")]
    return out


def synthetic_weights(cfg: PaddleCfg, seed: int) -> Dict[str, np.ndarray]:
    """Seeded synthetic checkpoint: per tensor a numpy PCG64 stream keyed by (seed, crc32(name)); linears N(0, 1/fan_in)
    (position / embedding tables N(0, 0.02^2)), biases N(0, 0.02^2), norm weights 1 + N(0, 0.05^2); every value rounded
    to fp16 and held as f32 (the reference's --dtype f16 weights, f32 compute)."""
    out = {}
    for name, shape, kind in tensor_specs(cfg):
        rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
        if kind == "w":
            fan_in = int(np.prod(shape[1:]))
            std = 0.02 if (name.endswith("embedding.weight") or "embed_tokens" in name) else 1.0 / math.sqrt(fan_in)
            a = rng.standard_normal(shape, dtype=F32) * F32(std)
        elif kind == "n":
            a = F32(1.0) + rng.standard_normal(shape, dtype=F32) * F32(0.05)
        else:
            a = rng.standard_normal(shape, dtype=F32) * F32(0.02)
        out[name] = a.astype(np.float16).astype(F32)
    return out


# ------------------------------------------------------------------ preprocessing (vision/preprocess.rs)
def smart_resize(height: int, width: int, factor: int, min_pixels: int, max_pixels: int) -> Tuple[int, int]:
    """smart_resize preprocess.rs:244-279 (f64 arithmetic, round half away from zero like Rust's f64::round)."""
    rnd = lambda x: math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)  # noqa: E731
    f = float(max(factor, 1))
    h, w = float(max(height, 1)), float(max(width, 1))
    if h < f:
        w = float(rnd((w * f) / h))
        h = f
    if w < f:
        h = float(rnd((h * f) / w))
        w = f
    if max(h, w) / min(h, w) > 200.0:
        raise ValueError("aspect ratio exceeds limit")
    hb, wb = rnd(h / f) * f, rnd(w / f) * f
    maxp, minp = float(max(max_pixels, 1)), float(max(min_pixels, 1))
    if hb * wb > maxp:
        beta = math.sqrt((h * w) / maxp)
        hb, wb = math.floor((h / beta) / f) * f, math.floor((w / beta) / f) * f
    elif hb * wb < minp:
        beta = math.sqrt(minp / (h * w))
        hb, wb = math.ceil((h * beta) / f) * f, math.ceil((w * beta) / f) * f
    if hb < f or wb < f:
        raise ValueError("resized dimensions smaller than factor")
    return int(hb), int(wb)


def resize_catmull_rom(rgb: np.ndarray, w: int, h: int) -> np.ndarray:
    """fast_image_resize Convolution(CatmullRom) through the engine library's host restatement (no GPU)."""
    from ._lib import check, lib
    src = np.ascontiguousarray(rgb, dtype=np.uint8)
    dst = np.empty((h, w, 3), np.uint8)
    check(lib().dsocr_resize_catmull_rom(src.ctypes.data_as(C.c_void_p), src.shape[1], src.shape[0],
                                         dst.ctypes.data_as(C.c_void_p), w, h))
    return dst


def preprocess_image(rgb: np.ndarray, cfg: VisionCfg, image_size: int = 0):
    """preprocess_image preprocess.rs:91-139 -> (patches [N][3*p*p] f32, grid (t, h, w), height_ids, width_ids)."""
    p, m = cfg.patch_size, cfg.spatial_merge_size
    max_px = MAX_PIXELS
    if image_size > 0:  # with_max_image_size :44-50
        max_px = min(MAX_PIXELS, max(image_size * image_size, MIN_PIXELS))
    oh, ow = rgb.shape[:2]
    rh, rw = smart_resize(oh, ow, p * m, MIN_PIXELS, max_px)
    img = rgb if (oh, ow) == (rh, rw) else resize_catmull_rom(rgb, rw, rh)
    x = img.astype(F32) * F32(1.0 / 255.0)
    x = (x - F32(0.5)) / F32(0.5)
    gh, gw = rh // p, rw // p
    # [gh, p, gw, p, C] -> [gh, gw, C, p, p]
    patches = x.reshape(gh, p, gw, p, 3).transpose(0, 2, 4, 1, 3).reshape(gh * gw, 3 * p * p)
    hid = np.repeat(np.arange(gh), gw)
    wid = np.tile(np.arange(gw), gh)
    return np.ascontiguousarray(patches), (1, gh, gw), hid, wid


# ------------------------------------------------------------------ math helpers
def layer_norm(x, w, b, eps):
    """PreciseLayerNorm encoder.rs:949-966 (mean, centred variance, / sqrt(var + eps), * w + b)."""
    mean = x.mean(-1, keepdims=True, dtype=F32)
    c = x - mean
    var = (c * c).mean(-1, keepdims=True, dtype=F32)
    return ((c / np.sqrt(var + F32(eps))) * w + b).astype(F32)


def rms_norm(x, w, eps):
    """candle_nn::ops::rms_norm: x / sqrt(mean(x^2) + eps) * w."""
    return ((x / np.sqrt((x * x).mean(-1, keepdims=True, dtype=F32) + F32(eps))) * w).astype(F32)


def gelu_tanh(x):
    """gelu_pytorch_tanh encoder.rs:765-780 (candle's Tensor::gelu is the same tanh form)."""
    return (((np.tanh((x + (x * x * x) * F32(0.044715)) * F32(0.7978846)) + F32(1.0)) * F32(0.5)) * x).astype(F32)


def silu(x):
    return (x / (F32(1.0) + np.exp(-x))).astype(F32)


def softmax(x):
    m = x.max(-1, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(-1, keepdims=True)).astype(F32)


def rotate_half(x):
    h = x.shape[-1] // 2
    return np.concatenate([-x[..., h:], x[..., :h]], -1)


def linear(x, w, b=None):
    y = x @ w.T
    return (y + b if b is not None else y).astype(F32)


def resize_positional_grid(base: np.ndarray, th: int, tw: int) -> np.ndarray:
    """resize_positional_grid encoder.rs:782-838: separable bilinear (half-pixel centres, clamped), rows first."""
    bh, bw, d = base.shape

    def coords(target, src):
        if src <= 1 or target <= 1:
            z = np.zeros(target, np.int64)
            return z, z, np.zeros(target, F32)
        scale = F32(src) / F32(target)
        real = (np.arange(target, dtype=F32) + F32(0.5)) * scale - F32(0.5)
        cl = np.clip(real, F32(0.0), F32(src - 1))
        lo = np.floor(cl).astype(np.int64)
        hi = np.minimum(lo + 1, src - 1)
        return lo, hi, (cl - lo.astype(F32)).astype(F32)

    if (th, tw) == (bh, bw):
        return base.reshape(bh * bw, d)
    y0, y1, fy = coords(th, bh)
    tmp = base[y0] + (base[y1] - base[y0]) * fy[:, None, None]
    if tw == bw:
        return tmp.reshape(th * bw, d).astype(F32)
    x0, x1, fx = coords(tw, bw)
    out = tmp[:, x0] + (tmp[:, x1] - tmp[:, x0]) * fx[None, :, None]
    return out.reshape(th * tw, d).astype(F32)


# ------------------------------------------------------------------ vision tower + projector
class SiglipVision:
    def __init__(self, cfg: PaddleCfg, W: Dict[str, np.ndarray]):
        self.cfg, self.W = cfg, W

    def _rotary(self, hid, wid):
        """build_rotary encoder.rs:459-481 with SiglipRotaryEmbedding :488-525 (head_dim / 2 base, step 2)."""
        v = self.cfg.vision
        hd = v.hidden_size // v.num_attention_heads
        base = max(hd // 2, 1)
        inv = np.array([F32(1.0) / np.power(F32(10000.0), F32(i) / F32(base)) for i in range(0, base, 2)], F32)
        if inv.size == 0:
            inv = np.ones(1, F32)
        size = int(max(hid.max(initial=0), wid.max(initial=0))) + 1
        table = np.arange(size, dtype=F32)[:, None] * inv[None, :]
        ang = np.concatenate([table[hid], table[wid]], -1)
        ang = np.concatenate([ang, ang], -1)
        return np.cos(ang).astype(F32), np.sin(ang).astype(F32)

    def forward(self, patches, grid, hid, wid):
        v, W = self.cfg.vision, self.W
        vp = "visual.vision_model."
        x = linear(patches, W[vp + "embeddings.patch_embedding.weight"].reshape(v.hidden_size, -1),
                   W[vp + "embeddings.patch_embedding.bias"])
        g = v.image_size // v.patch_size
        pos = resize_positional_grid(W[vp + "embeddings.position_embedding.weight"].reshape(g, g, v.hidden_size),
                                     grid[1], grid[2])
        x = (x + np.tile(pos, (grid[0], 1))).astype(F32)
        cos, sin = self._rotary(hid, wid) if self.cfg.use_3d_rope else (None, None)
        nh = v.num_attention_heads
        hd = v.hidden_size // nh
        n = x.shape[0]
        for i in range(v.num_hidden_layers):
            lp = f"{vp}encoder.layers.{i}."
            h = layer_norm(x, W[lp + "layer_norm1.weight"], W[lp + "layer_norm1.bias"], v.layer_norm_eps)
            qkv = [linear(h, W[lp + f"self_attn.{k}.weight"], W[lp + f"self_attn.{k}.bias"]).reshape(n, nh, hd)
                   .transpose(1, 0, 2) for k in ("q_proj", "k_proj", "v_proj")]
            q, k, vv = qkv
            if cos is not None:
                q = (q * cos + rotate_half(q) * sin).astype(F32)
                k = (k * cos + rotate_half(k) * sin).astype(F32)
            s = (q @ k.transpose(0, 2, 1)) / F32(math.sqrt(hd))
            ctx = (softmax(s) @ vv).transpose(1, 0, 2).reshape(n, v.hidden_size)
            x = (x + linear(ctx, W[lp + "self_attn.out_proj.weight"], W[lp + "self_attn.out_proj.bias"])).astype(F32)
            h = layer_norm(x, W[lp + "layer_norm2.weight"], W[lp + "layer_norm2.bias"], v.layer_norm_eps)
            h = gelu_tanh(linear(h, W[lp + "mlp.fc1.weight"], W[lp + "mlp.fc1.bias"]))
            x = (x + linear(h, W[lp + "mlp.fc2.weight"], W[lp + "mlp.fc2.bias"])).astype(F32)
        return layer_norm(x, W[vp + "post_layernorm.weight"], W[vp + "post_layernorm.bias"], v.layer_norm_eps)

    def project(self, feats, grid):
        """SiglipProjector::project_single projector.rs:79-118."""
        v, W = self.cfg.vision, self.W
        m = v.spatial_merge_size
        t, gh, gw = grid
        x = layer_norm(feats, W["mlp_AR.pre_norm.weight"], W["mlp_AR.pre_norm.bias"], 1e-5)
        x = x.reshape(t, gh // m, m, gw // m, m, v.hidden_size).transpose(0, 1, 3, 2, 4, 5)
        x = x.reshape(t * (gh // m) * (gw // m), m * m * v.hidden_size)
        x = gelu_tanh(linear(x, W["mlp_AR.linear_1.weight"], W["mlp_AR.linear_1.bias"]))
        return linear(x, W["mlp_AR.linear_2.weight"], W["mlp_AR.linear_2.bias"]), (t, gh // m, gw // m)


# ------------------------------------------------------------------ prompt / positions (model.rs)
def build_prompt_tokens(tokenizer, prompt: str, grids, cfg: PaddleCfg):
    """build_prompt_tokens model.rs:411-464."""
    segs = prompt.split("<image>")
    if len(segs) - 1 != len(grids):
        raise ValueError(f"prompt/image mismatch: {len(segs) - 1} slots vs {len(grids)} grids")
    end_id = tokenizer.token_to_id(IMAGE_END_TOKEN)
    m = cfg.vision.spatial_merge_size
    toks, mask = [], []
    if cfg.bos_token_id is not None:
        toks.append(int(cfg.bos_token_id))
        mask.append(0)
    for i, seg in enumerate(segs):
        if seg:
            ids = list(tokenizer.encode(seg, add_special_tokens=False).ids)
            toks += ids
            mask += [0] * len(ids)
        if i < len(grids):
            t, h, w = grids[i]
            if h % m or w % m:
                raise ValueError(f"grid {grids[i]} not divisible by merge size {m}")
            n = t * (h // m) * (w // m)
            toks.append(int(cfg.vision_start_token_id))
            mask.append(0)
            toks += [int(cfg.image_token_id)] * n
            mask += [1] * n
            if end_id is not None:
                toks.append(int(end_id))
                mask.append(0)
    return toks, mask


def compute_position_ids(cfg: PaddleCfg, ids, grids):
    """compute_position_ids / build_mrope_positions_for_row model.rs:566-818 for one row with an all-ones attention
    mask: text runs take scalar positions on all three axes, an image span base + (t', row, col) over the merged grid,
    the text after it base + token count; returns ([3][L] positions, delta = max + 1 - L)."""
    m = cfg.vision.spatial_merge_size
    L = len(ids)
    if not grids:  # attention mask given, no images (build_masked_text_positions)
        pos = np.arange(L, dtype=np.int64)
        return np.stack([pos, pos, pos]), int(max(1, L - 1) + 1 - L)
    at, ah, aw = [], [], []
    st, nxt, gi = 0, 0, 0
    while st < L:
        try:
            ed = ids.index(cfg.image_token_id, st)
        except ValueError:
            ed = None
        if ed is None:
            r = range(nxt, nxt + L - st)
            at += r; ah += r; aw += r  # noqa: E702
            nxt, st = L, L
            continue
        r = range(nxt, nxt + ed - st)
        at += r; ah += r; aw += r  # noqa: E702
        nxt += ed - st
        if gi >= len(grids):
            raise ValueError("not enough image grids for placeholders")
        t, h, w = grids[gi]
        gi += 1
        lh, lw = h // m, w // m
        block = t * lh * lw
        if ed + block > L or any(x != cfg.image_token_id for x in ids[ed:ed + block]):
            raise ValueError("placeholder span mismatch")
        for tt in range(t):
            tv = int(math.floor(tt * 0.0 * cfg.vision.tokens_per_second))
            for row in range(lh):
                for col in range(lw):
                    at.append(nxt + tv)
                    ah.append(nxt + row)
                    aw.append(nxt + col)
        nxt += block
        st = ed + block
    if gi != len(grids):
        raise ValueError("unused image grids remain after placeholder expansion")
    pos = np.array([at, ah, aw], np.int64)
    return pos, int(pos.max(initial=1) + 1 - L)


# ------------------------------------------------------------------ decoder (transformer/)
class ErnieDecoder:
    def __init__(self, cfg: PaddleCfg, W: Dict[str, np.ndarray]):
        self.cfg, self.W = cfg, W
        half = cfg.head_dim // 2
        self.inv = np.array([np.power(F32(cfg.rope_theta), -(F32(i) / F32(half))) for i in range(half)], F32)  # rope.rs:17-23
        self.sections = [2 * s for s in cfg.mrope_section]
        self.reset()

    def reset(self):
        self.k = [None] * self.cfg.num_hidden_layers
        self.v = [None] * self.cfg.num_hidden_layers

    def _cos_sin(self, pos):
        """ErnieRotaryEmbedding::cos_sin rope.rs:74-103 + select_sections attention.rs: dims of section k from axis k."""
        ang = pos.astype(F32)[:, :, None] * self.inv[None, None, :]   # [3][L][half]
        cos = np.concatenate([np.cos(ang), np.cos(ang)], -1)
        sin = np.concatenate([np.sin(ang), np.sin(ang)], -1)
        cs, sn, off = [], [], 0
        for k, w in enumerate(self.sections):
            cs.append(cos[k % 3, :, off:off + w])
            sn.append(sin[k % 3, :, off:off + w])
            off += w
        return np.concatenate(cs, -1).astype(F32), np.concatenate(sn, -1).astype(F32)

    def forward(self, x, pos):
        """ErnieDecoder::forward transformer/model.rs + decoder_layer_forward block.rs -> logits of the last row."""
        cfg, W = self.cfg, self.W
        L = x.shape[0]
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        cos, sin = self._cos_sin(pos)
        past = 0 if self.k[0] is None else self.k[0].shape[1]
        bias = None
        if past == 0 and L > 1:  # build_attention_bias block.rs:90-110 (causal, -1e9)
            bias = np.where(np.arange(L)[None, :] > np.arange(L)[:, None], F32(-1e9), F32(0.0)).astype(F32)
        b = (lambda n: W.get(n)) if cfg.use_bias else (lambda n: None)
        for i in range(cfg.num_hidden_layers):
            lp = f"model.layers.{i}."
            h = rms_norm(x, W[lp + "input_layernorm.weight"], cfg.rms_norm_eps)
            q = linear(h, W[lp + "self_attn.q_proj.weight"], b(lp + "self_attn.q_proj.bias")).reshape(L, nh, hd).transpose(1, 0, 2)
            k = linear(h, W[lp + "self_attn.k_proj.weight"], b(lp + "self_attn.k_proj.bias")).reshape(L, nkv, hd).transpose(1, 0, 2)
            v = linear(h, W[lp + "self_attn.v_proj.weight"], b(lp + "self_attn.v_proj.bias")).reshape(L, nkv, hd).transpose(1, 0, 2)
            q = (q * cos + rotate_half(q) * sin).astype(F32)
            k = (k * cos + rotate_half(k) * sin).astype(F32)
            rep = nh // nkv
            k = np.repeat(k, rep, axis=0)
            v = np.repeat(v, rep, axis=0)
            if self.k[i] is not None:
                k = np.concatenate([self.k[i], k], 1)
                v = np.concatenate([self.v[i], v], 1)
            self.k[i], self.v[i] = k, v
            s = (q @ k.transpose(0, 2, 1)) / F32(math.sqrt(hd))
            if bias is not None:
                s = s + bias
            ctx = (softmax(s) @ v).transpose(1, 0, 2).reshape(L, nh * hd)
            x = (x + linear(ctx, W[lp + "self_attn.o_proj.weight"], b(lp + "self_attn.o_proj.bias"))).astype(F32)
            h = rms_norm(x, W[lp + "post_attention_layernorm.weight"], cfg.rms_norm_eps)
            g = linear(h, W[lp + "mlp.gate_proj.weight"], b(lp + "mlp.gate_proj.bias"))
            u = linear(h, W[lp + "mlp.up_proj.weight"], b(lp + "mlp.up_proj.bias"))
            x = (x + linear(silu(g) * u, W[lp + "mlp.down_proj.weight"], b(lp + "mlp.down_proj.bias"))).astype(F32)
        n = rms_norm(x[-1:], W["model.norm.weight"], cfg.rms_norm_eps)
        return (n @ W["lm_head.weight"].T)[0].astype(F32)


# ------------------------------------------------------------------ token selection (core/src/sampling.rs)
def select_token_id(logits, context, repetition_penalty=1.0, no_repeat_ngram_size=None) -> int:
    """Greedy select_token_id sampling.rs:34-158: penalty once per distinct context token (divide positives,
    multiply negatives), the n-gram ban, first-index argmax skipping non-finite, then the un-banned / raw fallbacks."""
    adj = np.asarray(logits, F32).copy()
    if repetition_penalty > 0.0 and abs(repetition_penalty - 1.0) > np.finfo(F32).eps:
        pen = F32(max(repetition_penalty, np.finfo(F32).tiny))
        for t in dict.fromkeys(int(c) for c in context):
            if 0 <= t < adj.size:
                adj[t] = adj[t] / pen if adj[t] > 0 else adj[t] * pen
    filt = adj.copy()
    n = no_repeat_ngram_size
    ctx = [int(c) for c in context]
    if n is not None and n > 1 and len(ctx) >= n - 1:
        pre = ctx[len(ctx) - (n - 1):]
        for i in range(len(ctx) - n + 1):
            if ctx[i:i + n - 1] == pre and 0 <= ctx[i + n - 1] < filt.size:
                filt[ctx[i + n - 1]] = -np.inf
    if not np.any(np.isfinite(filt)):
        filt = adj
    for arr in (filt, adj, np.asarray(logits, F32)):
        a = np.where(np.isfinite(arr), arr, -np.inf)
        if np.any(np.isfinite(a)):
            return int(np.argmax(a))
    return 0


# ------------------------------------------------------------------ the engine
class PaddleOcrEngine:
    """OcrEngine for ModelKind::PaddleOcrVl (model.rs:286-416) on the host CPU."""

    def __init__(self, config_path: str = PADDLE_CONFIG, synthetic_seed: int = 0):
        self.cfg = PaddleCfg.load(config_path)
        self.W = synthetic_weights(self.cfg, synthetic_seed)
        self.vision = SiglipVision(self.cfg, self.W)
        self.decoder = ErnieDecoder(self.cfg, self.W)
        self.vocab = self.cfg.vocab_size
        self.eos_token_id = self.cfg.eos_token_id
        self.timings = {}

    def kind(self):
        return "paddleocr-vl"

    def device(self):
        return "cpu"

    def close(self):
        self.W.clear()

    def encode_image(self, rgb: np.ndarray, image_size: int = 0):
        """encode_image model.rs:157-191 -> (projected rows, original grid)."""
        patches, grid, hid, wid = preprocess_image(rgb, self.cfg.vision, image_size)
        feats = self.vision.forward(patches, grid, hid, wid)
        emb, _ = self.vision.project(feats, grid)
        return emb, grid

    def generate(self, tokenizer, prompt: str, images: Sequence[np.ndarray], image_size: int = 0,
                 max_new_tokens: int = 16, repetition_penalty: float = 1.0, no_repeat_ngram_size=None,
                 stream: Optional[Callable] = None, ignore_eos: bool = False):
        """decode model.rs:306-408 (use_cache, greedy) -> (generated ids, prompt length)."""
        import time
        t0 = time.perf_counter()
        enc = [self.encode_image(np.asarray(im), image_size) for im in images]
        t1 = time.perf_counter()
        grids = [g for _, g in enc]
        toks, mask = build_prompt_tokens(tokenizer, prompt, grids, self.cfg)
        n_img = sum(mask)
        avail = sum(e.shape[0] for e, _ in enc)
        if n_img != avail:
            raise ValueError(f"image placeholder span ({n_img}) mismatches projector outputs ({avail})")
        pos, delta = compute_position_ids(self.cfg, toks, grids)
        x = self.W["model.embed_tokens.weight"][np.asarray(toks, np.int64)].astype(F32)
        if enc:
            x[np.asarray(mask, bool)] = np.concatenate([e for e, _ in enc], 0)  # inject_image_embeddings
        self.decoder.reset()
        logits = self.decoder.forward(x, pos)
        t2 = time.perf_counter()
        ctx = list(toks)
        out = []
        nxt_pos = len(toks) + delta
        cur = select_token_id(logits, ctx, repetition_penalty, no_repeat_ngram_size)
        eos = None if ignore_eos else self.eos_token_id
        if max_new_tokens > 0 and not (eos is not None and cur == eos):
            while len(out) < max_new_tokens:
                ctx.append(cur)
                out.append(cur)
                if stream:
                    stream(len(out), list(out))
                if (eos is not None and cur == eos) or len(out) >= max_new_tokens:
                    break
                e = self.W["model.embed_tokens.weight"][[cur]].astype(F32)
                logits = self.decoder.forward(e, np.full((3, 1), nxt_pos, np.int64))
                nxt_pos += 1
                cur = select_token_id(logits, ctx, repetition_penalty, no_repeat_ngram_size)
        t3 = time.perf_counter()
        self.timings = {"vision_compute_ms": (t1 - t0) * 1e3, "decode_prefill_ms": (t2 - t1) * 1e3,
                        "decode_iterative_ms": (t3 - t2) * 1e3}
        return out, len(toks)

    def decode(self, tokenizer, prompt, images, vision, params, stream=None):
        """OcrEngine::decode (inference.rs:189-209) for this model kind: greedy only."""
        from .engine import DecodeOutcome, normalize_text
        if params.do_sample and params.temperature > 0.0:
            raise NotImplementedError("sampled decoding is not part of the PaddleOCR-VL CPU plumbing path")
        if not params.use_cache:
            raise ValueError("PaddleOCR decoder currently requires use_cache=true")  # model.rs:315-318
        rgbs = [np.asarray(im.convert("RGB")) if hasattr(im, "convert") else np.asarray(im) for im in images]
        ids, plen = self.generate(tokenizer, prompt, rgbs, vision.image_size, params.max_new_tokens,
                                  params.repetition_penalty, params.no_repeat_ngram_size, stream)
        text = normalize_text(tokenizer.decode([i for i in ids if i >= 0], skip_special_tokens=True))
        return DecodeOutcome(text=text, prompt_tokens=plen, response_tokens=len(ids), generated_tokens=ids)

    def last_timings(self):
        t = dict(self.timings)
        t.setdefault("vision_compute_ms", 0.0)
        t.update({"vision_prepare_ms": 0.0, "decode_generate_ms": sum(t.values())})
        return t


class PaddleSyntheticTokenizer:
    """The synthetic tokenizer (dsocr.synth) with PaddleOCR-VL's special tokens: <|IMAGE_END|>, </s>."""

    def __init__(self, cfg: PaddleCfg):
        from .synth import SyntheticTokenizer
        self._t = SyntheticTokenizer(min(cfg.vocab_size, cfg.image_token_id))
        self.special = {IMAGE_END_TOKEN: cfg.vision_start_token_id + 1, "</s>": cfg.eos_token_id}

    def token_to_id(self, tok):
        return self.special.get(tok)

    def encode(self, text, add_special_tokens=False):
        return self._t.encode(text, add_special_tokens)

    def decode(self, ids, skip_special_tokens=True):
        return self._t.decode(ids, skip_special_tokens)
