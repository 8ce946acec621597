"""Oracle: dots.ocr vision tower (DotsVisionTransformer) with the reference's bf16 semantics
(TEST INFRASTRUCTURE: only tests/ and bench.py's cpu_baseline import this).

Restates TimmyOVO/deepseek-ocr.rs crates/infer-dots:
  * vision/preprocess.rs: preprocess_image 103-145 (to_rgb8, smart_resize, normalise, patches),
    normalise_rgb 175-190, patches_from_normalised 192-235 (merge-group patch order),
    smart_resize 244-279;
  * vision/dots_vit.rs: DotsVisionModel::forward 80-96, SequenceLayout / build_frame_positions
    109-211, DotsPatchEmbed 220-262 (conv k=s=patch, RMSNorm), DotsVisionBlock::forward 305-315,
    VisionAttention::forward / forward_uniform 364-498 (f32 scores, softmax, probs.V:
    compute_dtype_for 584-589), apply_rotary / rotate_half 507-574, DotsSwiGLUFFN::forward 624-630,
    PatchMerger::forward 676-686 (LayerNorm eps 1e-6, Linear, gelu, Linear),
    VisionRotaryEmbedding 697-735 (2-D: [h * inv_freq | w * inv_freq]);
  * model.rs:149-160: pixel values cast to the model dtype before the tower;
  * quant.rs:124-160: linear = matmul (rounded to the activation dtype), then the bias added as a
    second bf16 op.
The model dtype is bf16 (BASELINE configs[3] "dots-ocr bf16"): every op output is a bf16 tensor
(f32 arithmetic inside the op, round-to-nearest-even at its boundary).  Element-wise activations
follow the reference's GPU kernels op by op (candle-kernels unary.cu silu_fwd / gelu_fwd computed
in the bf16 type: every multiply / add rounds to bf16) — a third-party crate (candle 0.9.2) not in
/root/reference, restated from its published kernels: parity of those two ops is unpinned.
The page resize (preprocess.rs:283-299) goes through fast_image_resize 5.3.0 (Cargo.lock), a
third-party crate not in /root/reference: `fir_resize_catmull_rom` restates its published
Convolution(CatmullRom) algorithm for U8x3 (i16 weights at the largest precision <= 14 bits,
horizontal pass then vertical); parity of the resize is unpinned against the crate (no Rust toolchain),
and tests/test_dots.py states how far it lies from Pillow's bicubic on the bench's 2048 -> 2044 page.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
PREPROC = {"patch_size": 14, "temporal_patch_size": 1, "merge_size": 2, "min_pixels": 3136,
           "max_pixels": 11289600,  # pinned by crates/infer-dots/tests/vision_preprocess.rs:9-12
           "image_mean": [0.48145466, 0.4578275, 0.40821073],  # upstream preprocessor_config.json (CLIP)
           "image_std": [0.26862954, 0.26130258, 0.27577711]}


def bf16(x):
    """Round f32 values to bf16 (RNE), returned as f32."""
    u = np.ascontiguousarray(x, F32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(F32)


# ----------------------------------------------------------------------------- preprocessing
def smart_resize(height, width, factor, min_pixels, max_pixels):
    """preprocess.rs:244-279 (f64 arithmetic, Rust's round = half away from zero)."""
    rnd = lambda v: math.floor(v + 0.5)
    factor = float(max(factor, 1))
    h, w = float(max(height, 1)), float(max(width, 1))
    if h < factor:
        w = float(rnd((w * factor) / h))
        h = factor
    if w < factor:
        h = float(rnd((h * factor) / w))
        w = factor
    if max(h, w) / min(h, w) > 200.0:
        raise ValueError("aspect ratio exceeds limit")
    h_bar = rnd(h / factor) * factor
    w_bar = rnd(w / factor) * factor
    area = h_bar * w_bar
    if area > max(max_pixels, 1):
        beta = math.sqrt((h * w) / max(max_pixels, 1))
        h_bar = math.floor((h / beta) / factor) * factor
        w_bar = math.floor((w / beta) / factor) * factor
    elif area < max(min_pixels, 1):
        beta = math.sqrt(max(min_pixels, 1) / (h * w))
        h_bar = math.ceil((h * beta) / factor) * factor
        w_bar = math.ceil((w * beta) / factor) * factor
    if h_bar < factor or w_bar < factor:
        raise ValueError("degenerate resize")
    return int(h_bar), int(w_bar)


def _catmull_rom(x):
    """fast_image_resize's cubic with B = 0, C = 0.5 (Mitchell-Netravali form)."""
    B, C = 0.0, 0.5
    x = abs(x)
    if x < 1.0:
        return ((12.0 - 9.0 * B - 6.0 * C) * x * x * x + (-18.0 + 12.0 * B + 6.0 * C) * x * x + (6.0 - 2.0 * B)) / 6.0
    if x < 2.0:
        return ((-B - 6.0 * C) * x * x * x + (6.0 * B + 30.0 * C) * x * x + (-12.0 * B - 48.0 * C) * x
                + (8.0 * B + 24.0 * C)) / 6.0
    return 0.0


def _round_away(v):
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def fir_coeffs(in_size, out_size):
    """Per output pixel (first tap, i16 weights) and the fixed-point precision of one axis."""
    scale = in_size / out_size
    fscale = max(scale, 1.0)
    radius = 2.0 * fscale
    rows, max_w = [], 0.0
    for x in range(out_size):
        centre = (x + 0.5) * scale
        x0 = max(0, math.floor(centre - radius))
        x1 = min(in_size, math.ceil(centre + radius))
        ws = [_catmull_rom((i - centre + 0.5) / fscale) for i in range(x0, x1)]
        tot = sum(ws)
        if tot != 0.0:
            ws = [w / tot for w in ws]
        max_w = max([max_w] + ws)
        rows.append((x0, ws))
    precision = 0
    for cur in range(15):
        precision = cur
        if _round_away(max_w * (1 << (cur + 1))) >= (1 << 15):
            break
    return [(x0, np.asarray([_round_away(w * (1 << precision)) for w in ws], np.int64)) for x0, ws in rows], precision


def _fir_pass(img, coeffs, precision):
    """Convolve axis 1 of img [rows][in][3] (uint8) -> [rows][out][3]."""
    out = np.empty((img.shape[0], len(coeffs), 3), np.uint8)
    src = img.astype(np.int64)
    for x, (x0, w) in enumerate(coeffs):
        acc = (1 << (precision - 1)) + np.einsum("rkc,k->rc", src[:, x0:x0 + len(w)], w)
        out[:, x] = np.clip(acc >> precision, 0, 255)
    return out


def fir_resize_catmull_rom(rgb, out_w, out_h):
    """fast_image_resize Convolution(CatmullRom), U8x3: horizontal pass, then vertical."""
    img = np.asarray(rgb, np.uint8)
    h, w = img.shape[:2]
    if out_w != w:
        cx, px = fir_coeffs(w, out_w)
        img = _fir_pass(img, cx, px)
    if out_h != h:
        cy, py = fir_coeffs(h, out_h)
        img = _fir_pass(img.transpose(1, 0, 2), cy, py).transpose(1, 0, 2)
    return np.ascontiguousarray(img)


def frame_positions(h, w, merge):
    """build_frame_positions dots_vit.rs:188-211: (hpos, wpos) in merge-group order."""
    pos = []
    for bh in range(h // merge):
        for bw in range(w // merge):
            for ih in range(merge):
                for iw in range(merge):
                    pos.append((bh * merge + ih, bw * merge + iw))
    return np.asarray(pos, np.int64)


def preprocess(rgb, cfg=PREPROC):
    """preprocess_image (preprocess.rs:103-145): returns (patches [N][3*p*p] f32 in merge-group order,
    grid (t, h, w)); pages off the smart_resize grid go through the Catmull-Rom resize (283-299)."""
    rgb = np.asarray(rgb, np.uint8)
    H, W = rgb.shape[:2]
    p, m = cfg["patch_size"], cfg["merge_size"]
    rh, rw = smart_resize(H, W, p * m, cfg["min_pixels"], cfg["max_pixels"])
    if (rh, rw) != (H, W):
        rgb = fir_resize_catmull_rom(rgb, rw, rh)
        H, W = rh, rw
    rescale = F32(1.0) / F32(255.0)
    mean = np.asarray(cfg["image_mean"], F32)
    std = np.asarray(cfg["image_std"], F32)
    norm = ((rgb.astype(F32) * rescale) - mean) / std                 # normalise_rgb 175-190
    gh, gw = H // p, W // p
    patches = norm.reshape(gh // m, m, p, gw // m, m, p, 3)               # [bh, ih, py, bw, iw, px, c]
    patches = patches.transpose(0, 3, 1, 4, 6, 2, 5)                    # [bh, bw, ih, iw, c, py, px]
    return np.ascontiguousarray(patches.reshape(gh * gw, 3 * p * p), F32), (1, gh, gw)


# ----------------------------------------------------------------------------- model
def rms_norm(x, w, eps):
    x = x.astype(F32, copy=False)
    ms = (x * x).sum(axis=-1, keepdims=True, dtype=F32) / F32(x.shape[-1])
    return (x / np.sqrt(ms + F32(eps))) * w


def layer_norm(x, w, b, eps):
    x = x.astype(F32, copy=False)
    mu = x.mean(-1, keepdims=True, dtype=F32)
    d = x - mu
    var = (d * d).mean(-1, keepdims=True, dtype=F32)
    return d / np.sqrt(var + F32(eps)) * w + b


def silu_bf16(x):
    """candle-kernels silu_fwd(x) = x / (1 + exp(-x)) with every op in bf16."""
    e = bf16(np.exp(-x))
    return bf16(x / bf16(F32(1.0) + e))


def gelu_bf16(x):
    """candle-kernels gelu_fwd (tanh form) in bf16: x_sq = x*x, x_cube = x_sq*x,
    alpha = x + 0.044715*x_cube, 0.5*x*(1 + tanh(sqrt(2/pi)*alpha)), every op rounded."""
    c = bf16(np.asarray(0.044715, F32))
    k = bf16(np.asarray(math.sqrt(2.0 / math.pi), F32))
    half = F32(0.5)
    x_sq = bf16(x * x)
    x_cube = bf16(x_sq * x)
    alpha = bf16(x + bf16(c * x_cube))
    t = bf16(np.tanh(bf16(k * alpha)))
    return bf16(bf16(half * x) * bf16(F32(1.0) + t))


class DotsVision:
    """dots.ocr vision tower with the weight names of the checkpoint (prefix `vision_tower.`)."""

    def __init__(self, vcfg: dict, weights, prefix="vision_tower."):
        self.c = vcfg
        self.W = weights
        self.p = prefix
        self.D = vcfg["embed_dim"]
        self.heads = vcfg["num_attention_heads"]
        self.hd = self.D // self.heads
        self.eps = vcfg["rms_norm_eps"]
        self.merge = vcfg["spatial_merge_size"]

    def w(self, name, shape):
        return bf16(self.W.get(self.p + name, shape))

    def has(self, name):
        return self.W.has(self.p + name)

    def linear(self, x, name, out_dim, in_dim, bias=None):
        y = bf16(x @ self.w(name + ".weight", (out_dim, in_dim)).T)
        use_bias = self.c.get("use_bias", False) if bias is None else bias
        if use_bias and self.has(name + ".bias"):
            y = bf16(y + self.w(name + ".bias", (out_dim,)))
        return y

    def rotary(self, positions):
        """VisionRotaryEmbedding (dots_vit.rs:697-735) -> cos, sin [N][head_dim] (cat [t, t])."""
        rope_dim = self.hd // 2
        axis = rope_dim // 2
        inv = np.asarray([F32(1.0) / (F32(10000.0) ** (F32(2 * i) / F32(rope_dim))) for i in range(axis)], F32)
        hp = positions[:, 0].astype(F32)[:, None]
        wp = positions[:, 1].astype(F32)[:, None]
        rope = np.concatenate([hp * inv[None], wp * inv[None]], 1).astype(F32)
        # f32 cos / sin, correctly rounded (computed in f64)
        cos = np.cos(rope.astype(np.float64)).astype(F32)
        sin = np.sin(rope.astype(np.float64)).astype(F32)
        return np.concatenate([cos, cos], 1), np.concatenate([sin, sin], 1)

    def attention(self, i, x, cos, sin):
        N, D, H, hd = x.shape[0], self.D, self.heads, self.hd
        qkv = self.linear(x, f"blocks.{i}.attn.qkv", 3 * D, D).reshape(N, 3, H, hd)
        q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]

        def rot(t):  # apply_rotary_to (f32), then back to bf16
            r = np.concatenate([-t[..., hd // 2:], t[..., :hd // 2]], -1)
            return bf16((t * cos[:, None, :]) + (r * sin[:, None, :]))
        q, k = rot(q), rot(k)
        scale = F32(1.0 / math.sqrt(hd))
        out = np.empty((N, H, hd), F32)
        for h in range(H):
            kt = np.ascontiguousarray(k[:, h].T)
            for q0 in range(0, N, 2048):  # query chunks (row-wise softmax: same math, bounded memory)
                s = (q[q0:q0 + 2048, h] @ kt) * scale
                s = s - s.max(-1, keepdims=True)
                e = np.exp(s)
                pr = e / e.sum(-1, keepdims=True, dtype=F32)
                out[q0:q0 + 2048, h] = pr @ v[:, h]
        ctx = bf16(out.reshape(N, D))
        return self.linear(ctx, f"blocks.{i}.attn.proj", D, D)

    def block(self, i, x, cos, sin):
        D, I = self.D, self.c["intermediate_size"]
        n1 = bf16(rms_norm(x, self.w(f"blocks.{i}.norm1.weight", (D,)), self.eps))
        x = bf16(x + self.attention(i, n1, cos, sin))
        n2 = bf16(rms_norm(x, self.w(f"blocks.{i}.norm2.weight", (D,)), self.eps))
        g = silu_bf16(self.linear(n2, f"blocks.{i}.mlp.fc1", I, D))
        u = self.linear(n2, f"blocks.{i}.mlp.fc3", I, D)
        h = bf16(g * u)
        return bf16(x + self.linear(h, f"blocks.{i}.mlp.fc2", D, I))

    def forward(self, patches, grid, layers=None):
        """DotsVisionModel::forward (dots_vit.rs:80-96) for one image -> [groups][hidden_size]."""
        D, P = self.D, self.c["patch_size"]
        t, gh, gw = grid
        x = bf16(patches)                                                  # model.rs:155-159
        x = bf16(x @ self.w("patch_embed.patchifier.proj.weight", (D, 3, P, P)).reshape(D, -1).T)
        if self.has("patch_embed.patchifier.proj.bias"):
            x = bf16(x + self.w("patch_embed.patchifier.proj.bias", (D,)))
        x = bf16(rms_norm(x, self.w("patch_embed.patchifier.norm.weight", (D,)), self.eps))
        pos = np.concatenate([frame_positions(gh, gw, self.merge)] * t, 0)
        cos, sin = self.rotary(pos)
        for i in range(self.c["num_hidden_layers"] if layers is None else layers):
            x = self.block(i, x, cos, sin)
        if self.c.get("post_norm", True):
            x = bf16(rms_norm(x, self.w("post_trunk_norm.weight", (D,)), self.eps))
        ln = bf16(layer_norm(x, self.w("merger.ln_q.weight", (D,)), self.w("merger.ln_q.bias", (D,)), 1e-6))
        G = D * self.merge * self.merge
        r = ln.reshape(-1, G)
        pre = gelu_bf16(self.linear(r, "merger.mlp.0", G, G, bias=True))
        return self.linear(pre, "merger.mlp.2", self.c["hidden_size"], G, bias=True)


def dots_tensor_names(vcfg, prefix="vision_tower."):
    """Names/shapes the vision tower reads (dots_vit.rs load paths; dsq-models adapters/dots_ocr.rs)."""
    D, I, P, C = vcfg["embed_dim"], vcfg["intermediate_size"], vcfg["patch_size"], vcfg["num_channels"]
    G = D * vcfg["spatial_merge_size"] ** 2
    t = {prefix + "patch_embed.patchifier.proj.weight": (D, C, P, P),
         prefix + "patch_embed.patchifier.proj.bias": (D,),
         prefix + "patch_embed.patchifier.norm.weight": (D,)}
    for i in range(vcfg["num_hidden_layers"]):
        b = f"{prefix}blocks.{i}."
        t[b + "norm1.weight"] = (D,)
        t[b + "norm2.weight"] = (D,)
        t[b + "attn.qkv.weight"] = (3 * D, D)
        t[b + "attn.proj.weight"] = (D, D)
        t[b + "mlp.fc1.weight"] = (I, D)
        t[b + "mlp.fc2.weight"] = (D, I)
        t[b + "mlp.fc3.weight"] = (I, D)
    t[prefix + "post_trunk_norm.weight"] = (D,)
    t[prefix + "merger.ln_q.weight"] = (D,)
    t[prefix + "merger.ln_q.bias"] = (D,)
    t[prefix + "merger.mlp.0.weight"] = (G, G)
    t[prefix + "merger.mlp.0.bias"] = (G,)
    t[prefix + "merger.mlp.2.weight"] = (vcfg["hidden_size"], G)
    t[prefix + "merger.mlp.2.bias"] = (vcfg["hidden_size"],)
    return t
