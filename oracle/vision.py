"""Oracle: SAM-ViTDet-B + CLIP-L vision tower, projector and token formatting
(TEST INFRASTRUCTURE).  f32 numpy restatement of vision/sam.rs, vision/clip.rs and
model/mod.rs:246-923.  Activations are kept NHWC like the reference's blocks
(sam.rs:243-246).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import erf as _erf

from .config import sam_params, clip_params, projector_params

F32 = np.float32


def layer_norm(x, w, b, eps):
    """candle_nn LayerNorm (remove_mean=true): (x-mean)/sqrt(var+eps)*w+b in f32."""
    x = x.astype(F32, copy=False)
    mean = x.mean(axis=-1, keepdims=True, dtype=F32)
    xc = x - mean
    var = (xc * xc).mean(axis=-1, keepdims=True, dtype=F32)
    return (xc / np.sqrt(var + F32(eps))) * w + b


def gelu_erf(x):
    """candle gelu_erf: 0.5*x*(1+erf(x/sqrt(2)))."""
    return (F32(0.5) * x * (F32(1.0) + _erf(x / F32(math.sqrt(2.0))).astype(F32))).astype(F32)


def sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def linear(x, w, b=None):
    y = x @ w.T
    if b is not None:
        y = y + b
    return y.astype(F32, copy=False)


def softmax(x, axis=-1):
    """candle_nn::ops::softmax: exp(x-max)/sum."""
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True, dtype=F32)


# ----------------------------------------------------------------------------- resizes
def _bicubic_filter_pillow(x):
    a = F32(-0.5)
    x = abs(F32(x))
    if x < 1.0:
        return F32(((a + F32(2.0)) * x - (a + F32(3.0))) * x * x + F32(1.0))
    if x < 2.0:
        return F32((((x - F32(5.0)) * x + F32(8.0)) * x - F32(4.0)) * a)
    return F32(0.0)


def _axis_weights_aa(in_len, out_len, scale):
    """sam.rs:1017-1064 compute_axis_weights_aa (f32)."""
    scale = F32(scale)
    support = F32(2.0) * scale if scale >= 1.0 else F32(2.0)
    invscale = F32(1.0) / scale if scale >= 1.0 else F32(1.0)
    ws, idx = [], []
    for o in range(out_len):
        center = scale * (F32(o) + F32(0.5))
        xmin = max(int(math.floor(center - support + F32(0.5))), 0)
        xmax = min(int(math.floor(center + support + F32(0.5))), in_len)
        xs = max(xmax - xmin, 0)
        xmc = F32(xmin) - center
        wts = []
        tot = F32(0.0)
        for j in range(xs):
            arg = (F32(j) + xmc + F32(0.5)) * invscale
            w = _bicubic_filter_pillow(arg)
            wts.append(w)
            tot = F32(tot + w)
        if tot != 0.0:
            wts = [F32(w / tot) for w in wts]
        ws.append(wts)
        idx.append(list(range(xmin, xmin + xs)))
    return ws, idx


def bicubic_resize_antialiased(inp, out_h, out_w):
    """sam.rs:1000-1123: [C,H,W] f32 -> [C,out_h,out_w]; vertical pass then horizontal."""
    c, in_h, in_w = inp.shape
    if in_h == out_h and in_w == out_w:
        return inp.copy()
    wy, iy = _axis_weights_aa(in_h, out_h, F32(in_h) / F32(out_h))
    wx, ix = _axis_weights_aa(in_w, out_w, F32(in_w) / F32(out_w))
    tmp = np.zeros((c, out_h, in_w), F32)
    for oh in range(out_h):
        acc = np.zeros((c, in_w), F32)
        for k, sy in enumerate(iy[oh]):
            acc += inp[:, sy, :] * wy[oh][k]
        tmp[:, oh, :] = acc
    out = np.zeros((c, out_h, out_w), F32)
    for ow in range(out_w):
        acc = np.zeros((c, out_h), F32)
        for k, sx in enumerate(ix[ow]):
            acc += tmp[:, :, sx] * wx[ow][k]
        out[:, :, ow] = acc
    return out


def get_rel_pos(q_size, k_size, rel):
    """sam.rs:1194-1247: linear resize of the rel-pos table + (q-k) gather."""
    orig_len, hd = rel.shape
    max_rel = 2 * max(q_size, k_size) - 1
    if orig_len == max_rel:
        res = rel
    else:
        res = np.zeros((max_rel, hd), F32)
        scale = F32(orig_len) / F32(max_rel)
        for i in range(max_rel):
            src = scale * (F32(i) + F32(0.5)) - F32(0.5)
            src = min(max(src, F32(0.0)), F32(orig_len - 1))
            lf = F32(math.floor(src))
            left = int(lf)
            right = min(left + 1, orig_len - 1)
            w = F32(min(max(src - lf, F32(0.0)), F32(1.0)))
            res[i] = rel[left] * (F32(1.0) - w) + rel[right] * w
    sq = max(F32(k_size) / F32(q_size), F32(1.0))
    sk = max(F32(q_size) / F32(k_size), F32(1.0))
    out = np.zeros((q_size, k_size, hd), F32)
    for qi in range(q_size):
        for ki in range(k_size):
            r = (F32(qi) * sq - F32(ki) * sk) + (F32(k_size) - F32(1.0)) * sk
            idx = int(min(max(math.floor(r), 0.0), float(max_rel - 1)))
            out[qi, ki] = res[idx]
    return out


# ----------------------------------------------------------------------------- SAM
class Sam:
    def __init__(self, cfg, W):
        self.p = sam_params(cfg)
        self.W = W
        self.pre = "model.sam_model."
        self._pos_cache = {}

    def g(self, name, shape):
        return self.W.get(self.pre + name, shape)

    def pos_embed(self, gh, gw):
        """adapt_position_embedding sam.rs:982-998 (AA bicubic when grid != 64)."""
        p = self.p
        t = p.image_size // p.patch_size
        if not self.W.has(self.pre + "pos_embed"):
            return None
        key = (gh, gw)
        if key not in self._pos_cache:
            pos = self.g("pos_embed", (1, t, t, p.embed_dim))[0]
            if (gh, gw) != (t, t):
                pos = bicubic_resize_antialiased(np.ascontiguousarray(pos.transpose(2, 0, 1)), gh, gw).transpose(1, 2, 0)
            self._pos_cache[key] = np.ascontiguousarray(pos, F32)
        return self._pos_cache[key]

    def attention(self, blk, x, window):
        """SamAttention::forward sam.rs:804-888 on x [N, h, w, C] (already windowed)."""
        p = self.p
        n, h, w, c = x.shape
        nh, hd = p.num_heads, c // p.num_heads
        qkv = linear(x.reshape(n * h * w, c), self.g(f"blocks.{blk}.attn.qkv.weight", (3 * c, c)),
                     self.g(f"blocks.{blk}.attn.qkv.bias", (3 * c,)) if self.W.has(self.pre + f"blocks.{blk}.attn.qkv.bias") else None)
        qkv = qkv.reshape(n, h * w, 3, nh, hd)
        q = qkv[:, :, 0].transpose(0, 2, 1, 3)
        k = qkv[:, :, 1].transpose(0, 2, 1, 3)
        v = qkv[:, :, 2].transpose(0, 2, 1, 3)
        use_rel = self.W.has(self.pre + f"blocks.{blk}.attn.rel_pos_h")
        if use_rel:
            tokens = window if window > 0 else p.image_size // p.patch_size
            rel_dim = 2 * tokens - 1
            Rh = get_rel_pos(h, h, self.g(f"blocks.{blk}.attn.rel_pos_h", (rel_dim, hd)))
            Rw = get_rel_pos(w, w, self.g(f"blocks.{blk}.attn.rel_pos_w", (rel_dim, hd)))
        out = np.empty((n, nh, h * w, hd), F32)
        scale = F32(1.0 / math.sqrt(hd))
        for i in range(n):
            for hh in range(nh):
                qi = q[i, hh]
                s = (qi @ k[i, hh].T) * scale
                if use_rel:
                    qg = qi.reshape(h, w, hd)
                    rel_h = np.einsum("hwc,hkc->hwk", qg, Rh, dtype=F32)   # [h,w,kh]
                    rel_w = np.einsum("hwc,wkc->hwk", qg, Rw, dtype=F32)   # [h,w,kw]
                    bias = rel_h[:, :, :, None] + rel_w[:, :, None, :]
                    s = s + bias.reshape(h * w, h * w)
                out[i, hh] = softmax(s.astype(F32)) @ v[i, hh]
        ctx = out.transpose(0, 2, 1, 3).reshape(n * h * w, c)
        y = linear(ctx, self.g(f"blocks.{blk}.attn.proj.weight", (c, c)),
                   self.g(f"blocks.{blk}.attn.proj.bias", (c,)) if self.W.has(self.pre + f"blocks.{blk}.attn.proj.bias") else None)
        return y.reshape(n, h, w, c)

    def block(self, blk, x):
        """SamBlock::forward sam.rs:731-748 incl. window_partition/unpartition 926-980."""
        p = self.p
        b, H, Wd, c = x.shape
        window = 0 if blk in p.global_attn_indexes else p.window_size
        normed = layer_norm(x, self.g(f"blocks.{blk}.norm1.weight", (c,)), self.g(f"blocks.{blk}.norm1.bias", (c,)), p.norm_eps)
        if window > 0:
            ph = (window - H % window) % window
            pw = (window - Wd % window) % window
            padded = np.zeros((b, H + ph, Wd + pw, c), F32)
            padded[:, :H, :Wd] = normed
            hp, wp = H + ph, Wd + pw
            win = padded.reshape(b, hp // window, window, wp // window, window, c).transpose(0, 1, 3, 2, 4, 5)
            win = win.reshape(-1, window, window, c)
            aw = self.attention(blk, win, window)
            rest = aw.reshape(b, hp // window, wp // window, window, window, c).transpose(0, 1, 3, 2, 4, 5)
            attn = rest.reshape(b, hp, wp, c)[:, :H, :Wd]
        else:
            attn = self.attention(blk, normed, 0)
        res = x + attn
        n2 = layer_norm(res, self.g(f"blocks.{blk}.norm2.weight", (c,)), self.g(f"blocks.{blk}.norm2.bias", (c,)), p.norm_eps)
        hid = int(c * p.mlp_ratio)
        fc1 = "mlp.fc1" if self.W.has(self.pre + f"blocks.{blk}.mlp.fc1.weight") else "mlp.lin1"
        fc2 = "mlp.fc2" if self.W.has(self.pre + f"blocks.{blk}.mlp.fc2.weight") else "mlp.lin2"
        h1 = linear(n2.reshape(-1, c), self.g(f"blocks.{blk}.{fc1}.weight", (hid, c)), self.g(f"blocks.{blk}.{fc1}.bias", (hid,)))
        h2 = linear(gelu_erf(h1), self.g(f"blocks.{blk}.{fc2}.weight", (c, hid)), self.g(f"blocks.{blk}.{fc2}.bias", (c,)))
        return res + h2.reshape(b, H, Wd, c)

    def forward(self, img):
        """SamBackbone::forward sam.rs:210-289.  img [B,3,H,W] -> NHWC [B,H/64,W/64,C_out]."""
        p = self.p
        b, _, H, Wd = img.shape
        ps = p.patch_size
        gh, gw = H // ps, Wd // ps
        cols = img.reshape(b, 3, gh, ps, gw, ps).transpose(0, 2, 4, 1, 3, 5).reshape(b * gh * gw, 3 * ps * ps)
        x = linear(cols, self.g("patch_embed.proj.weight", (p.embed_dim, 3, ps, ps)).reshape(p.embed_dim, -1),
                   self.g("patch_embed.proj.bias", (p.embed_dim,)))
        x = x.reshape(b, gh, gw, p.embed_dim)
        pos = self.pos_embed(gh, gw)
        if pos is not None:
            x = x + pos[None]
        for blk in range(p.depth):
            x = self.block(blk, x)
        # neck sam.rs:503-520 (NHWC throughout; LN2d == row LN over channels)
        nc = p.neck_channels
        x = conv2d_nhwc(x, self.g("neck.0.weight", (nc, p.embed_dim, 1, 1)), stride=1, pad=0)
        x = layer_norm(x, self.g("neck.1.weight", (nc,)), self.g("neck.1.bias", (nc,)), 1e-6)
        x = conv2d_nhwc(x, self.g("neck.2.weight", (nc, nc, 3, 3)), stride=1, pad=1)
        x = layer_norm(x, self.g("neck.3.weight", (nc,)), self.g("neck.3.bias", (nc,)), 1e-6)
        # downsample sam.rs:550-575
        c0, c1 = p.out_channels
        x = conv2d_nhwc(x, self.g("net_2.weight", (c0, nc, 3, 3)), stride=2, pad=1)
        x = conv2d_nhwc(x, self.g("net_3.weight", (c1, c0, 3, 3)), stride=2, pad=1)
        return x


def conv2d_nhwc(x, w, stride, pad):
    """Conv2d (no bias) on NHWC input with an [O,C,kh,kw] weight."""
    b, H, Wd, c = x.shape
    o, ci, kh, kw = w.shape
    assert ci == c
    xp = np.zeros((b, H + 2 * pad, Wd + 2 * pad, c), F32)
    xp[:, pad:pad + H, pad:pad + Wd] = x
    oh = (H + 2 * pad - kh) // stride + 1
    ow = (Wd + 2 * pad - kw) // stride + 1
    cols = np.empty((b, oh, ow, kh, kw, c), F32)
    for ky in range(kh):
        for kx in range(kw):
            cols[:, :, :, ky, kx, :] = xp[:, ky:ky + stride * oh:stride, kx:kx + stride * ow:stride, :]
    wm = w.transpose(0, 2, 3, 1).reshape(o, kh * kw * c)
    return (cols.reshape(b * oh * ow, -1) @ wm.T).reshape(b, oh, ow, o).astype(F32)


# ----------------------------------------------------------------------------- CLIP
class Clip:
    def __init__(self, cfg, W):
        self.p = clip_params(cfg)
        self.W = W
        self.pre = "model.vision_model."
        self._pos = {}

    def g(self, n, shape):
        return self.W.get(self.pre + n, shape)

    def pos(self, ntok):
        """adapt_position_embedding clip.rs:486-544."""
        p = self.p
        if ntok not in self._pos:
            tab = self.g("embeddings.position_embedding.weight", (p.seq_length + 1, p.hidden_size))
            if ntok == p.seq_length + 1:
                self._pos[ntok] = tab
            else:
                s = int(round(math.sqrt(p.seq_length)))
                t = int(round(math.sqrt(ntok - 1)))
                grid = np.ascontiguousarray(tab[1:].reshape(s, s, -1).transpose(2, 0, 1))
                r = bicubic_resize_antialiased(grid, t, t).transpose(1, 2, 0).reshape(t * t, -1)
                self._pos[ntok] = np.concatenate([tab[:1], r], 0).astype(F32)
        return self._pos[ntok]

    def forward(self, sam_nhwc):
        """ClipVisionModel::forward clip.rs:98-102 with SAM features as patch embeds."""
        p = self.p
        b, gh, gw, c = sam_nhwc.shape
        assert c == p.hidden_size and gh == gw
        patches = sam_nhwc.reshape(b, gh * gw, c)
        cls = np.broadcast_to(self.g("embeddings.class_embedding", (c,)), (b, 1, c))
        x = np.concatenate([cls, patches], 1) + self.pos(gh * gw + 1)[None]
        x = layer_norm(x, self.g("pre_layrnorm.weight", (c,)), self.g("pre_layrnorm.bias", (c,)), p.eps)
        nh, hd = p.num_heads, c // p.num_heads
        s = x.shape[1]
        for li in range(p.num_layers):
            pre = f"transformer.layers.{li}."
            n1 = layer_norm(x, self.g(pre + "layer_norm1.weight", (c,)), self.g(pre + "layer_norm1.bias", (c,)), p.eps)
            qkv = linear(n1.reshape(-1, c), self.g(pre + "self_attn.qkv_proj.weight", (3 * c, c)),
                         self.g(pre + "self_attn.qkv_proj.bias", (3 * c,))).reshape(b, s, 3, nh, hd)
            q = qkv[:, :, 0].transpose(0, 2, 1, 3)
            k = qkv[:, :, 1].transpose(0, 2, 1, 3)
            v = qkv[:, :, 2].transpose(0, 2, 1, 3)
            scale = F32(1.0 / math.sqrt(hd))
            att = softmax((q @ k.transpose(0, 1, 3, 2)) * scale) @ v
            att = att.transpose(0, 2, 1, 3).reshape(-1, c)
            x = x + linear(att, self.g(pre + "self_attn.out_proj.weight", (c, c)),
                           self.g(pre + "self_attn.out_proj.bias", (c,))).reshape(b, s, c)
            n2 = layer_norm(x, self.g(pre + "layer_norm2.weight", (c,)), self.g(pre + "layer_norm2.bias", (c,)), p.eps)
            h1 = linear(n2.reshape(-1, c), self.g(pre + "mlp.fc1.weight", (p.ffn_hidden_size, c)),
                        self.g(pre + "mlp.fc1.bias", (p.ffn_hidden_size,)))
            h1 = sigmoid(h1 * F32(1.702)) * h1                      # quick_gelu clip.rs:413-416
            x = x + linear(h1, self.g(pre + "mlp.fc2.weight", (c, p.ffn_hidden_size)),
                           self.g(pre + "mlp.fc2.bias", (c,))).reshape(b, s, c)
        return x


# ----------------------------------------------------------------------------- assembly
class Vision:
    """VisionContext (model/mod.rs:526-923): SAM -> CLIP -> concat -> project -> format."""

    def __init__(self, cfg, W):
        self.cfg = cfg
        self.W = W
        self.sam = Sam(cfg, W)
        self.clip = Clip(cfg, W)
        pc = projector_params(cfg)
        self.n_embed = pc["n_embed"]
        self.input_dim = pc["input_dim"]

    def project(self, x):
        """ImageProjector::project model/mod.rs:392-444."""
        w = self.W.get("model.projector.layers.weight", (self.n_embed, self.input_dim))
        b = self.W.get("model.projector.layers.bias", (self.n_embed,)) if self.W.has("model.projector.layers.bias") else None
        return linear(x, w, b)

    def newline(self):
        return self.W.get("model.image_newline", (self.n_embed,))

    def separator(self):
        return self.W.get("model.view_seperator", (self.n_embed,))

    def features(self, img):
        """compute_global / process_patch_batch: returns (pre [B,S,2048], post [B,S,n_embed])."""
        sam = self.sam.forward(img)
        clip = self.clip.forward(sam)
        b, gh, gw, c = sam.shape
        pre = np.concatenate([clip[:, 1:], sam.reshape(b, gh * gw, c)], -1)  # build_clip_sam_tokens 604-650
        post = self.project(pre.reshape(-1, pre.shape[-1])).reshape(b, gh * gw, -1)
        return pre, post

    def embeddings(self, glob, patches, crop):
        """process_input_full + assemble_artifacts: [local tokens, global tokens, view_separator]."""
        nl = self.newline()
        _, gpost = self.features(glob)
        side = int(round(math.sqrt(gpost.shape[1])))
        grid = gpost[0].reshape(side, side, -1)
        gtok = np.concatenate([grid, np.broadcast_to(nl, (side, 1, nl.shape[0]))], 1).reshape(-1, nl.shape[0])
        segs = []
        if patches is not None and len(patches) > 0:
            _, lpost = self.features(patches)
            wc, hc = crop
            ls = int(round(math.sqrt(lpost.shape[1])))
            g = lpost.reshape(hc, wc, ls, ls, -1).transpose(0, 2, 1, 3, 4).reshape(hc * ls, wc * ls, -1)
            segs.append(np.concatenate([g, np.broadcast_to(nl, (hc * ls, 1, nl.shape[0]))], 1).reshape(-1, nl.shape[0]))
        segs.append(gtok)
        segs.append(self.separator()[None])
        return np.concatenate(segs, 0).astype(F32)
