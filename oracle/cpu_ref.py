"""ctypes side of oracle/cpu_ref.cpp, the C++ / OpenMP CPU restatement of the decoder page path
(TEST / BENCH INFRASTRUCTURE: only tests/ and bench.py's cpu_baseline leg use it; never the product).

build() compiles oracle/_build/libcpuref.so (g++ -O3 -march=x86-64-v4 -fopenmp: AVX-512, which this container's
Xeon and the GPU box's EPYC both have).  CpuRef(cfg, weights) copies the decoder tensors the oracle's Weights
loader produces (the reference's --dtype f16 rounding applied) into the library: decoder linears / embeddings as
f16 (exact), lm_head as bf16 (exact), norms f32.  generate() = DeepseekOcrModel::generate (model/mod.rs:1870-2048,
greedy, EOS ignored) with the prefill and decode stage times.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .config import resolved_language_config, should_use_moe

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
_SO = os.path.join(_BUILD, "libcpuref.so")


def build() -> str:
    os.makedirs(_BUILD, exist_ok=True)
    src = os.path.join(_HERE, "cpu_ref.cpp")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O3", "-march=x86-64-v4", "-fopenmp", "-shared", "-fPIC", "-o", _SO, src])
    return _SO


def _lib():
    L = C.CDLL(_SO if os.path.exists(_SO) else build())
    i32, f32, vp = C.c_int, C.c_float, C.c_void_p
    L.cr_init.argtypes = [i32] * 13 + [f32, f32, f32, vp, i32]
    L.cr_set.argtypes = [C.c_char_p, vp, C.c_long, C.c_long, i32]
    L.cr_generate.argtypes = [vp, vp, i32, vp, i32, i32, i32, vp, vp]
    L.cr_free.restype = None
    L.cr_set_threads.argtypes = [i32]
    L.cr_set_threads.restype = None
    L.cv_init.argtypes = [i32, i32, i32, i32, vp, i32, i32, i32, i32, f32, i32, i32, i32, i32, f32, i32, i32, i32]
    L.cv_features.argtypes = [vp, i32, i32, i32, vp, vp, vp]
    return L


def decoder_tensor_names(cfg):
    """The decoder tensors (name -> shape) of oracle/specs.tensor_names."""
    from .specs import tensor_names
    return {n: s for n, s in tensor_names(cfg).items()
            if n.startswith("model.layers.") or n.startswith("model.embed_tokens.") or n in ("model.norm.weight", "lm_head.weight")}


class CpuRef:
    def __init__(self, cfg, weights, threads=0):
        self.L = _lib()
        lang = resolved_language_config(cfg)
        self.lang = lang
        H, nh = lang.hidden_size, lang.num_attention_heads
        flags = (C.c_int * lang.num_hidden_layers)(*[1 if should_use_moe(lang, i) else 0 for i in range(lang.num_hidden_layers)])
        rc = self.L.cr_init(H, nh, lang.num_key_value_heads or nh, H // nh, lang.num_hidden_layers, lang.vocab_size,
                            lang.intermediate_size, lang.moe_intermediate_size or 0, lang.n_routed_experts or 0,
                            lang.num_experts_per_tok or 0, lang.n_shared_experts or 0, 1 if lang.norm_topk_prob else 0,
                            1 if (lang.scoring_func or "softmax") == "softmax" else 0, float(lang.rms_norm_eps),
                            float(lang.rope_theta), float(lang.routed_scaling_factor or 1.0), flags, int(threads))
        if rc:
            raise RuntimeError(f"cpu_ref init failed ({rc})")
        for name, shape in decoder_tensor_names(cfg).items():
            if not weights.has(name):
                continue
            a = np.ascontiguousarray(weights.get(name, shape), dtype=np.float32)
            rows, cols = (shape[0], int(np.prod(shape[1:]))) if len(shape) > 1 else (1, shape[0])
            kind = 2 if name == "lm_head.weight" else (1 if len(shape) == 2 else 0)
            self.L.cr_set(name.encode(), a.ctypes.data_as(C.c_void_p), rows, cols, kind)
            weights._cache.pop(name, None)  # the library holds its own copy

    def generate(self, ids, mask, image_rows, max_new, ngram=20):
        ids = np.ascontiguousarray(ids, np.int64)
        m = np.ascontiguousarray(mask if mask is not None else np.zeros(len(ids)), np.uint8)
        rows = np.ascontiguousarray(image_rows if image_rows is not None else np.zeros((0, self.lang.hidden_size)), np.float32)
        out = np.zeros(max_new, np.int64)
        ms = np.zeros(2, np.float64)
        rc = self.L.cr_generate(ids.ctypes.data_as(C.c_void_p), m.ctypes.data_as(C.c_void_p), len(ids),
                                rows.ctypes.data_as(C.c_void_p), rows.shape[0], max_new, ngram,
                                out.ctypes.data_as(C.c_void_p), ms.ctypes.data_as(C.c_void_p))
        if rc:
            raise RuntimeError(f"cpu_ref generate failed ({rc})")
        return out.tolist(), {"prefill_ms": float(ms[0]), "decode_ms": float(ms[1])}

    def close(self):
        self.L.cr_free()


class CpuVision:
    """The vision tower (SAM-ViTDet-B + CLIP-L + projector) in C++ / OpenMP (cv_features in cpu_ref.cpp; oracle
    restatement oracle/vision.py of sam.rs / clip.rs / model/mod.rs:246-923).  The weight-only tables (position
    embeddings resized to each grid, rel-pos tables per block and grid) come from the oracle's own functions, once,
    for the view sizes given; the conv weights are re-laid [O][kh][kw][C] for the NHWC im2col.  embeddings(rgb) =
    Vision.embeddings with the features computed in C++; stage times in last_ms."""

    def __init__(self, cfg, weights, threads=0, sizes=(1024, 640)):
        from .config import clip_params, projector_params, sam_params
        from .vision import Clip, Sam, Vision, get_rel_pos
        self.L = _lib()
        sp, cp, pp = sam_params(cfg), clip_params(cfg), projector_params(cfg)
        self.sp, self.cp = sp, cp
        self.n_embed, self.in_dim = pp["n_embed"], pp["input_dim"]
        flags = (C.c_int * sp.depth)(*[1 if i in sp.global_attn_indexes else 0 for i in range(sp.depth)])
        rc = self.L.cv_init(sp.embed_dim, sp.depth, sp.num_heads, sp.window_size, flags, sp.neck_channels,
                            sp.out_channels[0], sp.out_channels[1], sp.patch_size, float(sp.norm_eps), cp.hidden_size,
                            cp.num_layers, cp.num_heads, cp.ffn_hidden_size, float(cp.eps), self.n_embed, self.in_dim,
                            int(threads))
        if rc:
            raise RuntimeError(f"cpu_ref vision init failed ({rc})")
        from .specs import tensor_names
        conv = {"model.sam_model.neck.0.weight": "cv.sam.neck.0", "model.sam_model.neck.2.weight": "cv.sam.neck.2",
                "model.sam_model.net_2.weight": "cv.sam.net_2", "model.sam_model.net_3.weight": "cv.sam.net_3"}
        for name, shape in tensor_names(cfg).items():
            if not name.startswith(("model.sam_model.", "model.vision_model.", "model.projector.")) or not weights.has(name):
                continue
            a = np.asarray(weights.get(name, shape), np.float32)
            if name in conv:
                a = a.transpose(0, 2, 3, 1)
                self._set(conv[name], a.reshape(a.shape[0], -1), 3)
            elif len(shape) >= 2 and "pos" not in name and "rel_pos" not in name:
                self._set(name, a.reshape(shape[0], -1), 3)  # bf16 values (exact), packed panels
            else:
                self._set(name, a.reshape(1, -1) if a.ndim < 2 else a.reshape(a.shape[0], -1), 0)
        sam, clip = Sam(cfg, weights), Clip(cfg, weights)
        self._vision = Vision(cfg, weights)
        hd = sp.embed_dim // sp.num_heads
        for size in sizes:
            g = size // sp.patch_size
            pos = sam.pos_embed(g, g)
            if pos is not None:
                self._set(f"cv.sam.pos.{g}x{g}", pos.reshape(g * g, -1), 0)
            for blk in range(sp.depth):
                pre = f"model.sam_model.blocks.{blk}.attn."
                if not weights.has(pre + "rel_pos_h"):
                    continue
                win = 0 if blk in sp.global_attn_indexes else sp.window_size
                n = g if win == 0 else win
                tokens = win if win > 0 else sp.image_size // sp.patch_size
                rel = (2 * tokens - 1, hd)
                self._set(f"cv.sam.relh.{blk}.{n}", get_rel_pos(n, n, weights.get(pre + "rel_pos_h", rel)).reshape(n, -1), 0)
                self._set(f"cv.sam.relw.{blk}.{n}", get_rel_pos(n, n, weights.get(pre + "rel_pos_w", rel)).reshape(n, -1), 0)
            go = g // 4
            self._set(f"cv.clip.pos.{go * go + 1}", clip.pos(go * go + 1), 0)
        self.last_ms = {}

    def _set(self, name, a, kind):
        a = np.ascontiguousarray(a, np.float32)
        self.L.cr_set(name.encode(), a.ctypes.data_as(C.c_void_p), a.shape[0], int(np.prod(a.shape[1:])), kind)

    def features(self, img, want_pre=False):
        """img [B,3,H,W] f32 -> (pre [B,G,in_dim] or None, post [B,G,n_embed])."""
        img = np.ascontiguousarray(img, np.float32)
        B, _, H, Wd = img.shape
        G = (H // 64) * (Wd // 64)
        post = np.zeros((B, G, self.n_embed), np.float32)
        pre = np.zeros((B, G, self.in_dim), np.float32) if want_pre else None
        ms = np.zeros(3, np.float64)
        rc = self.L.cv_features(img.ctypes.data_as(C.c_void_p), B, H, Wd, post.ctypes.data_as(C.c_void_p),
                                pre.ctypes.data_as(C.c_void_p) if want_pre else None, ms.ctypes.data_as(C.c_void_p))
        if rc:
            raise RuntimeError(f"cpu_ref vision failed ({rc})")
        for k, v in zip(("sam_ms", "clip_ms", "projector_ms"), ms):
            self.last_ms[k] = self.last_ms.get(k, 0.0) + float(v)
        return pre, post

    def embeddings(self, rgb, base=1024, image_size=640, crop_mode=True):
        """OracleModel.image_embeddings with the tower in C++ (preprocessing and token formatting as the oracle)."""
        from . import preprocess
        glob, patches, crop = preprocess.prepare_vision_input(rgb, base, image_size, crop_mode)
        self.last_ms = {}
        v = self._vision
        orig = v.features
        v.features = lambda img: self.features(img)
        try:
            return v.embeddings(glob, patches, crop), crop
        finally:
            v.features = orig


def set_threads(n: int) -> None:
    """OpenMP team size for every later CpuRef / CpuVision call in this process."""
    _lib().cr_set_threads(int(n))
