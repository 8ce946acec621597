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
