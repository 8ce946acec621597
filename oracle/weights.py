"""Oracle: weight access with the reference's dtype rules (TEST INFRASTRUCTURE).

Weight rounding follows the reference's `--dtype f16` load:
  * ``VarBuilder::from_mmaped_safetensors(.., F16, ..)`` (model/mod.rs:981-984)
    rounds every tensor the *language model* reads to f16; decoder linears then
    use an f32 copy (transformer/weights.rs:67-71), norms/router/embeddings are
    cast f16->f32 at use (block.rs:24-29, 1264; transformer/model.rs:116-127).
  * the final norm + lm_head (model/mod.rs:992-1025), the projector
    (model/mod.rs:1053-1055) and SAM/CLIP (model/mod.rs:1058-1063) are re-read
    directly as f32.
So: names under ``model.layers.`` / ``model.embed_tokens.`` -> f16-rounded,
everything else -> exact.  ``dtype='f32'`` (the reference's CPU default,
core/src/runtime.rs:27) keeps everything exact.

Sources: a safetensors file (read with the non-executing ``safetensors.numpy``
loader) or the deterministic synthetic generator of oracle/synth.c.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
_LIB = None


def build_synth() -> str:
    os.makedirs(_BUILD, exist_ok=True)
    so = os.path.join(_BUILD, "libsynth_oracle.so")
    src = os.path.join(_HERE, "synth.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", so, src])
    return so


def _lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build_synth())
        _LIB.dsocr_oracle_synth_bf16.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_double,
                                                 ctypes.c_double, ctypes.c_uint64, ctypes.c_void_p]
    return _LIB


def init_rule(name: str):
    """Synthetic init (same rule as the product's csrc/common/synth.hpp)."""
    is_norm_w = name.endswith(".weight") and (
        "norm" in name or ".neck.1." in name or ".neck.3." in name or ".ln_q." in name)
    if is_norm_w:
        return 1.0, 0.05
    return 0.0, 0.02


def synth_bf16(name: str, seed: int, n: int) -> np.ndarray:
    mean, std = init_rule(name)
    out = np.empty(n, dtype=np.uint16)
    _lib().dsocr_oracle_synth_bf16(name.encode(), ctypes.c_uint64(seed), mean, std, n,
                                   out.ctypes.data_as(ctypes.c_void_p))
    return out


def synthetic_has(name: str) -> bool:
    """Which optional tensors a synthetic checkpoint carries (DeepSeek-OCR layout:
    no attention/MLP biases in the decoder, no router correction bias, no CLIP
    patch conv because CLIP consumes SAM features, clip.rs:134-150)."""
    if name.startswith("model.layers.") and name.endswith(".bias"):
        return False
    if "e_score_correction_bias" in name:
        return False
    if "vision_model.embeddings.patch_embedding" in name:
        return False
    return True


def bf16_bits_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def round_f16(x: np.ndarray) -> np.ndarray:
    return x.astype(np.float16).astype(np.float32)


def is_language_tensor(name: str) -> bool:
    return name.startswith("model.layers.") or name.startswith("model.embed_tokens.")


class Weights:
    """name -> f32 numpy array, applying the dtype rule above."""

    def __init__(self, path: str | None = None, seed: int | None = None, dtype: str = "f16", shapes=None,
                 snapshot=None):
        assert (path is None) != (seed is None), "exactly one of path / seed"
        self.path, self.seed, self.dtype = path, seed, dtype
        # oracle.dsq.Snapshot: its records replace the base tensors, dequantised and stored fp16
        # (BASELINE config 5, dequant-on-load); a snapshot linear's bias comes from its record only
        # (crates/dsq-runtime/src/lib.rs:336-366)
        self.snapshot = snapshot
        self._cache = {}
        self._st = None
        if path is not None:
            from safetensors.numpy import load_file  # non-executing loader
            self._st = None
            self._raw = {}
            self._path = path
            self._load_file = load_file
        self.shapes = shapes  # for synthetic: name -> shape

    def _raw_f32(self, name, shape):
        if self.seed is not None:
            n = int(np.prod(shape))
            return bf16_bits_to_f32(synth_bf16(name, self.seed, n)).reshape(shape)
        if self._st is None:
            self._st = _read_safetensors_f32(self._path)
        if name not in self._st:
            raise KeyError(name)
        arr = self._st[name]
        if tuple(arr.shape) != tuple(shape):
            raise ValueError(f"shape mismatch for {name}: {arr.shape} vs {shape}")
        return arr

    def _snap_bias_owner(self, name):
        if self.snapshot is None or not name.endswith(".bias"):
            return None
        w = name[:-5] + ".weight"
        return w if self.snapshot.has(w) else None

    def has(self, name) -> bool:
        if self.snapshot is not None:
            if self.snapshot.has(name):
                return True
            owner = self._snap_bias_owner(name)
            if owner is not None:
                return self.snapshot.bias_for(owner) is not None
        if self.seed is not None:
            return synthetic_has(name)
        if self._st is None:
            self._st = _read_safetensors_f32(self._path)
        return name in self._st

    def get(self, name, shape=None):
        if name in self._cache:
            return self._cache[name]
        if shape is None:
            shape = self.shapes[name] if self.shapes is not None else None
        if self.snapshot is not None and self.snapshot.has(name):
            a = round_f16(self.snapshot.weight(name))
            if shape is not None and a.size != int(np.prod(shape)):
                raise ValueError(f"snapshot tensor {name} dims mismatch")
            a = np.ascontiguousarray(a.reshape(shape) if shape is not None else a, dtype=np.float32)
            self._cache[name] = a
            return a
        owner = self._snap_bias_owner(name)
        if owner is not None:
            b = self.snapshot.bias_for(owner)
            if b is None:
                raise KeyError(name)
            self._cache[name] = np.ascontiguousarray(b, dtype=np.float32)
            return self._cache[name]
        a = self._raw_f32(name, tuple(shape) if shape is not None else None)
        if self.dtype == "f16" and is_language_tensor(name):
            a = round_f16(a)
        a = np.ascontiguousarray(a, dtype=np.float32)
        self._cache[name] = a
        return a


def _read_safetensors_f32(path):
    """Read a safetensors file; bf16 payloads are widened bit-exactly to f32."""
    import json
    import struct
    out = {}
    with open(path, "rb") as f:
        (hlen,) = struct.unpack("<Q", f.read(8))
        header = json.loads(f.read(hlen))
        base = 8 + hlen
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    for name, meta in header.items():
        if name == "__metadata__":
            continue
        s, e = meta["data_offsets"]
        buf = mm[base + s: base + e]
        dt = meta["dtype"]
        shape = meta["shape"]
        if dt == "BF16":
            arr = bf16_bits_to_f32(np.frombuffer(buf, dtype=np.uint16)).reshape(shape)
        elif dt == "F16":
            arr = np.frombuffer(buf, dtype=np.float16).astype(np.float32).reshape(shape)
        elif dt == "F32":
            arr = np.frombuffer(buf, dtype=np.float32).reshape(shape).copy()
        else:
            raise ValueError(f"unsupported dtype {dt} for {name}")
        out[name] = arr
    return out
