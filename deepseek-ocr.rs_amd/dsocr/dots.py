"""dots.ocr vision tower (BASELINE configs[3]) bound to the C ABI (dsocr_dots_*).

Mirrors crates/infer-dots: ``preprocess`` = vision/preprocess.rs preprocess_image (patches in
merge-group order + grid_thw), ``DotsVision.embed`` = DotsVisionModel::forward
(vision/dots_vit.rs:80-96) on one page -> [groups][hidden] rows (bf16 values as float32).
All compute runs in libdsocr.so on a gfx950 GPU; this module only marshals.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import DsocrError, check, lib

_HERE = os.path.dirname(os.path.abspath(__file__))
DOTS_CONFIG = os.path.join(_HERE, "configs", "dots-ocr.json")
DOTS_TINY_CONFIG = os.path.join(_HERE, "configs", "dots-tiny.json")


def _rgb(img):
    if hasattr(img, "convert"):
        img = np.asarray(img.convert("RGB"))
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim != 3 or img.shape[2] != 3:
        raise DsocrError(1, "page must be HxWx3 uint8")
    return img


def preprocess(config_path: str, img):
    """Host preprocessing (dsocr_dots_preprocess): (patches [N][3*p*p] float32, (t, h, w))."""
    rgb = _rgb(img)
    n = C.c_size_t()
    grid = (C.c_uint32 * 3)()
    check(lib().dsocr_dots_preprocess(config_path.encode(), rgb.ctypes.data_as(C.c_void_p), rgb.shape[1], rgb.shape[0],
                                      None, 0, C.byref(n), grid))
    out = None
    with open(config_path) as f:
        import json
        v = json.load(f).get("vision_config", {})
    pd = 3 * v.get("patch_size", 14) ** 2
    out = np.empty((n.value, pd), np.float32)
    check(lib().dsocr_dots_preprocess(config_path.encode(), rgb.ctypes.data_as(C.c_void_p), rgb.shape[1], rgb.shape[0],
                                      out.ctypes.data_as(C.c_void_p), n.value, C.byref(n), grid))
    return out, (grid[0], grid[1], grid[2])


class DotsVision:
    def __init__(self, config_path: str = DOTS_CONFIG, weights_path=None, synthetic_seed: int = 0, device: int = 0):
        h = C.c_void_p()
        check(lib().dsocr_dots_load(config_path.encode(), weights_path.encode() if weights_path else None,
                                    synthetic_seed, device, C.byref(h)))
        self._h = h
        self.config_path = config_path
        hid, emb, nl, pd = C.c_size_t(), C.c_size_t(), C.c_size_t(), C.c_size_t()
        check(lib().dsocr_dots_info(h, C.byref(hid), C.byref(emb), C.byref(nl), C.byref(pd)))
        self.hidden, self.embed_dim, self.layers, self.patch_dim = hid.value, emb.value, nl.value, pd.value

    def embed(self, img):
        rgb = _rgb(img)
        n = C.c_size_t()
        grid = (C.c_uint32 * 3)()
        cap = (rgb.shape[0] * rgb.shape[1]) // 4 + 4096  # upper bound refined below
        check(lib().dsocr_dots_preprocess(self.config_path.encode(), rgb.ctypes.data_as(C.c_void_p), rgb.shape[1],
                                          rgb.shape[0], None, 0, C.byref(n), grid))
        cap = n.value // 4 + 1
        out = np.empty((cap, self.hidden), np.float32)
        check(lib().dsocr_dots_embed(self._h, rgb.ctypes.data_as(C.c_void_p), rgb.shape[1], rgb.shape[0],
                                     out.ctypes.data_as(C.c_void_p), cap, C.byref(n), grid))
        return out[:n.value], (grid[0], grid[1], grid[2])

    def embed_device(self, d_patches, grid, d_out, time_attention_layers: int = 0):
        check(lib().dsocr_dots_embed_device(self._h, d_patches, grid[0], grid[1], grid[2], d_out, time_attention_layers))

    def last_timings(self) -> dict:
        from ._lib import DotsTimingsC
        t = DotsTimingsC()
        check(lib().dsocr_dots_last_timings(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in DotsTimingsC._fields_}

    def close(self):
        if getattr(self, "_h", None):
            lib().dsocr_dots_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
