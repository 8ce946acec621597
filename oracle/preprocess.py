"""Oracle: host image preprocessing a1-a3 (TEST INFRASTRUCTURE).

Integer restatement of the reference's Pillow-compatible bicubic resampler
(vision/resample.rs:1-160), global view construction (model/mod.rs:2295-2330),
dynamic crop-grid selection (vision/preprocess.rs:67-138) and pixel
normalisation (model/mod.rs:2332-2347).  Bit-exact integer work.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 22
ROUNDING_BIAS = 1 << (PRECISION_BITS - 1)


def _bicubic_kernel(x: float) -> float:
    """resample.rs:32-42 (a = -0.5)."""
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0
    if x < 2.0:
        return (((x - 5.0) * x + 8.0) * x - 4.0) * a
    return 0.0


def _round_half_towards_zero(v: float) -> int:
    """resample.rs:24-30."""
    return math.floor(v + 0.5) if v >= 0.0 else math.ceil(v + 0.5)


def compute_resample_coeffs(in_size: int, out_size: int):
    """resample.rs:44-99: f64 weights normalised then quantised to 22-bit ints."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = []
    coeffs = np.zeros((out_size, ksize), dtype=np.int64)
    for o in range(out_size):
        center = (o + 0.5) * scale
        xmin = max(_round_half_towards_zero(center - support), 0)
        xmax = min(_round_half_towards_zero(center + support), in_size)
        if xmin >= in_size:
            xmin = max(in_size - 1, 0)
        if xmax <= xmin:
            xmax = xmin + 1
        length = xmax - xmin
        ss = 1.0 / filterscale
        row = [0.0] * ksize
        total = 0.0
        for i in range(length):
            w = _bicubic_kernel((xmin + i - center + 0.5) * ss)
            row[i] = w
            total += w
        if total != 0.0:
            for i in range(length):
                row[i] /= total
        for i in range(ksize):
            v = row[i]
            # Rust `as i32` truncates toward zero (resample.rs:90-94)
            coeffs[o, i] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0.0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds.append((xmin, length))
    return bounds, coeffs, ksize


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bicubic(src: np.ndarray, width: int, height: int) -> np.ndarray:
    """resample.rs:101-160.  src: HxWx3 uint8 -> height x width x 3 uint8."""
    sh, sw, _ = src.shape
    if width == 0 or height == 0:
        return np.zeros((height, width, 3), np.uint8)
    bx, cx, _ = compute_resample_coeffs(sw, width)
    by, cy, _ = compute_resample_coeffs(sh, height)
    s64 = src.astype(np.int64)
    horiz = np.empty((sh, width, 3), np.uint8)
    for x in range(width):
        start, ln = bx[x]
        acc = np.full((sh, 3), ROUNDING_BIAS, dtype=np.int64)
        for i in range(ln):
            acc += s64[:, start + i, :] * cx[x, i]
        horiz[:, x, :] = _clip8(acc)
    h64 = horiz.astype(np.int64)
    out = np.empty((height, width, 3), np.uint8)
    for y in range(height):
        start, ln = by[y]
        acc = np.full((width, 3), ROUNDING_BIAS, dtype=np.int64)
        for i in range(ln):
            acc += h64[start + i, :, :] * cy[y, i]
        out[y] = _clip8(acc)
    return out


def round_ties_to_even(v: float) -> float:
    """model/mod.rs:2295-2306 (Rust f64::round is half-away-from-zero)."""
    r = math.floor(abs(v) + 0.5) * (1 if v >= 0 else -1)
    if abs(v - r) != 0.5:
        return float(r)
    t = math.trunc(v)
    return float(t) if int(t) % 2 == 0 else float(t + math.copysign(1.0, v))


def build_global_view(img: np.ndarray, base: int) -> np.ndarray:
    """model/mod.rs:2308-2330: fit into base x base on a gray(127) canvas."""
    mean = int(0.5 * 255.0)
    canvas = np.full((base, base, 3), mean, np.uint8)
    h, w, _ = img.shape
    if w == 0 or h == 0:
        return canvas
    scale = min(base / w, base / h)
    nw = int(min(max(round_ties_to_even(w * scale), 1.0), float(base)))
    nh = int(min(max(round_ties_to_even(h * scale), 1.0), float(base)))
    resized = resize_bicubic(img, nw, nh)
    xo = int(round_ties_to_even((base - nw) * 0.5))
    yo = int(round_ties_to_even((base - nh) * 0.5))
    # imageops::replace clips to the canvas
    canvas[yo:yo + nh, xo:xo + nw] = resized[: base - yo, : base - xo]
    return canvas


def dynamic_preprocess(img: np.ndarray, tile: int, min_num: int = 2, max_num: int = 9):
    """preprocess.rs:67-138 with PreprocessParams::ocr1 (min 2, max 9, no-crop <= tile)."""
    h, w, _ = img.shape
    if w <= tile and h <= tile:
        return [], (1, 1)
    aspect = w / h
    ratios = sorted({(i, j) for n in range(min_num, max_num + 1) for i in range(1, n + 1)
                     for j in range(1, n + 1) if min_num <= i * j <= max_num})
    best = (1, 1)
    best_diff = float("inf")
    area = float(w * h)
    eps = 2.220446049250313e-16
    for (wr, hr) in ratios:  # BTreeSet order
        diff = abs(aspect - wr / hr)
        if diff < best_diff:
            best_diff = diff
            best = (wr, hr)
        elif abs(diff - best_diff) < eps and area > 0.5 * (tile * tile * wr * hr):
            best = (wr, hr)
    tw, th = tile * best[0], tile * best[1]
    resized = resize_bicubic(img, tw, th)
    tiles = []
    for i in range(best[0] * best[1]):
        x = (i % best[0]) * tile
        y = (i // best[0]) * tile
        tiles.append(resized[y:y + tile, x:x + tile].copy())
    return tiles, best


def image_to_tensor(img: np.ndarray) -> np.ndarray:
    """model/mod.rs:2332-2347: CHW f32, (v/255 - 0.5)/0.5 computed in f32."""
    v = img.astype(np.float32) / np.float32(255.0)
    v = (v - np.float32(0.5)) / np.float32(0.5)
    return np.ascontiguousarray(v.transpose(2, 0, 1))


def prepare_vision_input(img: np.ndarray, base: int = 1024, image_size: int = 640, crop_mode: bool = True):
    """model/mod.rs:1707-1758 (Ocr1 variant)."""
    gsize = base if crop_mode else image_size
    gview = build_global_view(img, gsize)
    glob = image_to_tensor(gview)[None]
    if crop_mode:
        tiles, crop = dynamic_preprocess(img, image_size)
        patches = np.stack([image_to_tensor(t) for t in tiles]) if tiles else None
        return glob, patches, crop
    return glob, None, None
