"""dots.ocr vision tower (BASELINE configs[3]; crates/infer-dots/src/vision/dots_vit.rs, preprocess.rs).

CPU: the oracle (oracle/dots.py) and the product's host preprocessing against the reference's own
tests (layout positions, constant-image preprocessing, config pins), and product == oracle pixels.
GPU: the tower through the C ABI vs the oracle — tiny config computed live, the full config
(42 layers, 1536 wide) against committed fixtures (tests/golden/dots_*.npz, made by
make_dots_golden.py): 448 px (1024 tokens) and the 2044 px page (21316 tokens: a 2048 px page
resized to it, the "2048px" config).

Tolerance (bf16 semantics: every op output is rounded to bf16, so f32 summation-order differences
flip single bf16 roundings that then propagate through the 42 blocks): relative Frobenius error of
the compared rows <= DOTS_REL = 0.05, and row sums within DOTS_REL of the mean row abs sum.  The noise
floor this is set against was measured: the oracle with its matmuls summed in f64 instead of f32
(both valid orders of the reference's f32 math) differs from the f32-summed oracle by 0.0209 on the
448 px page (tests/golden/make_dots_golden.py fixture), the engine by 0.0211.
"""
import json
import os

import numpy as np
import pytest

from oracle import dots as od

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG_DIR = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs")
FULL = os.path.join(CFG_DIR, "dots-ocr.json")
TINY = os.path.join(CFG_DIR, "dots-tiny.json")
GOLD = os.path.join(ROOT, "tests", "golden")
DOTS_REL = 5e-2
DOTS_ONE_BLOCK_REL = 5e-3  # one block: f32 summation order + the single bf16 roundings it flips (measured below)


# ---------------------------------------------------------------- CPU: oracle pinned to the reference's tests
def test_layout_positions_follow_merge_groups():
    """crates/infer-dots/tests/vision_dots_vit.rs:4-19."""
    pos = od.frame_positions(4, 4, 2)
    assert len(pos) == 16 and len(pos) // 4 == 4
    assert pos[:8].tolist() == [[0, 0], [0, 1], [1, 0], [1, 1], [0, 2], [0, 3], [1, 2], [1, 3]]


def test_preprocess_constant_image_oracle_and_product(tmp_path):
    """crates/infer-dots/tests/vision_preprocess.rs:15-47: 28x28 gray 128, min = max = 28*28 pixels,
    mean = std = 0.5 -> grid [1, 2, 2], pixel_values (4, 3, 14, 14), mean ((128/255) - 0.5) / 0.5."""
    cfg = dict(od.PREPROC, min_pixels=28 * 28, max_pixels=28 * 28, image_mean=[0.5] * 3, image_std=[0.5] * 3)
    img = np.full((28, 28, 3), 128, np.uint8)
    p, grid = od.preprocess(img, cfg)
    assert grid == (1, 2, 2) and p.shape == (4, 3 * 14 * 14)
    expected = ((128.0 / 255.0) - 0.5) / 0.5
    assert abs(float(p.sum()) / p.size - expected) < 1e-6
    from dsocr.dots import preprocess
    full = json.load(open(FULL))
    full["preprocessor_config"].update(min_pixels=28 * 28, max_pixels=28 * 28, image_mean=[0.5] * 3, image_std=[0.5] * 3)
    path = tmp_path / "cfg.json"
    path.write_text(json.dumps(full))
    q, g2 = preprocess(str(path), img)
    assert g2 == grid and np.array_equal(p, q)


def test_config_pins():
    """crates/infer-dots/tests/config.rs:4-11 and the dsq adapter's dots config (tests/adapters.rs:71-95)."""
    c = json.load(open(FULL))
    assert c["model_type"] == "dots_ocr" and c["image_token_id"] == 151665 and c["video_token_id"] == 151656
    assert c["num_hidden_layers"] == 28 and c["vision_config"]["num_hidden_layers"] == 42
    v = c["vision_config"]
    assert (v["embed_dim"], v["intermediate_size"], v["num_attention_heads"], v["patch_size"],
            v["spatial_merge_size"]) == (1536, 4224, 12, 14, 2)
    pp = c["preprocessor_config"]
    assert (pp["min_pixels"], pp["max_pixels"]) == (3136, 11289600)  # tests/vision_preprocess.rs:9-12


@pytest.mark.parametrize("hw", [(2048, 2048), (2044, 2044), (1000, 700), (20, 900), (5000, 4000), (28, 28),
                                (300, 411), (61, 1500)])
def test_preprocess_product_equals_oracle(hw):
    """smart_resize, the fast_image_resize Catmull-Rom resize (preprocess.rs:283-299; restated, parity
    unpinned against the crate) and the patch layout: product (C++ host) == oracle (numpy), bit for bit,
    on pages that need no resize, a downscale (2048 -> 2044, the bench page), upscales (20 x 900 and
    61 x 1500 grow to the 3136-pixel minimum) and a page over the pixel budget (5000 x 4000)."""
    from dsocr.dots import preprocess
    h, w = hw
    rh, rw = od.smart_resize(h, w, 28, 3136, 11289600)
    assert rh % 28 == 0 and rw % 28 == 0 and rh * rw <= 11289600
    img = np.random.default_rng(h * 7 + w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    if h * w > 4_000_000:  # the oracle's numpy resize of a 20 Mpixel page is slow: a smooth crop keeps it bounded
        img = np.ascontiguousarray(np.broadcast_to(img[:1, :1], (h, w, 3)))
    q, grid = preprocess(FULL, img)
    assert grid == (1, rh // 14, rw // 14) and q.shape == (rh * rw // 196, 588)
    p, g = od.preprocess(img)
    assert g == grid and np.array_equal(p, q)


def test_fir_catmull_rom_vs_pillow():
    """Where the restated fast_image_resize Catmull-Rom (i16 weights, <= 14-bit precision) and Pillow's
    bicubic (the same a = -0.5 cubic, 22-bit weights) part on the bench's 2048 -> 2044 page: the same
    cubic, so they differ only by fixed-point rounding — at most 1 (of 255) per value in each pass, stated
    here as max |diff| <= 2 and a small fraction of differing values."""
    from PIL import Image
    from dsocr.synth import synthetic_page
    img = synthetic_page(0, 2048, 2048)
    fir = od.fir_resize_catmull_rom(img, 2044, 2044)
    pil = np.asarray(Image.fromarray(img).resize((2044, 2044), Image.BICUBIC))
    d = np.abs(fir.astype(np.int16) - pil.astype(np.int16))
    frac = float((d > 0).mean())
    print(f"fir vs Pillow 2048->2044: max |diff| {d.max()}, differing values {frac:.4%}")
    assert d.max() <= 2 and frac < 0.05


# ---------------------------------------------------------------- GPU
def _rel_err(got, ref):
    return float(np.linalg.norm((got - ref).astype(np.float64)) / max(np.linalg.norm(ref.astype(np.float64)), 1e-30))


@pytest.mark.gpu
def test_dots_tiny_tower_matches_oracle(gpu):
    from dsocr.dots import DotsVision
    from dsocr.synth import synthetic_page
    from oracle.weights import Weights
    vcfg = json.load(open(TINY))["vision_config"]
    img = synthetic_page(3, 280, 224)
    eng = DotsVision(TINY, synthetic_seed=11)
    try:
        got, grid = eng.embed(img)
    finally:
        eng.close()
    patches, g = od.preprocess(img)
    ref = od.DotsVision(vcfg, Weights(seed=11, dtype="f32")).forward(patches, g)
    assert grid == g and got.shape == ref.shape == (224 * 280 // 784, vcfg["hidden_size"])
    err = _rel_err(got, ref)
    print(f"dots tiny rel err {err:.3e}")
    assert err <= DOTS_REL, err


@pytest.mark.gpu
@pytest.mark.parametrize("size", [448, 2044])
def test_dots_full_tower_matches_fixture(gpu, size):
    path = os.path.join(GOLD, f"dots_{size}.npz")
    if not os.path.exists(path):
        pytest.skip(f"fixture {path} not generated")
    fx = dict(np.load(path))
    from dsocr.dots import DotsVision
    from dsocr.synth import synthetic_page
    eng = DotsVision(FULL, synthetic_seed=int(fx["weights_seed"]))
    try:
        got, grid = eng.embed(synthetic_page(0, size, size))
        t = eng.last_timings()
    finally:
        eng.close()
    assert list(grid) == fx["grid"].tolist()
    rows = fx["rows"]
    err = _rel_err(got[rows], fx["row_vals"])
    rs = got.astype(np.float64).sum(1)
    rs_err = float(np.max(np.abs(rs - fx["row_sum"])) / max(float(fx["abs_total"]) / got.shape[0], 1e-30))
    print(json.dumps({"size": size, "rows_rel_err": err, "row_sum_err": rs_err, "ms": t["total_ms"]}))
    assert err <= DOTS_REL and rs_err <= DOTS_REL, (err, rs_err)


@pytest.mark.gpu
def test_dots_one_block_full_width_tight(gpu, tmp_path):
    """One full-width block (1536 wide, 12 heads, SwiGLU 4224) + post-norm + merger on a 448 px page
    (1024 patch tokens) vs the oracle at a tight bound: with a single block the only differences are f32
    summation order inside each op and the rare bf16 rounding flip it causes, so a systematic error in
    any one op (which the 42-block 0.05 bound could hide) shows here.  Bound DOTS_ONE_BLOCK_REL."""
    from dsocr.dots import DotsVision
    from dsocr.synth import synthetic_page
    from oracle.weights import Weights
    full = json.load(open(FULL))
    full["vision_config"]["num_hidden_layers"] = 1
    path = tmp_path / "dots-1block.json"
    path.write_text(json.dumps(full))
    img = synthetic_page(0, 448, 448)
    eng = DotsVision(str(path), synthetic_seed=3)
    try:
        got, grid = eng.embed(img)
    finally:
        eng.close()
    patches, g = od.preprocess(img)
    ref = od.DotsVision(full["vision_config"], Weights(seed=3, dtype="f32")).forward(patches, g)
    err = _rel_err(got, ref)
    mism = float(np.mean(got != ref))
    print(json.dumps({"one_block_rel_err": err, "values_not_bit_equal": mism}))
    assert tuple(grid) == tuple(g) and err <= DOTS_ONE_BLOCK_REL, err


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["tiny", "one_block"])
def test_dots_swiglu_fused_gemm_bitwise(gpu, tmp_path, monkeypatch, which):
    """The fc1|fc3 GEMM with the SwiGLU in its epilogue (interleaved weight rows, DSOCR_DOTS_SWIGLU_FUSE=1)
    and the q|k|v GEMM with the rotary in its epilogue (DSOCR_DOTS_ROPE_FUSE=1; 128-dim heads, so the
    one-block case), both defaults, against the separate GEMM + dots_swiglu8 / dots_rope8 launches: the
    tower outputs are bitwise equal."""
    from dsocr.dots import DotsVision
    from dsocr.synth import synthetic_page
    if which == "tiny":
        cfg, img, seed = TINY, synthetic_page(3, 280, 224), 11
    else:
        full = json.load(open(FULL))
        full["vision_config"]["num_hidden_layers"] = 1
        path = tmp_path / "dots-1block.json"
        path.write_text(json.dumps(full))
        cfg, img, seed = str(path), synthetic_page(0, 448, 448), 3
    outs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("DSOCR_DOTS_SWIGLU_FUSE", fuse)
        monkeypatch.setenv("DSOCR_DOTS_ROPE_FUSE", fuse)
        eng = DotsVision(cfg, synthetic_seed=seed)
        try:
            outs.append(eng.embed(img)[0])
        finally:
            eng.close()
    assert outs[0].shape == outs[1].shape
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32)), float(np.mean(outs[0] != outs[1]))
