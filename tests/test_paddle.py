"""PaddleOCR-VL CPU plumbing path (BASELINE configs[0]; dsocr/paddle.py restating crates/infer-paddleocr).

Mirrors the reference's own tests (crates/infer-paddleocr/tests/model.rs:88-157, transformer_model.rs) where they
run without a checkpoint (prompt builder, position ids, injection, decoder shapes), and pins the whole path —
preprocessing, SigLIP tower, projector, Ernie prefill + greedy decode — with the committed fixtures of
tests/golden/make_paddle_golden.py: the full PaddleOCR-VL-0.9B architecture on the reference's assets/sample_1.png
and a tiny architecture on a synthetic page.  The reference's PaddleOCR fixtures and checkpoint are not available
offline, so parity against the Candle path itself is unpinned.
"""
import io
import os

import numpy as np
import pytest

from dsocr import paddle
from dsocr.cli import build_parser, run_inference

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")

import sys  # noqa: E402

sys.path.insert(0, GOLD)
import make_paddle_golden as mk  # noqa: E402


@pytest.fixture(scope="module")
def tiny():
    eng = paddle.PaddleOcrEngine(paddle.PADDLE_TINY_CONFIG, synthetic_seed=0)
    yield eng
    eng.close()


def test_smart_resize_matches_the_reference_formula():
    # sample_1.png (2852 x 1756) at the CLI's image_size 640: max_pixels 409600, factor 28 -> (476, 812)
    assert paddle.smart_resize(1756, 2852, 28, paddle.MIN_PIXELS, 640 * 640) == (476, 812)
    # already a multiple of the factor and inside the pixel range: unchanged
    assert paddle.smart_resize(448, 448, 28, paddle.MIN_PIXELS, paddle.MAX_PIXELS) == (448, 448)
    # below min_pixels: scaled up with ceil
    h, w = paddle.smart_resize(100, 100, 28, paddle.MIN_PIXELS, paddle.MAX_PIXELS)
    assert h * w >= paddle.MIN_PIXELS and h % 28 == 0 and w % 28 == 0
    with pytest.raises(ValueError):
        paddle.smart_resize(1, 1000, 28, paddle.MIN_PIXELS, paddle.MAX_PIXELS)  # aspect > 200


def test_prompt_builder_matches_placeholder_tokens(tiny):
    """tests/model.rs:88-103."""
    tok = paddle.PaddleSyntheticTokenizer(tiny.cfg)
    grid = (1, 16, 16)
    toks, mask = paddle.build_prompt_tokens(tok, "Question: <image> Describe.", [grid], tiny.cfg)
    assert sum(mask) == 1 * (16 // 2) * (16 // 2)
    assert len(toks) == len(mask)
    i = toks.index(tiny.cfg.image_token_id)
    assert toks[0] == tiny.cfg.bos_token_id and toks[i - 1] == tiny.cfg.vision_start_token_id
    assert toks[i + 64] == tok.token_to_id(paddle.IMAGE_END_TOKEN)
    with pytest.raises(ValueError):
        paddle.build_prompt_tokens(tok, "no image slot", [grid], tiny.cfg)


def test_position_ids_cover_image_span(tiny):
    """tests/model.rs:105-131: [3, L] positions, consecutive image tokens share the time axis."""
    tok = paddle.PaddleSyntheticTokenizer(tiny.cfg)
    grid = (1, 16, 16)
    toks, _ = paddle.build_prompt_tokens(tok, "User: <image> end.", [grid], tiny.cfg)
    pos, delta = paddle.compute_position_ids(tiny.cfg, toks, [grid])
    assert pos.shape == (3, len(toks))
    i = toks.index(tiny.cfg.image_token_id)
    assert pos[0, i] == pos[0, i + 1]
    # rows / cols of the 8 x 8 merged grid on the h / w axes, offset by the text before the span
    assert pos[1, i + 8] == pos[1, i] + 1 and pos[2, i + 1] == pos[2, i] + 1
    # the text after the span continues at base + token count; delta = max + 1 - L
    assert pos[0, i + 64] == pos[0, i] + 64
    assert delta == int(pos.max()) + 1 - len(toks)


def test_mrope_sections_select_the_position_axes(tiny):
    """select_sections (attention.rs): dims [0, 2 s0) rotate by axis 0, then axis 1, then axis 2."""
    dec = tiny.decoder
    pos = np.array([[3], [5], [7]], np.int64)
    cos, _ = dec._cos_sin(pos)
    s0, s1, _ = dec.sections
    half = tiny.cfg.head_dim // 2
    inv = dec.inv
    assert np.allclose(cos[0, :s0], np.cos(np.float32(3) * inv[np.arange(s0) % half]))
    assert np.allclose(cos[0, s0:s0 + s1], np.cos(np.float32(5) * inv[np.arange(s0, s0 + s1) % half]))
    assert np.allclose(cos[0, s0 + s1:], np.cos(np.float32(7) * inv[np.arange(s0 + s1, 2 * half) % half]))


@pytest.mark.parametrize("name", ["tiny", "sample1"])
def test_paddle_greedy_ids_equal_fixture(name):
    """The whole path (preprocess -> SigLIP -> projector -> Ernie prefill + greedy decode with the 20-gram ban) on the
    committed fixture's input equals the fixture: ids, prompt ids, image mask, grid, 3-axis positions, image rows."""
    fx = dict(np.load(os.path.join(GOLD, f"paddle_{name}.npz")))
    got = mk.run(name)
    assert got["grid"].tolist() == fx["grid"].tolist()
    assert got["prompt_ids"].tolist() == fx["prompt_ids"].tolist()
    assert got["image_mask"].tolist() == fx["image_mask"].tolist()
    assert np.array_equal(got["positions"], fx["positions"]) and int(got["delta"]) == int(fx["delta"])
    assert abs(float(got["emb_sum"]) - float(fx["emb_sum"])) <= 1e-4 * float(fx["emb_abs_sum"])
    assert np.allclose(got["emb_row0"], fx["emb_row0"], rtol=1e-4, atol=1e-5)
    assert got["ids"].tolist() == fx["ids"].tolist()


def test_cli_runs_paddleocr_vl_on_cpu(tmp_path):
    img = np.random.default_rng(3).integers(0, 256, (120, 160, 3), dtype=np.uint8)
    from PIL import Image
    p = tmp_path / "page.png"
    Image.fromarray(img).save(p)
    args = build_parser().parse_args(["--model", "paddleocr-vl", "--model-config", paddle.PADDLE_TINY_CONFIG,
                                      "--device", "cpu", "--prompt", "<image>\nOCR:", "--image", str(p),
                                      "--max-new-tokens", "5", "--image-size", "224", "-q"])
    out, err = io.StringIO(), io.StringIO()
    assert run_inference(args, out, err) == 0
    assert out.getvalue().strip() != ""
