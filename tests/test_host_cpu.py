"""CPU tests: oracle pinning (Pillow, reference constants), host preprocessing of
the product library (host-only entry points, no GPU), synthetic-weight recipe,
and the C-ABI export surface."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest
from PIL import Image

from oracle import preprocess as opre
from oracle.config import clip_params, resolved_language_config, sam_params, should_use_moe
from oracle.decoder import banned_ngram_tokens, select_token_id
from oracle.weights import synth_bf16

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FULL = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "deepseek-ocr.json")
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")


def _lib():
    from dsocr._lib import lib
    return lib()


def _rand_img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


# ----------------------------------------------------------------- oracle pinned by Pillow
# The reference resampler reproduces Pillow's 22-bit integer bicubic (resample.rs:9-11) except
# one detail: its round_half_towards_zero(center - support) (resample.rs:24-30, 55) yields
# xmin = 1 where Pillow's (int)(x + 0.5) truncation yields 0, for center - support in (-0.5, 0)
# -- i.e. only at strong upscales (scale < 0.5).  We follow the reference; these cases are
# pinned against Pillow only where the two agree, and product == oracle bit-exactly everywhere.
PILLOW_EXACT = [((37, 53), (20, 31)), ((300, 420), (128, 256)), ((64, 64), (64, 64)),
                ((1024, 1024), (1280, 1280)), ((1756, 2852), (1280, 1920)), ((2852, 1756), (1024, 631))]
REF_ONLY = [((100, 80), (640, 512)), ((17, 900), (40, 300))]


@pytest.mark.parametrize("src,dst", PILLOW_EXACT)
def test_oracle_resize_matches_pillow(src, dst):
    img = _rand_img(src[0], src[1], 3)
    ref = np.asarray(Image.fromarray(img).resize((dst[1], dst[0]), Image.BICUBIC))
    got = opre.resize_bicubic(img, dst[1], dst[0])
    assert np.array_equal(got, ref)


def test_reference_xmin_rounding_deviation_is_the_only_pillow_gap():
    """Strong upscale: the only difference to Pillow comes from the xmin rounding above."""
    row = np.random.default_rng(3).integers(0, 256, (1, 10, 3), dtype=np.uint8)
    b, _, _ = opre.compute_resample_coeffs(10, 40)
    assert b[6][0] == 1  # center 1.625 - support 2 = -0.375 -> reference rounds to 1 (Pillow: 0)
    got = opre.resize_bicubic(row, 40, 1)
    ref = np.asarray(Image.fromarray(row).resize((40, 1), Image.BICUBIC))
    diff = np.nonzero(np.any(got != ref, axis=-1)[0])[0]
    assert set(diff.tolist()) <= {6, 7}


@pytest.mark.parametrize("src,dst", PILLOW_EXACT + REF_ONLY)
def test_product_resize_bit_exact_vs_oracle(src, dst):
    img = _rand_img(src[0], src[1], 5)
    out = np.empty((dst[0], dst[1], 3), np.uint8)
    assert _lib().dsocr_resize_bicubic(img.ctypes.data_as(C.c_void_p), src[1], src[0],
                                       out.ctypes.data_as(C.c_void_p), dst[1], dst[0]) == 0
    assert np.array_equal(out, opre.resize_bicubic(img, dst[1], dst[0]))


@pytest.mark.parametrize("hw,expect", [((1024, 1024), (2, 2)), ((1756, 2852), (3, 2)), ((600, 500), (1, 1)),
                                       ((2000, 700), (1, 3)), ((700, 2600), (4, 1))])
def test_crop_grid(hw, expect):
    """dynamic_preprocess_with_params (preprocess.rs:67-138); 1024^2 -> (2,2) is SURVEY §0's 4 tiles."""
    img = _rand_img(hw[0], hw[1], 1)
    _, grid = opre.dynamic_preprocess(img, 640)
    assert grid == expect


def test_placeholder_counts():
    """1024^2 page, crop (2,2): 420 local + 273 global = 693 image tokens."""
    from oracle.model import image_placeholder_count
    assert image_placeholder_count(1024, 640, True, (2, 2)) == 693
    assert image_placeholder_count(1024, 640, True, (1, 1)) == 273
    assert image_placeholder_count(1024, 640, False, None) == 111


@pytest.mark.parametrize("hw,vs", [((1024, 1024), (1024, 640, True)), ((300, 420), (256, 128, True)),
                                   ((500, 333), (1024, 640, True)), ((900, 1300), (1024, 640, False))])
def test_product_prepare_page_matches_oracle(hw, vs):
    from dsocr import Page, VisionSettings
    img = _rand_img(hw[0], hw[1], 11)
    page = Page(img, VisionSettings(*vs))
    g, tiles = page.pixels()
    og, otiles, ocrop = opre.prepare_vision_input(img, vs[0], vs[1], vs[2])
    assert np.array_equal(g, og[0])
    if otiles is None:
        assert tiles is None
    else:
        assert page.crop_shape == ocrop
        assert np.array_equal(tiles, otiles)
    from oracle.model import image_placeholder_count
    assert page.n_image_tokens == image_placeholder_count(vs[0], vs[1], vs[2], ocrop)


# ----------------------------------------------------------------- reference constants
def test_reference_config_constants():
    """tests/config.rs:32-58, vision_sam.rs:25-36, vision_clip.rs:9-20, transformer_weights.rs:32-43."""
    cfg = json.load(open(FULL))
    lang = resolved_language_config(cfg)
    assert (lang.hidden_size, lang.num_hidden_layers, lang.num_attention_heads) == (1280, 12, 10)
    assert lang.torch_dtype == "bfloat16"
    sp = sam_params(cfg)
    assert (sp.image_size, sp.patch_size, sp.embed_dim, sp.depth, sp.num_heads) == (1024, 16, 768, 12, 12)
    assert sp.global_attn_indexes == [2, 5, 8, 11]
    cp = clip_params(cfg)
    assert (cp.hidden_size, cp.num_heads, cp.num_layers, cp.patch_size, cp.image_size) == (1024, 16, 24, 14, 224)
    assert cp.seq_length + 1 == 257
    assert not should_use_moe(lang, 0) and should_use_moe(lang, 1)


def test_window_partition_math():
    """vision_sam.rs:70-81: (64, 48, 14) -> padded 70 x 56, tiles 5 x 4."""
    h, w, win = 64, 48, 14
    ph, pw = (win - h % win) % win, (win - w % win) % win
    assert (h + ph, w + pw, (h + ph) // win, (w + pw) // win) == (70, 56, 5, 4)


def test_clip_pos_downsample_shape():
    """vision_clip.rs:22-33: 257 -> 101 tokens."""
    from oracle.vision import bicubic_resize_antialiased
    tab = np.zeros((1024, 16, 16), np.float32)
    assert bicubic_resize_antialiased(tab, 10, 10).shape == (1024, 10, 10)


def test_aa_bicubic_matches_torch():
    """sam.rs:1000-1123 restates aten::_upsample_bicubic2d_aa; pin the oracle against torch."""
    torch = pytest.importorskip("torch")
    from oracle.vision import bicubic_resize_antialiased
    x = np.random.default_rng(0).standard_normal((8, 64, 64)).astype(np.float32)
    ref = torch.nn.functional.interpolate(torch.from_numpy(x)[None], size=(40, 40), mode="bicubic",
                                          align_corners=False, antialias=True)[0].numpy()
    got = bicubic_resize_antialiased(x, 40, 40)
    assert np.max(np.abs(got - ref)) < 1e-5


def test_rel_pos_resize_matches_torch_linear():
    """get_rel_pos_vec's resize = F.interpolate(mode='linear'), sam.rs:1202-1231."""
    torch = pytest.importorskip("torch")
    from oracle.vision import get_rel_pos
    rel = np.random.default_rng(1).standard_normal((127, 64)).astype(np.float32)
    ref = torch.nn.functional.interpolate(torch.from_numpy(rel.T)[None], size=79, mode="linear")[0].numpy().T
    out = get_rel_pos(40, 40, rel)  # [q, k, hd] gathered from the resized table
    for qi, ki in [(0, 0), (5, 17), (39, 0), (0, 39), (20, 20)]:
        assert np.max(np.abs(out[qi, ki] - ref[qi - ki + 39])) < 1e-6


# ----------------------------------------------------------------- sampling semantics
def test_ngram_ban_and_argmax_ties():
    seq = [1, 2, 3, 1, 2]
    assert banned_ngram_tokens(seq, 3) == {3}
    assert banned_ngram_tokens([5, 6], 3) == set()
    lg = np.zeros(8, np.float32)
    lg[3] = lg[5] = 2.0
    assert select_token_id(lg, [0], 1.0, None) == 3            # first index on ties
    assert select_token_id(lg, [1, 2, 3, 1, 2], 1.0, 3) == 5   # 3 banned
    lg2 = np.full(4, -np.inf, np.float32)
    assert select_token_id(lg2, [0], 1.0, None) == 0


def test_repetition_penalty():
    lg = np.array([1.0, -1.0, 0.5, 3.0], np.float32)
    assert select_token_id(lg, [3], 4.0, None) == 0            # 3.0/4 < 1.0


# ----------------------------------------------------------------- synthetic recipe + C ABI
@pytest.mark.parametrize("name", ["model.layers.3.mlp.experts.7.up_proj.weight", "model.sam_model.blocks.0.norm1.weight",
                                  "lm_head.weight"])
def test_synth_recipe_product_equals_oracle(name):
    n = 4097
    ora = synth_bf16(name, 1234, n)
    prod = np.empty(n, np.uint16)
    assert _lib().dsocr_synth_bf16(name.encode(), 1234, n, prod.ctypes.data_as(C.c_void_p)) == 0
    assert np.array_equal(ora, prod)


def test_c_abi_exports_every_declared_symbol():
    header = open(os.path.join(ROOT, "include", "dsocr.h")).read()
    declared = set(re.findall(r"\b(dsocr_[a-z0-9_]+)\s*\(", header)) - {"dsocr_stream_cb"}
    from dsocr._lib import EXPORTS
    assert declared == set(EXPORTS)
    L = _lib()
    for s in declared:
        assert hasattr(L, s), s


@pytest.mark.parametrize("waiting,api,cus,fits", [
    # dec_qkv_attn at its bound (24 chunks x 10 heads poll the q/k/v row): 4 blocks per CU (102 VGPRs) x 256 CUs
    (24 * 10, 4, 256, 1),
    # the same grid on a part that could hold one block per CU on 240 CUs: every slot could be a waiter
    (24 * 10, 1, 240, 0), (24 * 10, 1, 241, 1),
    # the 8-page polling merge: 8 pages x 10 heads merging blocks (the rest of the 1600-block grid never waits)
    (8 * 10, 4, 256, 1),
    # the API may over-admit one block per CU at 6..8: 7 reported -> 6 usable
    (6 * 256, 7, 256, 0), (6 * 256 - 1, 7, 256, 1), (8 * 256 - 1, 12, 256, 0), (7 * 256 - 1, 12, 256, 1),
    # no slot at all (occupancy query failed -> 0): never poll
    (1, 0, 256, 0), (0, 0, 256, 1)])
def test_poll_residency_rule(waiting, api, cus, fits):
    """Residency rule of the in-launch polled hand-offs (dec_qkv_attn, the dec_attn polling merge): the launch
    polls only if the blocks that may wait cannot fill every slot the device has for the kernel (HIP promises
    no dispatch order), else the engine takes the non-polling form.  Pure host decision through the C ABI."""
    assert _lib().dsocr_k_poll_wait_fits(waiting, api, cus) == fits


def test_engine_load_errors_without_gpu_are_loud():
    """The product path must fail loudly (never fall back to CPU) when no device/config is usable."""
    from dsocr import DsocrError, ModelLoadArgs, load_model
    with pytest.raises(DsocrError):
        load_model(ModelLoadArgs(config_path="/nonexistent/config.json"))


def test_moe_dispatch_kernel_names():
    """Which kernels the dispatch picks (host-only query; the bench labels its roofline with it)."""
    import ctypes as C
    from dsocr._lib import check, lib
    want = {1: ("moe_gateup_mix_kernel", "moe_down_mix_kernel"), 2: ("moe_gateup_slot_kernel", "moe_down_slot_kernel"),
            3: ("moe_gateup_mm_kernel", "moe_down_mm_kernel"), 8: ("moe_gateup_mm_kernel", "moe_down_mm_kernel"),
            9: ("moe_gateup2_kernel", "moe_down2_kernel")}
    for T, (gu, dn) in want.items():
        g, d = C.c_char_p(), C.c_char_p()
        check(lib().dsocr_k_moe_kernels(T, 1280, 64, 6, 896, 1792, 1, C.byref(g), C.byref(d)))
        assert (g.value.decode(), d.value.decode()) == (gu, dn), T
