"""Committed golden fixtures (tests/golden/tiny_pages.json, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces them (guards the oracle itself, which is pinned independently by
tests/test_oracle_crosscheck.py and the Pillow tests).  GPU: the engine reproduces them through
the C ABI without running the oracle on the box: greedy ids exact, image embeddings to 1e-3."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402

GOLD = json.load(open(os.path.join(HERE, "golden", "tiny_pages.json")))


def _page(p):
    return mg.image(p["image_seed"], p["height"], p["width"])


@pytest.fixture(scope="module")
def oracle_model():
    from oracle.model import OracleModel
    from oracle.weights import Weights
    return OracleModel(json.load(open(mg.TINY)), Weights(seed=GOLD["weights_seed"], dtype="f16"))


@pytest.mark.parametrize("i", range(len(GOLD["pages"])))
def test_oracle_reproduces_golden(oracle_model, i):
    from oracle.preprocess import prepare_vision_input
    p = GOLD["pages"][i]
    img = _page(p)
    glob, tiles, crop = prepare_vision_input(img, 256, 128, True)
    assert mg.digest(glob) == p["global_pixels_sha"]
    assert (mg.digest(tiles) if tiles is not None else None) == p["tiles_sha"]
    emb, crop = oracle_model.image_embeddings(img, 256, 128, True)
    assert list(crop) == p["crop"] and emb.shape[0] == p["n_image_rows"]
    assert abs(float(emb.astype(np.float64).sum()) - p["embedding_sum"]) <= 1e-5 * p["embedding_abs_sum"]
    gen, _ = oracle_model.generate(p["prompt_ids"], p["image_mask"], emb, len(p["generated"]), eos_token_id=1,
                                   no_repeat_ngram_size=20)
    assert gen == p["generated"]


@pytest.mark.gpu
def test_engine_reproduces_golden(gpu):
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, load_model
    eng = load_model(ModelLoadArgs(config_path=mg.TINY, synthetic_seed=GOLD["weights_seed"], dtype="f16"))
    try:
        vs = VisionSettings(256, 128, True)
        for p in GOLD["pages"]:
            page = Page(_page(p), vs)
            assert list(page.crop_shape) == p["crop"]
            emb = eng.image_embeddings([page])[0]
            assert emb.shape[0] == p["n_image_rows"]
            assert abs(float(emb.astype(np.float64).sum()) - p["embedding_sum"]) <= 1e-3 * p["embedding_abs_sum"]
            assert np.allclose(emb[0, :8], p["embedding_row0_head"], rtol=1e-3, atol=1e-4)
            got = eng.generate(p["prompt_ids"], p["image_mask"], page, None,
                               DecodeParameters(max_new_tokens=len(p["generated"])))
            assert got == p["generated"]
    finally:
        eng.close()


def test_oracle_generate_without_cache_matches_cached(oracle_model):
    """The oracle's generate_without_cache restatement gives the cached path's ids (text-only prompt)."""
    ids = [0] + list(range(40, 70))
    a = oracle_model.generate_without_cache(ids, None, None, 8, eos_token_id=1, no_repeat_ngram_size=20)
    b, _ = oracle_model.generate(ids, [0] * len(ids), None, 8, eos_token_id=1, no_repeat_ngram_size=20)
    assert a == b


# ---------------------------------------------------------------- a16: the product's prompt builder
@pytest.mark.parametrize("prompt,counts", [
    ("<image>\n<|grounding|>Convert the document to markdown.", [693]),
    ("<image>\nFree OCR.", [273]),
    ("Compare <image> with <image>, then summarise.", [100, 257]),
    ("<image><image>", [5, 7]),
    ("No image at all, just text.", []),
])
def test_product_prompt_builder_equals_oracle(prompt, counts):
    """dsocr.build_prompt_tokens (the product's host builder) gives the oracle's ids and mask
    (oracle/model.py build_prompt_tokens, model/mod.rs:2536-2603) for single, multiple and no images."""
    from dsocr import build_prompt_tokens
    from dsocr.synth import SyntheticTokenizer
    from oracle.model import build_prompt_tokens as oracle_build
    tok = SyntheticTokenizer(129280)
    ids, mask = build_prompt_tokens(tok, prompt, counts)
    segs = [list(tok.encode(s, add_special_tokens=False).ids) for s in prompt.split("<image>")]
    rids, rmask = oracle_build(segs, tok.token_to_id("<image>"), counts)
    assert ids == rids and mask == rmask
    assert sum(mask) == sum(counts)


def test_product_prompt_builder_mismatch_is_einval():
    """slots != images -> the reference's 'prompt/image embedding mismatch' (400 class, DSOCR_EINVAL)."""
    from dsocr import build_prompt_tokens
    from dsocr._lib import DsocrError
    from dsocr.synth import SyntheticTokenizer
    with pytest.raises(DsocrError) as e:
        build_prompt_tokens(SyntheticTokenizer(512), "<image> and <image>", [10])
    assert "mismatch" in str(e.value)
