"""End-to-end parity of the MI355X engine against the CPU oracle (same seeded
synthetic checkpoint, same pages, same prompt ids).

Contract: greedy token ids bit-exact; image embeddings within
max-abs 1e-3 of the oracle (reference's own projector tolerance vs Python is 2.0,
tests/baseline.rs:805); batched generate == per-page generate.
"""
import json
import os

import numpy as np
import pytest

from dsocr import DecodeParameters, DsocrError, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
from dsocr.synth import SyntheticTokenizer, synthetic_page
from oracle.model import OracleModel, build_prompt_tokens as o_build
from oracle.weights import Weights

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")
FULL = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "deepseek-ocr.json")
TINY_VS = VisionSettings(256, 128, True)
SEED = 7


@pytest.fixture(scope="module")
def tiny_engine(gpu):
    eng = load_model(ModelLoadArgs(config_path=TINY, synthetic_seed=SEED, dtype="f16"))
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def tiny_oracle():
    return OracleModel(json.load(open(TINY)), Weights(seed=SEED, dtype="f16"))


def _img(seed, h, w):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("hw", [(300, 420), (256, 256), (100, 90), (700, 200)])
def test_tiny_image_embeddings(tiny_engine, tiny_oracle, hw):
    img = _img(hw[0] + hw[1], *hw)
    page = Page(img, TINY_VS)
    got = tiny_engine.image_embeddings([page])[0]
    ref, crop = tiny_oracle.image_embeddings(img, 256, 128, True)
    assert page.crop_shape == crop
    assert got.shape == ref.shape
    assert np.max(np.abs(got - ref)) < 1e-3 * max(1.0, np.max(np.abs(ref)))


def _prompt(tok, page):
    return build_prompt_tokens(tok, "<image>\nConvert the document to markdown.", [page.n_image_tokens])


@pytest.mark.parametrize("hw,max_new", [((300, 420), 24), ((256, 256), 40), ((120, 500), 16)])
def test_tiny_generate_matches_oracle(tiny_engine, tiny_oracle, hw, max_new):
    img = _img(hw[0] * 3 + hw[1], *hw)
    tok = SyntheticTokenizer(512)
    page = Page(img, TINY_VS)
    ids, mask = _prompt(tok, page)
    params = DecodeParameters(max_new_tokens=max_new)
    got = tiny_engine.generate(ids, mask, page, None, params)
    emb, _ = tiny_oracle.image_embeddings(img, 256, 128, True)
    ref, _ = tiny_oracle.generate(ids, mask, emb, max_new, eos_token_id=1, no_repeat_ngram_size=20)
    assert got == ref


def test_tiny_generate_host_rows_and_stream(tiny_engine, tiny_oracle):
    """image rows supplied by the caller (the `image_embeddings` seam) + stream callback."""
    img = _img(5, 260, 300)
    tok = SyntheticTokenizer(512)
    page = Page(img, TINY_VS)
    rows = tiny_engine.image_embeddings([page])[0]
    ids, mask = _prompt(tok, page)
    seen = []
    got = tiny_engine.generate(ids, mask, None, rows, DecodeParameters(max_new_tokens=12),
                               stream=lambda n, toks: seen.append(list(toks)))
    ref, _ = tiny_oracle.generate(ids, mask, rows, 12, eos_token_id=1, no_repeat_ngram_size=20)
    assert got == ref
    assert seen and seen[-1] == got[: len(seen[-1])]


@pytest.mark.parametrize("n", [2, 4])
def test_tiny_batch_equals_single(tiny_engine, n):
    """B <= 2 runs the norm-fused decode kernels, B > 2 the separate-RMSNorm variant: same ids."""
    tok = SyntheticTokenizer(512)
    reqs, singles = [], []
    params = DecodeParameters(max_new_tokens=20)
    for i, hw in enumerate([(300, 420), (256, 256), (500, 140), (130, 130)][:n]):
        page = Page(_img(100 + i, *hw), TINY_VS)
        ids, mask = _prompt(tok, page)
        reqs.append((ids, mask, page, None))
        singles.append(tiny_engine.generate(ids, mask, page, None, params))
    batch = tiny_engine.generate_batch(reqs, params)
    assert batch == singles


def test_tiny_text_only_and_penalty(tiny_engine, tiny_oracle):
    ids = [0] + list(range(20, 60))
    params = DecodeParameters(max_new_tokens=16, repetition_penalty=1.3, no_repeat_ngram_size=3)
    got = tiny_engine.generate(ids, None, None, None, params)
    ref, _ = tiny_oracle.generate(ids, [0] * len(ids), None, 16, eos_token_id=1, repetition_penalty=1.3,
                                  no_repeat_ngram_size=3)
    assert got == ref


def test_eos_stops_generation(tiny_engine, tiny_oracle):
    """With EOS ignored the engine produces max_new tokens; with the real EOS it stops where the oracle does."""
    ids = [0] + list(range(30, 50))
    p = DecodeParameters(max_new_tokens=30)
    full = tiny_engine.generate(ids, None, None, None, p, ignore_eos=True)
    assert len(full) == 30
    stop = tiny_engine.generate(ids, None, None, None, p)
    ref, _ = tiny_oracle.generate(ids, [0] * len(ids), None, 30, eos_token_id=1, no_repeat_ngram_size=20)
    assert stop == ref


def test_mask_mismatch_is_einval(tiny_engine):
    tok = SyntheticTokenizer(512)
    page = Page(_img(1, 300, 300), TINY_VS)
    ids, mask = _prompt(tok, page)
    mask = list(mask)
    mask[-1] = 1  # one extra <image> slot (the last text token)
    with pytest.raises(DsocrError) as e:
        tiny_engine.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=4))
    assert e.value.status == 1 and "mismatch" in e.value.message


def test_safetensors_checkpoint_matches_synthetic(tiny_engine, tmp_path):
    """Loading a real .safetensors file (bf16, the reference's checkpoint format) gives the same engine."""
    from safetensors.numpy import save_file
    from oracle.weights import synth_bf16, synthetic_has
    import oracle.config as oc
    cfg = json.load(open(TINY))
    from oracle.specs import tensor_names
    names = tensor_names(cfg)
    tensors = {}
    for n, shape in names.items():
        if not synthetic_has(n):
            continue
        tensors[n] = synth_bf16(n, SEED, int(np.prod(shape))).reshape(shape)
    # safetensors.numpy has no bf16 dtype: write raw bits with a BF16 header ourselves
    path = tmp_path / "model.safetensors"
    _write_bf16_safetensors(path, tensors)
    eng = load_model(ModelLoadArgs(config_path=TINY, weights_path=str(path), dtype="f16"))
    tok = SyntheticTokenizer(512)
    page = Page(_img(77, 300, 420), TINY_VS)
    ids, mask = _prompt(tok, page)
    p = DecodeParameters(max_new_tokens=16)
    assert eng.generate(ids, mask, page, None, p) == tiny_engine.generate(ids, mask, page, None, p)
    eng.close()
    del save_file, oc


def _write_bf16_safetensors(path, tensors):
    import struct
    header, off, blobs = {}, 0, []
    for n, a in tensors.items():
        b = np.ascontiguousarray(a, np.uint16).tobytes()
        header[n] = {"dtype": "BF16", "shape": list(a.shape), "data_offsets": [off, off + len(b)]}
        blobs.append(b)
        off += len(b)
    h = json.dumps(header).encode()
    h += b" " * ((8 - len(h) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(h)))
        f.write(h)
        for b in blobs:
            f.write(b)


# ------------------------------------------------------------------ full-size DeepSeek-OCR
@pytest.fixture(scope="module")
def full_engine(gpu):
    eng = load_model(ModelLoadArgs(config_path=FULL, synthetic_seed=SEED, dtype="f16"))
    yield eng
    eng.close()


def test_full_decoder_parity(full_engine):
    """Full-size decoder (12 layers, 64 experts, vocab 129280): host image rows, 706-token prompt."""
    cfg = json.load(open(FULL))
    orc = OracleModel(cfg, Weights(seed=SEED, dtype="f16"))
    tok = SyntheticTokenizer(129280)
    rng = np.random.default_rng(3)
    rows = (rng.standard_normal((693, 1280)) * 0.05).astype(np.float32)
    ids, mask = build_prompt_tokens(tok, "<image>\n<|grounding|>Convert the document to markdown.", [693])
    got = full_engine.generate(ids, mask, None, rows, DecodeParameters(max_new_tokens=6), ignore_eos=True)
    ref, logs = orc.generate(ids, mask, rows, 6, eos_token_id=None, record_logits=True)
    assert got == ref, (got, ref)


def test_full_page_vision_parity(full_engine):
    """Full-size SAM + CLIP + projector on one synthetic 1024x1024 page (693 rows)."""
    cfg = json.load(open(FULL))
    orc = OracleModel(cfg, Weights(seed=SEED, dtype="f16"))
    img = synthetic_page(0)
    page = Page(img, VisionSettings())
    got = full_engine.image_embeddings([page])[0]
    ref, _ = orc.image_embeddings(img)
    assert got.shape == ref.shape == (693, 1280)
    err = np.max(np.abs(got - ref))
    assert err < 1e-3 * max(1.0, np.max(np.abs(ref))), err


def test_tiny_device_resident_page_equals_host(tiny_engine):
    """dsocr_page_to_device: HBM-resident pixels (device-to-device gather) give the same ids."""
    tok = SyntheticTokenizer(512)
    p = DecodeParameters(max_new_tokens=16)
    reqs_h, reqs_d = [], []
    for i, hw in enumerate([(300, 420), (220, 180)]):
        img = _img(300 + i, *hw)
        ph, pd = Page(img, TINY_VS), Page(img, TINY_VS).to_device(tiny_engine)
        ids, mask = _prompt(tok, ph)
        reqs_h.append((ids, mask, ph, None))
        reqs_d.append((ids, mask, pd, None))
    assert tiny_engine.generate_batch(reqs_d, p) == tiny_engine.generate_batch(reqs_h, p)


def test_full_screened_selection_equals_exact(full_engine, monkeypatch):
    """Screened greedy selection (int8 lm_head intervals + exact rescoring, lmhead.hip) picks the
    same tokens as the exact bf16 lm_head path on a full-size page with the 20-gram ban on."""
    tok = SyntheticTokenizer(129280)
    page = Page(synthetic_page(5), VisionSettings())
    ids, mask = build_prompt_tokens(tok, "<image>\n<|grounding|>Convert the document to markdown.", [page.n_image_tokens])
    p = DecodeParameters(max_new_tokens=48)
    monkeypatch.setenv("DSOCR_SCREEN", "1")
    screened = full_engine.generate(ids, mask, page, None, p, ignore_eos=True)
    monkeypatch.setenv("DSOCR_SCREEN", "0")
    exact = full_engine.generate(ids, mask, page, None, p, ignore_eos=True)
    assert screened == exact, (screened, exact)


def test_full_spans_do_not_change_ids(full_engine):
    """In-context launch spans (dsocr_engine_set_spans: 1 = wave spans stamped by every gate/up, down and
    attention wave, 2 = HIP events around those launches inside the replayed step graph, 4 = chain spans: five
    launches per layer stamped into their own regions, one fold per step) record without changing what is
    decoded: ids equal with spans off and in every mode, records present with the stated dims, and
    profile_decode (whose replays rewrite the last K/V slot) leaves a following generate unchanged."""
    tok = SyntheticTokenizer(129280)
    page = Page(synthetic_page(2), VisionSettings())
    ids, mask = build_prompt_tokens(tok, "<image>\n<|grounding|>Convert the document to markdown.", [page.n_image_tokens])
    n = 24
    p = DecodeParameters(max_new_tokens=n)
    full_engine.set_spans(0)
    ref = full_engine.generate(ids, mask, page, None, p, ignore_eos=True)
    layers = json.load(open(FULL))["language_config"]["num_hidden_layers"]
    try:
        for mode in (1, 2, 4):
            full_engine.set_spans(mode)
            got = full_engine.generate(ids, mask, page, None, p, ignore_eos=True)
            assert got == ref, (mode, got, ref)
            sp = full_engine.spans()
            kinds = ("moe_gateup", "moe_down", "attention") + (("o_proj", "router") if mode == 4 else ())
            assert set(sp) == set(kinds), sp.keys()
            steps = n + 1 if mode == 4 else n
            for kind in kinds:
                a = sp[kind]
                assert a.shape == (layers, steps, 5), (kind, a.shape)
                moe = kind in ("moe_gateup", "moe_down", "router")
                rows = a[1:, 1:n] if moe else a[:, 1:n]     # layer 0 is dense: no MoE launches
                if mode in (1, 4):
                    assert np.all(rows[..., 1] > rows[..., 0]), kind   # exit after entry in every step
                else:
                    assert np.all(rows[..., 4] > 0), kind              # event duration in every step
                if moe and mode == 1:
                    assert np.all((rows[..., 2] >= 6) & (rows[..., 2] <= 64)), kind  # distinct experts
            if mode == 4:  # one chain: every launch starts after its predecessor's last wave left
                for k, pk in (("moe_gateup", "router"), ("moe_down", "moe_gateup"), ("o_proj", "attention"),
                              ("router", "o_proj")):
                    assert np.all(sp[k][1:, 1:n, 0] > sp[pk][1:, 1:n, 1]), (k, pk)
    finally:
        full_engine.set_spans(0)
    full_engine.profile_decode(2)
    assert full_engine.generate(ids, mask, page, None, p, ignore_eos=True) == ref


def test_tiny_generate_without_cache(tiny_engine, tiny_oracle):
    """use_cache = false (generate_without_cache, model/mod.rs:2051-2283): every step re-runs the whole
    forward on prompt + generated tokens; ids equal the oracle's no-cache restatement and the cached path."""
    img = _img(21, 300, 420)
    tok = SyntheticTokenizer(512)
    page = Page(img, TINY_VS)
    ids, mask = _prompt(tok, page)
    emb, _ = tiny_oracle.image_embeddings(img, 256, 128, True)
    seen = []
    got = tiny_engine.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=12, use_cache=False),
                               stream=lambda n, toks: seen.append(list(toks)))
    ref = tiny_oracle.generate_without_cache(ids, mask, emb, 12, eos_token_id=1, no_repeat_ngram_size=20)
    assert got == ref
    assert got == tiny_engine.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=12))
    assert [len(s) for s in seen] == list(range(1, len(got) + 1)) and seen[-1] == got
    # batch of two pages without cache == per-page
    page2 = Page(_img(22, 256, 256), TINY_VS)
    ids2, mask2 = _prompt(tok, page2)
    p = DecodeParameters(max_new_tokens=10, use_cache=False)
    bat = tiny_engine.generate_batch([(ids, mask, page, None), (ids2, mask2, page2, None)], p)
    assert bat == [tiny_engine.generate(ids, mask, page, None, p), tiny_engine.generate(ids2, mask2, page2, None, p)]


def test_tiny_stream_callback_every_token(tiny_engine):
    """The stream callback runs after every token, the first one included (model/mod.rs:1980-1982)."""
    ids = [0] + list(range(30, 50))
    seen = []
    got = tiny_engine.generate(ids, None, None, None, DecodeParameters(max_new_tokens=6),
                               stream=lambda n, toks: seen.append((n, list(toks))), ignore_eos=True)
    assert [n for n, _ in seen] == list(range(1, 7)) and seen[-1][1] == got
