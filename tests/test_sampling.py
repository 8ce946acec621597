"""Stochastic token selection (select_token_id's do_sample branch, core/src/sampling.rs:67-86).

CPU: the oracle's ChaCha block function against the RFC 7539 A.1 keystream vectors (the only
published vectors for this path; rand's seed expansion / float sampling are restated from the
crates' algorithms — parity unpinned vs the Rust crates, see oracle/sampling.py), plus the
documented behaviours of apply_top_k / apply_top_p / WeightedIndex on hand-checked cases.
GPU: `dsocr_k_sample_stoch` and the engine's sampled generate against the oracle — same ids
for the same seed (successive draws carry the RNG state), batch == single.
"""
import json
import math
import os
import struct

import numpy as np
import pytest

from oracle.decoder import select_token_id
from oracle.sampling import (MAX_RAND, StdRng, WeightedIndex, apply_top_k, apply_top_p, chacha_block,
                             pcg32_seed_bytes, uniform_f64_new)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")


def test_chacha20_rfc7539_vectors():
    b0 = struct.pack("<16I", *chacha_block([0] * 8, 0, 0, 20)).hex()
    b1 = struct.pack("<16I", *chacha_block([0] * 8, 1, 0, 20)).hex()
    assert b0 == ("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                  "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")
    assert b1 == ("9f07e7be5551387a98ba977c732d080dcb0f29a048e3656912c6533e32ee7aed"
                  "29b721769ce64e43d57133b074d839d531ed1f28510afb45ace10a1f4b794d6f")


def test_stdrng_buffering():
    # four blocks per refill, consecutive counters; u64 = low word first; an odd index straddles
    r = StdRng(7)
    key = list(struct.unpack("<8I", pcg32_seed_bytes(7)))
    words = sum((chacha_block(key, c, 0, 12) for c in range(8)), [])
    assert [r.next_u64() for _ in range(32)] == [words[2 * i] | (words[2 * i + 1] << 32) for i in range(32)]
    r2 = StdRng(7)
    for _ in range(63):
        r2.next_u32()
    assert r2.next_u64() == words[63] | (words[64] << 32)
    assert pcg32_seed_bytes(0) != pcg32_seed_bytes(1) and len(pcg32_seed_bytes(5)) == 32


def test_uniform_and_weighted_index():
    for total in (1.0, 3.0, 0.7, 1e-300, 12345.678):
        low, scale = uniform_f64_new(0.0, total)
        assert scale * MAX_RAND + low < total and scale <= total
    w = WeightedIndex([0.0, 2.0, 0.0, 1.0])
    assert w.cum == [0.0, 2.0, 2.0] and w.total == 3.0
    with pytest.raises(ValueError):
        WeightedIndex([0.0, 0.0])
    r = StdRng(3)
    counts = np.bincount([w.sample(r) for _ in range(3000)], minlength=4)
    assert counts[0] == 0 and counts[2] == 0 and 1800 < counts[1] < 2200


def test_top_k_stable_ties_and_top_p():
    lg = [1.0, 3.0, 3.0, -math.inf, 2.0, 3.0]
    apply_top_k(lg, 2)  # ties keep the lower index first (stable sort_by)
    assert [math.isfinite(v) for v in lg] == [False, True, True, False, False, False]
    lg = [math.log(p) for p in (0.1, 0.5, 0.25, 0.15)]
    apply_top_p(lg, 0.7)  # sorted shares .5, .25 -> .75 > .7: keep two
    assert [math.isfinite(v) for v in lg] == [False, True, True, False]
    lg = [0.0, 1.0]
    apply_top_p(lg, 0.0)  # the first share already exceeds 0: keep one
    assert [math.isfinite(v) for v in lg] == [False, True]
    lg = [0.0, 1.0]
    apply_top_p(lg, 1.0)  # outside [0, 1): no-op
    assert all(math.isfinite(v) for v in lg)


def test_select_token_id_sampling_fallbacks():
    lg = np.array([0.0, 5.0, 1.0], np.float32)
    # temperature 0 with do_sample: greedy (sampling.rs:67)
    assert select_token_id(lg, [], do_sample=True, temperature=0.0, rng=StdRng(1)) == 1
    # all candidates banned -> the ban is dropped, sampling proceeds over all three
    ctx = [1, 1, 1, 1]
    toks = {select_token_id(lg, ctx, 1.0, 2, do_sample=True, temperature=5.0, rng=StdRng(s)) for s in range(40)}
    assert toks <= {0, 1, 2} and len(toks) >= 2


# ---------------------------------------------------------------- GPU
def _oracle_draws(logits, ctx, pen, ngram, T, k, p, seed, draws):
    rng = StdRng(seed)
    return [select_token_id(logits, ctx, pen, ngram if ngram > 1 else None, do_sample=True, temperature=T,
                            top_k=k if k else None, top_p=p if 0.0 <= p < 1.0 else None, rng=rng)
            for _ in range(draws)]


@pytest.mark.gpu
@pytest.mark.parametrize("V,T,k,p,ngram,pen", [
    (5000, 0.7, 0, -1.0, 0, 1.0),     # temperature only: every finite logit is a candidate
    (5000, 1.0, 40, -1.0, 3, 1.0),    # top-k with the n-gram ban
    (5000, 0.8, 0, 0.9, 0, 1.3),      # top-p with the repetition penalty
    (5000, 1.2, 50, 0.5, 20, 1.0),    # both
    (129280, 0.6, 0, 0.95, 20, 1.0),  # full vocabulary, top-p
    (129280, 0.7, 0, -1.0, 0, 1.0),   # full vocabulary, temperature only: the early-stop fold crosses many tiles
    (129280, 1.1, 64, -1.0, 20, 1.0), # full vocabulary, top-k only (radix select of the k-th key)
])
def test_sample_stoch_matches_oracle(gpu, V, T, k, p, ngram, pen):
    from dsocr._lib import check, lib
    from _dev import Dev
    rng = np.random.default_rng(V + k)
    B, cap, draws = 2, 64, (12 if V > 100000 else 6)
    logits = (rng.standard_normal((B, V)) * 3).astype(np.float32)
    logits[0, 5] = -np.inf
    logits[1, 7] = np.nan
    logits[1, 100:110] = logits[1, 99]  # ties
    ctx = np.zeros((B, cap), np.int32)
    lens = np.array([40, 12], np.int32)
    for b in range(B):
        seq = np.tile(rng.integers(0, 60, 4), 20)[: lens[b]]
        ctx[b, : lens[b]] = seq
    dl, dc, dn = Dev(logits), Dev(ctx), Dev(lens)
    dt = Dev.zeros(draws * B, np.int32)
    seed = 1234 + V
    check(lib().dsocr_k_sample_stoch(B, V, dl.ptr, dc.ptr, cap, dn.ptr, ngram, pen, T, k, p, seed, draws, dt.ptr))
    got = dt.get().reshape(draws, B)
    for b in range(B):
        ref = _oracle_draws(logits[b], ctx[b, : lens[b]].tolist(), pen, ngram, T, k, p, seed, draws)
        assert got[:, b].tolist() == ref, (b, got[:, b].tolist(), ref)


@pytest.mark.gpu
def test_engine_sampled_generate_matches_oracle(gpu):
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import SyntheticTokenizer
    from oracle.model import OracleModel
    from oracle.weights import Weights
    vs = VisionSettings(256, 128, True)
    img = np.random.default_rng(11).integers(0, 256, (300, 420, 3), dtype=np.uint8)
    eng = load_model(ModelLoadArgs(config_path=TINY, synthetic_seed=7, dtype="f16"))
    try:
        page = Page(img, vs)
        ids, mask = build_prompt_tokens(SyntheticTokenizer(512), "<image>\nConvert the document to markdown.",
                                        [page.n_image_tokens])
        orc = OracleModel(json.load(open(TINY)), Weights(seed=7, dtype="f16"))
        emb, _ = orc.image_embeddings(img, 256, 128, True)
        for T, k, p, seed in [(0.9, None, 0.95, 5), (1.5, 20, 1.0, 6)]:
            prm = DecodeParameters(max_new_tokens=24, do_sample=True, temperature=T, top_k=k, top_p=p, seed=seed)
            got = eng.generate(ids, mask, page, None, prm)
            ref, _ = orc.generate(ids, mask, emb, 24, eos_token_id=1, do_sample=True, temperature=T, top_k=k,
                                  top_p=p if p < 1.0 else None, seed=seed)
            assert got == ref, (T, k, p, got, ref)
            # every page of a batch starts from init_rng(seed): batch == single
            bat = eng.generate_batch([(ids, mask, page, None), (ids, mask, page, None)], prm)
            assert bat == [got, got]
        # greedy when temperature is 0 even with do_sample (sampling.rs:67)
        g0 = eng.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=8))
        g1 = eng.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=8, do_sample=True, temperature=0.0))
        assert g0 == g1
    finally:
        eng.close()
