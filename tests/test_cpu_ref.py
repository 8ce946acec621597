"""The C++ / OpenMP CPU restatement (oracle/cpu_ref.cpp, bench.py's cpu_baseline) against the numpy oracle
(oracle/decoder.py: transformer/block.rs, model/mod.rs:1870-2048) on the tiny config: the same greedy ids
(prefill with injected image rows, KV-cached decode, the 20-gram ban)."""
import json
import os

import numpy as np
import pytest

from oracle import cpu_ref
from oracle.model import OracleModel
from oracle.weights import Weights

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")


@pytest.mark.parametrize("seed,P,n_img,max_new,ngram", [(3, 40, 12, 24, 20), (5, 17, 0, 30, 3), (9, 64, 30, 16, 20)])
def test_cpu_ref_matches_oracle_tiny(seed, P, n_img, max_new, ngram):
    cfg = json.load(open(TINY))
    rng = np.random.default_rng(seed)
    ids = rng.integers(2, 500, P).astype(np.int64)
    mask = np.zeros(P, np.uint8)
    if n_img:
        mask[1:1 + n_img] = 1
    rows = (rng.standard_normal((n_img, 128)) * 0.5).astype(np.float32) if n_img else None
    orc = OracleModel(cfg, Weights(seed=seed, dtype="f16"))
    ref, _ = orc.generate(ids.tolist(), mask.tolist(), rows, max_new, eos_token_id=None, no_repeat_ngram_size=ngram)
    cr = cpu_ref.CpuRef(cfg, Weights(seed=seed, dtype="f16"), threads=4)
    try:
        got, ms = cr.generate(ids, mask, rows, max_new, ngram=ngram)
    finally:
        cr.close()
    assert got == ref, (got, ref)
    assert ms["prefill_ms"] > 0 and ms["decode_ms"] > 0


@pytest.mark.parametrize("seed", [7, 11])
def test_cpu_vision_matches_oracle_tiny(seed):
    """The C++ vision tower (cv_features: SAM blocks with windowed / global attention and the decomposed rel-pos
    bias, neck, downsample, CLIP, projector) against the numpy oracle (oracle/vision.py) on a crop-mode page:
    the formatted image rows within 1e-4 relative (f32 summation order only)."""
    cfg = json.load(open(TINY))
    img = np.random.default_rng(seed).integers(0, 256, (300, 420, 3), dtype=np.uint8)
    orc = OracleModel(cfg, Weights(seed=seed, dtype="f16"))
    ref, crop = orc.image_embeddings(img, 256, 128, True)
    cv = cpu_ref.CpuVision(cfg, Weights(seed=seed, dtype="f16"), threads=4, sizes=(256, 128))
    got, crop2 = cv.embeddings(img, 256, 128, True)
    assert crop == crop2 and got.shape == ref.shape
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-4
    assert cv.last_ms["sam_ms"] > 0 and cv.last_ms["clip_ms"] > 0
