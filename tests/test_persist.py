"""The one-page persistent decode step (decode_persist.hip): every decoder layer of a step as ONE launch.

At the bench configuration (BASELINE configs[1]: full-size synthetic DeepSeek-OCR, one 1024^2 page, 706-token
prompt, greedy 512 tokens) the persistent launch must give:

* the oracle's greedy ids over all 512 steps and the traced logits within LOGIT_TOL at the oracle's top-8 and probe
  indices (the committed fixture of tests/golden/make_full_golden.py, oracle/decoder.py layer() per step:
  TransformerBlock::forward_internal, block.rs:124-191);
* the same ids as the per-layer launch chain (DSOCR_PERSIST=0) and logits within LOGIT_TOL of it (only the f32
  summation orders differ: split-K down projection, per-dim attention merge);
* its diagnostics (dsocr_engine_persist_info): one timed launch per decode step, phase clocks in order.
"""
import os

import numpy as np
import pytest

from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
from dsocr.synth import SyntheticTokenizer

from test_full_parity import FULL, LOGIT_TOL, PROMPT, check_stream, fixture, page_image

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine(gpu):
    old = os.environ.get("DSOCR_PERSIST")
    os.environ["DSOCR_PERSIST"] = "1"  # the persistent step is opt-in (DSOCR_PERSIST=1)
    eng = load_model(ModelLoadArgs(config_path=FULL, synthetic_seed=7, dtype="f16"))
    yield eng
    eng.close()
    if old is None:
        os.environ.pop("DSOCR_PERSIST", None)
    else:
        os.environ["DSOCR_PERSIST"] = old


@pytest.fixture(scope="module")
def bench_page(engine):
    fx = fixture("synthetic0")
    page = Page(page_image("synthetic0"), VisionSettings(), engine)
    ids, mask = build_prompt_tokens(SyntheticTokenizer(engine.vocab), PROMPT, [page.n_image_tokens])
    assert ids == fx["prompt_ids"].tolist()
    return fx, page, ids, mask


def _trace(engine, page, ids, mask, n, persist):
    old = os.environ.get("DSOCR_PERSIST")
    os.environ["DSOCR_PERSIST"] = "1" if persist else "0"
    try:
        outs, logits = engine.generate_trace([(ids, mask, page, None)], DecodeParameters(max_new_tokens=n),
                                             ignore_eos=True)
    finally:
        os.environ["DSOCR_PERSIST"] = old if old is not None else "1"
    return outs[0], logits[0]


def test_persist_page_512_tokens_matches_oracle(engine, bench_page):
    fx, page, ids, mask = bench_page
    n = int(fx["max_new"])
    got, logits = _trace(engine, page, ids, mask, n, True)
    assert engine.persist_info()["used"], "the persistent decode did not run at the bench shape"
    check_stream("synthetic0/persistent", fx, got, logits, n)


def test_persist_equals_launch_chain(engine, bench_page):
    _, page, ids, mask = bench_page
    n = 64
    a, la = _trace(engine, page, ids, mask, n, True)
    assert engine.persist_info()["used"]
    b, lb = _trace(engine, page, ids, mask, n, False)
    assert not engine.persist_info()["used"]
    assert a == b
    d = float(np.abs(la[:n] - lb[:n]).max())
    print(f"persistent vs launch chain: max |logit diff| over {n} steps = {d:.3g}")
    assert d <= LOGIT_TOL


def test_persist_timed_launches_and_phase_clocks(engine, bench_page):
    _, page, ids, mask = bench_page
    n = 24
    ref = engine.generate_batch([(ids, mask, page, None)], DecodeParameters(max_new_tokens=n), ignore_eos=True)[0]
    engine.set_persist_stamps(1)
    got = engine.generate_batch([(ids, mask, page, None)], DecodeParameters(max_new_tokens=n), ignore_eos=True)[0]
    info = engine.persist_info(layers=engine.num_layers)
    assert got == ref
    assert info["used"] and len(info["launch_us"]) == n - 1
    assert np.all(info["launch_us"] > 0) and np.all(np.isfinite(info["launch_us"]))
    st = info["stamps"][: n - 1].astype(np.int64)  # [steps][256][layers][9]
    assert np.all(st > 0)
    assert np.all(np.diff(st, axis=-1) >= 0), "phase clocks out of order inside a layer"
    # a layer starts after the previous one's reduction on the same workgroup
    assert np.all(st[:, :, 1:, 0] >= st[:, :, :-1, 8])
    print(f"persistent launch: median {np.median(info['launch_us']):.1f} us over {n - 1} steps")
