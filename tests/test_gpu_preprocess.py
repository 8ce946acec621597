"""Page preprocessing on the GPU: dsocr_prepare_page_device must produce the
host path's pixels (dsocr_prepare_page, itself pinned against the oracle and Pillow in
test_host_cpu.py / test_golden.py) bit for bit — same tile grid, same f32 CHW values — for
upscales, downscales, identity sizes, pages needing no tiles and crop_mode off; and a page prepared
on the GPU generates the same ids."""
import os

import numpy as np
import pytest

from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
from dsocr.synth import SyntheticTokenizer, synthetic_page

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")


@pytest.fixture(scope="module")
def engine(gpu):
    eng = load_model(ModelLoadArgs(config_path=TINY, synthetic_seed=7, dtype="f16"))
    yield eng
    eng.close()


SIZES = [(1024, 1024), (420, 300), (300, 2000), (90, 100), (200, 700), (2000, 3000), (640, 640), (100, 641), (1, 1)]
SETTINGS = [VisionSettings(1024, 640, True), VisionSettings(256, 128, True), VisionSettings(1024, 640, False)]


@pytest.mark.parametrize("vs", SETTINGS, ids=["1024-640", "256-128", "nocrop"])
@pytest.mark.parametrize("hw", SIZES, ids=[f"{h}x{w}" for h, w in SIZES])
def test_device_pixels_equal_host(engine, hw, vs):
    img = np.random.default_rng(hw[0] * 7 + hw[1]).integers(0, 256, (hw[0], hw[1], 3), dtype=np.uint8)
    host = Page(img, vs)
    dev = Page(img, vs, engine)
    assert dev.crop_shape == host.crop_shape and dev.n_tiles == host.n_tiles
    assert dev.n_image_tokens == host.n_image_tokens
    hg, ht = host.pixels()
    dg, dt = dev.pixels()
    assert np.array_equal(hg.view(np.uint32), dg.view(np.uint32))
    if ht is None:
        assert dt is None
    else:
        assert np.array_equal(ht.view(np.uint32), dt.view(np.uint32))


def test_document_page_equal_host(engine):
    img = synthetic_page(0)
    vs = VisionSettings(1024, 640, True)
    hg, ht = Page(img, vs).pixels()
    dg, dt = Page(img, vs, engine).pixels()
    assert np.array_equal(hg, dg) and np.array_equal(ht, dt)


def test_generate_from_device_page(engine):
    img = np.random.default_rng(3).integers(0, 256, (300, 420, 3), dtype=np.uint8)
    vs = VisionSettings(256, 128, True)
    tok = SyntheticTokenizer(512)
    host, dev = Page(img, vs), Page(img, vs, engine)
    ids, mask = build_prompt_tokens(tok, "<image>\nConvert the document to markdown.", [host.n_image_tokens])
    p = DecodeParameters(max_new_tokens=16)
    assert engine.generate(ids, mask, dev, None, p) == engine.generate(ids, mask, host, None, p)
    assert np.array_equal(engine.image_embeddings([dev])[0], engine.image_embeddings([host])[0])
