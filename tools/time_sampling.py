"""Decode-step cost of the GPU sampler (full DeepSeek-OCR config, synthetic weights, one page):
greedy vs do_sample with temperature only / top-k / top-p.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))
import dsocr  # noqa: E402
from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model  # noqa: E402
from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page  # noqa: E402

eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16"))
page = Page(synthetic_page(0), VisionSettings(), eng)
ids, mask = build_prompt_tokens(SyntheticTokenizer(eng.vocab), BENCH_PROMPT, [page.n_image_tokens])
out = {}
for name, kw in [("greedy", {}), ("temperature", dict(do_sample=True, temperature=0.8, seed=1)),
                 ("top_k50", dict(do_sample=True, temperature=0.8, top_k=50, seed=1)),
                 ("top_p0.9", dict(do_sample=True, temperature=0.8, top_p=0.9, seed=1))]:
    prm = DecodeParameters(max_new_tokens=256, **kw)
    eng.generate(ids, mask, page, None, prm, ignore_eos=True)
    t = eng.last_timings()
    out[name] = round(t["decode_iterative_ms"] * 1e3 / max(t["decode_steps"], 1), 1)
print(json.dumps({"decode_us_per_step": out}))
eng.close()
