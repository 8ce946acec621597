"""Dev tool: per-kernel decode timings (HIP events on the engine stream) after one page.

    python tools/prof_decode.py [--max-new 256] [--iters 20] [--pages 1]

Prints one JSON line per kernel: avg_us, algorithmic bytes, GB/s, plus the whole-layer-stack
graph replay (layers_step) and the decode.iterative ms/token of the generate() it followed.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "deepseek-ocr.rs_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-new", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pages", type=int, default=1)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import dsocr
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16", device=0))
    tok = SyntheticTokenizer(eng.vocab)
    vs = VisionSettings(1024, 640, True)
    reqs = []
    for i in range(a.pages):
        page = Page(synthetic_page(i), vs).to_device(eng)
        ids, mask = build_prompt_tokens(tok, BENCH_PROMPT, [page.n_image_tokens])
        reqs.append((ids, mask, page, None))
    params = DecodeParameters(max_new_tokens=a.max_new)
    eng.generate_batch(reqs, params, ignore_eos=True)
    eng.generate_batch(reqs, params, ignore_eos=True)
    t = eng.last_timings()
    prof = eng.profile_decode(a.iters)
    out = {"tag": a.tag, "pages": a.pages, "kv_len": prof["kv_len"], "experts_touched": prof["experts_touched"],
           "vision_ms": round(t["vision_compute_ms"], 2), "prefill_ms": round(t["decode_prefill_ms"], 2),
           "iter_us_per_step": round(1e3 * t["decode_iterative_ms"] / max(1, a.max_new - 1), 1)}
    for k, v in prof.items():
        if isinstance(v, dict) and v["avg_us"] > 0:
            out[k] = {"us": round(v["avg_us"], 2), "MB": round(v["bytes"] / 1e6, 2),
                      "GB/s": round(v["bytes"] / (v["avg_us"] * 1e-6) / 1e9, 0)}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
