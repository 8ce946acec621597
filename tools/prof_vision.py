"""Dev tool: the vision tower + prefill of one 1024 px page, repeated, for a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o pv -- python tools/prof_vision.py [--reps 3]

Prints the engine's own stage timings (vision_compute_ms, decode_prefill_ms) per repetition; the
trace gives each launch's duration and grid (tools/kstats.py summarises it).
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pages", type=int, default=1)
    ap.add_argument("--lib", default=None, help="another libdsocr.so build (A/B of two kernel versions)")
    ap.add_argument("--variant", action="append", help="name:ENV=VAL,ENV2=VAL (same-process A/B, alternating)")
    a = ap.parse_args()
    import dsocr
    if a.lib:
        import dsocr._lib
        dsocr._lib.LIB_PATH = os.path.abspath(a.lib)
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16", device=0))
    tok = SyntheticTokenizer(eng.vocab)
    vs = VisionSettings(1024, 640, True)
    reqs = []
    for i in range(a.pages):
        page = Page(synthetic_page(i), vs, eng)
        ids, mask = build_prompt_tokens(tok, BENCH_PROMPT, [page.n_image_tokens])
        reqs.append((ids, mask, page, None))
    params = DecodeParameters(max_new_tokens=2)
    variants = [v.partition(":") for v in (a.variant or [":"])]
    eng.generate_batch(reqs, params, ignore_eos=True)  # warm-up
    for r in range(a.reps):
        for name, _, env in variants:  # same-process A/B: each variant's environment set before its pass
            for k, v in (kv.partition("=")[::2] for kv in filter(None, env.split(","))):
                os.environ[k] = v
            eng.generate_batch(reqs, params, ignore_eos=True)
            t = eng.last_timings()
            print(json.dumps({"rep": r, "variant": name, "vision_ms": round(t["vision_compute_ms"], 2),
                              "prefill_ms": round(t["decode_prefill_ms"], 2)}), flush=True)
            for k in (kv.partition("=")[0] for kv in filter(None, env.split(","))):
                os.environ.pop(k, None)
    eng.close()


if __name__ == "__main__":
    main()
