#!/usr/bin/env python3
"""Same-process A/B of decode kernel variants under a rocprofv3 kernel trace.

One engine, one prepared bench page; every round generates the page once per variant (a variant = a set
of environment switches the engine reads when it captures the step graph).  Run it under
    ROC_AQL_QUEUE_SIZE=131072 rocprofv3 --kernel-trace --stats -d DIR -o g --output-format csv -- \
        python tools/ab_trace.py --tokens 64 --rounds 3 --variant base: --variant x:DSOCR_FOO=1
and read the per-variant kernel durations with tools/ab_stats.py DIR/g_kernel_trace.csv gpurun_out/ab_order.json.
Without the profiler it still prints each generate's decode ms (host clock, whole generate).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))


def parse_variant(v):
    name, _, rest = v.partition(":")
    env = {}
    for kv in filter(None, rest.split(",")):
        k, _, val = kv.partition("=")
        env[k] = val
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pages", type=int, default=1)
    ap.add_argument("--text-pages", action="store_true")
    ap.add_argument("--variant", action="append", required=True, help="name:ENV=VAL,ENV2=VAL")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab_order.json"))
    ap.add_argument("--lib", default=None, help="another libdsocr.so build (A/B of two kernel versions)")
    args = ap.parse_args()
    import dsocr
    if args.lib:
        import dsocr._lib
        dsocr._lib.LIB_PATH = os.path.abspath(args.lib)
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page, text_page_prompt
    variants = [parse_variant(v) for v in args.variant]
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16", device=0))
    tok = SyntheticTokenizer(eng.vocab)
    vs = VisionSettings(1024, 640, True)
    reqs = []
    for idx in range(args.pages):
        if args.text_pages:
            reqs.append((text_page_prompt(idx, vocab=eng.vocab), None, None, None))
        else:
            page = Page(synthetic_page(idx), vs, eng)
            ids, mask = build_prompt_tokens(tok, BENCH_PROMPT, [page.n_image_tokens])
            reqs.append((ids, mask, page, None))
    params = DecodeParameters(max_new_tokens=args.tokens)
    base_env = {k: os.environ.get(k) for _, e in variants for k in e}
    order, ref = [], None
    eng.generate_batch(reqs, params, ignore_eos=True)  # warm-up (not counted: index -1 in the order file)
    order.append({"variant": "_warmup"})
    for r in range(args.rounds):
        for name, env in variants:
            for k, v in base_env.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            os.environ.update(env)
            t = time.perf_counter()
            out = eng.generate_batch(reqs, params, ignore_eos=True)
            dt = time.perf_counter() - t
            tm = eng.last_timings()
            same = ref is None or out == ref
            ref = ref or out
            order.append({"variant": name, "round": r, "wall_ms": dt * 1e3,
                          "decode_ms": tm["decode_iterative_ms"], "same_ids": same})
            print(f"[ab] round {r} {name:12s} decode {tm['decode_iterative_ms']:8.2f} ms  ids {'same' if same else 'DIFFER'}",
                  flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump({"tokens": args.tokens, "pages": args.pages, "order": order}, open(args.out, "w"), indent=1)
    eng.close()
    if not all(o.get("same_ids", True) for o in order):
        sys.exit(1)


if __name__ == "__main__":
    main()
