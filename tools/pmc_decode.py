#!/usr/bin/env python3
"""Decode workload for the rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) with the routing of every MoE launch.

One batch of the bench's workload (1 page, 8 image pages or 8 text pages) is generated twice: first with
in-kernel wave spans on (each MoE gate/up and down launch records the distinct experts it streamed), then
plainly.  The routing is deterministic (same batch, same ids: checked), so the second generate's MoE launches,
the LAST ones of each MoE kernel in the PMC pass's dispatch order, are priced from the first one's records:
the dry step before the decode graph (it repeats step 1's routing), then steps 1 .. N-1, layers in order.
Writes {kind: [distinct experts per launch in dispatch order]} for tools/pmc_summary.py --routing.

    DSOCR_NO_GRAPH=1 rocprofv3 --pmc FETCH_SIZE -d DIR -o pmc --output-format csv -- \
        python tools/pmc_decode.py --pages 8 --text-pages --tokens 16 --out gpurun_out/routing_b8.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", type=int, default=1)
    ap.add_argument("--text-pages", action="store_true")
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import dsocr
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page, text_page_prompt
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16", device=0))
    tok = SyntheticTokenizer(eng.vocab)
    vs = VisionSettings(1024, 640, True)
    reqs = []
    for idx in range(args.pages):  # bench.py's first batch (page indices 0 .. pages - 1)
        if args.text_pages:
            reqs.append((text_page_prompt(idx, vocab=eng.vocab), None, None, None))
        else:
            page = Page(synthetic_page(idx), vs, eng)
            ids, mask = build_prompt_tokens(tok, BENCH_PROMPT, [page.n_image_tokens])
            reqs.append((ids, mask, page, None))
    params = DecodeParameters(max_new_tokens=args.tokens)
    eng.set_spans(eng.SPAN_WAVES)
    ids_a = eng.generate_batch(reqs, params, ignore_eos=True)
    spans = eng.spans()
    eng.set_spans(0)
    ids_b = eng.generate_batch(reqs, params, ignore_eos=True)
    if ids_a != ids_b:
        raise SystemExit("the two generates emitted different ids: routing not reproducible")
    out = {"pages": args.pages, "text_pages": args.text_pages, "tokens": args.tokens}
    for kind in ("moe_gateup", "moe_down"):
        arr = spans[kind]  # [layers][steps][5]
        layers = [l for l in range(arr.shape[0]) if arr[l, 1:, 2].any()]
        seq = [int(arr[l, 1, 2]) for l in layers]  # the dry step (= step 1's routing)
        for st in range(1, args.tokens):
            seq += [int(arr[l, st, 2]) for l in layers]
        out[kind] = seq
    json.dump(out, open(args.out, "w"))
    eng.close()


if __name__ == "__main__":
    main()
