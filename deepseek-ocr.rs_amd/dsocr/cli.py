"""`deepseek-ocr-cli` for the MI355X engine: same flags, same stdout/stderr behaviour.

Mirrors crates/cli (args.rs:10-101, app.rs:40-330, prompt.rs:7-19, bench.rs:200-260) and the
shared flags of crates/config/src/args.rs:9-92.  What differs, and why:

* The reference resolves model files through its app-config TOML and downloads missing ones
  (`prepare_model_paths`); this CLI takes explicit paths (`--model-config`, `--weights`,
  `--tokenizer`, `--snapshot`) — there is no network and the config store is control plane.
  Without `--weights` the engine builds the deterministic synthetic checkpoint (same names
  and shapes), selected by `--synthetic-seed`.
* `--device` accepts `hip` / `hip:N` (also the reference spellings `cuda` / `cuda:N`, mapped
  to the HIP ordinal); `cpu` / `metal` are refused — the product path has no CPU engine.
* Sampling flags behave as the reference's: `--do-sample true --temperature T [--top-k K]
  [--top-p P] [--seed S]` samples on the GPU with the reference's RNG (sampling.hip); without a
  positive temperature selection is greedy (sampling.rs:67).

Usage: python -m dsocr.cli --prompt "<image>\\nConvert the document to markdown." --image page.png
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List, Optional

from . import FULL_CONFIG
from ._lib import DsocrError
from .engine import DecodeParameters, ModelLoadArgs, VisionSettings, load_model, render_prompt
from .streaming import DeltaTracker, decode_ids


def _bool(v: str) -> bool:
    s = v.strip().lower()
    if s in ("1", "true", "yes", "on"):
        return True
    if s in ("0", "false", "no", "off"):
        return False
    raise argparse.ArgumentTypeError(f"invalid boolean {v!r}")


def add_model_args(p: argparse.ArgumentParser) -> None:
    """CommonModelArgs (config/src/args.rs:9-29)."""
    g = p.add_argument_group("Application")
    g.add_argument("--config", metavar="PATH", help="application config (accepted for compatibility; unused)")
    g.add_argument("--model", metavar="ID", default="deepseek-ocr",
                   help="model id: deepseek-ocr (MI355X engine) or paddleocr-vl (host CPU plumbing path, configs[0])")
    g.add_argument("--model-config", metavar="PATH", help="model config.json (default: bundled DeepSeek-OCR)")
    g.add_argument("--tokenizer", metavar="PATH", help="tokenizer.json (default: synthetic tokenizer)")
    g.add_argument("--weights", metavar="PATH", help="model .safetensors (default: synthetic weights)")
    g.add_argument("--snapshot", metavar="PATH", help="DSQ snapshot (.dsq) to dequantise on load")
    g.add_argument("--synthetic-seed", type=int, default=0, help="seed of the synthetic checkpoint")


def add_inference_args(p: argparse.ArgumentParser) -> None:
    """CommonInferenceArgs (config/src/args.rs:31-92)."""
    g = p.add_argument_group("Inference")
    g.add_argument("--device", default="hip", help="hip | hip:N (cuda[:N] is accepted as an alias)")
    g.add_argument("--dtype", default="f16", choices=["f32", "f16", "bf16"])
    g.add_argument("--template", default="plain")
    g.add_argument("--base-size", type=int, default=1024)
    g.add_argument("--image-size", type=int, default=640)
    g.add_argument("--crop-mode", type=_bool, default=True, metavar="BOOL")
    g.add_argument("--max-new-tokens", type=int, default=512)
    g.add_argument("--no-cache", action="store_true")
    g.add_argument("--do-sample", type=_bool, default=False, metavar="BOOL")
    g.add_argument("--temperature", type=float, default=0.0)
    g.add_argument("--top-p", type=float, default=1.0)
    g.add_argument("--top-k", type=int, default=None)
    g.add_argument("--repetition-penalty", type=float, default=1.0)
    g.add_argument("--no-repeat-ngram-size", type=int, default=20)
    g.add_argument("--seed", type=int, default=None)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="deepseek-ocr-cli", description="DeepSeek-OCR CLI (MI355X engine)")
    add_model_args(p)
    add_inference_args(p)
    pr = p.add_mutually_exclusive_group()
    pr.add_argument("--prompt", help="prompt text; `<image>` marks image slots")
    pr.add_argument("--prompt-file", metavar="PATH", help="UTF-8 prompt file")
    p.add_argument("--image", dest="images", action="append", default=[], metavar="PATH",
                   help="image files for the <image> placeholders, in order")
    b = p.add_argument_group("Benchmark")
    b.add_argument("--bench", action="store_true", help="print per-stage timings")
    b.add_argument("--bench-output", metavar="PATH", help="write benchmark events to a JSON file")
    p.add_argument("-q", "--quiet", action="store_true", help="print only the final result")
    return p


def parse_device(spec: str) -> int:
    s = spec.strip().lower()
    for pre in ("hip", "cuda"):
        if s == pre:
            return 0
        if s.startswith(pre + ":") and s[len(pre) + 1:].isdigit():
            return int(s[len(pre) + 1:])
    raise DsocrError(1, f"device {spec!r} is not supported by the MI355X engine (use hip or hip:N)")


def load_prompt(args) -> str:
    """prompt.rs:7-19."""
    if args.prompt_file:
        with open(args.prompt_file, encoding="utf-8") as f:
            return f.read()
    if args.prompt is not None:
        return args.prompt
    raise DsocrError(1, "prompt is required (use --prompt or --prompt-file)")


def decode_params(args) -> DecodeParameters:
    return DecodeParameters(max_new_tokens=args.max_new_tokens, do_sample=args.do_sample,
                            temperature=args.temperature, top_p=args.top_p, top_k=args.top_k,
                            repetition_penalty=args.repetition_penalty,
                            no_repeat_ngram_size=args.no_repeat_ngram_size, seed=args.seed,
                            use_cache=not args.no_cache)


def load_tokenizer(path: Optional[str], vocab_size: int):
    if path:
        from tokenizers import Tokenizer
        return Tokenizer.from_file(path)
    from .synth import SyntheticTokenizer
    return SyntheticTokenizer(vocab_size)


def open_image(path: str):
    from PIL import Image
    try:
        with Image.open(path) as im:
            return im.convert("RGB")
    except (OSError, ValueError) as e:
        raise DsocrError(3, f"failed to open image at {path}: {e}") from e


def stage_report(events: List[dict]) -> dict:
    """bench.rs:200-245: events + per-stage totals (count/total/avg/min/max ms)."""
    totals = {}
    for ev in events:
        t = totals.setdefault(ev["stage"], [])
        t.append(ev["duration_ms"])
    stage_totals = [{"stage": k, "count": len(v), "total_ms": sum(v), "total_ns": str(int(sum(v) * 1e6)),
                     "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)} for k, v in sorted(totals.items())]
    return {"events": events, "stage_totals": stage_totals}


def _event(stage: str, ms: float, **fields) -> dict:
    return {"stage": stage, "duration_ms": ms, "duration_ns": str(int(ms * 1e6)),
            "fields": [{"key": k, "value": v} for k, v in fields.items()]}


def run_inference(args, out=sys.stdout, err=sys.stderr) -> int:
    def info(msg):
        if not args.quiet:
            print(msg, file=err, flush=True)

    prompt_raw = load_prompt(args)
    if args.model in PADDLE_IDS:
        return run_paddle(args, prompt_raw, out, err)
    device = parse_device(args.device)
    if args.model not in ("deepseek-ocr", "deepseek"):
        raise DsocrError(1, f"model `{args.model}` is not served by the MI355X engine (deepseek-ocr only)")
    config = args.model_config or FULL_CONFIG
    vocab = _vocab_of(config)
    events = []
    t0 = time.perf_counter()
    engine = load_model(ModelLoadArgs(config_path=config, weights_path=args.weights, snapshot_path=args.snapshot,
                                      device=device, dtype=args.dtype, synthetic_seed=args.synthetic_seed))
    load_ms = (time.perf_counter() - t0) * 1e3
    events.append(_event("model.load", load_ms, model=args.model, kind="Deepseek", device=f"hip:{device}",
                         dtype=args.dtype))
    info(f"Model ready in {load_ms / 1e3:.2f}s (kind=Deepseek, flash-attn: true, weights="
         f"{args.weights or f'synthetic(seed={args.synthetic_seed})'})")
    try:
        tokenizer = load_tokenizer(args.tokenizer, vocab)
        prompt = render_prompt(args.template, "", prompt_raw)
        slots = prompt.count("<image>")
        if slots != len(args.images):
            raise DsocrError(1, f"prompt includes {slots} <image> tokens but {len(args.images)} image paths "
                                f"were provided")
        images = [open_image(p) for p in args.images]
        vision = VisionSettings(args.base_size, args.image_size, args.crop_mode)
        params = decode_params(args)

        tracker = DeltaTracker()
        state = {"last": 0, "prefill_s": None}
        start = time.perf_counter()

        def on_token(count, ids):
            if count > 0 and state["prefill_s"] is None:
                state["prefill_s"] = time.perf_counter() - start
            if count <= state["last"]:
                state["last"] = count
                return
            delta = tracker.advance(decode_ids(tokenizer, ids[:count]), False)
            state["last"] = count
            if delta:
                out.write(delta)
                out.flush()

        info(f"Starting generation with requested budget {params.max_new_tokens} tokens")
        outcome = engine.decode(tokenizer, prompt, images, vision, params, None if args.quiet else on_token)
        elapsed = time.perf_counter() - start
        decoded = decode_ids(tokenizer, outcome.generated_tokens)
        if args.quiet:
            out.write(outcome.text + "\n")
        else:
            tail = tracker.advance(decoded, True)
            if tail:
                out.write(tail)
            out.write("\n")
            out.flush()
            info(f"Final output:\n{outcome.text}")
        prefill_s = state["prefill_s"] if state["prefill_s"] is not None and state["prefill_s"] <= elapsed \
            else elapsed
        decode_s = max(elapsed - prefill_s, 0.0)
        info(f"Throughput: prefill={outcome.prompt_tokens} tok in {prefill_s:.2f}s "
             f"({outcome.prompt_tokens / prefill_s if prefill_s > 0 else 0.0:.2f} tok/s); "
             f"generation={outcome.response_tokens} tok in {decode_s:.2f}s "
             f"({outcome.response_tokens / decode_s if decode_s > 0 else 0.0:.2f} tok/s)")
        if args.bench or args.bench_output:
            t = engine.last_timings()
            events += [_event("vision.prepare_inputs", t["vision_prepare_ms"]),
                       _event("vision.compute_embeddings", t["vision_compute_ms"]),
                       _event("decode.prefill", t["decode_prefill_ms"], tokens=outcome.prompt_tokens),
                       _event("decode.iterative", t["decode_iterative_ms"], tokens=outcome.response_tokens),
                       _event("decode.generate", t["decode_generate_ms"])]
            report = stage_report(events)
            if args.bench_output:
                d = os.path.dirname(args.bench_output)
                if d:
                    os.makedirs(d, exist_ok=True)
                with open(args.bench_output, "w") as f:
                    json.dump(report, f, indent=2)
            if args.bench:
                for s in report["stage_totals"]:
                    print(f"[bench] {s['stage']:<28} count={s['count']:<3} total={s['total_ms']:.2f}ms "
                          f"avg={s['avg_ms']:.2f}ms", file=err)
    finally:
        engine.close()
    return 0


PADDLE_IDS = ("paddleocr-vl", "paddleocr", "paddle-ocr-vl")


def run_paddle(args, prompt_raw: str, out=sys.stdout, err=sys.stderr) -> int:
    """ModelKind::PaddleOcrVl on the host CPU (crates/infer-paddleocr model.rs:286-416; BASELINE configs[0]:
    Candle CPU backend plumbing): dsocr.paddle's numpy restatement with a seeded synthetic checkpoint."""
    from . import paddle

    def info(msg):
        if not args.quiet:
            print(msg, file=err, flush=True)

    if args.device.strip().lower() not in ("cpu", "hip", "cuda") and not args.device.lower().startswith(("hip:", "cuda:")):
        raise DsocrError(1, f"device {args.device!r} is not supported")
    if args.weights or args.snapshot:
        raise DsocrError(1, "the PaddleOCR-VL CPU path runs the seeded synthetic checkpoint only (no weights offline)")
    t0 = time.perf_counter()
    engine = paddle.PaddleOcrEngine(args.model_config or paddle.PADDLE_CONFIG, synthetic_seed=args.synthetic_seed)
    load_ms = (time.perf_counter() - t0) * 1e3
    info(f"Model ready in {load_ms / 1e3:.2f}s (kind=PaddleOcrVl, device=cpu, weights=synthetic(seed={args.synthetic_seed}))")
    if args.tokenizer:
        from tokenizers import Tokenizer
        tokenizer = Tokenizer.from_file(args.tokenizer)
    else:
        tokenizer = paddle.PaddleSyntheticTokenizer(engine.cfg)
    prompt = render_prompt(args.template, "", prompt_raw)
    slots = prompt.count("<image>")
    if slots != len(args.images):
        raise DsocrError(1, f"prompt includes {slots} <image> tokens but {len(args.images)} image paths were provided")
    images = [open_image(p) for p in args.images]
    vision = VisionSettings(args.base_size, args.image_size, args.crop_mode)
    outcome = engine.decode(tokenizer, prompt, images, vision, decode_params(args))
    out.write(outcome.text + "\n")
    info(f"generated {outcome.response_tokens} tokens: {outcome.generated_tokens}")
    if args.bench or args.bench_output:
        t = engine.last_timings()
        events = [_event("model.load", load_ms, model=args.model, kind="PaddleOcrVl", device="cpu"),
                  _event("vision.compute_embeddings", t["vision_compute_ms"]),
                  _event("decode.prefill", t["decode_prefill_ms"], tokens=outcome.prompt_tokens),
                  _event("decode.iterative", t["decode_iterative_ms"], tokens=outcome.response_tokens)]
        report = stage_report(events)
        if args.bench_output:
            with open(args.bench_output, "w") as f:
                json.dump(report, f, indent=2)
        if args.bench:
            for s_ in report["stage_totals"]:
                print(f"[bench] {s_['stage']:<28} count={s_['count']:<3} total={s_['total_ms']:.2f}ms", file=err)
    engine.close()
    return 0


def _vocab_of(config_path: str) -> int:
    with open(config_path) as f:
        cfg = json.load(f)
    lang = cfg.get("language_config") or {}
    return int(lang.get("vocab_size") or cfg.get("vocab_size") or 129280)


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    try:
        return run_inference(args)
    except DsocrError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
