"""Host-side mirror of the reference engine surface, bound to the C ABI.

Mirrors (TimmyOVO/deepseek-ocr.rs):
  * ``ModelLoadArgs`` / ``load_model``           core/src/inference.rs:178-186, model/mod.rs:90-115
  * ``VisionSettings`` / ``DecodeParameters``    core/src/inference.rs:13-79 (same defaults)
  * ``DecodeOutcome``                            core/src/inference.rs:161-167
  * ``OcrEngine.decode``                         model/mod.rs:2370-2455
  * ``build_prompt_tokens``                      model/mod.rs:2536-2603
  * ``render_prompt`` (plain template)           core/src/inference.rs:212-225, conversation/mod.rs:115-125
  * ``normalize_text``                           core/src/inference.rs:228-233
All compute runs in libdsocr.so on a gfx950 GPU; this module only marshals.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import numpy as np

from ._lib import (DTYPES, DecodeParamsC, DsocrError, LoadArgs, RequestC, ResultC, STREAM_CB, TimingsC,
                   VisionSettingsC, check, lib)


@dataclass
class VisionSettings:
    base_size: int = 1024
    image_size: int = 640
    crop_mode: bool = True


@dataclass
class DecodeParameters:
    """DecodeParameters::default (inference.rs:65-79)."""
    max_new_tokens: int = 512
    do_sample: bool = False
    temperature: float = 0.0
    top_p: Optional[float] = 1.0
    top_k: Optional[int] = None
    repetition_penalty: float = 1.0
    no_repeat_ngram_size: Optional[int] = 20
    seed: Optional[int] = None
    use_cache: bool = True


@dataclass
class DecodeOutcome:
    text: str
    prompt_tokens: int
    response_tokens: int
    generated_tokens: list = field(default_factory=list)


@dataclass
class ModelLoadArgs:
    kind: str = "deepseek"
    config_path: Optional[str] = None
    weights_path: Optional[str] = None   # None -> deterministic synthetic checkpoint
    snapshot_path: Optional[str] = None
    device: int = 0
    dtype: str = "f16"
    synthetic_seed: int = 0


def render_prompt(template: str, system_prompt: str, raw_prompt: str) -> str:
    """Only the `plain` template (the CLI default, config.rs:209-221): message trimmed, empty separators."""
    if template != "plain":
        raise ValueError(f"unknown conversation template {template}")
    return raw_prompt.strip()


def normalize_text(s: str) -> str:
    return s.replace("\r\n", "\n").replace("<｜end▁of▁sentence｜>", "").strip()


def _encode(tokenizer, text: str) -> list:
    enc = tokenizer.encode(text, add_special_tokens=False)
    return list(enc.ids) if hasattr(enc, "ids") else list(enc)


def build_prompt_tokens(tokenizer, prompt: str, image_token_counts: Sequence[int]):
    """model/mod.rs:2536-2603: [BOS=0] + encode(segment) + <image> x count per image; mask marks slots."""
    image_token_id = tokenizer.token_to_id("<image>")
    if image_token_id is None:
        raise DsocrError(1, "tokenizer missing <image> token")
    segments = prompt.split("<image>")
    if len(segments) - 1 != len(image_token_counts):
        raise DsocrError(1, f"prompt formatting failed: prompt/image embedding mismatch: {len(segments) - 1} slots vs "
                            f"{len(image_token_counts)} embeddings")
    ids, mask = [0], [0]
    for i, seg in enumerate(segments):
        t = _encode(tokenizer, seg)
        ids += t
        mask += [0] * len(t)
        if i < len(image_token_counts):
            ids += [int(image_token_id)] * int(image_token_counts[i])
            mask += [1] * int(image_token_counts[i])
    return ids, mask


class Page:
    """Preprocessed page pixels (a1-a3): global view + crop tiles.

    ``engine=None``: host C++ (dsocr_prepare_page); with an engine: on that engine's GPU
    (dsocr_prepare_page_device, bit-identical pixels, device-resident)."""

    def __init__(self, rgb, vision: VisionSettings, engine=None):
        if hasattr(rgb, "convert"):  # PIL image
            rgb = np.asarray(rgb.convert("RGB"))
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        if rgb.ndim != 3 or rgb.shape[2] != 3:
            raise DsocrError(1, "page must be HxWx3 uint8")
        vs = VisionSettingsC(vision.base_size, vision.image_size, 1 if vision.crop_mode else 0)
        h = C.c_void_p()
        if engine is None:
            check(lib().dsocr_prepare_page(rgb.ctypes.data_as(C.c_void_p), rgb.shape[1], rgb.shape[0], C.byref(vs),
                                           C.byref(h)))
        else:
            check(lib().dsocr_prepare_page_device(engine._h, rgb.ctypes.data_as(C.c_void_p), rgb.shape[1],
                                                  rgb.shape[0], C.byref(vs), C.byref(h)))
        self.on_device = engine is not None
        self._h = h
        cw, ch, nt, ntok = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_size_t()
        check(lib().dsocr_page_info(h, C.byref(cw), C.byref(ch), C.byref(nt), C.byref(ntok)))
        self.crop_shape = (cw.value, ch.value)
        self.n_tiles = nt.value
        self.n_image_tokens = ntok.value

    def to_device(self, engine) -> "Page":
        """Stage the pixels in the engine's HBM (dsocr_page_to_device); returns self."""
        check(lib().dsocr_page_to_device(engine._h, self._h))
        return self

    def pixels(self):
        g, gs, t, ts = C.c_void_p(), C.c_uint32(), C.c_void_p(), C.c_uint32()
        check(lib().dsocr_page_pixels_view(self._h, C.byref(g), C.byref(gs), C.byref(t), C.byref(ts)))
        if self.on_device:
            glob = np.empty((3, gs.value, gs.value), np.float32)
            tiles = np.empty((self.n_tiles, 3, ts.value, ts.value), np.float32) if self.n_tiles else None
            check(lib().dsocr_page_read_device(self._h, glob.ctypes.data_as(C.c_void_p),
                                               tiles.ctypes.data_as(C.c_void_p) if tiles is not None else None))
            return glob, tiles
        glob = np.ctypeslib.as_array(C.cast(g, C.POINTER(C.c_float)), (3, gs.value, gs.value)).copy()
        tiles = None
        if self.n_tiles:
            tiles = np.ctypeslib.as_array(C.cast(t, C.POINTER(C.c_float)),
                                          (self.n_tiles, 3, ts.value, ts.value)).copy()
        return glob, tiles

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().dsocr_page_free(self._h)
                self._h = None
        except Exception:
            pass


def _params_c(p: DecodeParameters, eos: int, ignore_eos: bool) -> DecodeParamsC:
    return DecodeParamsC(max_new_tokens=p.max_new_tokens, do_sample=1 if p.do_sample else 0,
                         temperature=p.temperature, top_p=p.top_p if p.top_p is not None else -1.0,
                         top_k=p.top_k or 0, repetition_penalty=p.repetition_penalty,
                         no_repeat_ngram_size=p.no_repeat_ngram_size or 0, seed=p.seed or 0,
                         use_cache=1 if p.use_cache else 0, eos_token_id=eos, ignore_eos=1 if ignore_eos else 0,
                         has_seed=0 if p.seed is None else 1)


class DeepseekOcrEngine:
    """OcrEngine implementation backed by the MI355X engine (one per GPU)."""

    def __init__(self, args: ModelLoadArgs):
        if args.kind != "deepseek":
            raise DsocrError(1, f"ModelKind::{args.kind} cannot be loaded by the Deepseek engine")
        if args.config_path is None:
            raise DsocrError(1, "config_path is required")
        la = LoadArgs(args.config_path.encode(), args.weights_path.encode() if args.weights_path else None,
                      args.snapshot_path.encode() if args.snapshot_path else None, args.device, DTYPES[args.dtype],
                      args.synthetic_seed)
        h = C.c_void_p()
        check(lib().dsocr_engine_load(C.byref(la), C.byref(h)))
        self._h = h
        self.args = args
        hid, voc, eos, nl = C.c_size_t(), C.c_size_t(), C.c_int64(), C.c_size_t()
        check(lib().dsocr_engine_info(h, C.byref(hid), C.byref(voc), C.byref(eos), C.byref(nl)))
        self.hidden, self.vocab, self.eos_token_id, self.num_layers = hid.value, voc.value, eos.value, nl.value

    # OcrEngine accessors (inference.rs:189-198)
    def kind(self):
        return "deepseek"

    def device(self):
        return f"hip:{self.args.device}"

    def dtype(self):
        return self.args.dtype

    def weights_path(self):
        return self.args.weights_path

    def flash_attention_enabled(self):
        return True

    def close(self):
        if getattr(self, "_h", None):
            lib().dsocr_engine_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ lower seams
    def image_embeddings(self, pages: Sequence[Page]):
        n = len(pages)
        arr = (C.c_void_p * n)(*[p._h for p in pages])
        cap = sum(p.n_image_tokens for p in pages)
        out = np.empty((max(cap, 1), self.hidden), np.float32)
        rows = (C.c_size_t * n)()
        check(lib().dsocr_image_embeddings(self._h, arr, n, out.ctypes.data_as(C.c_void_p), cap, rows))
        res, off = [], 0
        for i in range(n):
            res.append(out[off:off + rows[i]].copy())
            off += rows[i]
        return res

    def _request(self, ids, mask, page, image_rows, keep):
        ids = np.ascontiguousarray(ids, np.int64)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        rows = None if image_rows is None else np.ascontiguousarray(image_rows, np.float32)
        keep += [ids, m, rows]
        return RequestC(ids.ctypes.data_as(C.POINTER(C.c_int64)),
                        None if m is None else m.ctypes.data_as(C.POINTER(C.c_uint8)), len(ids),
                        page._h if page is not None else None,
                        None if rows is None else rows.ctypes.data_as(C.POINTER(C.c_float)),
                        0 if rows is None else rows.shape[0])

    def generate(self, ids, mask=None, page: Optional[Page] = None, image_rows=None,
                 params: DecodeParameters = DecodeParameters(), stream: Optional[Callable] = None,
                 ignore_eos: bool = False):
        keep = []
        req = self._request(ids, mask, page, image_rows, keep)
        pc = _params_c(params, self.eos_token_id, ignore_eos)
        out = np.empty(max(params.max_new_tokens, 1), np.int64)
        n = C.c_size_t()
        cb = STREAM_CB(lambda k, toks, _u: stream(k, [toks[i] for i in range(k)])) if stream else STREAM_CB()
        check(lib().dsocr_generate(self._h, C.byref(req), C.byref(pc), cb, None, out.ctypes.data_as(C.c_void_p),
                                   len(out), C.byref(n)))
        return out[:n.value].tolist()

    def generate_batch(self, requests, params: DecodeParameters = DecodeParameters(), ignore_eos: bool = False):
        """requests: list of (ids, mask, page_or_None, image_rows_or_None)."""
        keep = []
        reqs = (RequestC * len(requests))(*[self._request(*r, keep) for r in requests])
        outs = [np.empty(max(params.max_new_tokens, 1), np.int64) for _ in requests]
        res = (ResultC * len(requests))(*[ResultC(o.ctypes.data_as(C.POINTER(C.c_int64)), len(o), 0, 0)
                                          for o in outs])
        pc = _params_c(params, self.eos_token_id, ignore_eos)
        check(lib().dsocr_generate_batch(self._h, len(requests), reqs, C.byref(pc), res))
        return [outs[i][:res[i].n_out].tolist() for i in range(len(requests))]

    def generate_trace(self, requests, params: DecodeParameters = DecodeParameters(), ignore_eos: bool = False):
        """generate_batch + the raw logits of every step (dsocr_generate_trace): returns
        (ids per page, logits [n][max_new][vocab] float32; rows past a page's last token are 0)."""
        keep = []
        reqs = (RequestC * len(requests))(*[self._request(*r, keep) for r in requests])
        outs = [np.empty(max(params.max_new_tokens, 1), np.int64) for _ in requests]
        res = (ResultC * len(requests))(*[ResultC(o.ctypes.data_as(C.POINTER(C.c_int64)), len(o), 0, 0)
                                          for o in outs])
        logits = np.zeros((len(requests), max(params.max_new_tokens, 1), self.vocab), np.float32)
        pc = _params_c(params, self.eos_token_id, ignore_eos)
        check(lib().dsocr_generate_trace(self._h, len(requests), reqs, C.byref(pc), res,
                                         logits.ctypes.data_as(C.c_void_p), logits.size))
        return [outs[i][:res[i].n_out].tolist() for i in range(len(requests))], logits

    def last_timings(self) -> dict:
        t = TimingsC()
        check(lib().dsocr_last_timings(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in TimingsC._fields_}

    SPAN_KINDS = ("moe_gateup", "moe_down", "attention", "o_proj", "router")  # the last two: chain spans only

    SPAN_WAVES, SPAN_EVENTS, SPAN_CHAIN = 1, 2, 4

    def set_spans(self, mode: int):
        """In-context launch spans for the following generates (dsocr_engine_set_spans): 0 off, bit 1 wave
        spans, bit 2 HIP events around the launches inside the replayed step graph, 4 (alone) chain spans
        (every layer's gate/up, down, attention, o_proj and router launches, one fold per step)."""
        check(lib().dsocr_engine_set_spans(self._h, int(mode)))

    def spans(self) -> dict:
        """Launch spans of the last generate run with spans on: {kind: array [layers][steps][5] uint64
        (entry, exit (100 MHz wall clock), distinct experts, waves, HIP-event dispatch duration ns)};
        only the decode steps (index 1 .. steps - 1) of the layers that have the launch are non-zero."""
        k, l, st = C.c_size_t(), C.c_size_t(), C.c_size_t()
        check(lib().dsocr_engine_spans(self._h, None, 0, C.byref(k), C.byref(l), C.byref(st)))
        if st.value == 0:
            return {}
        buf = np.zeros((k.value, l.value, st.value, 5), np.uint64)
        check(lib().dsocr_engine_spans(self._h, buf.ctypes.data_as(C.c_void_p), buf.size, None, None, None))
        return {name: buf[i] for i, name in enumerate(self.SPAN_KINDS[:k.value])}

    def set_persist_stamps(self, mode: int = 1):
        """The next generate times every persistent decode launch (HIP events) and records its phase clocks."""
        check(lib().dsocr_engine_set_persist_stamps(self._h, int(mode)))

    def persist_info(self, layers: int = 0) -> dict:
        """{used, launch_us [steps], stamps [steps][256][layers][9] uint64} of the last generate
        (dsocr_engine_persist_info)."""
        used, nd, ns = C.c_int(), C.c_size_t(), C.c_size_t()
        check(lib().dsocr_engine_persist_info(self._h, C.byref(used), None, 0, C.byref(nd), None, 0, C.byref(ns)))
        d = np.zeros(nd.value, np.float64)
        st = np.zeros(ns.value, np.uint64)
        check(lib().dsocr_engine_persist_info(self._h, None, d.ctypes.data_as(C.c_void_p), d.size, None,
                                              st.ctypes.data_as(C.c_void_p), st.size, None))
        out = {"used": bool(used.value), "launch_us": d}
        if layers and st.size:
            out["stamps"] = st.reshape(-1, 256, layers, 9)
        return out

    def profile_decode(self, iters: int = 3) -> dict:
        """HIP-event timings + algorithmic bytes of the dominant decode kernels (see dsocr.h)."""
        from ._lib import DecodeProfileC
        p = DecodeProfileC()
        check(lib().dsocr_profile_decode(self._h, iters, C.byref(p)))
        out = {}
        for k in ("moe_gateup", "moe_down", "attention", "lm_head", "qkv", "o_proj", "router", "layers_step",
                  "lm_head_screened"):
            kp = getattr(p, k)
            out[k] = {"avg_us": kp.avg_us, "bytes": kp.bytes, "flops": kp.flops, "launches": kp.launches,
                      "replay_us": kp.replay_us, "ctx_us": kp.ctx_us}
        out.update(experts_touched=p.experts_touched, tokens=p.tokens, kv_len=p.kv_len,
                   moe_gateup_kernel=(p.moe_gateup_kernel or b"").decode(),
                   moe_down_kernel=(p.moe_down_kernel or b"").decode())
        return out

    # ------------------------------------------------------------------ OcrEngine::decode
    def decode(self, tokenizer, prompt: str, images: Sequence, vision: VisionSettings,
               params: DecodeParameters, stream: Optional[Callable] = None) -> DecodeOutcome:
        pages = [Page(im, vision, self) for im in images]
        ids, mask = build_prompt_tokens(tokenizer, prompt, [p.n_image_tokens for p in pages])
        if len(pages) > 1:
            # several <image> slots: the pages' rows in image order (compute_image_embeddings over the
            # list, model/mod.rs:2387), injected at the mask positions in that order
            rows = np.concatenate(self.image_embeddings(pages), axis=0)
            gen = self.generate(ids, mask, None, rows, params, stream)
        else:
            gen = self.generate(ids, mask, pages[0] if pages else None, None, params, stream)
        text = ""
        if hasattr(tokenizer, "decode"):
            try:
                text = tokenizer.decode([int(t) for t in gen], skip_special_tokens=True)
            except TypeError:
                text = tokenizer.decode([int(t) for t in gen])
        return DecodeOutcome(normalize_text(text), len(ids), len(gen), gen)


def load_model(args: ModelLoadArgs) -> DeepseekOcrEngine:
    return DeepseekOcrEngine(args)
