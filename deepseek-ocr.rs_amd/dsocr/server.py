"""OpenAI-compatible HTTP server over the MI355X engine (`deepseek-ocr-server`).

Mirrors crates/server: routes (routes.rs:20-232: GET /v1/health, GET/OPTIONS /v1/models,
POST /v1/responses, POST /v1/chat/completions), request/response shapes (models.rs:1-145),
message flattening and image loading (generation.rs:177-313), error classes (error.rs:10-50:
400 `invalid_request_error` / 500 `internal_error`, with engine messages containing
"prompt formatting failed" / "prompt/image embedding mismatch" mapped to 400,
generation.rs:108-118), the missing-image fallback (routes.rs:240-246) and the SSE event
sequence (stream.rs:140-374).  The engine sits behind one lock (Send-not-Sync, state.rs:22)
and decodes on a worker thread (spawn_blocking, generation.rs:38-49).

Not carried over: multi-model hot swapping from the app config (one DeepSeek-OCR engine per
process/GPU here) and fetching http(s) image URLs (no network on the target boxes: such
URLs are refused with 400, like any other unsupported URL scheme in the reference).
"""

import base64
import io
import json
import queue
import threading
import time
import uuid
from dataclasses import dataclass, field, replace
from typing import Any, List, Optional, Tuple

from ._lib import DsocrError
from .engine import DecodeParameters, VisionSettings
from .streaming import DeltaTracker, decode_ids

EMPTY_GENERATION_ERROR = ("generation failed: model returned empty output (response_tokens=0 and text is empty)")

MISSING_IMAGE_MARKDOWN = (
    "⚠️ **Image Required**\n\n- This OCR backend expects at least one `<image>` placeholder or attached image.\n"
    "- Please include `input_image` / `image_url`, or add `<image>` inside the prompt.\n\n---\n\n"
    "⚠️ **需要图像输入**\n\n- 当前 OCR 模型需要至少一个 `<image>` 占位符或实际图片。\n"
    "- 请在请求中附带 `input_image`/`image_url`，或在 prompt 中插入 `<image>`。")

_PATCH_FIELDS = ("max_new_tokens", "do_sample", "temperature", "top_p", "top_k", "repetition_penalty",
                 "no_repeat_ngram_size", "seed", "use_cache")


class ApiError(Exception):
    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status
        self.message = message

    @staticmethod
    def bad_request(msg):
        return ApiError(400, msg)

    @staticmethod
    def internal(msg):
        return ApiError(500, msg)

    def body(self) -> dict:
        return {"error": {"message": self.message,
                          "type": "invalid_request_error" if self.status == 400 else "internal_error"}}


# ---------------------------------------------------------------- message conversion (generation.rs:177-313)
def load_image(url: str):
    """generation.rs:261-296: data: URLs (base64) only; http(s) fetching is not available offline."""
    if url.startswith("data:"):
        meta, sep, payload = url[5:].partition(",")
        if not sep:
            raise ApiError.bad_request("invalid data URL")
        if not meta.endswith(";base64"):
            raise ApiError.bad_request("data URLs must specify base64 encoding")
        try:
            raw = base64.b64decode(payload, validate=True)
        except (ValueError, TypeError) as e:
            raise ApiError.bad_request(f"invalid base64 image payload: {e}")
        from PIL import Image
        try:
            with Image.open(io.BytesIO(raw)) as im:
                return im.convert("RGB")
        except (OSError, ValueError) as e:
            raise ApiError.bad_request(f"failed to decode inline image: {e}")
    if url.startswith("http://") or url.startswith("https://"):
        raise ApiError.bad_request(f"failed to fetch {url}: remote image URLs are not available on this host")
    raise ApiError.bad_request("only data: URIs or http(s) image URLs are supported")


def _image_url(part: dict) -> str:
    v = part.get("image_url")
    if isinstance(v, dict):
        v = v.get("url")
    if not isinstance(v, str):
        raise ApiError.bad_request("image part is missing image_url")
    return v


def flatten_content(content: Any) -> Tuple[str, list]:
    """generation.rs:238-259.  Parts are visited in REVERSE order, as the reference does."""
    if content is None:
        return "", []
    if isinstance(content, str):
        return content.strip(), []
    if not isinstance(content, list):
        raise ApiError.bad_request("message content must be a string or a list of parts")
    buf, images = "", []
    for part in reversed(content):
        kind = part.get("type") if isinstance(part, dict) else None
        if kind in ("image_url", "input_image"):
            buf += "<image>"
            images.append(load_image(_image_url(part)))
        elif kind in ("text", "input_text"):
            if buf:
                buf += "\n"
            buf += str(part.get("text", ""))
        else:
            raise ApiError.bad_request(f"unsupported message part type {kind!r}")
    return buf.strip(), images


def collect_prompt_sections(messages: List[dict]) -> Tuple[List[str], list]:
    """generation.rs:193-236: system messages before the LAST user message, then that user message."""
    user_idx = None
    for i in range(len(messages) - 1, -1, -1):
        if str(messages[i].get("role", "")).lower() == "user":
            user_idx = i
            break
    if user_idx is None:
        raise ApiError.bad_request("request must include at least one user message")
    sections, images = [], []
    for m in messages[:user_idx]:
        if str(m.get("role", "")).lower() != "system":
            continue
        text, imgs = flatten_content(m.get("content"))
        if text:
            sections.append(text)
        images += imgs
    text, imgs = flatten_content(messages[user_idx].get("content"))
    if text:
        sections.append(text)
    images += imgs
    if not sections and not images:
        raise ApiError.bad_request("user content must include text or images")
    return sections, images


def convert_messages(messages: List[dict]) -> Tuple[str, list]:
    """generation.rs:177-191 (DeepSeek: sections joined by a blank line, trimmed)."""
    sections, images = collect_prompt_sections(messages)
    return "\n\n".join(sections).strip(), images


def merge_decode(defaults: DecodeParameters, req: dict, max_tokens: Optional[int]) -> DecodeParameters:
    """DecodeParameters + DecodeParametersPatch (routes.rs:79-85): max tokens first, then the
    request's flattened patch fields."""
    p = replace(defaults, max_new_tokens=max_tokens if max_tokens is not None else defaults.max_new_tokens)
    patch = {k: req[k] for k in _PATCH_FIELDS if k in req and req[k] is not None}
    return replace(p, **patch)


# ---------------------------------------------------------------- state
@dataclass
class ServerState:
    engine: Any
    tokenizer: Any
    model_id: str = "deepseek-ocr"
    vision: VisionSettings = field(default_factory=VisionSettings)
    defaults: DecodeParameters = field(default_factory=DecodeParameters)
    lock: threading.Lock = field(default_factory=threading.Lock)

    def validate_model(self, requested: str):
        if requested != self.model_id:
            raise ApiError.bad_request(f"requested model `{requested}` is not available")


def _now() -> int:
    return int(time.time())


def generate_blocking(state: ServerState, prompt: str, images: list, params: DecodeParameters, on_token=None):
    """generation.rs:75-163."""
    with state.lock:
        try:
            outcome = state.engine.decode(state.tokenizer, prompt, images, state.vision, params, on_token)
        except DsocrError as e:
            msg = str(e)
            if "prompt formatting failed" in msg or "prompt/image embedding mismatch" in msg:
                raise ApiError.bad_request(msg)
            raise ApiError.internal(f"generation failed: {msg}")
    if outcome.response_tokens == 0 and not outcome.text.strip():
        raise ApiError.internal(EMPTY_GENERATION_ERROR)
    return outcome


class StreamController:
    """stream.rs:120-374: initial event, per-token deltas through DeltaTracker, final event, [DONE]."""

    def __init__(self, tokenizer, kind: str, model: str):
        self.tokenizer, self.kind, self.model = tokenizer, kind, model
        self.created = _now()
        self.q: "queue.Queue[Optional[str]]" = queue.Queue()
        self.delta = DeltaTracker()
        self.last_count = 0
        self.role_sent = False
        self.finished = False
        if kind == "chat":
            self.id = f"chatcmpl-{uuid.uuid4()}"
        else:
            self.id = f"resp-{uuid.uuid4()}"
            self.output_id = f"msg-{uuid.uuid4()}"

    def _send(self, obj):
        self.q.put(json.dumps(obj, ensure_ascii=False))

    def _head(self):
        return {"id": self.id, "object": "response", "created": self.created, "model": self.model}

    def send_initial(self):
        if self.kind == "chat":
            self._send({"id": self.id, "object": "chat.completion.chunk", "created": self.created,
                        "model": self.model,
                        "choices": [{"index": 0, "delta": {"role": "assistant"}, "finish_reason": None}]})
            self.role_sent = True
        else:
            self._send({"type": "response.created", "response": self._head()})

    def emit_delta(self, text: str, include_role: bool):
        if self.kind == "chat":
            delta = {"content": text}
            if include_role:
                delta["role"] = "assistant"
            self._send({"id": self.id, "object": "chat.completion.chunk", "created": self.created,
                        "model": self.model, "choices": [{"index": 0, "delta": delta, "finish_reason": None}]})
        else:
            self._send({"type": "response.output_text.delta", "response": self._head(),
                        "output_id": self.output_id, "output_index": 0, "delta": text})

    def process_tokens(self, count: int, ids, is_final: bool):
        if count == 0:
            return
        if count <= self.last_count:
            self.last_count = count
            return
        include_role = self.kind == "chat" and not self.role_sent
        full = decode_ids(self.tokenizer, ids[:count])
        emit = None
        if full:
            d = self.delta.advance(full, is_final)
            if include_role or d:
                emit = d
                if include_role:
                    self.role_sent = True
        self.last_count = count
        if emit is not None:
            self.emit_delta(emit, include_role)

    def callback(self):
        return lambda count, ids: self.process_tokens(count, ids, False)

    def flush_remaining(self, ids):
        if ids:
            self.process_tokens(len(ids), ids, True)

    def finalize(self, normalized: str, prompt_tokens: int, completion_tokens: int):
        if self.finished:
            return
        self.finished = True
        if self.kind == "chat":
            self._send({"id": self.id, "object": "chat.completion.chunk", "created": self.created,
                        "model": self.model, "choices": [{"index": 0, "delta": {}, "finish_reason": "stop"}],
                        "usage": {"prompt_tokens": prompt_tokens, "completion_tokens": completion_tokens,
                                  "total_tokens": prompt_tokens + completion_tokens}})
        else:
            self._send({"type": "response.completed", "response": dict(self._head(), output=[
                {"id": self.output_id, "type": "message", "role": "assistant",
                 "content": [{"type": "output_text", "text": normalized}]}],
                usage={"input_tokens": prompt_tokens, "output_tokens": completion_tokens,
                       "total_tokens": prompt_tokens + completion_tokens})})
        self.q.put("[DONE]")
        self.q.put(None)

    def send_error(self, message: str):
        if self.finished:
            return
        self.finished = True
        self._send({"type": "response.error", "error": {"message": message}})
        self.q.put("[DONE]")
        self.q.put(None)

    def emit_fallback(self, text: str):
        self.emit_delta(text, True)
        self.finalize(text, 0, 0)

    def events(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            yield f"data: {item}\n\n"


def _chat_response(model, text, pt, ct):
    return {"id": f"chatcmpl-{uuid.uuid4()}", "object": "chat.completion", "created": _now(), "model": model,
            "choices": [{"index": 0, "message": {"role": "assistant", "content": text}, "finish_reason": "stop"}],
            "usage": {"prompt_tokens": pt, "completion_tokens": ct, "total_tokens": pt + ct}}


def _responses_response(model, text, pt, ct):
    return {"id": f"resp-{uuid.uuid4()}", "object": "response", "created": _now(), "model": model,
            "output": [{"id": f"msg-{uuid.uuid4()}", "type": "message", "role": "assistant",
                        "content": [{"type": "output_text", "text": text}]}],
            "usage": {"prompt_tokens": pt, "completion_tokens": ct, "total_tokens": pt + ct}}


def handle_generation(state: ServerState, req: dict, kind: str):
    """Shared body of responses_endpoint / chat_completions_endpoint (routes.rs:55-222).
    Returns ("json", dict) or ("stream", StreamController)."""
    if not isinstance(req, dict):
        raise ApiError.bad_request("request body must be a JSON object")
    model = req.get("model")
    if not isinstance(model, str):
        raise ApiError.bad_request("missing field `model`")
    state.validate_model(model)
    messages = req.get("input" if kind == "responses" else "messages") or []
    prompt, images = convert_messages(messages)
    stream = bool(req.get("stream"))
    if "<image>" not in prompt:
        if stream:
            c = StreamController(state.tokenizer, kind, model)
            c.send_initial()
            c.emit_fallback(MISSING_IMAGE_MARKDOWN)
            return "stream", c
        mk = _chat_response if kind == "chat" else _responses_response
        return "json", mk(model, MISSING_IMAGE_MARKDOWN, 0, 0)
    max_tokens = req.get("max_output_tokens") if kind == "responses" else None
    if max_tokens is None:
        max_tokens = req.get("max_tokens")
    params = merge_decode(state.defaults, req, max_tokens)
    if stream:
        c = StreamController(state.tokenizer, kind, model)

        def work():
            try:
                c.send_initial()
                out = generate_blocking(state, prompt, images, params, c.callback())
                c.flush_remaining(out.generated_tokens)
                c.finalize(out.text, out.prompt_tokens, out.response_tokens)
            except ApiError as e:
                c.send_error(e.message)
            except Exception as e:  # noqa: BLE001 - reported to the client like generation.rs:60-70
                c.send_error(f"generation task failed: {e}")

        threading.Thread(target=work, daemon=True).start()
        return "stream", c
    out = generate_blocking(state, prompt, images, params)
    mk = _chat_response if kind == "chat" else _responses_response
    return "json", mk(model, out.text, out.prompt_tokens, out.response_tokens)


def create_app(state: ServerState):
    """The FastAPI application (app.rs:11-63: routes mounted under /v1, permissive CORS)."""
    from fastapi import FastAPI, Request
    from fastapi.middleware.cors import CORSMiddleware
    from fastapi.responses import JSONResponse, PlainTextResponse, Response, StreamingResponse
    from starlette.concurrency import run_in_threadpool

    app = FastAPI(title="DeepSeek-OCR API Server (MI355X)")
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"])

    @app.exception_handler(ApiError)
    async def _api_error(_req, exc: ApiError):
        return JSONResponse(exc.body(), status_code=exc.status)

    @app.get("/v1/health")
    async def health():
        return PlainTextResponse("ok")

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": state.model_id, "object": "model", "created": _now(),
                                            "owned_by": "deepseek-ocr"}]}

    @app.options("/v1/models")
    async def options_models():
        return Response(status_code=200)

    async def _run(request: Request, kind: str):
        try:
            req = await request.json()
        except (ValueError, UnicodeDecodeError) as e:
            raise ApiError.bad_request(f"invalid JSON body: {e}")
        how, val = await run_in_threadpool(handle_generation, state, req, kind)
        if how == "stream":
            return StreamingResponse(val.events(), media_type="text/event-stream")
        return JSONResponse(val)

    @app.post("/v1/responses")
    async def responses(request: Request):
        return await _run(request, "responses")

    @app.post("/v1/chat/completions")
    async def chat(request: Request):
        return await _run(request, "chat")

    return app


def main(argv=None) -> int:
    """`deepseek-ocr-server` (server/src/args.rs + config defaults host 0.0.0.0, port 8000)."""
    import argparse

    from .cli import _vocab_of, add_inference_args, add_model_args, decode_params, load_tokenizer, parse_device
    from . import FULL_CONFIG
    from .engine import ModelLoadArgs, load_model

    p = argparse.ArgumentParser(prog="deepseek-ocr-server", description="DeepSeek-OCR API Server (MI355X engine)")
    add_model_args(p)
    add_inference_args(p)
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    args = p.parse_args(argv)
    config = args.model_config or FULL_CONFIG
    engine = load_model(ModelLoadArgs(config_path=config, weights_path=args.weights, snapshot_path=args.snapshot,
                                      device=parse_device(args.device), dtype=args.dtype,
                                      synthetic_seed=args.synthetic_seed))
    state = ServerState(engine, load_tokenizer(args.tokenizer, _vocab_of(config)), args.model,
                        VisionSettings(args.base_size, args.image_size, args.crop_mode), decode_params(args))
    import uvicorn
    uvicorn.run(create_app(state), host=args.host, port=args.port)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
