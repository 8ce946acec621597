"""CLI / HTTP server bridge over the engine surface.

CPU tests drive the host logic with a stand-in engine object that records what it is asked
(the product engine needs a GPU); the `gpu` tests run the same CLI and server over the real
MI355X engine on the tiny config and check the generated ids against the CPU oracle.

Reference behaviour pinned here: crates/cli/src/app.rs:150-157 (slot/image count check),
prompt.rs:7-19, bench.rs:200-245 (report shape); crates/server/src/generation.rs:177-313
(reverse part order, last user message + earlier system messages, data-URL images),
routes.rs:55-246 (missing-image fallback, max tokens precedence), error.rs:36-50 (400/500
bodies), stream.rs:140-374 (SSE event sequence); core/src/streaming.rs (UTF-8-safe deltas).
"""
import base64
import io
import json
import os

import numpy as np
import pytest

from dsocr import DecodeOutcome, DecodeParameters, DsocrError, VisionSettings
from dsocr import cli, server
from dsocr.streaming import DeltaTracker, extract_delta
from dsocr.synth import SyntheticTokenizer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")


def _png_bytes(h=40, w=60, seed=0):
    from PIL import Image
    arr = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="PNG")
    return b.getvalue(), arr


def _data_url(png):
    return "data:image/png;base64," + base64.b64encode(png).decode()


class FakeEngine:
    """Records decode calls; streams a fixed token list through the callback."""

    def __init__(self, tokens=(20, 21, 22), error=None):
        self.tokens, self.error, self.calls, self.closed = list(tokens), error, [], False

    def decode(self, tokenizer, prompt, images, vision, params, stream=None):
        self.calls.append(dict(prompt=prompt, images=images, vision=vision, params=params))
        if self.error:
            raise self.error
        for k in range(1, len(self.tokens) + 1):
            if stream:
                stream(k, self.tokens[:k])
        text = tokenizer.decode(self.tokens, skip_special_tokens=True)
        return DecodeOutcome(text, 10, len(self.tokens), list(self.tokens))

    def last_timings(self):
        return dict(vision_prepare_ms=1.0, vision_compute_ms=2.0, decode_prefill_ms=3.0, decode_iterative_ms=4.0,
                    decode_generate_ms=9.0, decode_steps=2, pages=1)

    def close(self):
        self.closed = True


# ---------------------------------------------------------------- streaming.rs
def test_extract_delta_and_tracker():
    assert extract_delta("abc", "abcdef") == "def"
    assert extract_delta("abX", "abcd") == "cd"
    t = DeltaTracker()
    assert t.advance("he", False) == "he"
    assert t.advance("hello", False) == "llo"
    # an incomplete multi-byte char decodes to U+FFFD: held back until complete
    assert t.advance("hello w�", False) == " w"
    assert t.snapshot() == "hello w"
    assert t.advance("hello w�", False) == ""
    assert t.advance("hello wé", False) == "é"
    assert t.advance("hello wé�", True) == "�"


# ---------------------------------------------------------------- generation.rs message conversion
def test_convert_messages_reverse_parts_and_system():
    png, _ = _png_bytes()
    msgs = [{"role": "system", "content": "be precise"},
            {"role": "assistant", "content": "ignored"},
            {"role": "user", "content": "old turn"},
            {"role": "user", "content": [{"type": "text", "text": "Convert."},
                                         {"type": "image_url", "image_url": {"url": _data_url(png)}}]}]
    prompt, images = server.convert_messages(msgs)
    # parts visited in reverse: image first, then text on a new line; system text precedes
    assert prompt == "be precise\n\n<image>\nConvert."
    assert len(images) == 1 and images[0].size == (60, 40)
    p2, im2 = server.convert_messages([{"role": "user", "content": [
        {"type": "input_image", "image_url": _data_url(png)}, {"type": "input_text", "text": "x"}]}])
    assert p2 == "x<image>" and len(im2) == 1  # an image part appends no separator (generation.rs:244-247)


@pytest.mark.parametrize("msgs,needle", [
    ([], "at least one user message"),
    ([{"role": "assistant", "content": "hi"}], "at least one user message"),
    ([{"role": "user", "content": "   "}], "must include text or images"),
    ([{"role": "user", "content": [{"type": "image_url", "image_url": "data:image/png,abc"}]}], "base64 encoding"),
    ([{"role": "user", "content": [{"type": "image_url", "image_url": "data:image/png;base64,@@@"}]}], "invalid base64"),
    ([{"role": "user", "content": [{"type": "image_url", "image_url": "data:image/png;base64,AAAA"}]}],
     "failed to decode inline image"),
    ([{"role": "user", "content": [{"type": "image_url", "image_url": "ftp://x/y.png"}]}], "only data: URIs"),
    ([{"role": "user", "content": [{"type": "image_url", "image_url": "https://x/y.png"}]}], "failed to fetch"),
])
def test_convert_messages_errors_are_400(msgs, needle):
    with pytest.raises(server.ApiError) as e:
        server.convert_messages(msgs)
    assert e.value.status == 400 and needle in e.value.message


def test_merge_decode_precedence():
    d = DecodeParameters()
    p = server.merge_decode(d, {"max_new_tokens": 7, "no_repeat_ngram_size": 3}, 100)
    assert p.max_new_tokens == 7 and p.no_repeat_ngram_size == 3  # patch applies after max_tokens
    assert server.merge_decode(d, {}, 33).max_new_tokens == 33
    assert server.merge_decode(d, {}, None).max_new_tokens == 512


# ---------------------------------------------------------------- routes.rs over a stand-in engine
@pytest.fixture()
def client_engine():
    from starlette.testclient import TestClient
    eng = FakeEngine()
    st = server.ServerState(eng, SyntheticTokenizer(512), "deepseek-ocr", VisionSettings(256, 128, True),
                            DecodeParameters(max_new_tokens=64))
    return TestClient(server.create_app(st)), eng, st


def _sse(text):
    out = []
    for block in text.split("\n\n"):
        if block.startswith("data: "):
            d = block[6:]
            out.append(d if d == "[DONE]" else json.loads(d))
    return out


def test_health_and_models(client_engine):
    c, _, _ = client_engine
    assert c.get("/v1/health").text == "ok"
    m = c.get("/v1/models").json()
    assert m["object"] == "list" and m["data"][0]["id"] == "deepseek-ocr"
    assert m["data"][0]["owned_by"] == "deepseek-ocr"
    assert c.options("/v1/models").status_code == 200


def test_chat_completion_json(client_engine):
    c, eng, _ = client_engine
    png, _ = _png_bytes()
    r = c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "max_tokens": 5, "messages": [
        {"role": "user", "content": [{"type": "text", "text": "OCR"},
                                     {"type": "image_url", "image_url": {"url": _data_url(png)}}]}]})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["object"] == "chat.completion" and body["choices"][0]["finish_reason"] == "stop"
    assert body["choices"][0]["message"]["content"] == "<20> <21> <22>"
    assert body["usage"] == {"prompt_tokens": 10, "completion_tokens": 3, "total_tokens": 13}
    assert eng.calls[0]["prompt"] == "<image>\nOCR" and eng.calls[0]["params"].max_new_tokens == 5


def test_responses_json_max_output_tokens(client_engine):
    c, eng, _ = client_engine
    png, _ = _png_bytes()
    r = c.post("/v1/responses", json={"model": "deepseek-ocr", "max_output_tokens": 9, "max_tokens": 4,
                                      "input": [{"role": "user", "content": [
                                          {"type": "input_image", "image_url": _data_url(png)}]}]})
    body = r.json()
    assert r.status_code == 200 and body["object"] == "response"
    assert body["output"][0]["content"][0] == {"type": "output_text", "text": "<20> <21> <22>"}
    assert eng.calls[0]["params"].max_new_tokens == 9


def test_chat_stream_event_sequence(client_engine):
    c, _, _ = client_engine
    png, _ = _png_bytes()
    r = c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "stream": True, "messages": [
        {"role": "user", "content": [{"type": "image_url", "image_url": {"url": _data_url(png)}}]}]})
    ev = _sse(r.text)
    assert ev[-1] == "[DONE]"
    assert ev[0]["choices"][0]["delta"] == {"role": "assistant"}
    text = "".join(e["choices"][0]["delta"].get("content", "") for e in ev[1:-1])
    assert text == "<20> <21> <22>"
    assert ev[-2]["choices"][0]["finish_reason"] == "stop" and ev[-2]["usage"]["completion_tokens"] == 3


def test_responses_stream_event_sequence(client_engine):
    c, _, _ = client_engine
    png, _ = _png_bytes()
    r = c.post("/v1/responses", json={"model": "deepseek-ocr", "stream": True, "input": [
        {"role": "user", "content": [{"type": "input_image", "image_url": _data_url(png)}]}]})
    ev = _sse(r.text)
    assert ev[0]["type"] == "response.created" and ev[-1] == "[DONE]"
    assert ev[-2]["type"] == "response.completed"
    assert ev[-2]["response"]["usage"] == {"input_tokens": 10, "output_tokens": 3, "total_tokens": 13}
    assert "".join(e["delta"] for e in ev if isinstance(e, dict) and e.get("type") ==
                   "response.output_text.delta") == "<20> <21> <22>"


def test_missing_image_fallback(client_engine):
    c, eng, _ = client_engine
    r = c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "messages": [{"role": "user", "content": "hi"}]})
    assert r.status_code == 200 and "Image Required" in r.json()["choices"][0]["message"]["content"]
    assert r.json()["usage"]["total_tokens"] == 0 and not eng.calls
    ev = _sse(c.post("/v1/responses", json={"model": "deepseek-ocr", "stream": True,
                                            "input": [{"role": "user", "content": "hi"}]}).text)
    assert ev[-1] == "[DONE]" and "Image Required" in ev[1]["delta"]


def test_error_classes(client_engine):
    c, eng, _ = client_engine
    png, _ = _png_bytes()
    msg = [{"role": "user", "content": [{"type": "image_url", "image_url": {"url": _data_url(png)}}]}]
    r = c.post("/v1/chat/completions", json={"model": "other", "messages": msg})
    assert r.status_code == 400 and r.json()["error"]["type"] == "invalid_request_error"
    assert "`other` is not available" in r.json()["error"]["message"]
    eng.error = DsocrError(1, "prompt formatting failed: prompt/image embedding mismatch")
    assert c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "messages": msg}).status_code == 400
    eng.error = DsocrError(6, "device lost")
    r = c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "messages": msg})
    assert r.status_code == 500 and r.json()["error"]["type"] == "internal_error"
    eng.error = None
    eng.tokens = []
    r = c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "messages": msg})
    assert r.status_code == 500 and "empty output" in r.json()["error"]["message"]


# ---------------------------------------------------------------- cli (args.rs / app.rs)
def test_cli_parser_and_device():
    a = cli.build_parser().parse_args(["--prompt", "<image>\nx", "--image", "a.png", "--crop-mode", "false",
                                       "--max-new-tokens", "7", "--device", "cuda:1"])
    assert a.images == ["a.png"] and a.crop_mode is False and a.max_new_tokens == 7
    assert cli.parse_device(a.device) == 1 and cli.parse_device("hip") == 0
    with pytest.raises(DsocrError):
        cli.parse_device("cpu")
    with pytest.raises(SystemExit):
        cli.build_parser().parse_args(["--prompt", "a", "--prompt-file", "b"])
    with pytest.raises(DsocrError, match="prompt is required"):
        cli.load_prompt(cli.build_parser().parse_args([]))


def _run_cli(monkeypatch, argv, eng):
    monkeypatch.setattr(cli, "load_model", lambda la: eng)
    out, err = io.StringIO(), io.StringIO()
    rc = cli.run_inference(cli.build_parser().parse_args(argv), out, err)
    return rc, out.getvalue(), err.getvalue()


def test_cli_stream_and_bench(monkeypatch, tmp_path):
    png, _ = _png_bytes()
    p = tmp_path / "page.png"
    p.write_bytes(png)
    bo = tmp_path / "b" / "bench.json"
    eng = FakeEngine()
    rc, out, err = _run_cli(monkeypatch, ["--model-config", TINY, "--prompt", "<image>\nConvert.", "--image", str(p),
                                          "--bench", "--bench-output", str(bo)], eng)
    assert rc == 0 and out == "<20> <21> <22>\n" and eng.closed
    assert "Throughput: prefill=10 tok" in err and "[bench] decode.iterative" in err
    rep = json.loads(bo.read_text())
    stages = {s["stage"]: s for s in rep["stage_totals"]}
    assert stages["decode.iterative"]["total_ms"] == 4.0 and stages["vision.compute_embeddings"]["count"] == 1
    assert "model.load" in stages
    assert eng.calls[0]["images"][0].size == (60, 40)


def test_cli_quiet_and_slot_mismatch(monkeypatch, tmp_path):
    png, _ = _png_bytes()
    p = tmp_path / "page.png"
    p.write_bytes(png)
    rc, out, err = _run_cli(monkeypatch, ["--model-config", TINY, "-q", "--prompt", "<image>x", "--image", str(p)],
                            FakeEngine())
    assert out == "<20> <21> <22>\n" and err == ""
    eng = FakeEngine()
    with pytest.raises(DsocrError, match="prompt includes 2 <image> tokens but 1 image paths"):
        _run_cli(monkeypatch, ["--model-config", TINY, "--prompt", "<image><image>", "--image", str(p)], eng)
    assert eng.closed
    with pytest.raises(DsocrError, match="failed to open image"):
        _run_cli(monkeypatch, ["--model-config", TINY, "--prompt", "<image>", "--image", str(tmp_path / "no.png")],
                 FakeEngine())


# ---------------------------------------------------------------- the same bridges over the MI355X engine
def _oracle_ids(img, prompt, max_new, **sampling):
    from oracle.model import OracleModel
    from oracle.weights import Weights
    from dsocr import Page, build_prompt_tokens
    orc = OracleModel(json.load(open(TINY)), Weights(seed=7, dtype="f16"))
    vs = VisionSettings(256, 128, True)
    ids, mask = build_prompt_tokens(SyntheticTokenizer(512), prompt, [Page(img, vs).n_image_tokens])
    emb, _ = orc.image_embeddings(img, 256, 128, True)
    ref, _ = orc.generate(ids, mask, emb, max_new, eos_token_id=1, **sampling)
    return ref


@pytest.mark.gpu
def test_gpu_cli_matches_oracle(gpu, tmp_path):
    png, arr = _png_bytes(300, 420, seed=3)
    p = tmp_path / "page.png"
    p.write_bytes(png)
    out = io.StringIO()
    args = cli.build_parser().parse_args(["--model-config", TINY, "--synthetic-seed", "7", "--prompt",
                                          "<image>\nConvert the document to markdown.", "--image", str(p),
                                          "--base-size", "256", "--image-size", "128", "--max-new-tokens", "12",
                                          "-q"])
    assert cli.run_inference(args, out, io.StringIO()) == 0
    ref = _oracle_ids(arr, "<image>\nConvert the document to markdown.", 12)
    assert out.getvalue() == SyntheticTokenizer(512).decode(ref) + "\n"


@pytest.mark.gpu
def test_gpu_server_chat_matches_oracle(gpu):
    from starlette.testclient import TestClient
    from dsocr import ModelLoadArgs, load_model
    png, arr = _png_bytes(256, 256, seed=5)
    eng = load_model(ModelLoadArgs(config_path=TINY, synthetic_seed=7, dtype="f16"))
    try:
        st = server.ServerState(eng, SyntheticTokenizer(512), "deepseek-ocr", VisionSettings(256, 128, True),
                                DecodeParameters(max_new_tokens=10))
        c = TestClient(server.create_app(st))
        msg = [{"role": "user", "content": [{"type": "text", "text": "Convert the document to markdown."},
                                            {"type": "image_url", "image_url": {"url": _data_url(png)}}]}]
        body = c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "messages": msg}).json()
        ref = _oracle_ids(arr, "<image>\nConvert the document to markdown.", 10)
        assert body["choices"][0]["message"]["content"] == SyntheticTokenizer(512).decode(ref)
        ev = _sse(c.post("/v1/chat/completions", json={"model": "deepseek-ocr", "messages": msg,
                                                       "stream": True}).text)
        assert "".join(e["choices"][0]["delta"].get("content", "") for e in ev[1:-1]) == \
            SyntheticTokenizer(512).decode(ref)
        # sampling fields flatten into the request (DecodeParametersPatch), seeded -> reproducible
        req = {"model": "deepseek-ocr", "messages": msg, "do_sample": True, "temperature": 0.7, "top_k": 30,
               "seed": 99}
        r = c.post("/v1/chat/completions", json=req)
        assert r.status_code == 200
        ref = _oracle_ids(arr, "<image>\nConvert the document to markdown.", 10, do_sample=True, temperature=0.7,
                          top_k=30, top_p=None, seed=99)
        assert r.json()["choices"][0]["message"]["content"] == SyntheticTokenizer(512).decode(ref)
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_decode_two_images_matches_oracle(gpu):
    """OcrEngine::decode with two <image> slots: rows of both pages injected in image order."""
    from dsocr import ModelLoadArgs, Page, build_prompt_tokens, load_model
    from oracle.model import OracleModel
    from oracle.weights import Weights
    vs = VisionSettings(256, 128, True)
    a = np.random.default_rng(21).integers(0, 256, (300, 420, 3), dtype=np.uint8)
    b = np.random.default_rng(22).integers(0, 256, (200, 200, 3), dtype=np.uint8)
    prompt = "<image>\nfirst page\n<image>\nsecond page"
    tok = SyntheticTokenizer(512)
    eng = load_model(ModelLoadArgs(config_path=TINY, synthetic_seed=7, dtype="f16"))
    try:
        out = eng.decode(tok, prompt, [a, b], vs, DecodeParameters(max_new_tokens=12))
    finally:
        eng.close()
    orc = OracleModel(json.load(open(TINY)), Weights(seed=7, dtype="f16"))
    ids, mask = build_prompt_tokens(tok, prompt, [Page(a, vs).n_image_tokens, Page(b, vs).n_image_tokens])
    rows = np.concatenate([orc.image_embeddings(x, 256, 128, True)[0] for x in (a, b)], axis=0)
    ref, _ = orc.generate(ids, mask, rows, 12, eos_token_id=1)
    assert out.generated_tokens == ref and out.prompt_tokens == len(ids)
