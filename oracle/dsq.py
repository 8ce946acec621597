"""Oracle: DSQ snapshot container + GGML block dequantisation (TEST INFRASTRUCTURE).

Restates, for the parity tests only:
  * the `.dsq` container (crates/dsq/src/lib.rs): magic ``DSQSNAP`` (14), version 1 (15),
    u32-length strings (521-528), header = candle_version / model_id / backend / default qdtype
    u32 / block_size u32 / tensor_count u32 (314-339), records = name / out_dim u32 / in_dim u32 /
    q_dtype u32 / q_offset u64 / q_len u64 / bias_offset u64 / bias_len u64 / bias_dtype u32
    (341-369; bias_len 0 = no bias), and the validation rules (393-519).  The writer layout
    (crates/dsq-writer/src/lib.rs:410-531: header, records with payload offsets shifted by the
    metadata length, payload) is restated by :func:`write_dsq`.
  * dtype codes (lib.rs:60-110): Q8_0 = 8, Q4_K = 12, Q6_K = 14, F16 = 1, BF16 = 16, F32 = 0;
    bias codes (137-168): U8 0, U32 1, I64 2, F16 3, F32 4, F64 5, BF16 6.
  * block dequantisation as Candle's k-quants ``to_float`` computes it (third-party candle-core
    0.9.2, not vendored; the GGML block layouts it mirrors): Q4_K 256 elements / 144 bytes
    (d f16, dmin f16, 12 packed 6-bit scale/min bytes, 128 nibble bytes; y = (d*sc)*q - dmin*m),
    Q6_K 256 / 210 (ql[128], qh[64], int8 scales[16], d f16; y = (d*sc)*q), Q8_0 32 / 34
    (d f16, int8 qs[32]; y = d*q).  Every product / difference is one IEEE f32 operation in that
    order (no fused multiply-add), as the Rust code evaluates it.
  * the reference writer's Q8_0 quantiser (dsq-writer/src/lib.rs:555-598).  Q4_K / Q6_K encoders
    here are this repo's own (the reference encodes through Candle's ``from_float``, which is not
    available offline): any valid block decodes the same way, and the tests only need encodings.

Parity status: the reference's own DSQ tests need Rust + Candle (dsq-writer/tests/writer.rs) and
there is no GGML implementation in this image, so block decoding is **parity unpinned** against
the reference; it is pinned by exact round trips of this file's encoders and by the documented
layout.  The GPU dequantiser (csrc/kernels/dsq.hip) must match this module bit for bit.
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC = b"DSQSNAP"
VERSION = 1
Q8_0, Q4K, Q6K, F16, BF16, F32 = 8, 12, 14, 1, 16, 0
BLOCK = {Q8_0: 32, Q4K: 256, Q6K: 256}
BLOCK_BYTES = {Q8_0: 34, Q4K: 144, Q6K: 210}
ELEM = {F16: 2, BF16: 2, F32: 4}
BIAS_U8, BIAS_U32, BIAS_I64, BIAS_F16, BIAS_F32, BIAS_F64, BIAS_BF16 = 0, 1, 2, 3, 4, 5, 6
_BIAS_NP = {BIAS_U8: np.uint8, BIAS_U32: np.uint32, BIAS_I64: np.int64, BIAS_F16: np.float16,
            BIAS_F32: np.float32, BIAS_F64: np.float64}


class DsqError(ValueError):
    pass


def payload_bytes(qtype: int, out_dim: int, in_dim: int) -> int:
    if qtype in BLOCK:
        return out_dim * (in_dim // BLOCK[qtype]) * BLOCK_BYTES[qtype]
    return out_dim * in_dim * ELEM[qtype]


# ------------------------------------------------------------------ container
def parse_dsq(buf: bytes):
    """(header dict, [record dict]) with lib.rs's validation; raises DsqError."""
    mv = memoryview(buf)
    pos = 0

    def take(n):
        nonlocal pos
        if pos + n > len(mv):
            raise DsqError("truncated snapshot")
        out = bytes(mv[pos:pos + n])
        pos += n
        return out

    def u32():
        return struct.unpack("<I", take(4))[0]

    def u64():
        return struct.unpack("<Q", take(8))[0]

    def string():
        n = u32()
        return take(n).decode("utf-8")

    magic = take(7)
    if magic != MAGIC:
        raise DsqError(f"invalid snapshot magic: found {magic!r}")
    version = u32()
    if version != VERSION:
        raise DsqError(f"unsupported snapshot version {version}, expected {VERSION}")
    hdr = {"version": version, "candle_version": string(), "model_id": string(), "backend": string()}
    hdr["default_qdtype"] = _dtype(u32())
    hdr["block_size"] = u32()
    if hdr["block_size"] == 0:
        raise DsqError("block_size must be non-zero")
    count = u32()
    hdr["tensor_count"] = count
    recs = []
    for _ in range(count):
        r = {"name": string(), "out_dim": u32(), "in_dim": u32(), "q_dtype": _dtype(u32()),
             "q_offset": u64(), "q_len": u64()}
        boff, blen, bdt = u64(), u64(), u32()
        if blen == 0:
            r["bias_offset"] = r["bias_len"] = r["bias_dtype"] = None
        else:
            if bdt not in (0, 1, 2, 3, 4, 5, 6):
                raise DsqError(f"unsupported bias dtype code {bdt}")
            r["bias_offset"], r["bias_len"], r["bias_dtype"] = boff, blen, bdt
        recs.append(r)
    meta = pos
    # validate_header (lib.rs:393-407)
    if hdr["default_qdtype"] not in BLOCK:
        raise DsqError(f"snapshot dtype {hdr['default_qdtype']} not supported")
    if hdr["block_size"] != BLOCK[hdr["default_qdtype"]]:
        raise DsqError(f"snapshot block size {hdr['block_size']} mismatches expected "
                       f"{BLOCK[hdr['default_qdtype']]}")
    # validate_records (lib.rs:409-494)
    total = len(mv)
    names = set()
    for r in recs:
        if r["q_len"] == 0:
            raise DsqError(f"tensor `{r['name']}` has empty quantized payload")
        if r["q_offset"] < meta:
            raise DsqError(f"tensor `{r['name']}` q_offset {r['q_offset']} overlaps metadata ({meta} bytes)")
        if r["q_offset"] + r["q_len"] > total:
            raise DsqError(f"tensor `{r['name']}` quantized slice exceeds file size {total}")
        if r["bias_len"] is not None and r["bias_offset"] + r["bias_len"] > total:
            raise DsqError(f"tensor `{r['name']}` bias slice exceeds file size {total}")
        q = r["q_dtype"]
        if q in BLOCK:
            if r["in_dim"] % BLOCK[q]:
                raise DsqError(f"tensor `{r['name']}` in_dim {r['in_dim']} not divisible by block_size {BLOCK[q]}")
        elif r["q_len"] != r["out_dim"] * r["in_dim"] * ELEM[q]:
            raise DsqError(f"tensor `{r['name']}` has q_len {r['q_len']} but expected "
                           f"{r['out_dim'] * r['in_dim'] * ELEM[q]} bytes")
        if r["name"] in names:
            raise DsqError(f"duplicate tensor record `{r['name']}`")
        names.add(r["name"])
    return hdr, recs


def _dtype(code: int) -> int:
    if code not in (Q8_0, Q4K, Q6K, F16, BF16, F32):
        raise DsqError(f"unsupported tensor dtype code {code}")
    return code


def write_dsq(path: str, tensors, default_qdtype: int = Q4K, candle_version="dsocr-test",
              model_id="deepseek-ocr", backend="HIP") -> None:
    """tensors: [(name, out_dim, in_dim, qtype, payload bytes, bias f32 array | None)]."""
    payload = bytearray()
    pending = []
    for name, out_dim, in_dim, qtype, qbytes, bias in tensors:
        qoff = len(payload)
        payload += qbytes
        b = None
        if bias is not None:
            bb = np.asarray(bias, dtype="<f4").tobytes()
            b = (len(payload), len(bb), BIAS_F32)
            payload += bb
        pending.append((name, out_dim, in_dim, qtype, qoff, len(qbytes), b))

    def s(v):
        e = v.encode()
        return struct.pack("<I", len(e)) + e

    head = MAGIC + struct.pack("<I", VERSION) + s(candle_version) + s(model_id) + s(backend)
    head += struct.pack("<III", default_qdtype, BLOCK[default_qdtype], len(pending))
    meta = len(head) + sum(52 + len(p[0].encode()) for p in pending)
    recs = bytearray()
    for name, out_dim, in_dim, qtype, qoff, qlen, b in pending:
        recs += s(name) + struct.pack("<IIIQQ", out_dim, in_dim, qtype, qoff + meta, qlen)
        recs += struct.pack("<QQI", b[0] + meta, b[1], b[2]) if b else struct.pack("<QQI", 0, 0, 0)
    assert len(head) + len(recs) == meta
    with open(path, "wb") as f:
        f.write(head)
        f.write(recs)
        f.write(payload)


def record_payload(buf: bytes, r) -> bytes:
    return bytes(memoryview(buf)[r["q_offset"]:r["q_offset"] + r["q_len"]])


def record_bias(buf: bytes, r):
    if r["bias_len"] is None:
        return None
    raw = bytes(memoryview(buf)[r["bias_offset"]:r["bias_offset"] + r["bias_len"]])
    if r["bias_dtype"] == BIAS_BF16:
        return (np.frombuffer(raw, "<u2").astype(np.uint32) << 16).view(np.float32)
    return np.frombuffer(raw, np.dtype(_BIAS_NP[r["bias_dtype"]]).newbyteorder("<")).astype(np.float32)


# ------------------------------------------------------------------ dequantisation (f32, Candle's order)
def _f16(raw: np.ndarray) -> np.ndarray:
    return raw.view("<f2").astype(np.float32)


def _scale_min_k4(sc: np.ndarray, j: int):
    """get_scale_min_k4 over a [nblocks, 12] byte array (GGML k-quants)."""
    if j < 4:
        d = sc[:, j] & 63
        m = sc[:, j + 4] & 63
    else:
        d = (sc[:, j + 4] & 0xF) | ((sc[:, j - 4] >> 6) << 4)
        m = (sc[:, j + 4] >> 4) | ((sc[:, j] >> 6) << 4)
    return d.astype(np.float32), m.astype(np.float32)


def dequant_q4k(payload: bytes, rows: int, cols: int) -> np.ndarray:
    b = np.frombuffer(payload, np.uint8).reshape(-1, 144)
    d, dmin = _f16(b[:, 0:2].copy()).ravel(), _f16(b[:, 2:4].copy()).ravel()
    sc, qs = b[:, 4:16], b[:, 16:144]
    out = np.empty((b.shape[0], 256), np.float32)
    for c in range(4):  # 64-element chunks
        q = qs[:, 32 * c:32 * c + 32]
        s1, m1 = _scale_min_k4(sc, 2 * c)
        s2, m2 = _scale_min_k4(sc, 2 * c + 1)
        d1, mm1 = (d * s1)[:, None], (dmin * m1)[:, None]
        d2, mm2 = (d * s2)[:, None], (dmin * m2)[:, None]
        out[:, 64 * c:64 * c + 32] = d1 * (q & 0xF).astype(np.float32) - mm1
        out[:, 64 * c + 32:64 * c + 64] = d2 * (q >> 4).astype(np.float32) - mm2
    return out.reshape(rows, cols)


def dequant_q6k(payload: bytes, rows: int, cols: int) -> np.ndarray:
    b = np.frombuffer(payload, np.uint8).reshape(-1, 210)
    ql, qh = b[:, 0:128], b[:, 128:192]
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = _f16(b[:, 208:210].copy()).ravel()[:, None]
    out = np.empty((b.shape[0], 256), np.float32)
    for n in range(2):
        L, H, S = ql[:, 64 * n:64 * n + 64], qh[:, 32 * n:32 * n + 32], sc[:, 8 * n:8 * n + 8]
        q1 = ((L[:, :32] & 0xF) | (((H >> 0) & 3) << 4)).astype(np.int32) - 32
        q2 = ((L[:, 32:] & 0xF) | (((H >> 2) & 3) << 4)).astype(np.int32) - 32
        q3 = ((L[:, :32] >> 4) | (((H >> 4) & 3) << 4)).astype(np.int32) - 32
        q4 = ((L[:, 32:] >> 4) | (((H >> 6) & 3) << 4)).astype(np.int32) - 32
        isx = np.arange(32) // 16
        for k, q in enumerate((q1, q2, q3, q4)):
            s = S[:, isx + 2 * k]
            out[:, 128 * n + 32 * k:128 * n + 32 * k + 32] = (d * s) * q.astype(np.float32)
    return out.reshape(rows, cols)


def dequant_q8_0(payload: bytes, rows: int, cols: int) -> np.ndarray:
    b = np.frombuffer(payload, np.uint8).reshape(-1, 34)
    d = _f16(b[:, 0:2].copy()).ravel()[:, None]
    return (d * b[:, 2:].view(np.int8).astype(np.float32)).reshape(rows, cols)


def dequant(qtype: int, payload: bytes, rows: int, cols: int) -> np.ndarray:
    if qtype == Q4K:
        return dequant_q4k(payload, rows, cols)
    if qtype == Q6K:
        return dequant_q6k(payload, rows, cols)
    if qtype == Q8_0:
        return dequant_q8_0(payload, rows, cols)
    if qtype == F16:
        return np.frombuffer(payload, "<f2").astype(np.float32).reshape(rows, cols)
    if qtype == BF16:
        return (np.frombuffer(payload, "<u2").astype(np.uint32) << 16).view(np.float32).reshape(rows, cols)
    if qtype == F32:
        return np.frombuffer(payload, "<f4").astype(np.float32).reshape(rows, cols)
    raise DsqError(f"unsupported tensor dtype code {qtype}")


# ------------------------------------------------------------------ encoders
def quantize_q8_0(w: np.ndarray) -> bytes:
    """The reference writer's Q8_0 (dsq-writer/src/lib.rs:555-598): f16(amax/127), round half
    away from zero of value * (1/scale) with the f32 scale, clamp [-128, 127]."""
    w = np.asarray(w, np.float32).reshape(-1, 32)
    amax = np.abs(w).max(axis=1)
    scale = np.where(amax > 0, amax / np.float32(127.0), np.float32(0.0)).astype(np.float32)
    out = np.zeros((w.shape[0], 34), np.uint8)
    out[:, 0:2] = scale.astype("<f2").view(np.uint8).reshape(-1, 2)
    inv = np.where(scale > 0, np.float32(1.0) / np.where(scale > 0, scale, 1), 0).astype(np.float32)
    v = w * inv[:, None]
    q = np.clip(np.sign(v) * np.floor(np.abs(v) + np.float32(0.5)), -128, 127).astype(np.int8)
    q[scale == 0] = 0
    out[:, 2:] = q.view(np.uint8)
    return out.tobytes()


def quantize_q4k(w: np.ndarray) -> bytes:
    """This repo's Q4_K encoder (min/max per 32-element sub-block, 6-bit scale / min codes
    against per-block f16 d / dmin).  Produces valid blocks; not Candle's from_float."""
    w = np.asarray(w, np.float32).reshape(-1, 256)
    nb = w.shape[0]
    sub = w.reshape(nb, 8, 32)
    lo = np.minimum(sub.min(axis=2), 0.0)
    hi = sub.max(axis=2)
    step = np.maximum((hi - lo) / 15.0, 1e-12).astype(np.float32)   # per sub-block scale
    mins = (-lo).astype(np.float32)                                    # per sub-block min (>= 0)
    d = (step.max(axis=1) / 63.0).astype(np.float16)
    dmin = (mins.max(axis=1) / 63.0).astype(np.float16)
    df, dmf = d.astype(np.float32), dmin.astype(np.float32)
    sc = np.clip(np.rint(step / np.where(df > 0, df, 1)[:, None]), 0, 63).astype(np.uint8)
    mc = np.clip(np.rint(mins / np.where(dmf > 0, dmf, 1)[:, None]), 0, 63).astype(np.uint8)
    scales = np.zeros((nb, 12), np.uint8)
    scales[:, 0:4] = sc[:, 0:4] | ((sc[:, 4:8] >> 4) << 6)
    scales[:, 4:8] = mc[:, 0:4] | ((mc[:, 4:8] >> 4) << 6)
    scales[:, 8:12] = (sc[:, 4:8] & 0xF) | ((mc[:, 4:8] & 0xF) << 4)
    dd = (df[:, None] * sc.astype(np.float32))                          # decoded sub-block scales
    mm = (dmf[:, None] * mc.astype(np.float32))
    q = np.clip(np.rint((sub + mm[:, :, None]) / np.where(dd > 0, dd, 1)[:, :, None]), 0, 15).astype(np.uint8)
    qs = np.zeros((nb, 128), np.uint8)
    for c in range(4):
        qs[:, 32 * c:32 * c + 32] = q[:, 2 * c] | (q[:, 2 * c + 1] << 4)
    out = np.zeros((nb, 144), np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dmin.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = scales
    out[:, 16:] = qs
    return out.tobytes()


def quantize_q6k(w: np.ndarray) -> bytes:
    """This repo's Q6_K encoder (absmax per 16-element group, int8 scales against f16 d)."""
    w = np.asarray(w, np.float32).reshape(-1, 256)
    nb = w.shape[0]
    g = w.reshape(nb, 16, 16)
    gs = (np.abs(g).max(axis=2) / 31.0).astype(np.float32)
    d = (gs.max(axis=1) / 127.0).astype(np.float16)
    df = d.astype(np.float32)
    sc = np.clip(np.rint(gs / np.where(df > 0, df, 1)[:, None]), -128, 127).astype(np.int8)
    ds = df[:, None] * sc.astype(np.float32)
    q = (np.clip(np.rint(g / np.where(ds != 0, ds, 1)[:, :, None]), -32, 31).astype(np.int32) + 32).reshape(nb, 256)
    ql = np.zeros((nb, 128), np.uint8)
    qh = np.zeros((nb, 64), np.uint8)
    for n in range(2):
        Q = q[:, 128 * n:128 * n + 128]
        q1, q2, q3, q4 = Q[:, 0:32], Q[:, 32:64], Q[:, 64:96], Q[:, 96:128]
        ql[:, 64 * n:64 * n + 32] = (q1 & 0xF) | ((q3 & 0xF) << 4)
        ql[:, 64 * n + 32:64 * n + 64] = (q2 & 0xF) | ((q4 & 0xF) << 4)
        qh[:, 32 * n:32 * n + 32] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
    out = np.zeros((nb, 210), np.uint8)
    out[:, 0:128] = ql
    out[:, 128:192] = qh
    out[:, 192:208] = sc.view(np.uint8)
    out[:, 208:210] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    return out.tobytes()


def quantize(qtype: int, w: np.ndarray) -> bytes:
    w = np.asarray(w, np.float32)
    if qtype == Q4K:
        return quantize_q4k(w)
    if qtype == Q6K:
        return quantize_q6k(w)
    if qtype == Q8_0:
        return quantize_q8_0(w)
    if qtype == F16:
        return w.astype("<f2").tobytes()
    if qtype == F32:
        return w.astype("<f4").tobytes()
    if qtype == BF16:
        b = w.view(np.uint32)
        r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16).astype("<u2")  # RNE
        return r.tobytes()
    raise DsqError(f"unsupported tensor dtype code {qtype}")


class Snapshot:
    """A parsed snapshot file: name -> dequantised f32 (cached), biases."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            self.buf = f.read()
        self.header, recs = parse_dsq(self.buf)
        self.records = {r["name"]: r for r in recs}
        self._cache = {}

    def has(self, name: str) -> bool:
        return name in self.records

    def weight(self, name: str) -> np.ndarray:
        if name not in self._cache:
            r = self.records[name]
            self._cache[name] = dequant(r["q_dtype"], record_payload(self.buf, r), r["out_dim"], r["in_dim"])
        return self._cache[name]

    def bias_for(self, weight_name: str):
        r = self.records.get(weight_name)
        return None if r is None else record_bias(self.buf, r)


# ------------------------------------------------------------------ which linears a snapshot holds
def discover_linears(cfg: dict, include_projector: bool = True):
    """(name, out_dim, in_dim, bias name) of every linear the reference's DeepSeek-OCR adapter
    puts in a snapshot (crates/dsq-models/src/adapters/deepseek_ocr.rs:41-140): q/k/v/o per layer,
    routed experts + fused shared experts on MoE layers (should_use_moe 160-168), the dense MLP
    otherwise, lm_head (unless ``lm_head`` is false), the projector."""
    lang = cfg.get("language_config", cfg)
    H, nl, nh = lang["hidden_size"], lang["num_hidden_layers"], lang["num_attention_heads"]
    nkv = lang.get("num_key_value_heads") or nh
    hd = H // nh
    vhd = lang.get("v_head_dim") or hd
    inter = lang["intermediate_size"]
    moe_i = lang.get("moe_intermediate_size") or inter
    n_routed = lang.get("n_routed_experts") or 0
    n_shared = lang.get("n_shared_experts") or 0
    freq = lang.get("moe_layer_freq") or 1
    first_dense = lang.get("first_k_dense_replace") or 0
    out = []

    def mlp(prefix, inner):
        return [(f"{prefix}.gate_proj.weight", inner, H, f"{prefix}.gate_proj.bias"),
                (f"{prefix}.up_proj.weight", inner, H, f"{prefix}.up_proj.bias"),
                (f"{prefix}.down_proj.weight", H, inner, f"{prefix}.down_proj.bias")]

    for l in range(nl):
        a = f"model.layers.{l}.self_attn"
        out += [(f"{a}.q_proj.weight", nh * hd, H, f"{a}.q_proj.bias"),
                (f"{a}.k_proj.weight", nkv * hd, H, f"{a}.k_proj.bias"),
                (f"{a}.v_proj.weight", nkv * vhd, H, f"{a}.v_proj.bias"),
                (f"{a}.o_proj.weight", H, nh * vhd, f"{a}.o_proj.bias")]
        m = f"model.layers.{l}.mlp"
        if n_routed and l >= first_dense and freq and l % freq == 0:
            for e in range(n_routed):
                out += mlp(f"{m}.experts.{e}", moe_i)
            if n_shared:
                out += mlp(f"{m}.shared_experts", moe_i * n_shared)
        else:
            out += mlp(m, inter)
    if lang.get("lm_head", True):
        out.append(("lm_head.weight", lang["vocab_size"], H, None))
    if include_projector:
        p = cfg["projector_config"]
        out.append(("model.projector.layers.weight", p["n_embed"], p["input_dim"], "model.projector.layers.bias"))
    return out
