"""DSQ snapshots (BASELINE config 5: Q4_K snapshot, dequant-on-load -> fp16).

CPU (oracle / host): container layout and the reader's validation rules (crates/dsq/src/lib.rs),
block decoding cross-checked against a second, loop-level restatement of the GGML layouts, the
reference writer's Q8_0 rounding, encoder round trips, and the committed fixture
(tests/golden/dsq_small.dsq, made by tests/golden/make_dsq_fixture.py).
GPU: the HIP dequantiser (dsocr_k_dsq_dequant) equals the oracle bit for bit (fp16 RNE of the f32
value), and an engine loaded with a snapshot generates the oracle's ids (tiny256 config, every
dtype the snapshot format allows in one file).

Parity status: decoding is restated from the published GGML block layouts (Candle's k-quants);
the reference's own tests for it need Rust + Candle, so it is "parity unpinned" against the
reference (documented in DESIGN.md).
"""
import json
import os
import struct

import numpy as np
import pytest

from oracle import dsq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
TINY256 = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny256.json")
SEED = 11


# ------------------------------------------------------------------ loop-level restatement
def _f16(b0, b1):
    return float(np.frombuffer(bytes([b0, b1]), "<f2")[0])


def _loop_q4k(block: bytes):
    d, dmin = np.float32(_f16(block[0], block[1])), np.float32(_f16(block[2], block[3]))
    sc, qs = block[4:16], block[16:]
    out = []
    for j in range(8):
        if j < 4:
            s, m = sc[j] & 63, sc[j + 4] & 63
        else:
            s = (sc[j + 4] & 0xF) | ((sc[j - 4] >> 6) << 4)
            m = (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4)
        c, hi = j // 2, j % 2
        d1, m1 = np.float32(d * np.float32(s)), np.float32(dmin * np.float32(m))
        for l in range(32):
            q = qs[32 * c + l]
            nib = (q >> 4) if hi else (q & 0xF)
            out.append(np.float32(np.float32(d1 * np.float32(nib)) - m1))
    return np.array(out, np.float32)


def _loop_q6k(block: bytes):
    ql, qh, sc = block[0:128], block[128:192], np.frombuffer(block[192:208], np.int8)
    d = np.float32(_f16(block[208], block[209]))
    y = np.zeros(256, np.float32)
    for n in range(2):
        for l in range(32):
            isx = l // 16
            L, Hh, S = ql[64 * n:], qh[32 * n:], sc[8 * n:]
            q1 = ((L[l] & 0xF) | (((Hh[l] >> 0) & 3) << 4)) - 32
            q2 = ((L[l + 32] & 0xF) | (((Hh[l] >> 2) & 3) << 4)) - 32
            q3 = ((L[l] >> 4) | (((Hh[l] >> 4) & 3) << 4)) - 32
            q4 = ((L[l + 32] >> 4) | (((Hh[l] >> 6) & 3) << 4)) - 32
            for k, q in enumerate((q1, q2, q3, q4)):
                y[128 * n + 32 * k + l] = np.float32(np.float32(d * np.float32(S[isx + 2 * k])) * np.float32(q))
    return y


def _random_blocks(rng, qtype, nblocks):
    raw = rng.integers(0, 256, (nblocks, dsq.BLOCK_BYTES[qtype]), dtype=np.uint8)
    d = (rng.standard_normal(nblocks) * 0.01).astype(np.float16).view(np.uint8).reshape(-1, 2)
    if qtype == dsq.Q4K:
        raw[:, 0:2] = d
        raw[:, 2:4] = (np.abs(rng.standard_normal(nblocks)) * 0.01).astype(np.float16).view(np.uint8).reshape(-1, 2)
    elif qtype == dsq.Q6K:
        raw[:, 208:210] = d
    else:
        raw[:, 0:2] = d
    return raw.tobytes()


def test_dequant_matches_loop_restatement():
    rng = np.random.default_rng(0)
    for qtype, loop in ((dsq.Q4K, _loop_q4k), (dsq.Q6K, _loop_q6k)):
        raw = _random_blocks(rng, qtype, 6)
        got = dsq.dequant(qtype, raw, 3, 512).reshape(6, 256)
        nb = dsq.BLOCK_BYTES[qtype]
        for b in range(6):
            ref = loop(raw[b * nb:(b + 1) * nb])
            assert np.array_equal(got[b].view(np.uint32), ref.view(np.uint32)), (qtype, b)
    raw = _random_blocks(rng, dsq.Q8_0, 4)
    got = dsq.dequant(dsq.Q8_0, raw, 2, 64).reshape(4, 32)
    for b in range(4):
        blk = raw[b * 34:(b + 1) * 34]
        d = np.float32(_f16(blk[0], blk[1]))
        ref = np.array([np.float32(d * np.float32(v)) for v in np.frombuffer(blk[2:], np.int8)], np.float32)
        assert np.array_equal(got[b], ref)


def test_q4k_scale_packing_known_answer():
    # d = 1, dmin = 0.5; sub-block j gets scale code j+1 and min code 2j (j >= 4 uses the split
    # high-bit packing); every nibble = 3 -> y = (j+1)*3 - 0.5*2j
    blk = bytearray(144)
    blk[0:2] = np.float16(1.0).tobytes()
    blk[2:4] = np.float16(0.5).tobytes()
    sc = [j + 1 for j in range(8)]
    mn = [2 * j for j in range(8)]
    for j in range(8):
        if j < 4:
            blk[4 + j] = sc[j]
            blk[4 + j + 4] = mn[j]
        else:
            blk[4 + j + 4] = (sc[j] & 0xF) | ((mn[j] & 0xF) << 4)
            blk[4 + j - 4] |= (sc[j] >> 4) << 6
            blk[4 + j] |= (mn[j] >> 4) << 6
    for i in range(128):
        blk[16 + i] = 0x33
    y = dsq.dequant_q4k(bytes(blk), 1, 256)[0]
    for j in range(8):
        c, hi = j // 2, j % 2
        seg = y[64 * c + 32 * hi:64 * c + 32 * hi + 32]
        assert np.all(seg == np.float32((j + 1) * 3 - 0.5 * 2 * j)), j


def test_q8_0_writer_rounding():
    # amax 127 -> scale 1, values round half away from zero, zero block stays zero
    w = np.zeros((2, 32), np.float32)
    w[0, :4] = [127.0, -2.5, 2.5, 0.49]
    b = dsq.quantize_q8_0(w)
    assert len(b) == 68
    assert np.frombuffer(b[0:2], "<f2")[0] == 1.0
    q = np.frombuffer(b[2:34], np.int8)
    assert list(q[:4]) == [127, -3, 3, 0]
    assert b[34:] == bytes(34)


@pytest.mark.parametrize("qtype,tol", [(dsq.Q4K, 0.15), (dsq.Q6K, 0.04), (dsq.Q8_0, 0.01)])
def test_encoder_round_trip(qtype, tol):
    rng = np.random.default_rng(int(qtype))
    w = (rng.standard_normal((4, 512)) * 0.02).astype(np.float32)
    raw = dsq.quantize(qtype, w)
    assert len(raw) == dsq.payload_bytes(qtype, 4, 512)
    y = dsq.dequant(qtype, raw, 4, 512)
    assert np.mean(np.abs(y - w)) <= tol * np.mean(np.abs(w))


def _container(tmp_path, tensors, **kw):
    p = str(tmp_path / "s.dsq")
    dsq.write_dsq(p, tensors, **kw)
    return p, open(p, "rb").read()


def test_container_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    w = (rng.standard_normal((2, 256)) * 0.1).astype(np.float32)
    bias = np.array([0.25, -0.5], np.float32)
    p, buf = _container(tmp_path, [("a.weight", 2, 256, dsq.Q4K, dsq.quantize(dsq.Q4K, w), None),
                                   ("b.weight", 2, 256, dsq.F32, dsq.quantize(dsq.F32, w), bias)])
    hdr, recs = dsq.parse_dsq(buf)
    assert hdr["version"] == 1 and hdr["default_qdtype"] == dsq.Q4K and hdr["block_size"] == 256
    assert [r["name"] for r in recs] == ["a.weight", "b.weight"]
    assert recs[0]["q_len"] == 288 and recs[0]["bias_len"] is None
    assert recs[1]["bias_dtype"] == dsq.BIAS_F32
    s = dsq.Snapshot(p)
    assert np.array_equal(s.weight("b.weight"), w)
    assert np.array_equal(s.bias_for("b.weight"), bias)
    # metadata length = header + 52 + len(name) per record (dsq-writer/src/lib.rs:529-531)
    head = 7 + 4 + 3 * 4 + len(b"dsocr-test") + len(b"deepseek-ocr") + len(b"HIP") + 12
    assert recs[0]["q_offset"] == head + 52 + 8 + 52 + 8


def _patch(buf, off, fmt, val):
    b = bytearray(buf)
    struct.pack_into(fmt, b, off, val)
    return bytes(b)


def test_container_validation(tmp_path):
    w = np.zeros((1, 256), np.float32)
    p, buf = _container(tmp_path, [("a.weight", 1, 256, dsq.Q4K, dsq.quantize(dsq.Q4K, w), None)])
    with pytest.raises(dsq.DsqError, match="magic"):
        dsq.parse_dsq(b"XSQSNAP" + buf[7:])
    with pytest.raises(dsq.DsqError, match="version"):
        dsq.parse_dsq(_patch(buf, 7, "<I", 2))
    hdr_end = 7 + 4 + 4 + len(b"dsocr-test") + 4 + len(b"deepseek-ocr") + 4 + len(b"HIP")
    with pytest.raises(dsq.DsqError, match="block size"):
        dsq.parse_dsq(_patch(buf, hdr_end + 4, "<I", 32))
    with pytest.raises(dsq.DsqError, match="non-zero"):
        dsq.parse_dsq(_patch(buf, hdr_end + 4, "<I", 0))
    rec = hdr_end + 12
    off_q = rec + 4 + len(b"a.weight") + 12
    with pytest.raises(dsq.DsqError, match="overlaps metadata"):
        dsq.parse_dsq(_patch(buf, off_q, "<Q", 3))
    with pytest.raises(dsq.DsqError, match="exceeds file size"):
        dsq.parse_dsq(_patch(buf, off_q + 8, "<Q", 10 ** 6))
    with pytest.raises(dsq.DsqError, match="empty"):
        dsq.parse_dsq(_patch(buf, off_q + 8, "<Q", 0))
    with pytest.raises(dsq.DsqError, match="not divisible"):
        dsq.parse_dsq(_patch(buf, rec + 4 + len(b"a.weight") + 4, "<I", 255))
    with pytest.raises(dsq.DsqError, match="dtype code"):
        dsq.parse_dsq(_patch(buf, rec + 4 + len(b"a.weight") + 8, "<I", 3))
    _, buf2 = _container(tmp_path, [("a.weight", 1, 4, dsq.F16, b"\0" * 8, None), ("a.weight", 1, 4, dsq.F16, b"\0" * 8, None)])
    with pytest.raises(dsq.DsqError, match="duplicate"):
        dsq.parse_dsq(buf2)
    _, buf3 = _container(tmp_path, [("f.weight", 1, 4, dsq.F16, b"\0" * 6, None)])
    with pytest.raises(dsq.DsqError, match="q_len"):
        dsq.parse_dsq(buf3)


def test_golden_fixture():
    p = os.path.join(GOLDEN, "dsq_small.dsq")
    exp = np.load(os.path.join(GOLDEN, "dsq_small_expected.npz"))
    s = dsq.Snapshot(p)
    assert sorted(s.records) == sorted(k for k in exp.files if not k.endswith(".bias"))
    for name in s.records:
        assert np.array_equal(s.weight(name).view(np.uint32), exp[name].view(np.uint32)), name
    assert np.array_equal(s.bias_for("q8.weight"), exp["q8.weight.bias"])


def test_adapter_discovery_full_config():
    cfg = json.load(open(os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "deepseek-ocr.json")))
    specs = dsq.discover_linears(cfg)
    names = [s[0] for s in specs]
    # 12 layers x 4 attention + layer 0 dense (3) + 11 MoE layers x (64 experts + shared) x 3 + lm_head + projector
    assert len(specs) == 12 * 4 + 3 + 11 * 65 * 3 + 2
    assert "model.layers.1.mlp.shared_experts.down_proj.weight" in names
    assert ("model.layers.0.mlp.gate_proj.weight", 6848, 1280, "model.layers.0.mlp.gate_proj.bias") in specs
    assert specs[-2][:3] == ("lm_head.weight", 129280, 1280)


def test_synthetic_snapshot_generator(tmp_path):
    """dsocr.synth.write_synthetic_snapshot (the bench's configs[4] input): the adapter's record list,
    the quantizer's dtype choice (lm_head / projector Q8_0, Q4_K unless in_dim % 256 falls back to
    Q8_0), a container the reader accepts, values of the synthetic checkpoint's scale."""
    import dsocr
    from dsocr.synth import snapshot_dtype, snapshot_linears, write_synthetic_snapshot
    for cfgp in (TINY256, dsocr.FULL_CONFIG):
        cfg = json.load(open(cfgp))
        assert [r[:3] for r in snapshot_linears(cfg)] == [r[:3] for r in dsq.discover_linears(cfg)]
    assert snapshot_dtype("model.layers.1.mlp.experts.3.down_proj.weight", 896) == dsq.Q8_0
    assert snapshot_dtype("model.layers.0.mlp.down_proj.weight", 6848) == dsq.Q8_0
    assert snapshot_dtype("model.layers.1.mlp.shared_experts.down_proj.weight", 1792) == dsq.Q4K
    assert snapshot_dtype("lm_head.weight", 1280) == dsq.Q8_0
    cfg = json.load(open(TINY256))
    path = str(tmp_path / "synth.dsq")
    info = write_synthetic_snapshot(cfg, path, seed=3)
    snap = dsq.Snapshot(path)
    assert info["records"] == len(snap.records) and info["bytes"] == os.path.getsize(path)
    assert snap.header["default_qdtype"] == dsq.Q4K and snap.header["block_size"] == 256
    for name, out_dim, in_dim, bias in dsq.discover_linears(cfg):
        r = snap.records[name]
        assert (r["out_dim"], r["in_dim"], r["q_dtype"]) == (out_dim, in_dim, snapshot_dtype(name, in_dim))
        w = snap.weight(name)
        assert np.isfinite(w).all() and 0.01 < float(w.std()) < 0.04 and abs(float(w.mean())) < 0.005
        assert (snap.bias_for(name) is not None) == name.startswith("model.projector")


# ------------------------------------------------------------------ GPU
def make_tiny256_snapshot(path):
    """Every linear of the tiny256 model from the seeded synthetic checkpoint (bf16 values), in
    the dtypes the format allows: Q4_K / Q6_K / Q8_0 (+ projector bias) / F16 / BF16 / F32."""
    from oracle.weights import Weights
    cfg = json.load(open(TINY256))
    base = Weights(seed=SEED, dtype="f32")
    tensors = []
    for name, out_dim, in_dim, bias in dsq.discover_linears(cfg):
        w = base.get(name, (out_dim, in_dim))
        if name == "lm_head.weight":
            qt = dsq.Q8_0
        elif name.startswith("model.projector"):
            qt = dsq.Q8_0
        elif name.endswith("o_proj.weight"):
            qt = {0: dsq.BF16, 1: dsq.F16, 2: dsq.F32}[int(name.split(".")[2])]
        elif "down_proj" in name or "shared_experts" in name:
            qt = dsq.Q6K
        else:
            qt = dsq.Q4K
        b = base.get(bias, (out_dim,)) if bias and base.has(bias) else None
        tensors.append((name, out_dim, in_dim, qt, dsq.quantize(qt, w), b))
    dsq.write_dsq(path, tensors, default_qdtype=dsq.Q4K)
    return cfg


@pytest.mark.gpu
@pytest.mark.parametrize("qtype", [dsq.Q4K, dsq.Q6K, dsq.Q8_0, dsq.F16, dsq.BF16, dsq.F32])
def test_dequant_kernel_bit_exact(gpu, qtype):
    from _dev import Dev
    from dsocr._lib import check, lib
    rng = np.random.default_rng(100 + qtype)
    rows, cols = 37, 512
    if qtype in dsq.BLOCK:
        raw = _random_blocks(rng, qtype, rows * cols // dsq.BLOCK[qtype])
    else:
        raw = dsq.quantize(qtype, (rng.standard_normal((rows, cols)) * 3).astype(np.float32))
    src = Dev(np.frombuffer(raw, np.uint8))
    out = Dev.zeros((rows, cols), np.uint16)
    check(lib().dsocr_k_dsq_dequant(qtype, src.ptr, len(raw), rows, cols, out.ptr))
    ref = dsq.dequant(qtype, raw, rows, cols).astype(np.float16).view(np.uint16)
    got = out.get()
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]


@pytest.mark.gpu
def test_dequant_kernel_rejects_bad_sizes(gpu):
    from _dev import Dev
    from dsocr._lib import DsocrError, check, lib
    src = Dev(np.zeros(144, np.uint8))
    out = Dev.zeros((1, 256), np.uint16)
    with pytest.raises(DsocrError, match="EINVAL"):
        check(lib().dsocr_k_dsq_dequant(dsq.Q4K, src.ptr, 100, 1, 256, out.ptr))
    with pytest.raises(DsocrError, match="EINVAL"):
        check(lib().dsocr_k_dsq_dequant(3, src.ptr, 144, 1, 256, out.ptr))


@pytest.fixture(scope="module")
def snap_path(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("dsq") / "tiny256.dsq")
    make_tiny256_snapshot(p)
    return p


@pytest.mark.gpu
def test_snapshot_engine_matches_oracle(gpu, snap_path):
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import SyntheticTokenizer
    from oracle.model import OracleModel
    from oracle.weights import Weights
    cfg = json.load(open(TINY256))
    eng = load_model(ModelLoadArgs(config_path=TINY256, synthetic_seed=SEED, dtype="f16", snapshot_path=snap_path))
    try:
        oracle = OracleModel(cfg, Weights(seed=SEED, dtype="f16", snapshot=dsq.Snapshot(snap_path)))
        img = np.random.default_rng(5).integers(0, 256, (300, 260, 3), dtype=np.uint8)
        vs = VisionSettings(256, 128, True)
        page = Page(img, vs)
        got_emb = eng.image_embeddings([page])[0]
        ref_emb, _ = oracle.image_embeddings(img, 256, 128, True)
        assert np.max(np.abs(got_emb - ref_emb)) < 1e-3 * max(1.0, np.max(np.abs(ref_emb)))
        tok = SyntheticTokenizer(512)
        ids, mask = build_prompt_tokens(tok, "<image>\nConvert the document to markdown.", [page.n_image_tokens])
        got = eng.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=24))
        ref, _ = oracle.generate(ids, mask, ref_emb, 24, eos_token_id=1, no_repeat_ngram_size=20)
        assert got == ref
    finally:
        eng.close()


@pytest.mark.gpu
def test_snapshot_load_errors(gpu, snap_path, tmp_path):
    from dsocr import DsocrError, ModelLoadArgs, load_model
    with pytest.raises(DsocrError, match="EINVAL"):
        load_model(ModelLoadArgs(config_path=TINY256, synthetic_seed=SEED, dtype="f32", snapshot_path=snap_path))
    bad = tmp_path / "bad.dsq"
    bad.write_bytes(b"XSQSNAP" + open(snap_path, "rb").read()[7:])
    with pytest.raises(DsocrError, match="EINVAL"):
        load_model(ModelLoadArgs(config_path=TINY256, synthetic_seed=SEED, dtype="f16", snapshot_path=str(bad)))
    with pytest.raises(DsocrError, match="ENOENT"):
        load_model(ModelLoadArgs(config_path=TINY256, synthetic_seed=SEED, dtype="f16",
                                 snapshot_path=str(tmp_path / "missing.dsq")))
    # a record whose dims disagree with the config
    wrong = str(tmp_path / "wrong.dsq")
    dsq.write_dsq(wrong, [("lm_head.weight", 256, 512, dsq.Q8_0, dsq.quantize(dsq.Q8_0, np.zeros((256, 512), np.float32)), None)])
    with pytest.raises(DsocrError, match="EINVAL"):
        load_model(ModelLoadArgs(config_path=TINY256, synthetic_seed=SEED, dtype="f16", snapshot_path=wrong))


@pytest.mark.gpu
def test_full_q4k_snapshot_engine_matches_oracle(gpu, tmp_path):
    """configs[4] at its size: a full-size synthetic Q4_K snapshot (the bench's input: 1491 Q4_K and
    707 Q8_0 records, 2.05 GB) loaded through the engine's dequant-on-load path; text prompts so the
    oracle only dequantises the experts it routes to.  One page: ids and per-step logits (the same
    2e-3 bar as tests/test_full_parity.py) vs the oracle; 8 pages (the matrix-core decode of the
    configs[2]/[4] batch): ids vs the oracle per page."""
    import dsocr
    from dsocr import DecodeParameters, ModelLoadArgs, load_model
    from dsocr.synth import write_synthetic_snapshot
    from oracle.model import OracleModel
    from oracle.weights import Weights
    cfg = json.load(open(dsocr.FULL_CONFIG))
    path = str(tmp_path / "full_q4k.dsq")
    write_synthetic_snapshot(cfg, path, seed=0)
    n_new = 12
    rng = np.random.default_rng(9)
    prompts = [rng.integers(16, 129000, int(rng.integers(6, 20))).astype(np.int64) for _ in range(8)]
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16", snapshot_path=path))
    try:
        params = DecodeParameters(max_new_tokens=n_new)
        ids1, logits = eng.generate_trace([(prompts[0], None, None, None)], params, ignore_eos=True)
        # without the trace the screened head selects (the snapshot's lm_head is f16: int8 screening of the
        # f16 rows, exact rescoring in f16): one page and the 8-page matrix-core form
        ids1s = eng.generate_batch([(prompts[0], None, None, None)], params, ignore_eos=True)
        ids8 = eng.generate_batch([(p, None, None, None) for p in prompts], params, ignore_eos=True)
    finally:
        eng.close()
    oracle = OracleModel(cfg, Weights(seed=0, dtype="f16", snapshot=dsq.Snapshot(path)))
    for i, p in enumerate(prompts):
        ref, lg = oracle.generate(p, np.zeros(len(p), np.uint8), None, n_new, eos_token_id=None,
                                  record_logits=(i == 0), ignore_eos=True)
        if i == 0:
            assert ids1[0] == ref
            assert ids1s[0] == ref, (ids1s[0], ref)
            err = max(float(np.max(np.abs(logits[0, s] - lg[s]))) for s in range(n_new))
            assert err < 2e-3, err
        assert ids8[i] == ref, (i, ids8[i], ref)


@pytest.mark.gpu
def test_full_q4k_snapshot_page_matches_fixture(gpu, tmp_path):
    """configs[4] with a page: the full-size synthetic Q4_K snapshot (the projector from its Q8_0 record)
    through vision -> projector -> 706-token prefill -> the fixture's greedy tokens on the bench's synthetic 1024 px
    page (512 tokens): ids equal and the raw logits at the oracle's top-8 and probe indices within 2e-3 of the
    committed fixture
    (tests/golden/full_q4k_synthetic0.npz, make_full_golden.py --snapshot q4k: the oracle reading the
    same snapshot)."""
    import os
    import dsocr
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page, write_synthetic_snapshot
    fxp = os.path.join(os.path.dirname(__file__), "golden", "full_q4k_synthetic0.npz")
    fx = dict(np.load(fxp))
    cfg = json.load(open(dsocr.FULL_CONFIG))
    path = str(tmp_path / "full_q4k.dsq")
    write_synthetic_snapshot(cfg, path, seed=0)
    n = int(fx["max_new"])
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=int(fx["weights_seed"]), dtype="f16",
                                   snapshot_path=path))
    try:
        page = Page(synthetic_page(0), VisionSettings(), eng)
        ids, mask = build_prompt_tokens(SyntheticTokenizer(eng.vocab), BENCH_PROMPT, [page.n_image_tokens])
        assert ids == fx["prompt_ids"].tolist()
        outs, logits = eng.generate_trace([(ids, mask, page, None)], DecodeParameters(max_new_tokens=n), ignore_eos=True)
        # the bench path: the screened head over the f16 lm_head rows (no trace)
        screened = eng.generate(ids, mask, page, None, DecodeParameters(max_new_tokens=n), ignore_eos=True)
    finally:
        eng.close()
    from test_full_parity import check_stream
    check_stream("q4k_synthetic0", fx, outs[0], logits[0], n)
    assert screened == fx["ids"].tolist(), "screened selection over the f16 lm_head differs from the fixture"
