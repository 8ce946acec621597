"""Kernel-level parity on MI355X (gfx950) through the C ABI entry points.

Tolerances (f32 accumulation in a different order than the oracle's BLAS):
  GEMM/GEMV/attention/MoE: |got - ref| <= 2e-5 * sum_k |a_k w_k| + 1e-6 (per element bound)
  norms: 1e-5 relative.  Greedy token selection: exact.
"""
import ctypes as C
import math

import numpy as np
import pytest

from _dev import Dev, bf16_round, bf16_to_f32, f16_bits
from dsocr._lib import check, lib
from oracle.decoder import rms_norm, select_token_id, softmax
from oracle.vision import gelu_erf, get_rel_pos, layer_norm, sigmoid

pytestmark = pytest.mark.gpu


def _weights(rng, n, k, wdtype):
    w = (rng.standard_normal((n, k)) * 0.05).astype(np.float32)
    if wdtype == 0:
        bits = bf16_round(w)
        return bits, bf16_to_f32(bits)
    bits = f16_bits(w)
    return bits, bits.view(np.float16).astype(np.float32)


def _bound(a, w):
    return 2e-5 * (np.abs(a) @ np.abs(w).T) + 1e-6


ACTS = {0: lambda x: x, 1: gelu_erf, 2: lambda x: sigmoid(x * np.float32(1.702)) * x,
        3: lambda x: x / (np.float32(1) + np.exp(-x))}


@pytest.mark.parametrize("M,N,K,wdt,act,acc", [(256, 256, 256, 0, 0, 0), (1000, 770, 768, 0, 1, 0),
                                              (77, 130, 24, 1, 0, 1), (4096, 2304, 768, 0, 0, 0),
                                              (300, 4096, 1024, 1, 2, 0), (129, 64, 1280, 1, 3, 1)])
def test_gemm(gpu, M, N, K, wdt, act, acc):
    rng = np.random.default_rng(M + N + K)
    a = rng.standard_normal((M, K)).astype(np.float32)
    bits, w = _weights(rng, N, K, wdt)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    c0 = rng.standard_normal((M, N)).astype(np.float32) if acc else np.zeros((M, N), np.float32)
    dA, dW, dB, dC = Dev(a), Dev(bits), Dev(bias), Dev(c0)
    check(lib().dsocr_k_gemm(M, N, K, dA.ptr, dW.ptr, wdt, dB.ptr, dC.ptr, act, acc))
    ref = ACTS[act]((a.astype(np.float64) @ w.T.astype(np.float64)).astype(np.float32) + bias) + (c0 if acc else 0)
    got = dC.get()
    bound = _bound(a, w) * (2.0 if act else 1.0)
    assert np.all(np.abs(got - ref) <= bound + 1e-5 * np.abs(ref)), np.max(np.abs(got - ref))


@pytest.mark.parametrize("M,N,K,wdt,act,acc,splits", [(256, 256, 256, 0, 0, 0, 1), (1000, 770, 768, 0, 1, 0, 0),
                                                      (6400, 768, 3072, 0, 0, 1, 0), (257, 3072, 1024, 0, 2, 0, 0),
                                                      (77, 130, 96, 0, 0, 1, 3), (4096, 2304, 768, 0, 0, 0, 1),
                                                      (693, 1280, 2048, 0, 0, 0, 0), (706, 3840, 1280, 1, 0, 0, 0),
                                                      (706, 1280, 1280, 1, 0, 1, 0), (1412, 13696, 1280, 1, 3, 0, 0),
                                                      (100, 64, 1280, 1, 0, 0, 2),
                                                      # split-K reduce over more than one batch of 8 slices,
                                                      # four columns per thread, accumulate + activation
                                                      (300, 512, 1152, 0, 1, 1, 9)])
def test_gemm_f32a(gpu, M, N, K, wdt, act, acc, splits):
    """Vision (bf16 weights: 3 exact bf16 planes of the f32 activations) and prefill (f16 weights, split into
    hi / lo bf16 as well: 5 products) linears on the fused-split kernel vs an f64 matmul, incl. split-K and
    the accumulate epilogue."""
    rng = np.random.default_rng(M * 7 + N + K)
    a = rng.standard_normal((M, K)).astype(np.float32)
    bits, w = _weights(rng, N, K, wdt)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    c0 = rng.standard_normal((M, N)).astype(np.float32) if acc else np.zeros((M, N), np.float32)
    dA, dW, dB, dC = Dev(a), Dev(bits), Dev(bias), Dev(c0)
    check(lib().dsocr_k_gemm_f32a(M, N, K, dA.ptr, dW.ptr, wdt, dB.ptr, dC.ptr, act, acc, splits))
    ref = ACTS[act]((a.astype(np.float64) @ w.T.astype(np.float64)).astype(np.float32) + bias) + (c0 if acc else 0)
    got = dC.get()
    bound = _bound(a, w) * (2.0 if act else 1.0)
    assert np.all(np.abs(got - ref) <= bound + 1e-5 * np.abs(ref)), np.max(np.abs(got - ref))


@pytest.mark.parametrize("T,E,topk,N,K,wdt,act,acc,kernel", [
    (300, 64, 6, 1792, 1280, 1, 0, 0, 1),   # one page's routed gate/up (~28 rows per expert)
    (300, 64, 6, 1280, 896, 1, 0, 1, 1),    # ... down, accumulate epilogue
    (37, 16, 3, 200, 96, 0, 3, 0, 1),       # bf16 weights, ragged N, empty experts, SiLU epilogue
    (3000, 64, 6, 1792, 1280, 1, 0, 0, 0),  # many rows per expert: the engine dispatch (128-row tiles)
    (3000, 64, 6, 1792, 1280, 1, 0, 0, 1),  # ... the 32-row tiles at the same size
    (300, 64, 6, 1280, 896, 1, 0, 1, 2),    # 128-row tiles with few rows (padding rows, accumulate)
    (37, 16, 3, 200, 96, 0, 3, 0, 2)])      # ... bf16, ragged N, empty experts
def test_gemm_grouped(gpu, T, E, topk, N, K, wdt, act, acc, kernel):
    """Prefill routed experts (block.rs:1215-1395: expert e on the rows that picked it) through the grouped
    exact-f32 GEMM: rows gathered by a sorted row list, weights of each expert's slab, rows scattered back,
    vs an f64 matmul per expert (same per-element bound as test_gemm)."""
    rng = np.random.default_rng(T + E + N)
    a = rng.standard_normal((T, K)).astype(np.float32)
    picks = np.stack([rng.choice(E // 2 if E > 16 else E - 4, topk, replace=False) for _ in range(T)])  # some experts empty
    flat = picks.reshape(-1)
    order = np.argsort(flat, kind="stable")
    arow = (order // topk).astype(np.int32)                 # sorted position -> token
    counts = np.bincount(flat, minlength=E)
    eoff = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    M = T * topk
    crow = np.arange(M, dtype=np.int32)[::-1].copy()        # scatter to reversed rows
    ws, wf = zip(*[_weights(rng, N, K, wdt) for _ in range(E)])
    bits = np.stack(ws)
    bias = (rng.standard_normal((E, N)) * 0.1).astype(np.float32)
    c0 = rng.standard_normal((M, N)).astype(np.float32) if acc else np.zeros((M, N), np.float32)
    dA, dW, dB, dC, dR, dO, dCr = Dev(a), Dev(bits), Dev(bias), Dev(c0), Dev(arow), Dev(eoff), Dev(crow)
    check(lib().dsocr_k_gemm_grouped(M, N, K, dA.ptr, K, dR.ptr, dW.ptr, wdt, N * K, dB.ptr, N, dC.ptr, N, dCr.ptr, act,
                                     acc, dO.ptr, E, int(counts.max()), kernel))
    got = dC.get()
    ref = c0.copy()
    for e in range(E):
        rows = np.arange(eoff[e], eoff[e + 1])
        if rows.size == 0:
            continue
        x = a[arow[rows]]
        y = ACTS[act]((x.astype(np.float64) @ wf[e].T.astype(np.float64)).astype(np.float32) + bias[e])
        bound = _bound(x, wf[e]) * (2.0 if act else 1.0)
        r = crow[rows]
        exp = y + (c0[r] if acc else 0)
        assert np.all(np.abs(got[r] - exp) <= bound + 1e-5 * np.abs(exp)), (e, np.max(np.abs(got[r] - exp)))


@pytest.mark.parametrize("M,N,K,wdt,norm", [(1, 1280, 1280, 1, True), (1, 129280, 1280, 0, True),
                                            (2, 3840, 1280, 1, True), (3, 3840, 1280, 1, False),
                                            (8, 896, 1792, 1, False), (16, 100, 64, 0, False),
                                            (21, 513, 128, 0, True), (1, 64, 1280, 1, True), (4, 9000, 256, 0, False),
                                            (8, 3840, 1280, 1, True), (5, 1280, 1280, 1, True), (8, 1280, 1280, 1, False),
                                            (7, 200, 512, 0, True)])
def test_gemv(gpu, M, N, K, wdt, norm):
    """Decode linear (dec_gemv) with the optional fused RMSNorm prologue (block.rs:24-29)."""
    rng = np.random.default_rng(N + K + M)
    x = rng.standard_normal((M, K)).astype(np.float32)
    bits, w = _weights(rng, N, K, wdt)
    nw = (1.0 + 0.05 * rng.standard_normal(K)).astype(np.float32)
    y0 = rng.standard_normal((M, N)).astype(np.float32)
    acc = int(M % 2 == 1)
    dx, dW, dy, dn = Dev(x), Dev(bits), Dev(y0 if acc else np.zeros((M, N), np.float32)), Dev(nw)
    check(lib().dsocr_k_gemv(M, N, K, dx.ptr, dn.ptr if norm else None, 1e-6, dW.ptr, wdt, None, dy.ptr, 0, acc))
    xn = rms_norm(x, nw, 1e-6) if norm else x
    ref = (xn.astype(np.float64) @ w.T.astype(np.float64)).astype(np.float32) + (y0 if acc else 0)
    assert np.all(np.abs(dy.get() - ref) <= _bound(xn, w) + 1e-6 * np.abs(ref))


@pytest.mark.parametrize("M,N,K,acc", [(8, 1280, 6848, True), (3, 1280, 6848, False), (5, 200, 640, True)])
def test_gemv_splitk(gpu, M, N, K, acc):
    """Long-K decode linear on the matrix cores (the dense layer-0 down projection at 3..8 pages):
    split-K pieces of 512 with per-(row, piece) scaled f16 planes, in-launch ordered sum."""
    rng = np.random.default_rng(N + K + M)
    x = (rng.standard_normal((M, K)) * np.exp(rng.standard_normal((M, 1)) * 3)).astype(np.float32)
    bits, w = _weights(rng, N, K, 1)
    y0 = rng.standard_normal((M, N)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    dx, dW, dy, db = Dev(x), Dev(bits), Dev(y0 if acc else np.zeros((M, N), np.float32)), Dev(bias)
    check(lib().dsocr_k_gemv_splitk(M, N, K, dx.ptr, dW.ptr, 1, db.ptr, dy.ptr, int(acc)))
    ref = (x.astype(np.float64) @ w.T.astype(np.float64)).astype(np.float32) + bias + (y0 if acc else 0)
    assert np.all(np.abs(dy.get() - ref) <= _bound(x, w) + 1e-6 * np.abs(ref))


@pytest.mark.parametrize("rows,cols,eps", [(4096, 768, 1e-6), (257, 1024, 1e-5), (100, 256, 1e-6)])
def test_layernorm(gpu, rows, cols, eps):
    rng = np.random.default_rng(rows)
    x = (rng.standard_normal((rows, cols)) * 3 + 1).astype(np.float32)
    w = rng.standard_normal(cols).astype(np.float32)
    b = rng.standard_normal(cols).astype(np.float32)
    dx, dw, db, dy = Dev(x), Dev(w), Dev(b), Dev.zeros((rows, cols))
    check(lib().dsocr_k_layernorm(rows, cols, dx.ptr, dw.ptr, db.ptr, eps, dy.ptr))
    ref = layer_norm(x, w, b, eps)
    assert np.max(np.abs(dy.get() - ref)) <= 1e-5 * (1 + np.max(np.abs(ref)))


def test_rmsnorm(gpu):
    rng = np.random.default_rng(7)
    x = rng.standard_normal((706, 1280)).astype(np.float32) * 0.01
    w = (1 + rng.standard_normal(1280) * 0.05).astype(np.float32)
    dx, dw, dy = Dev(x), Dev(w), Dev.zeros((706, 1280))
    check(lib().dsocr_k_rmsnorm(706, 1280, dx.ptr, dw.ptr, 1e-6, dy.ptr))
    ref = rms_norm(x, w, 1e-6)
    assert np.max(np.abs(dy.get() - ref)) <= 1e-5 * np.max(np.abs(ref))


def _attn_ref(q, k, v, scale, causal=False, bias=None):
    s = (q.astype(np.float64) @ k.T.astype(np.float64)) * scale
    if bias is not None:
        s = s + bias
    if causal:
        s = s + np.triu(np.full(s.shape, -1e9), 1)
    s = s - s.max(-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(-1, keepdims=True)
    return p @ v.astype(np.float64)


@pytest.mark.parametrize("n_seq,L,heads,hd,causal", [(2, 257, 16, 64, 0), (3, 101, 4, 32, 0), (1, 706, 10, 128, 1),
                                                     (5, 196, 12, 64, 0), (2, 33, 2, 128, 1), (3, 300, 4, 64, 1),
                                                     (1, 1217, 10, 128, 1), (2, 20, 4, 64, 0), (1, 97, 3, 64, 0)])
def test_attention(gpu, n_seq, L, heads, hd, causal):
    """Flash attention vs f64 math (block.rs:1504-1526 causal prefill; sam.rs / clip.rs bidirectional).  The
    causal cases run the prefill's key-piece form (one block per (128-query block, 128-key piece) + the piece
    combine)."""
    rng = np.random.default_rng(L * heads)
    C_ = heads * hd
    q, k, v = (rng.standard_normal((n_seq * L, C_)).astype(np.float32) for _ in range(3))
    dq, dk, dv, do = Dev(q), Dev(k), Dev(v), Dev.zeros((n_seq * L, C_))
    scale = 1.0 / math.sqrt(hd)
    check(lib().dsocr_k_attention(n_seq, L, heads, hd, scale, causal, dq.ptr, dk.ptr, dv.ptr, do.ptr, None, None, 0, 0))
    got = do.get()
    for s in range(n_seq):
        for h in range(heads):
            sl, hl = slice(s * L, (s + 1) * L), slice(h * hd, (h + 1) * hd)
            ref = _attn_ref(q[sl, hl], k[sl, hl], v[sl, hl], scale, bool(causal))
            assert np.max(np.abs(got[sl, hl] - ref)) < 2e-5, (s, h)


@pytest.mark.parametrize("g,rel_len", [(14, 27), (16, 31), (40, 127), (64, 127)])
def test_attention_sam_relpos(gpu, g, rel_len):
    """SamAttention::forward with the decomposed rel-pos bias (sam.rs:804-888, 1124-1247)."""
    rng = np.random.default_rng(g)
    heads, hd, n_seq, L = 2, 64, 1, g * g
    q, k, v = (rng.standard_normal((L, heads * hd)).astype(np.float32) for _ in range(3))
    relh = rng.standard_normal((rel_len, hd)).astype(np.float32) * 0.2
    relw = rng.standard_normal((rel_len, hd)).astype(np.float32) * 0.2
    Rh, Rw = get_rel_pos(g, g, relh), get_rel_pos(g, g, relw)       # [g, g, hd]
    # direct construction of the resized table from get_rel_pos: idx = qi - ki + g - 1
    tab_h = np.zeros((2 * g - 1, hd), np.float32)
    tab_w = np.zeros((2 * g - 1, hd), np.float32)
    for qi in range(g):
        for ki in range(g):
            tab_h[qi - ki + g - 1] = Rh[qi, ki]
            tab_w[qi - ki + g - 1] = Rw[qi, ki]
    dq, dk, dv, do = Dev(q), Dev(k), Dev(v), Dev.zeros((L, heads * hd))
    dh, dw = Dev(tab_h), Dev(tab_w)
    scale = 1.0 / math.sqrt(hd)
    check(lib().dsocr_k_attention(n_seq, L, heads, hd, scale, 0, dq.ptr, dk.ptr, dv.ptr, do.ptr, dh.ptr, dw.ptr, g, g))
    got = do.get()
    for h in range(heads):
        hl = slice(h * hd, (h + 1) * hd)
        qg = q[:, hl].reshape(g, g, hd).astype(np.float64)
        rel_h = np.einsum("hwc,hkc->hwk", qg, Rh)
        rel_w = np.einsum("hwc,wkc->hwk", qg, Rw)
        bias = (rel_h[:, :, :, None] + rel_w[:, :, None, :]).reshape(L, L)
        ref = _attn_ref(q[:, hl], k[:, hl], v[:, hl], scale, False, bias)
        assert np.max(np.abs(got[:, hl] - ref)) < 5e-5


@pytest.mark.parametrize("B,heads,kvh,hd,max_len,prerot", [
    (1, 10, 10, 128, 1218, 0), (3, 4, 4, 32, 300, 0), (5, 12, 4, 64, 700, 0), (2, 10, 10, 128, 257, 0),
    (1, 10, 10, 128, 64, 0), (8, 10, 10, 128, 1218, 0), (2, 10, 10, 128, 2000, 0),
    # the one-page decode loop's form: q / k pre-rotated by the projection's epilogue
    (1, 10, 10, 128, 1218, 1), (1, 10, 10, 128, 130, 1), (1, 10, 10, 128, 2000, 1)])
def test_decode_attention(gpu, B, heads, kvh, hd, max_len, prerot):
    """Fused decode attention (block.rs:608-789 at seq_len 1): RoPE on q / new k (block.rs:1403-1471) in the
    kernel or already applied (prerot), K/V append at pos = kv_pos[b], flash-decoding over pos + 1 keys of the
    f32 cache (64-key chunks; polled merge up to 24 chunks, ticket beyond).  The cache past the position holds
    NaN: keys past the position must contribute nothing."""
    from types import SimpleNamespace
    from oracle.decoder import apply_rope, rope_tables
    rng = np.random.default_rng(B * hd + max_len + prerot)
    qkvw = (heads + 2 * kvh) * hd
    qkv = rng.standard_normal((B, qkvw)).astype(np.float32)
    kc = rng.standard_normal((B, kvh, max_len, hd)).astype(np.float32)
    vc = rng.standard_normal((B, kvh, max_len, hd)).astype(np.float32)
    pos = rng.integers(0, max_len, B).astype(np.int32)
    pos[0] = max_len - 1
    if B > 1:
        pos[1] = 0
    if B > 2:
        pos[2] = 63
    for b in range(B):
        kc[b, :, pos[b] + 1:] = np.nan
        vc[b, :, pos[b] + 1:] = np.nan
    lang = SimpleNamespace(rope_theta=10000.0)
    cos, sin = rope_tables(lang, max_len, hd)
    rot = qkv.copy()
    for b in range(B):
        cs, sn = cos[pos[b]][None], sin[pos[b]][None]
        rot[b, :heads * hd] = apply_rope(qkv[b, :heads * hd].reshape(heads, hd), cs, sn, False).reshape(-1)
        rot[b, heads * hd:(heads + kvh) * hd] = apply_rope(qkv[b, heads * hd:(heads + kvh) * hd].reshape(kvh, hd),
                                                           cs, sn, False).reshape(-1)
    dqkv, dk, dv, dp, do = Dev(rot if prerot else qkv), Dev(kc), Dev(vc), Dev(pos), Dev.zeros((B, heads * hd))
    dcos, dsin = Dev(cos), Dev(sin)
    scale = 1.0 / math.sqrt(hd)
    check(lib().dsocr_k_decode_attention(B, heads, kvh, hd, hd, max_len, scale, dqkv.ptr, dcos.ptr, dsin.ptr,
                                         dk.ptr, dv.ptr, dp.ptr, do.ptr, prerot))
    got, gk, gv = do.get(), dk.get(), dv.get()
    for b in range(B):
        p = pos[b]
        q = rot[b, :heads * hd].reshape(heads, hd)
        kn = rot[b, heads * hd:(heads + kvh) * hd].reshape(kvh, hd)
        vn = qkv[b, (heads + kvh) * hd:].reshape(kvh, hd)
        assert np.max(np.abs(gk[b, :, p] - kn)) < 1e-5 and np.array_equal(gv[b, :, p], vn)
        K = kc[b].copy(); V = vc[b].copy()
        K[:, p] = kn; V[:, p] = vn
        for h in range(heads):
            g = h // (heads // kvh)
            ref = _attn_ref(q[h][None], K[g, :p + 1], V[g, :p + 1], scale)[0]
            assert np.max(np.abs(got[b, h * hd:(h + 1) * hd] - ref)) < 2e-5, (b, h)


SENT = 0x7FBADBAD  # DSOCR_HANDOFF_SENTINEL


@pytest.mark.parametrize("max_len,p0", [(1219, 1200), (1219, 700), (130, 60), (64 * 24, 64 * 24 - 3)])
def test_qkv_attention_fused_back_to_back(gpu, max_len, p0):
    """One page's q/k/v projection + decode attention as ONE launch (dec_qkv_attn: attention blocks poll the
    sentinel-filled q/k/v row the projection blocks of the same grid write) for three launches back to back
    (positions p0, p0+1, p0+2: the row and the merge records refilled by each launch are what the next one
    polls), against the two-launch form (dec_qkv_rope + dec_attn) on the same inputs and against f64 math
    (block.rs:446-804 at seq_len 1: RMSNorm, q/k/v = W x, RoPE, K/V append, softmax attention).  Checks the
    outputs, the appended K / V slots, and that the row holds only sentinels again afterwards."""
    from types import SimpleNamespace
    from oracle.decoder import apply_rope, rope_tables
    H, heads, hd, steps = 1280, 10, 128, 3
    rng = np.random.default_rng(max_len + p0)
    x = rng.standard_normal((steps, H)).astype(np.float32)
    nw = (1.0 + 0.1 * rng.standard_normal(H)).astype(np.float32)
    bits, w = _weights(rng, 3 * H, H, 1)
    kc = rng.standard_normal((heads, max_len, hd)).astype(np.float32)
    vc = rng.standard_normal((heads, max_len, hd)).astype(np.float32)
    kc[:, p0:] = np.nan
    vc[:, p0:] = np.nan
    pos = np.arange(p0, p0 + steps, dtype=np.int32)
    cos, sin = rope_tables(SimpleNamespace(rope_theta=10000.0), max_len, hd)
    scale, eps = 1.0 / math.sqrt(hd), 1e-6
    dW, dx, dn, dcos, dsin, dp = Dev(bits), Dev(x), Dev(nw), Dev(cos), Dev(sin), Dev(pos)
    outs = {}
    for fused in (1, 0):
        row = Dev(np.full(3 * H, SENT, np.uint32))
        dk, dv, do = Dev(kc), Dev(vc), Dev.zeros((steps, H))
        used = C.c_int(-1)
        check(lib().dsocr_k_qkv_attention(fused, steps, H, heads, hd, max_len, scale, eps, dx.ptr, dn.ptr, dW.ptr, 1,
                                          dcos.ptr, dsin.ptr, dk.ptr, dv.ptr, dp.ptr, row.ptr, do.ptr, C.byref(used)))
        assert used.value == fused, "the residency rule refused the fused launch at this size"
        if fused:
            assert np.all(row.get() == SENT), "the q/k/v hand-off row was not refilled with sentinels"
        outs[fused] = (do.get(), dk.get(), dv.get())
    (o1, k1, v1), (o0, k0, v0) = outs[1], outs[0]
    # the two forms' projection epilogues are separate instantiations (the fused one stores write-through):
    # equal up to the f32 rounding of the RoPE epilogue (a few ulp), the rest of the cache untouched
    sl = slice(p0, p0 + steps)
    assert np.allclose(k1[:, sl], k0[:, sl], rtol=4e-7, atol=4e-7), np.max(np.abs(k1[:, sl] - k0[:, sl]))
    assert np.allclose(v1[:, sl], v0[:, sl], rtol=4e-7, atol=4e-7), np.max(np.abs(v1[:, sl] - v0[:, sl]))
    assert np.array_equal(k1[:, :p0], kc[:, :p0]) and np.array_equal(v1[:, :p0], vc[:, :p0])
    assert np.max(np.abs(o1 - o0)) <= 1e-5, np.max(np.abs(o1 - o0))
    K, V = kc.copy(), vc.copy()
    for s in range(steps):
        p = pos[s]
        xn = rms_norm(x[s][None], nw, eps)[0]
        qkv = (xn.astype(np.float64) @ w.T.astype(np.float64)).astype(np.float32)
        cs, sn = cos[p][None], sin[p][None]
        q = apply_rope(qkv[:H].reshape(heads, hd), cs, sn, False)
        kn = apply_rope(qkv[H:2 * H].reshape(heads, hd), cs, sn, False)
        vn = qkv[2 * H:].reshape(heads, hd)
        assert np.max(np.abs(k1[:, p] - kn)) < 1e-4 and np.max(np.abs(v1[:, p] - vn)) < 1e-4
        K[:, p], V[:, p] = k1[:, p], v1[:, p]
        for h in range(heads):
            ref = _attn_ref(q[h][None], K[h, :p + 1], V[h, :p + 1], scale)[0]
            assert np.max(np.abs(o1[s, h * hd:(h + 1) * hd] - ref)) < 1e-4, (s, h)


@pytest.mark.parametrize("T,H,E,topk,I,ns,norm", [(3, 256, 16, 6, 64, 2, False), (1, 256, 16, 6, 64, 2, True),
                                                  (2, 1280, 64, 6, 896, 2, True), (9, 128, 8, 3, 32, 1, False),
                                                  (4, 256, 16, 6, 64, 2, False)])
def test_moe_decode_layer(gpu, T, H, E, topk, I, ns, norm):
    """Decode MoE (north-star kernel chain) vs the oracle's run_moe (block.rs:1215-1395).
    T <= 2: slot mode (gate/up blocks route themselves); 3..8: grouped (the router launch writes the
    expert groups); T > 8: one block groups the assignments by expert."""
    from oracle.decoder import Decoder
    rng = np.random.default_rng(5 + T)
    Is = I * ns
    x = rng.standard_normal((T, H)).astype(np.float32)
    router = f16_bits(rng.standard_normal((E, H)) * 0.1)
    gate = [f16_bits(rng.standard_normal((I, H)) * 0.05) for _ in range(E)]
    up = [f16_bits(rng.standard_normal((I, H)) * 0.05) for _ in range(E)]
    down = [f16_bits(rng.standard_normal((H, I)) * 0.05) for _ in range(E)]
    sg, su, sd = (f16_bits(rng.standard_normal(s) * 0.05) for s in [(Is, H), (Is, H), (H, Is)])
    Wgu = np.stack([np.concatenate([gate[e], up[e]]) for e in range(E)])
    Wd = np.stack(down)
    sWgu = np.concatenate([sg, su])
    out0 = rng.standard_normal((T, H)).astype(np.float32)
    dx, dr, dgu, dd, dsgu, dsd, dout = Dev(x), Dev(router), Dev(Wgu), Dev(Wd), Dev(sWgu), Dev(sd), Dev(out0)
    ids = np.zeros(T * topk, np.int32)
    wts = np.zeros(T * topk, np.float32)
    nw = (1.0 + 0.05 * rng.standard_normal(H)).astype(np.float32)
    dn = Dev(nw)
    check(lib().dsocr_k_moe(T, H, E, topk, I, Is, dx.ptr, dn.ptr if norm else None, 1e-6, dr.ptr, dgu.ptr, dd.ptr,
                            dsgu.ptr, dsd.ptr, 1, 0, 1.0, dout.ptr, ids.ctypes.data_as(C.c_void_p),
                            wts.ctypes.data_as(C.c_void_p)))
    if norm:
        x = rms_norm(x, nw, 1e-6)

    f = lambda b: b.view(np.float16).astype(np.float32)
    W = {"l.mlp.gate.weight": f(router), "l.mlp.shared_experts.gate_proj.weight": f(sg),
         "l.mlp.shared_experts.up_proj.weight": f(su), "l.mlp.shared_experts.down_proj.weight": f(sd)}
    for e in range(E):
        W[f"l.mlp.experts.{e}.gate_proj.weight"] = f(gate[e])
        W[f"l.mlp.experts.{e}.up_proj.weight"] = f(up[e])
        W[f"l.mlp.experts.{e}.down_proj.weight"] = f(down[e])

    class _W:
        def get(self, n, shape=None):
            return W[n.replace("model.layers.1.", "l.")]

        def has(self, n):
            return n.replace("model.layers.1.", "l.") in W

    dec = Decoder.__new__(Decoder)
    dec.W = _W()
    dec.H = H

    class _L:
        n_routed_experts, num_experts_per_tok, moe_intermediate_size = E, topk, I
        topk_method, scoring_func, norm_topk_prob, routed_scaling_factor, n_shared_experts = "greedy", "softmax", False, 1.0, ns
    dec.lang = _L()
    ref = dec.moe(1, x) + out0
    logits = x @ f(router).T
    order = np.argsort(-softmax(logits), axis=-1, kind="stable")[:, :topk]
    assert np.array_equal(ids.reshape(T, topk), order)
    assert np.max(np.abs(dout.get() - ref)) < 1e-4


@pytest.mark.parametrize("ngram,pen", [(0, 1.0), (3, 1.0), (20, 1.0), (3, 1.3)])
def test_sample_greedy(gpu, ngram, pen):
    rng = np.random.default_rng(ngram)
    B, V, cap = 3, 5000, 64
    logits = rng.standard_normal((B, V)).astype(np.float32)
    ctx = np.zeros((B, cap), np.int32)
    lens = np.array([40, 25, 3], np.int32)
    for b in range(B):
        base = rng.integers(0, 50, 5)
        seq = np.tile(base, 20)[: lens[b]]
        ctx[b, : lens[b]] = seq
        logits[b, seq] += 3.0  # make the repeated tokens the likely argmax
    dl, dc, dn, dt = Dev(logits), Dev(ctx), Dev(lens), Dev.zeros(B, np.int32)
    check(lib().dsocr_k_sample_greedy(B, V, dl.ptr, dc.ptr, cap, dn.ptr, ngram, pen, dt.ptr))
    got = dt.get()
    for b in range(B):
        ref = select_token_id(logits[b], ctx[b, : lens[b]].tolist(), pen, ngram if ngram > 1 else None)
        assert got[b] == ref, (b, got[b], ref)


# ---------------------------------------------------------------- decode MoE: the production dispatch
@pytest.mark.parametrize("T,H,E,topk,I,ns,norm", [(1, 1280, 64, 6, 896, 2, True),   # mix kernels (bench, 1 page)
                                                  (2, 1280, 64, 6, 896, 2, True),   # slot kernels
                                                  (3, 1280, 64, 6, 896, 2, True),   # grouped kernels ...
                                                  (8, 1280, 64, 6, 896, 2, True),   # ... at 8 pages (configs[2])
                                                  (5, 256, 16, 6, 64, 2, True),     # many tokens per expert
                                                  (8, 256, 8, 3, 32, 1, False)])    # every record full (8 tokens)
def test_moe_decode_full_size_dispatch(gpu, T, H, E, topk, I, ns, norm):
    """dsocr_k_moe runs the engine's own decode dispatch (launch_moe_decode): at full size
    (H 1280, 64 experts, I 896, 2 shared = Is 1792) one token takes moe_gateup_mix + moe_down_mix,
    3..8 tokens the grouped kernels (each distinct expert streamed once) - vs the oracle's run_moe
    (block.rs:1215-1395), ids exact, outputs <= 1e-4."""
    test_moe_decode_layer(gpu, T, H, E, topk, I, ns, norm)


# ---------------------------------------------------------------- screened lm_head: ties / near ties
@pytest.mark.parametrize("B", [2, 3, 8])
def test_screened_head_ties_first_index(gpu, B):
    """The screened selection (int8 intervals + exact rescoring) against the exact lm_head GEMV's
    first-index argmax (argmax_index, sampling.rs:104-118) on rows built to tie: two identical
    dominant rows (first index wins), a row one bf16 ulp away in one element (a near tie far below
    the int8 quantisation error), and a ban list that removes the first of the tied rows.  B = 2: the
    single-token kernel per page; B = 3, 8: one int8 stream for every row on the int8 matrix cores (two int8
    planes per token row, its representation error in the bound)."""
    rng = np.random.default_rng(99)
    V, K = 20000, 1280
    x = rng.standard_normal((B, K)).astype(np.float32)
    nw = (1.0 + 0.05 * rng.standard_normal(K)).astype(np.float32)
    w = (rng.standard_normal((V, K)) * 0.02).astype(np.float32)
    xn = rms_norm(x, nw, 1e-6)
    dom = (xn[0] / np.linalg.norm(xn[0]) * 0.5).astype(np.float32)
    bits = bf16_round(w)
    dbits = bf16_round(dom)
    A, Bt, Cn = 777, 15000, 300
    bits[A] = dbits
    bits[Bt] = dbits                       # exact tie with A
    bits[Cn] = dbits
    j = int(np.argmax(np.abs(dom)))
    bits[Cn, j] = dbits[j] + 1             # one ulp in one element: a near tie
    bits[:, :][4000] = dbits               # a third copy (after A)
    ban_ld = 8
    ban = np.zeros((B, ban_ld), np.int32)
    ban[1, 0], ban[1, 1] = 2, A            # page 1: A banned
    ban[1, 2] = Cn
    if B > 3:
        ban[B - 1, 0], ban[B - 1, 1:6] = 5, [int(t) for t in rng.integers(0, V, 5)]  # a longer list
    dx, dn, dW, dban, dt = Dev(x), Dev(nw), Dev(bits), Dev(ban), Dev.zeros(B, np.int32)
    check(lib().dsocr_k_lmhead_screened(B, V, K, dx.ptr, dn.ptr, 1e-6, dW.ptr, dban.ptr, ban_ld, dt.ptr))
    got = dt.get()
    # the exact path: dec_gemv over the same rows (the engine's exact lm_head kernel for V > 16384)
    dy = Dev.zeros((B, V))
    check(lib().dsocr_k_gemv(B, V, K, dx.ptr, dn.ptr, 1e-6, dW.ptr, 0, None, dy.ptr, 0, 0))
    ex = dy.get()
    for b in range(B):
        row = ex[b].copy()
        for t in ban[b, 1:1 + ban[b, 0]]:
            row[t] = -np.inf
        assert got[b] == int(np.argmax(row)), (b, got[b], int(np.argmax(row)), row[[A, Bt, Cn, 4000]])
    assert got[1] != A and got[1] != Cn


@pytest.mark.parametrize("B,V", [(3, 50000), (8, 129280), (5, 1000)])
def test_screened_head_multi_token_random(gpu, B, V):
    """3..8 rows on the int8 matrix cores over random rows (vocab sizes incl. the model's 129280 and a
    partial last 16-row tile): the selected token of every row equals the exact GEMV's first-index argmax,
    with each row's top candidates placed at tile edges and a ban list on one row."""
    rng = np.random.default_rng(B * 7 + V)
    K = 1280
    x = rng.standard_normal((B, K)).astype(np.float32)
    nw = (1.0 + 0.05 * rng.standard_normal(K)).astype(np.float32)
    bits = bf16_round((rng.standard_normal((V, K)) * 0.02).astype(np.float32))
    xn = rms_norm(x, nw, 1e-6)
    for b in range(B):  # a strong row per page at a tile edge (row 16 t + 15) or the last row
        r = V - 1 if b == 0 else (int(rng.integers(0, V // 16)) * 16 + 15) % V
        bits[r] = bf16_round((xn[b] / np.linalg.norm(xn[b]) * 0.06 + rng.standard_normal(K) * 0.01).astype(np.float32))
    ban_ld = 8
    ban = np.zeros((B, ban_ld), np.int32)
    dy = Dev.zeros((B, V))
    dx, dn, dW = Dev(x), Dev(nw), Dev(bits)
    check(lib().dsocr_k_gemv(B, V, K, dx.ptr, dn.ptr, 1e-6, dW.ptr, 0, None, dy.ptr, 0, 0))
    ex = dy.get()
    ban[B - 1, 0], ban[B - 1, 1] = 1, int(np.argmax(ex[B - 1]))  # the last row's best is banned
    dban, dt = Dev(ban), Dev.zeros(B, np.int32)
    check(lib().dsocr_k_lmhead_screened(B, V, K, dx.ptr, dn.ptr, 1e-6, dW.ptr, dban.ptr, ban_ld, dt.ptr))
    got = dt.get()
    for b in range(B):
        row = ex[b].copy()
        for t in ban[b, 1:1 + ban[b, 0]]:
            row[t] = -np.inf
        assert got[b] == int(np.argmax(row)), (b, got[b], int(np.argmax(row)))


# ---------------------------------------------------------------- bf16-matrix-core attention (dots.ocr ViT)
@pytest.mark.parametrize("L,planes", [(1000, 3), (4133, 3), (130, 3), (20, 3), (1000, 2)])
def test_attention_bf16_pingpong_bitwise(gpu, monkeypatch, L, planes):
    """The 8-wave ping-pong kernel (128-dim heads, two wave groups one interval apart) runs the 4-wave kernel's
    products and sums in the same order per query: bitwise equal outputs (f32 and bf16 out), ragged lengths and
    fewer keys than one tile included."""
    rng = np.random.default_rng(L)
    heads, hd = 2, 128
    D = heads * hd
    qkv = rng.standard_normal((L, 3 * D)).astype(np.float32)
    qkv[:, :D] *= 0.6
    dq = Dev(bf16_round(qkv))
    outs = []
    for pp in ("1", "0"):
        monkeypatch.setenv("DSOCR_DOTS_ATTN_PP", pp)
        monkeypatch.setenv("DSOCR_DOTS_PV_PLANES", str(planes))
        do = Dev.zeros((L, D))
        check(lib().dsocr_k_attention_bf16(1, L, heads, hd, 1.0 / math.sqrt(hd), dq.ptr, 3 * D, do.ptr, D, 0))
        outs.append(do.get())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.parametrize("n_seq,L,heads,hd", [(1, 1000, 2, 128), (2, 257, 3, 64), (1, 64, 1, 128), (1, 4133, 2, 128),
                                              (1, 20, 2, 128), (2, 130, 2, 128), (1, 300, 1, 128)])
def test_attention_bf16_f32_math(gpu, n_seq, L, heads, hd):
    """attention_bf16 (dots_vit.rs:433-498 math: f32 scores / softmax / probs.V on bf16 q, k, v):
    exact bf16 products and a 3-plane exact split of P, so the result is an f32 attention up to
    summation order: <= 2e-5 of the f64 reference (the same bound as the f32-MFMA kernel)."""
    import ctypes as C
    rng = np.random.default_rng(L + hd)
    D = heads * hd
    qkv = rng.standard_normal((n_seq * L, 3 * D)).astype(np.float32)
    qkv[:, :D] *= 0.6
    bits = bf16_round(qkv)
    vals = bf16_to_f32(bits)
    dq = Dev(bits)
    do = Dev.zeros((n_seq * L, D))
    check(lib().dsocr_k_attention_bf16(n_seq, L, heads, hd, 1.0 / math.sqrt(hd), dq.ptr, 3 * D, do.ptr, D, 0))
    got = do.get()
    for s in range(n_seq):
        for h in range(heads):
            sl = slice(s * L, (s + 1) * L)
            q = vals[sl, h * hd:(h + 1) * hd]
            k = vals[sl, D + h * hd:D + (h + 1) * hd]
            v = vals[sl, 2 * D + h * hd:2 * D + (h + 1) * hd]
            ref = _attn_ref(q, k, v, 1.0 / math.sqrt(hd))
            assert np.max(np.abs(got[sl, h * hd:(h + 1) * hd] - ref)) < 2e-5, (s, h)
