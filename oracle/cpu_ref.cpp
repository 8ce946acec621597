// C++ / OpenMP CPU restatement of the DeepSeek-OCR decoder page path — TEST / BENCH INFRASTRUCTURE ONLY.
//
// bench.py's cpu_baseline leg times this on the GPU box's host cores (the reference's CPU backend is Rust +
// Candle, not buildable here: SURVEY §8c).  It is never linked into the product (deepseek-ocr.rs_amd/).
// Same f32 math as the numpy oracle (oracle/decoder.py, oracle/model.py), which restates:
//   * TransformerBlock::forward_internal  transformer/block.rs:124-191 (pre-norm, residual adds)
//   * rms_norm_slow                       block.rs:24-29       x / sqrt(mean(x^2) + eps) * w
//   * attention_forward                   block.rs:446-804     q/k/v linears, RoPE rotate_half on the full head
//                                                              (rope.rs:172-207, block.rs:1403-1471), causal -1e9
//                                                              bias in the prefill (block.rs:1504-1526), f32 KV
//                                                              cache (block.rs:776-789), softmax, o_proj
//   * run_dense_mlp                       block.rs:1179-1213   down(silu(gate x) * up x)
//   * run_moe                             block.rs:1215-1395   softmax router (+ correction bias), stable
//                                                              descending top-k, optional renormalise, scaling,
//                                                              per-expert SwiGLU, weighted combine + shared experts
//   * final norm + lm_head                transformer/model.rs:207-270
//   * select_token_id (greedy)            core/src/sampling.rs:34-158: n-gram ban over prompt + generated,
//                                                              first-index argmax skipping non-finite, fallbacks
//   * generate                            model/mod.rs:1870-2048 (prefill, then one forward per token)
// Weights arrive from the oracle's loader (oracle/weights.py: the reference's --dtype f16 rounding already
// applied); the decoder's 16-bit values are kept as f16 (exact) and widened to f32 at use, the lm_head as
// bf16 (exact), norms in f32.  Linear algebra: AVX-512 dot-product micro-kernels, OpenMP over output rows.
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct Tensor {
    int kind = 0;  // 0 f32, 1 f16, 2 bf16
    std::vector<float> f;
    std::vector<uint16_t> h;
    long rows = 0, cols = 0;
};
std::unordered_map<std::string, Tensor> g_w;

struct Cfg {
    int H, heads, kv_heads, hd, layers, vocab, inter, moe_inter, E, topk, n_shared, norm_topk, softmax_scoring;
    float eps, rope_theta, scaling;
};
Cfg g_c;
std::vector<int> g_moe;

inline uint16_t f32_to_f16_bits(float v) { return (uint16_t)_cvtss_sh(v, _MM_FROUND_TO_NEAREST_INT); }

const Tensor& W(const std::string& n) {
    auto it = g_w.find(n);
    if (it == g_w.end()) throw std::runtime_error("cpu_ref: missing tensor " + n);
    return it->second;
}
bool has(const std::string& n) { return g_w.count(n) != 0; }

inline __m512 load16(const Tensor& t, long off) {
    if (t.kind == 1) return _mm512_cvtph_ps(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(t.h.data() + off)));
    if (t.kind == 2) {
        const __m512i v = _mm512_cvtepu16_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(t.h.data() + off)));
        return _mm512_castsi512_ps(_mm512_slli_epi32(v, 16));
    }
    return _mm512_loadu_ps(t.f.data() + off);
}
inline float load1(const Tensor& t, long off) {
    if (t.kind == 1) return _cvtsh_ss(t.h[off]);
    if (t.kind == 2) {
        uint32_t b = (uint32_t)t.h[off] << 16;
        float f;
        memcpy(&f, &b, 4);
        return f;
    }
    return t.f[off];
}

// Y[m][n] = X[m] . W[n] (+ b[n]) for m < M, n < N (K % 16 == 0): MR x NR register tiles of 16-wide dot
// accumulators (MR x NR + NR + 1 <= 32 zmm: 4 x 4 for the prefill GEMMs, 1 x 8 for the decode GEMVs), the
// weight type a template parameter (no branch in the k loop), M chunked so the activation rows stay in L2,
// OpenMP over NR-row weight blocks.
template <int KIND>
inline __m512 ld16(const uint16_t* h, const float* f, long off) {
    if (KIND == 1) return _mm512_cvtph_ps(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(h + off)));
    if (KIND == 2) {
        const __m512i v = _mm512_cvtepu16_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(h + off)));
        return _mm512_castsi512_ps(_mm512_slli_epi32(v, 16));
    }
    return _mm512_loadu_ps(f + off);
}

template <int KIND, int MR, int NR>
inline void tile(const float* X, int K, const Tensor& w, const Tensor* b, float* Y, int N, int m0, int n0, int nn) {
    const uint16_t* h = w.h.data();
    const float* f = w.f.data();
    __m512 acc[MR][NR];
    for (int i = 0; i < MR; ++i)
        for (int j = 0; j < NR; ++j) acc[i][j] = _mm512_setzero_ps();
    long wo[NR];
    for (int j = 0; j < NR; ++j) wo[j] = (long)(n0 + std::min(j, nn - 1)) * K;
    const float* xr[MR];
    for (int i = 0; i < MR; ++i) xr[i] = X + (long)(m0 + i) * K;
    for (int k = 0; k < K; k += 16) {
        __m512 wv[NR];
        for (int j = 0; j < NR; ++j) wv[j] = ld16<KIND>(h, f, wo[j] + k);
        for (int i = 0; i < MR; ++i) {
            const __m512 xv = _mm512_loadu_ps(xr[i] + k);
            for (int j = 0; j < NR; ++j) acc[i][j] = _mm512_fmadd_ps(xv, wv[j], acc[i][j]);
        }
    }
    for (int i = 0; i < MR; ++i)
        for (int j = 0; j < nn; ++j) {
            float v = _mm512_reduce_add_ps(acc[i][j]);
            if (b) v += b->f[n0 + j];
            Y[(long)(m0 + i) * N + n0 + j] = v;
        }
}

template <int KIND>
void linear_t(const float* X, int M, int K, const Tensor& w, const Tensor* b, float* Y, int N) {
    if (M < 4) {  // decode: GEMV-shaped, 8 weight rows per tile (memory-bound)
        const int nb = (N + 7) / 8;
#pragma omp parallel for schedule(static)
        for (int ib = 0; ib < nb; ++ib) {
            const int n0 = ib * 8, nn = std::min(8, N - n0);
            for (int m = 0; m < M; ++m) tile<KIND, 1, 8>(X, K, w, b, Y, N, m, n0, nn);
        }
        return;
    }
    const int nb = (N + 3) / 4;
    for (int m0 = 0; m0 < M; m0 += 128) {
        const int mc = std::min(128, M - m0);
#pragma omp parallel for schedule(static)
        for (int ib = 0; ib < nb; ++ib) {
            const int n0 = ib * 4, nn = std::min(4, N - n0);
            int mm = 0;
            for (; mm + 4 <= mc; mm += 4) tile<KIND, 4, 4>(X, K, w, b, Y, N, m0 + mm, n0, nn);
            for (; mm < mc; ++mm) tile<KIND, 1, 4>(X, K, w, b, Y, N, m0 + mm, n0, nn);
        }
    }
}

// kind 3 (the vision tower's bf16 weights, round 5): packed 32-column panels for the large-M GEMMs.  Panel p holds
// columns 32p .. 32p + 31 as [K][16] dwords, dword i = bf16(W[32p + i][k]) | bf16(W[32p + 16 + i][k]) << 16, so a
// k-step is one 64-B load, a shift (columns 0..15) and a mask (16..31).  The micro-kernel keeps MR rows x 32
// columns in 2 MR accumulators and broadcasts one activation per row and k (outer products), instead of the
// dot-product tiles' per-tile horizontal reductions.
template <int MR>
inline void pk_tile(const float* X, long ldx, int K, const uint32_t* P, const float* bias, float* Y, long ldy, int nc) {
    __m512 a0[MR], a1[MR];
    for (int r = 0; r < MR; ++r) { a0[r] = _mm512_setzero_ps(); a1[r] = _mm512_setzero_ps(); }
    const __m512i hi_mask = _mm512_set1_epi32((int)0xffff0000u);
    for (int k = 0; k < K; ++k) {
        const __m512i raw = _mm512_loadu_si512(P + (size_t)k * 16);
        const __m512 w0 = _mm512_castsi512_ps(_mm512_slli_epi32(raw, 16));
        const __m512 w1 = _mm512_castsi512_ps(_mm512_and_si512(raw, hi_mask));
        for (int r = 0; r < MR; ++r) {
            const __m512 xb = _mm512_set1_ps(X[(long)r * ldx + k]);
            a0[r] = _mm512_fmadd_ps(xb, w0, a0[r]);
            a1[r] = _mm512_fmadd_ps(xb, w1, a1[r]);
        }
    }
    const __mmask16 m0 = nc >= 16 ? (__mmask16)0xffff : (__mmask16)((1u << nc) - 1);
    const __mmask16 m1 = nc >= 32 ? (__mmask16)0xffff : (nc > 16 ? (__mmask16)((1u << (nc - 16)) - 1) : (__mmask16)0);
    const __m512 b0 = bias ? _mm512_maskz_loadu_ps(m0, bias) : _mm512_setzero_ps();
    const __m512 b1 = bias ? _mm512_maskz_loadu_ps(m1, bias + 16) : _mm512_setzero_ps();
    for (int r = 0; r < MR; ++r) {
        _mm512_mask_storeu_ps(Y + (long)r * ldy, m0, _mm512_add_ps(a0[r], b0));
        _mm512_mask_storeu_ps(Y + (long)r * ldy + 16, m1, _mm512_add_ps(a1[r], b1));
    }
}

void linear_packed(const float* X, int M, int K, const Tensor& w, const Tensor* b, float* Y, int N) {
    const int np = (N + 31) / 32;
    constexpr int MB = 96;  // rows per work item (8 tiles of 12): the panel stays in L1 / L2 across them
    const int nmb = (M + MB - 1) / MB;
    const uint32_t* P = reinterpret_cast<const uint32_t*>(w.h.data());
#pragma omp parallel for schedule(dynamic, 2) collapse(2)
    for (int mb = 0; mb < nmb; ++mb)
        for (int p = 0; p < np; ++p) {
            const uint32_t* pp = P + (size_t)p * K * 16;
            const int nc = std::min(32, N - 32 * p);
            const float* bias = b ? b->f.data() + 32 * p : nullptr;
            int m = mb * MB;
            const int me = std::min(M, m + MB);
            for (; m + 12 <= me; m += 12) pk_tile<12>(X + (long)m * K, K, K, pp, bias, Y + (long)m * N + 32 * p, N, nc);
            for (; m + 4 <= me; m += 4) pk_tile<4>(X + (long)m * K, K, K, pp, bias, Y + (long)m * N + 32 * p, N, nc);
            for (; m < me; ++m) pk_tile<1>(X + (long)m * K, K, K, pp, bias, Y + (long)m * N + 32 * p, N, nc);
        }
}

double g_lin_ms = 0, g_att_ms = 0;  // stage clocks (cr_profile)

void linear(const float* X, int M, int K, const Tensor& w, const Tensor* b, float* Y, int N) {
    if (K % 16) throw std::runtime_error("cpu_ref: K % 16 != 0");
    struct Clk {
        std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
        ~Clk() { g_lin_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count(); }
    } clk;
    if (w.kind == 3) linear_packed(X, M, K, w, b, Y, N);
    else if (w.kind == 1) linear_t<1>(X, M, K, w, b, Y, N);
    else if (w.kind == 2) linear_t<2>(X, M, K, w, b, Y, N);
    else linear_t<0>(X, M, K, w, b, Y, N);
}

void rms_norm(const float* x, int M, int K, const float* w, float eps, float* y) {
#pragma omp parallel for schedule(static) if (M > 8)
    for (int m = 0; m < M; ++m) {
        const float* xr = x + (long)m * K;
        float s = 0.f;
        for (int k = 0; k < K; ++k) s += xr[k] * xr[k];
        const float den = std::sqrt(s / (float)K + eps);
        for (int k = 0; k < K; ++k) y[(long)m * K + k] = (xr[k] / den) * w[k];
    }
}

inline float silu(float v) { return v / (1.f + std::exp(-v)); }

struct KV {
    std::vector<float> k, v;  // [kv_heads][cap][hd]
    int cap = 0;
};
std::vector<KV> g_kv;
int g_past = 0;
std::vector<float> g_cos, g_sin;  // [cap][hd]

void rope_tables(int cap) {
    const int hd = g_c.hd, half = hd / 2;
    g_cos.assign((size_t)cap * hd, 0.f);
    g_sin.assign((size_t)cap * hd, 0.f);
    std::vector<float> inv(half);
    for (int i = 0; i < half; ++i) inv[i] = 1.0f / std::pow(g_c.rope_theta, (float)(i * 2.0) / (float)hd);
    for (int p = 0; p < cap; ++p)
        for (int i = 0; i < half; ++i) {
            const float a = (float)p * inv[i];
            g_cos[(size_t)p * hd + i] = g_cos[(size_t)p * hd + half + i] = std::cos(a);
            g_sin[(size_t)p * hd + i] = g_sin[(size_t)p * hd + half + i] = std::sin(a);
        }
}

void rope(float* v, int pos) {  // rotate_half over the head
    const int hd = g_c.hd, half = hd / 2;
    const float* c = g_cos.data() + (size_t)pos * hd;
    const float* s = g_sin.data() + (size_t)pos * hd;
    float t[512];
    for (int i = 0; i < hd; ++i) t[i] = i < half ? -v[i + half] : v[i - half];
    for (int i = 0; i < hd; ++i) v[i] = v[i] * c[i] + t[i] * s[i];
}

// one layer's attention over S new rows (positions g_past ..), xn normalised input, out += o_proj
void attention(int li, const float* xn, int S, float* out) {
    const Cfg& c = g_c;
    const std::string pre = "model.layers." + std::to_string(li) + ".self_attn.";
    const int qn = c.heads * c.hd, kn = c.kv_heads * c.hd;
    std::vector<float> q((size_t)S * qn), k((size_t)S * kn), v((size_t)S * kn);
    auto bias = [&](const std::string& n) { return has(n) ? &W(n) : nullptr; };
    linear(xn, S, c.H, W(pre + "q_proj.weight"), bias(pre + "q_proj.bias"), q.data(), qn);
    linear(xn, S, c.H, W(pre + "k_proj.weight"), bias(pre + "k_proj.bias"), k.data(), kn);
    linear(xn, S, c.H, W(pre + "v_proj.weight"), bias(pre + "v_proj.bias"), v.data(), kn);
    KV& kv = g_kv[li];
    for (int s = 0; s < S; ++s) {
        for (int h = 0; h < c.heads; ++h) rope(q.data() + (size_t)s * qn + h * c.hd, g_past + s);
        for (int h = 0; h < c.kv_heads; ++h) {
            rope(k.data() + (size_t)s * kn + h * c.hd, g_past + s);
            memcpy(kv.k.data() + ((size_t)h * kv.cap + g_past + s) * c.hd, k.data() + (size_t)s * kn + h * c.hd, c.hd * 4);
            memcpy(kv.v.data() + ((size_t)h * kv.cap + g_past + s) * c.hd, v.data() + (size_t)s * kn + h * c.hd, c.hd * 4);
        }
    }
    std::vector<float> o((size_t)S * qn);
    const auto ta = std::chrono::steady_clock::now();
    const float scale = 1.0f / std::sqrt((float)c.hd);
    const int rep = c.heads / c.kv_heads;
    const int L = g_past + S;
#pragma omp parallel
    {
        std::vector<float> sc(L);
#pragma omp for schedule(dynamic) collapse(2)
        for (int h = 0; h < c.heads; ++h)
            for (int s = 0; s < S; ++s) {
                const float* qr = q.data() + (size_t)s * qn + h * c.hd;
                const float* K = kv.k.data() + (size_t)(h / rep) * kv.cap * c.hd;
                const float* V = kv.v.data() + (size_t)(h / rep) * kv.cap * c.hd;
                // the prefill's causal bias puts -1e9 on the keys past s: their exp underflows to exactly 0, so
                // they are skipped (the same softmax)
                const int n = (S > 1 && g_past == 0) ? s + 1 : L;
                float mx = -INFINITY;
                for (int t = 0; t < n; ++t) {
                    const float* kr = K + (size_t)t * c.hd;
                    __m512 acc = _mm512_setzero_ps();
                    for (int i = 0; i < c.hd; i += 16) acc = _mm512_fmadd_ps(_mm512_loadu_ps(qr + i), _mm512_loadu_ps(kr + i), acc);
                    const float d = _mm512_reduce_add_ps(acc) * scale;
                    sc[t] = d;
                    mx = std::max(mx, d);
                }
                float sum = 0.f;
                for (int t = 0; t < n; ++t) { sc[t] = std::exp(sc[t] - mx); sum += sc[t]; }
                float* orow = o.data() + (size_t)s * qn + h * c.hd;
                for (int i = 0; i < c.hd; ++i) orow[i] = 0.f;
                for (int t = 0; t < n; ++t) {
                    const float p = sc[t] / sum;
                    if (p == 0.f) continue;
                    for (int i = 0; i < c.hd; ++i) orow[i] += p * V[(size_t)t * c.hd + i];
                }
            }
    }
    g_att_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
    std::vector<float> y((size_t)S * c.H);
    linear(o.data(), S, qn, W(pre + "o_proj.weight"), bias(pre + "o_proj.bias"), y.data(), c.H);
    for (size_t i = 0; i < y.size(); ++i) out[i] += y[i];
}

// down(silu(gate x) * up x) for M rows of x
void dense_mlp(const float* x, int M, const std::string& pre, int inter, float* y) {
    std::vector<float> g((size_t)M * inter), u((size_t)M * inter);
    linear(x, M, g_c.H, W(pre + "gate_proj.weight"), nullptr, g.data(), inter);
    linear(x, M, g_c.H, W(pre + "up_proj.weight"), nullptr, u.data(), inter);
    for (size_t i = 0; i < g.size(); ++i) g[i] = silu(g[i]) * u[i];
    linear(g.data(), M, inter, W(pre + "down_proj.weight"), nullptr, y, g_c.H);
}

void moe(int li, const float* xn, int T, float* out) {
    const Cfg& c = g_c;
    const std::string pre = "model.layers." + std::to_string(li) + ".mlp.";
    std::vector<float> lg((size_t)T * c.E);
    linear(xn, T, c.H, W(pre + "gate.weight"), nullptr, lg.data(), c.E);
    const std::string cb = pre + "gate.e_score_correction_bias";
    std::vector<int> pick((size_t)T * c.topk);
    std::vector<float> pw((size_t)T * c.topk);
    for (int t = 0; t < T; ++t) {
        float* l = lg.data() + (size_t)t * c.E;
        if (has(cb))
            for (int e = 0; e < c.E; ++e) l[e] += W(cb).f[e];
        std::vector<float> sc(c.E);
        if (c.softmax_scoring) {
            float mx = -INFINITY, sum = 0.f;
            for (int e = 0; e < c.E; ++e) mx = std::max(mx, l[e]);
            for (int e = 0; e < c.E; ++e) { sc[e] = std::exp(l[e] - mx); sum += sc[e]; }
            for (int e = 0; e < c.E; ++e) sc[e] /= sum;
        } else {
            for (int e = 0; e < c.E; ++e) sc[e] = 1.f / (1.f + std::exp(-l[e]));
        }
        std::vector<int> ord(c.E);
        for (int e = 0; e < c.E; ++e) ord[e] = e;
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return sc[a] > sc[b]; });
        float ws = 0.f;
        for (int k = 0; k < c.topk; ++k) { pick[t * c.topk + k] = ord[k]; pw[t * c.topk + k] = sc[ord[k]]; ws += sc[ord[k]]; }
        for (int k = 0; k < c.topk; ++k) {
            if (c.topk > 1 && c.norm_topk) pw[t * c.topk + k] /= (ws + 1e-20f);
            if (c.scaling != 1.0f) pw[t * c.topk + k] *= c.scaling;
        }
    }
    // experts in ascending id order over the rows that picked them
    std::vector<float> outs((size_t)T * c.topk * c.H, 0.f);
    for (int e = 0; e < c.E; ++e) {
        std::vector<int> rows, slots;
        for (int t = 0; t < T; ++t)
            for (int k = 0; k < c.topk; ++k)
                if (pick[t * c.topk + k] == e) { rows.push_back(t); slots.push_back(k); }
        if (rows.empty()) continue;
        const int n = (int)rows.size();
        std::vector<float> xs((size_t)n * c.H), ys((size_t)n * c.H);
        for (int i = 0; i < n; ++i) memcpy(xs.data() + (size_t)i * c.H, xn + (size_t)rows[i] * c.H, c.H * 4);
        dense_mlp(xs.data(), n, pre + "experts." + std::to_string(e) + ".", c.moe_inter, ys.data());
        for (int i = 0; i < n; ++i)
            memcpy(outs.data() + ((size_t)rows[i] * c.topk + slots[i]) * c.H, ys.data() + (size_t)i * c.H, c.H * 4);
    }
    std::vector<float> sh;
    if (c.n_shared > 0) {
        sh.resize((size_t)T * c.H);
        dense_mlp(xn, T, pre + "shared_experts.", c.moe_inter * c.n_shared, sh.data());
    }
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < c.H; ++j) {
            float comb = 0.f;
            for (int k = 0; k < c.topk; ++k) comb += outs[((size_t)t * c.topk + k) * c.H + j] * pw[t * c.topk + k];
            if (c.n_shared > 0) comb += sh[(size_t)t * c.H + j];
            out[(size_t)t * c.H + j] += comb;
        }
}

// rows x [S][H] (positions g_past ..) through every layer -> last row's logits
void forward(std::vector<float>& x, int S, std::vector<float>& logits) {
    const Cfg& c = g_c;
    std::vector<float> xn((size_t)S * c.H), m((size_t)S * c.H);
    for (int li = 0; li < c.layers; ++li) {
        const std::string pre = "model.layers." + std::to_string(li) + ".";
        rms_norm(x.data(), S, c.H, W(pre + "input_layernorm.weight").f.data(), c.eps, xn.data());
        attention(li, xn.data(), S, x.data());  // h = x + attn
        rms_norm(x.data(), S, c.H, W(pre + "post_attention_layernorm.weight").f.data(), c.eps, xn.data());
        if (g_moe[li]) {
            moe(li, xn.data(), S, x.data());
        } else {
            dense_mlp(xn.data(), S, pre + "mlp.", c.inter, m.data());
            for (size_t i = 0; i < m.size(); ++i) x[i] += m[i];
        }
    }
    g_past += S;
    std::vector<float> last(c.H);
    rms_norm(x.data() + (size_t)(S - 1) * c.H, 1, c.H, W("model.norm.weight").f.data(), c.eps, last.data());
    logits.resize(c.vocab);
    linear(last.data(), 1, c.H, W("lm_head.weight"), nullptr, logits.data(), c.vocab);
}

// greedy select_token_id (sampling.rs:34-158) without repetition penalty
int select(const std::vector<float>& lg, const std::vector<int>& ctx, int ngram) {
    std::vector<char> ban(lg.size(), 0);
    const int n = (int)ctx.size();
    if (ngram > 1 && n >= ngram - 1)
        for (int i = 0; i <= n - ngram; ++i) {
            bool match = true;
            for (int j = 0; j < ngram - 1; ++j)
                if (ctx[i + j] != ctx[n - ngram + 1 + j]) { match = false; break; }
            if (match) ban[ctx[i + ngram - 1]] = 1;
        }
    int best = -1;
    float bv = -INFINITY;
    for (size_t v = 0; v < lg.size(); ++v)
        if (!ban[v] && std::isfinite(lg[v]) && (best < 0 || lg[v] > bv)) { bv = lg[v]; best = (int)v; }
    if (best >= 0) return best;
    for (size_t v = 0; v < lg.size(); ++v)
        if (std::isfinite(lg[v]) && (best < 0 || lg[v] > bv)) { bv = lg[v]; best = (int)v; }
    return best < 0 ? 0 : best;
}


// ====================================================================== vision tower (round 5)
// SAM-ViTDet-B + CLIP-L + linear projector, the same f32 math as the numpy oracle (oracle/vision.py), which
// restates vision/sam.rs, vision/clip.rs and model/mod.rs:246-923:
//   * patch embed (16x16 conv as im2col + linear)    sam.rs:210-246
//   * SamBlock: LN -> (window partition, pad with zeros) -> attention with the decomposed rel-pos bias
//     (sam.rs:804-888: scores * scale + q.Rh[qh][kh] + q.Rw[qw][kw]) -> unpartition -> residual -> LN ->
//     fc1 -> GELU-erf -> fc2 -> residual                 sam.rs:731-748, 926-980
//   * neck (1x1 conv, LN2d, 3x3 conv, LN2d) + two stride-2 3x3 convs      sam.rs:503-575
//   * CLIP: class token + patches + position table, pre-LN, 24 x (LN, MHA, residual, LN, fc1, quick-GELU,
//     fc2, residual)                                    clip.rs:98-102, 349-416
//   * projector over [clip tokens 1.. | sam tokens]     model/mod.rs:392-444, 604-650
// The position-embedding resizes and the rel-pos tables depend only on the weights and the grid: the Python
// side (CpuVision) computes them once with the oracle's functions and hands them over as tensors.
struct VCfg {
    int embed, depth, heads, window, neck, c0, c1, patch;
    float sam_eps;
    int clip_h, clip_layers, clip_heads, clip_ffn;
    float clip_eps;
    int n_embed, in_dim;
    std::vector<int> global;
};
VCfg g_v;
double g_vis_prof[6];  // ms: layer norms, activations, window / im2col copies, residual adds (DSOCR_CV_PROF=1)
struct VClk {
    int slot;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    explicit VClk(int s) : slot(s) {}
    ~VClk() { g_vis_prof[slot] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count(); }
};

const Tensor* opt(const std::string& n) { return has(n) ? &W(n) : nullptr; }

void layer_norm_rows(const float* x, long M, int C, const float* w, const float* b, float eps, float* y) {
    VClk clk(0);
#pragma omp parallel for schedule(static)
    for (long m = 0; m < M; ++m) {
        const float* xr = x + m * C;
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += xr[c];
        const float mean = s / (float)C;
        float v = 0.f;
        for (int c = 0; c < C; ++c) v += (xr[c] - mean) * (xr[c] - mean);
        const float den = std::sqrt(v / (float)C + eps);
        float* yr = y + m * C;
        for (int c = 0; c < C; ++c) yr[c] = ((xr[c] - mean) / den) * w[c] + b[c];
    }
}

// multi-head attention over n sequences of L rows: qkv [n][L][3C] (q | k | v, head-major inside each), ctx
// [n][L][C]; optional decomposed rel-pos bias (L = h * w, tables [h][h][hd] and [w][w][hd]).  Scores for a
// block of 4 query rows against every key by broadcast FMAs over K^T (built once per sequence and head),
// softmax (exp(s - max) / sum), then P.V with the 4 rows' dims in registers.
// exp on 16 lanes: n = round(x log2 e), r = x - n ln2 (two-part ln2), degree-6 polynomial, scaled by 2^n
// (within ~2 ulp of expf over the softmax's range x <= 0; the vision leg's tolerance vs the oracle is 1e-4)
inline __m512 exp16(__m512 x) {
    x = _mm512_max_ps(x, _mm512_set1_ps(-87.3f));
    const __m512 n = _mm512_roundscale_ps(_mm512_mul_ps(x, _mm512_set1_ps(1.44269504088896341f)), _MM_FROUND_TO_NEAREST_INT);
    __m512 r = _mm512_fnmadd_ps(n, _mm512_set1_ps(0.693359375f), x);
    r = _mm512_fnmadd_ps(n, _mm512_set1_ps(-2.12194440e-4f), r);
    __m512 p = _mm512_set1_ps(1.3981999507e-3f);
    p = _mm512_fmadd_ps(p, r, _mm512_set1_ps(8.3334519073e-3f));
    p = _mm512_fmadd_ps(p, r, _mm512_set1_ps(4.1665795894e-2f));
    p = _mm512_fmadd_ps(p, r, _mm512_set1_ps(1.6666665459e-1f));
    p = _mm512_fmadd_ps(p, r, _mm512_set1_ps(5.0000001201e-1f));
    p = _mm512_fmadd_ps(p, _mm512_mul_ps(r, r), _mm512_add_ps(r, _mm512_set1_ps(1.0f)));
    return _mm512_scalef_ps(p, n);
}

// multi-head attention over n sequences of L rows: qkv [n][L][3C] (q | k | v, head-major inside each), ctx
// [n][L][C]; optional decomposed rel-pos bias (L = h * w, tables [h][h][hd] and [w][w][hd]).  K^T and V are
// copied once per (sequence, head) into contiguous [hd][Lp] / [L][hd] buffers; a work item is 16 query rows:
// their scores against every key by broadcast FMAs over K^T, scale + bias, softmax (exp(s - max) / sum), then
// P.V for 8 rows x 32 dims at a time.
template <int ND>  // hd / 16
void attention_core(const float* qkv, int n, int L, int C, int nh, const float* Rh, const float* Rw, int h, int w,
                    float* ctx) {
    constexpr int hd = ND * 16, QB = 16;
    const int Lp = (L + 15) & ~15, C3 = 3 * C;
    const float scale = 1.0f / std::sqrt((float)hd);
    std::vector<float> kt((size_t)n * nh * hd * Lp, 0.f), vv((size_t)n * nh * L * hd);
#pragma omp parallel for schedule(static) collapse(2)
    for (int i = 0; i < n; ++i)
        for (int hh = 0; hh < nh; ++hh) {
            float* K = kt.data() + ((size_t)i * nh + hh) * hd * Lp;
            float* V = vv.data() + ((size_t)i * nh + hh) * L * hd;
            for (int k = 0; k < L; ++k) {
                const float* kr = qkv + ((size_t)i * L + k) * C3 + C + hh * hd;
                for (int d = 0; d < hd; ++d) K[(size_t)d * Lp + k] = kr[d];
                memcpy(V + (size_t)k * hd, kr + C, hd * 4);
            }
        }
    const int nqb = (L + QB - 1) / QB;
#pragma omp parallel
    {
        std::vector<float> S((size_t)QB * Lp);
        std::vector<float> rh((size_t)QB * std::max(h, 1)), rw((size_t)QB * std::max(w, 1));
#pragma omp for schedule(dynamic, 2) collapse(3)
        for (int i = 0; i < n; ++i)
            for (int hh = 0; hh < nh; ++hh)
                for (int qb = 0; qb < nqb; ++qb) {
                    const int q0 = qb * QB, nq = std::min(QB, L - q0);
                    const float* K = kt.data() + ((size_t)i * nh + hh) * hd * Lp;
                    const float* V = vv.data() + ((size_t)i * nh + hh) * L * hd;
                    const float* Q[QB];
                    for (int r = 0; r < QB; ++r) Q[r] = qkv + ((size_t)i * L + q0 + std::min(r, nq - 1)) * C3 + hh * hd;
                    // 8 query rows x 32 keys per pass (2 K^T loads + 8 broadcasts per 16 FMAs)
                    for (int rh0 = 0; rh0 < QB; rh0 += 8)
                        for (int kb = 0; kb < Lp; kb += 32) {
                            const bool two = kb + 16 < Lp;
                            __m512 a0[8], a1[8];
                            for (int r = 0; r < 8; ++r) { a0[r] = _mm512_setzero_ps(); a1[r] = _mm512_setzero_ps(); }
                            for (int d = 0; d < hd; ++d) {
                                const __m512 k0 = _mm512_loadu_ps(K + (size_t)d * Lp + kb);
                                const __m512 k1 = two ? _mm512_loadu_ps(K + (size_t)d * Lp + kb + 16) : _mm512_setzero_ps();
                                for (int r = 0; r < 8; ++r) {
                                    const __m512 qb_ = _mm512_set1_ps(Q[rh0 + r][d]);
                                    a0[r] = _mm512_fmadd_ps(qb_, k0, a0[r]);
                                    a1[r] = _mm512_fmadd_ps(qb_, k1, a1[r]);
                                }
                            }
                            for (int r = 0; r < 8; ++r) {
                                _mm512_storeu_ps(S.data() + (size_t)(rh0 + r) * Lp + kb, a0[r]);
                                if (two) _mm512_storeu_ps(S.data() + (size_t)(rh0 + r) * Lp + kb + 16, a1[r]);
                            }
                        }
                    if (Rh) {
                        for (int r = 0; r < nq; ++r) {
                            const int q = q0 + r, qh = q / w, qw = q % w;
                            for (int kh = 0; kh < h; ++kh) {
                                const float* t = Rh + ((size_t)qh * h + kh) * hd;
                                __m512 a = _mm512_setzero_ps();
                                for (int d = 0; d < hd; d += 16) a = _mm512_fmadd_ps(_mm512_loadu_ps(Q[r] + d), _mm512_loadu_ps(t + d), a);
                                rh[r * h + kh] = _mm512_reduce_add_ps(a);
                            }
                            for (int kw = 0; kw < w; ++kw) {
                                const float* t = Rw + ((size_t)qw * w + kw) * hd;
                                __m512 a = _mm512_setzero_ps();
                                for (int d = 0; d < hd; d += 16) a = _mm512_fmadd_ps(_mm512_loadu_ps(Q[r] + d), _mm512_loadu_ps(t + d), a);
                                rw[r * w + kw] = _mm512_reduce_add_ps(a);
                            }
                        }
                    }
                    for (int r = 0; r < QB; ++r) {
                        float* sr = S.data() + (size_t)r * Lp;
                        if (r >= nq) { std::fill(sr, sr + Lp, 0.f); continue; }
                        __m512 mv = _mm512_set1_ps(-INFINITY);
                        const __m512 sc = _mm512_set1_ps(scale);
                        for (int k = 0; k < Lp; k += 16) {
                            const __mmask16 mk = (L - k) >= 16 ? (__mmask16)0xffff : (__mmask16)((1u << (L - k)) - 1);
                            __m512 v = _mm512_mul_ps(_mm512_loadu_ps(sr + k), sc);
                            if (Rh && w % 16 == 0) {  // the 16 keys share kh = k / w; kw = k % w .. + 15
                                v = _mm512_add_ps(v, _mm512_add_ps(_mm512_set1_ps(rh[r * h + k / w]), _mm512_loadu_ps(&rw[r * w + k % w])));
                            } else if (Rh) {
                                alignas(64) float bias[16];
                                for (int t = 0; t < 16; ++t) {
                                    const int kk = std::min(k + t, L - 1);
                                    bias[t] = rh[r * h + kk / w] + rw[r * w + kk % w];
                                }
                                v = _mm512_add_ps(v, _mm512_load_ps(bias));
                            }
                            v = _mm512_mask_blend_ps(mk, _mm512_set1_ps(-INFINITY), v);
                            _mm512_storeu_ps(sr + k, v);
                            mv = _mm512_max_ps(mv, v);
                        }
                        const __m512 mx = _mm512_set1_ps(_mm512_reduce_max_ps(mv));
                        __m512 sv = _mm512_setzero_ps();
                        for (int k = 0; k < Lp; k += 16) {
                            const __mmask16 mk = (L - k) >= 16 ? (__mmask16)0xffff : (__mmask16)((1u << (L - k)) - 1);
                            const __m512 e = _mm512_maskz_mov_ps(mk, exp16(_mm512_sub_ps(_mm512_loadu_ps(sr + k), mx)));
                            _mm512_storeu_ps(sr + k, e);
                            sv = _mm512_add_ps(sv, e);
                        }
                        const __m512 sum = _mm512_set1_ps(_mm512_reduce_add_ps(sv));
                        for (int k = 0; k < Lp; k += 16) _mm512_storeu_ps(sr + k, _mm512_div_ps(_mm512_loadu_ps(sr + k), sum));
                    }
                    for (int r0 = 0; r0 < nq; r0 += 8) {
                        for (int j = 0; j < ND; j += 2) {
                            __m512 o0[8], o1[8];
                            for (int r = 0; r < 8; ++r) { o0[r] = _mm512_setzero_ps(); o1[r] = _mm512_setzero_ps(); }
                            for (int k = 0; k < L; ++k) {
                                const __m512 v0 = _mm512_loadu_ps(V + (size_t)k * hd + 16 * j);
                                const __m512 v1 = _mm512_loadu_ps(V + (size_t)k * hd + 16 * j + 16);
                                for (int r = 0; r < 8; ++r) {
                                    const __m512 pb = _mm512_set1_ps(S[(size_t)(r0 + r) * Lp + k]);
                                    o0[r] = _mm512_fmadd_ps(pb, v0, o0[r]);
                                    o1[r] = _mm512_fmadd_ps(pb, v1, o1[r]);
                                }
                            }
                            for (int r = 0; r < 8 && r0 + r < nq; ++r) {
                                float* orow = ctx + ((size_t)i * L + q0 + r0 + r) * C + hh * hd + 16 * j;
                                _mm512_storeu_ps(orow, o0[r]);
                                _mm512_storeu_ps(orow + 16, o1[r]);
                            }
                        }
                    }
                }
    }
}

void attention_any(const float* qkv, int n, int L, int C, int nh, const float* Rh, const float* Rw, int h, int w,
                   float* ctx) {
    const int hd = C / nh;
    if (hd == 64) attention_core<4>(qkv, n, L, C, nh, Rh, Rw, h, w, ctx);
    else if (hd == 32) attention_core<2>(qkv, n, L, C, nh, Rh, Rw, h, w, ctx);
    else if (hd == 128) attention_core<8>(qkv, n, L, C, nh, Rh, Rw, h, w, ctx);
    else throw std::runtime_error("cpu_ref vision: head dim must be 32, 64 or 128");
}

inline float gelu_erf(float v) { return 0.5f * v * (1.0f + std::erf(v * 0.70710678118654752f)); }

// conv (no bias) on NHWC x [B][H][W][C] with the weight re-laid [O][kh][kw][C] (CpuVision does it): im2col + linear
void conv_nhwc(const float* x, int B, int H, int Wd, int C, const Tensor& w, int O, int k, int stride, int pad,
               std::vector<float>& y, int& oh, int& ow) {
    oh = (H + 2 * pad - k) / stride + 1;
    ow = (Wd + 2 * pad - k) / stride + 1;
    const long rows = (long)B * oh * ow, K = (long)k * k * C;
    VClk clk2(2);
    std::vector<float> cols((size_t)rows * K);
#pragma omp parallel for schedule(static)
    for (long r = 0; r < rows; ++r) {
        const int b = (int)(r / ((long)oh * ow)), oy = (int)(r / ow % oh), ox = (int)(r % ow);
        float* cr = cols.data() + (size_t)r * K;
        for (int ky = 0; ky < k; ++ky)
            for (int kx = 0; kx < k; ++kx) {
                const int iy = oy * stride + ky - pad, ix = ox * stride + kx - pad;
                float* dst = cr + ((size_t)ky * k + kx) * C;
                if (iy < 0 || iy >= H || ix < 0 || ix >= Wd) std::fill(dst, dst + C, 0.f);
                else memcpy(dst, x + (((size_t)b * H + iy) * Wd + ix) * C, (size_t)C * 4);
            }
    }
    y.assign((size_t)rows * O, 0.f);
    linear(cols.data(), (int)rows, (int)K, w, nullptr, y.data(), O);
}

// SamBackbone::forward: img [B][3][H][W] -> NHWC [B][H/64][W/64][c1] (out, resized)
void sam_forward(const float* img, int B, int H, int Wd, std::vector<float>& out, int& oh, int& ow) {
    const VCfg& v = g_v;
    const std::string pre = "model.sam_model.";
    const int ps = v.patch, gh = H / ps, gw = Wd / ps, C = v.embed, K0 = 3 * ps * ps;
    const long T = (long)B * gh * gw;
    std::vector<float> cols((size_t)T * K0), x((size_t)T * C);
#pragma omp parallel for schedule(static)
    for (long r = 0; r < T; ++r) {
        const int b = (int)(r / ((long)gh * gw)), gy = (int)(r / gw % gh), gx = (int)(r % gw);
        for (int c = 0; c < 3; ++c)
            for (int ky = 0; ky < ps; ++ky)
                memcpy(cols.data() + (size_t)r * K0 + ((size_t)c * ps + ky) * ps,
                       img + (((size_t)b * 3 + c) * H + gy * ps + ky) * Wd + gx * ps, (size_t)ps * 4);
    }
    linear(cols.data(), (int)T, K0, W(pre + "patch_embed.proj.weight"), opt(pre + "patch_embed.proj.bias"), x.data(), C);
    const std::string pk = "cv.sam.pos." + std::to_string(gh) + "x" + std::to_string(gw);
    if (has(pk)) {
        const float* pos = W(pk).f.data();
        for (long r = 0; r < T; ++r)
            for (int c = 0; c < C; ++c) x[(size_t)r * C + c] += pos[(size_t)(r % ((long)gh * gw)) * C + c];
    }
    std::vector<float> nrm((size_t)T * C), attn((size_t)T * C);
    for (int blk = 0; blk < v.depth; ++blk) {
        const std::string bp = pre + "blocks." + std::to_string(blk) + ".";
        layer_norm_rows(x.data(), T, C, W(bp + "norm1.weight").f.data(), W(bp + "norm1.bias").f.data(), v.sam_eps, nrm.data());
        const bool glob = std::find(v.global.begin(), v.global.end(), blk) != v.global.end();
        const int ws = glob ? 0 : v.window;
        int n, h, w;
        std::vector<float> win;
        const float* xin;
        int hp = gh, wp = gw;
        if (ws > 0) {
            hp = gh + (ws - gh % ws) % ws;
            wp = gw + (ws - gw % ws) % ws;
            const int nwy = hp / ws, nwx = wp / ws;
            n = B * nwy * nwx;
            h = w = ws;
            win.assign((size_t)n * ws * ws * C, 0.f);
#pragma omp parallel for schedule(static) collapse(2)
            for (int b = 0; b < B; ++b)
                for (int y = 0; y < gh; ++y)
                    for (int xx = 0; xx < gw; ++xx) {
                        const int wi = (b * nwy + y / ws) * nwx + xx / ws, t = (y % ws) * ws + xx % ws;
                        memcpy(win.data() + ((size_t)wi * ws * ws + t) * C, nrm.data() + (((size_t)b * gh + y) * gw + xx) * C,
                               (size_t)C * 4);
                    }
            xin = win.data();
        } else {
            n = B;
            h = gh;
            w = gw;
            xin = nrm.data();
        }
        const int L = h * w;
        std::vector<float> qkv((size_t)n * L * 3 * C), ctx((size_t)n * L * C), y((size_t)n * L * C);
        linear(xin, n * L, C, W(bp + "attn.qkv.weight"), opt(bp + "attn.qkv.bias"), qkv.data(), 3 * C);
        const float *Rh = nullptr, *Rw = nullptr;
        if (has(bp + "attn.rel_pos_h")) {
            Rh = W("cv.sam.relh." + std::to_string(blk) + "." + std::to_string(h)).f.data();
            Rw = W("cv.sam.relw." + std::to_string(blk) + "." + std::to_string(w)).f.data();
        }
        const auto ta = std::chrono::steady_clock::now();
        attention_any(qkv.data(), n, L, C, v.heads, Rh, Rw, h, w, ctx.data());
        g_att_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
        linear(ctx.data(), n * L, C, W(bp + "attn.proj.weight"), opt(bp + "attn.proj.bias"), y.data(), C);
        if (ws > 0) {
            const int nwy = hp / ws, nwx = wp / ws;
#pragma omp parallel for schedule(static) collapse(2)
            for (int b = 0; b < B; ++b)
                for (int yy = 0; yy < gh; ++yy)
                    for (int xx = 0; xx < gw; ++xx) {
                        const int wi = (b * nwy + yy / ws) * nwx + xx / ws, t = (yy % ws) * ws + xx % ws;
                        memcpy(attn.data() + (((size_t)b * gh + yy) * gw + xx) * C, y.data() + ((size_t)wi * ws * ws + t) * C,
                               (size_t)C * 4);
                    }
        } else {
            attn.swap(y);
            y.assign(attn.size(), 0.f);
        }
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < x.size(); ++i) x[i] += attn[i];
        layer_norm_rows(x.data(), T, C, W(bp + "norm2.weight").f.data(), W(bp + "norm2.bias").f.data(), v.sam_eps, nrm.data());
        const std::string f1 = has(bp + "mlp.fc1.weight") ? "mlp.fc1" : "mlp.lin1";
        const std::string f2 = has(bp + "mlp.fc2.weight") ? "mlp.fc2" : "mlp.lin2";
        const int hid = (int)W(bp + f1 + ".weight").rows;
        std::vector<float> h1((size_t)T * hid), h2((size_t)T * C);
        linear(nrm.data(), (int)T, C, W(bp + f1 + ".weight"), opt(bp + f1 + ".bias"), h1.data(), hid);
        {
            VClk clk(1);
#pragma omp parallel for schedule(static)
            for (size_t i = 0; i < h1.size(); ++i) h1[i] = gelu_erf(h1[i]);
        }
        linear(h1.data(), (int)T, hid, W(bp + f2 + ".weight"), opt(bp + f2 + ".bias"), h2.data(), C);
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < x.size(); ++i) x[i] += h2[i];
    }
    // neck + downsample (NHWC; LN2d = LN over channels per position)
    std::vector<float> a, bbuf;
    int h1, w1;
    conv_nhwc(x.data(), B, gh, gw, C, W("cv.sam.neck.0"), v.neck, 1, 1, 0, a, h1, w1);
    bbuf.resize(a.size());
    layer_norm_rows(a.data(), (long)B * h1 * w1, v.neck, W(pre + "neck.1.weight").f.data(), W(pre + "neck.1.bias").f.data(), 1e-6f, bbuf.data());
    conv_nhwc(bbuf.data(), B, h1, w1, v.neck, W("cv.sam.neck.2"), v.neck, 3, 1, 1, a, h1, w1);
    layer_norm_rows(a.data(), (long)B * h1 * w1, v.neck, W(pre + "neck.3.weight").f.data(), W(pre + "neck.3.bias").f.data(), 1e-6f, bbuf.data());
    int h2, w2;
    conv_nhwc(bbuf.data(), B, h1, w1, v.neck, W("cv.sam.net_2"), v.c0, 3, 2, 1, a, h2, w2);
    conv_nhwc(a.data(), B, h2, w2, v.c0, W("cv.sam.net_3"), v.c1, 3, 2, 1, out, oh, ow);
}

// ClipVisionModel::forward with the SAM features as patch embeddings: sam [B][g*g][C] -> x [B][1+g*g][C]
void clip_forward(const float* sam, int B, int G, std::vector<float>& x) {
    const VCfg& v = g_v;
    const std::string pre = "model.vision_model.";
    const int C = v.clip_h, S = G + 1;
    const long T = (long)B * S;
    x.assign((size_t)T * C, 0.f);
    const float* cls = W(pre + "embeddings.class_embedding").f.data();
    const float* pos = W("cv.clip.pos." + std::to_string(S)).f.data();
    for (int b = 0; b < B; ++b)
        for (int t = 0; t < S; ++t)
            for (int c = 0; c < C; ++c)
                x[((size_t)b * S + t) * C + c] = (t == 0 ? cls[c] : sam[((size_t)b * G + t - 1) * C + c]) + pos[(size_t)t * C + c];
    std::vector<float> n1((size_t)T * C);
    layer_norm_rows(x.data(), T, C, W(pre + "pre_layrnorm.weight").f.data(), W(pre + "pre_layrnorm.bias").f.data(), v.clip_eps, n1.data());
    x.swap(n1);
    std::vector<float> qkv((size_t)T * 3 * C), ctx((size_t)T * C), y((size_t)T * C), h1((size_t)T * v.clip_ffn);
    for (int li = 0; li < v.clip_layers; ++li) {
        const std::string lp = pre + "transformer.layers." + std::to_string(li) + ".";
        layer_norm_rows(x.data(), T, C, W(lp + "layer_norm1.weight").f.data(), W(lp + "layer_norm1.bias").f.data(), v.clip_eps, n1.data());
        linear(n1.data(), (int)T, C, W(lp + "self_attn.qkv_proj.weight"), opt(lp + "self_attn.qkv_proj.bias"), qkv.data(), 3 * C);
        const auto ta = std::chrono::steady_clock::now();
        attention_any(qkv.data(), B, S, C, v.clip_heads, nullptr, nullptr, 0, 0, ctx.data());
        g_att_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
        linear(ctx.data(), (int)T, C, W(lp + "self_attn.out_proj.weight"), opt(lp + "self_attn.out_proj.bias"), y.data(), C);
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < x.size(); ++i) x[i] += y[i];
        layer_norm_rows(x.data(), T, C, W(lp + "layer_norm2.weight").f.data(), W(lp + "layer_norm2.bias").f.data(), v.clip_eps, n1.data());
        linear(n1.data(), (int)T, C, W(lp + "mlp.fc1.weight"), opt(lp + "mlp.fc1.bias"), h1.data(), v.clip_ffn);
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < h1.size(); ++i) h1[i] = (1.0f / (1.0f + std::exp(-(h1[i] * 1.702f)))) * h1[i];
        linear(h1.data(), (int)T, v.clip_ffn, W(lp + "mlp.fc2.weight"), opt(lp + "mlp.fc2.bias"), y.data(), C);
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < x.size(); ++i) x[i] += y[i];
    }
}

}  // namespace

extern "C" {

int cr_init(int H, int heads, int kv_heads, int hd, int layers, int vocab, int inter, int moe_inter, int E, int topk,
            int n_shared, int norm_topk, int softmax_scoring, float eps, float rope_theta, float scaling,
            const int* moe_flags, int threads) {
    g_c = Cfg{H, heads, kv_heads, hd, layers, vocab, inter, moe_inter, E, topk, n_shared, norm_topk, softmax_scoring,
              eps, rope_theta, scaling};
    g_moe.assign(moe_flags, moe_flags + layers);
    if (H % 16 || hd % 16 || hd > 512) return 1;
    if (threads > 0) omp_set_num_threads(threads);
    g_w.clear();
    return 0;
}

// kind: 0 keep f32, 1 store f16 (values already f16-rounded), 2 store bf16 (values already bf16), 3 store bf16 as
// the packed 32-column panels of linear_packed (rows = N outputs, cols = K)
int cr_set(const char* name, const float* data, long rows, long cols, int kind) {
    Tensor t;
    t.kind = kind;
    t.rows = rows;
    t.cols = cols;
    const long n = rows * cols;
    if (kind == 3) {
        const long np = (rows + 31) / 32;
        t.h.assign((size_t)np * cols * 32, 0);
        uint32_t* P = reinterpret_cast<uint32_t*>(t.h.data());
#pragma omp parallel for schedule(static)
        for (long p = 0; p < np; ++p)
            for (long k = 0; k < cols; ++k)
                for (int i = 0; i < 32; ++i) {
                    const long r = 32 * p + i;
                    uint32_t bits = 0;
                    if (r < rows) memcpy(&bits, data + r * cols + k, 4);
                    const uint32_t v = bits >> 16;
                    P[((size_t)p * cols + k) * 16 + (i & 15)] |= i < 16 ? v : (v << 16);
                }
        g_w[name] = std::move(t);
        return 0;
    }
    if (kind == 0) {
        t.f.assign(data, data + n);
    } else {
        t.h.resize(n);
#pragma omp parallel for schedule(static)
        for (long i = 0; i < n; ++i) {
            if (kind == 1) {
                t.h[i] = f32_to_f16_bits(data[i]);
            } else {
                uint32_t b;
                memcpy(&b, data + i, 4);
                t.h[i] = (uint16_t)(b >> 16);
            }
        }
    }
    g_w[name] = std::move(t);
    return 0;
}

// generate (model/mod.rs:1870-2048, greedy, EOS ignored): prompt ids with image rows injected at mask slots,
// max_new tokens; ms[0] = prefill, ms[1] = the (max_new - 1) decode forwards
int cr_generate(const int64_t* ids, const uint8_t* mask, int P, const float* img, int n_img, int max_new, int ngram,
                int64_t* out, double* ms) {
    try {
        const Cfg& c = g_c;
        const int cap = P + max_new + 1;
        g_kv.assign(c.layers, KV());
        for (auto& kv : g_kv) {
            kv.cap = cap;
            kv.k.assign((size_t)c.kv_heads * cap * c.hd, 0.f);
            kv.v.assign((size_t)c.kv_heads * cap * c.hd, 0.f);
        }
        rope_tables(cap);
        g_past = 0;
        const Tensor& emb = W("model.embed_tokens.weight");
        std::vector<float> x((size_t)P * c.H);
        int r = 0;
        for (int i = 0; i < P; ++i) {
            if (mask && mask[i]) {
                if (r >= n_img) return 2;
                memcpy(x.data() + (size_t)i * c.H, img + (size_t)r * c.H, c.H * 4);
                ++r;
            } else {
                for (int j = 0; j < c.H; ++j) x[(size_t)i * c.H + j] = load1(emb, (long)ids[i] * c.H + j);
            }
        }
        std::vector<int> ctx(ids, ids + P);
        std::vector<float> lg;
        auto t0 = std::chrono::steady_clock::now();
        forward(x, P, lg);
        int cur = select(lg, ctx, ngram);
        auto t1 = std::chrono::steady_clock::now();
        for (int s = 0; s < max_new; ++s) {
            out[s] = cur;
            ctx.push_back(cur);
            if (s + 1 == max_new) break;
            std::vector<float> xe(c.H);
            for (int j = 0; j < c.H; ++j) xe[j] = load1(emb, (long)cur * c.H + j);
            forward(xe, 1, lg);
            cur = select(lg, ctx, ngram);
        }
        auto t2 = std::chrono::steady_clock::now();
        ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
        ms[1] = std::chrono::duration<double, std::milli>(t2 - t1).count();
        return 0;
    } catch (...) {
        return 3;
    }
}


// ---- vision (round 5).  cv_init keeps the tensors already set (the decoder's cr_init clears them).
int cv_init(int embed, int depth, int heads, int window, const int* global_flags, int neck, int c0, int c1, int patch,
            float sam_eps, int clip_h, int clip_layers, int clip_heads, int clip_ffn, float clip_eps, int n_embed,
            int in_dim, int threads) {
    g_v = VCfg{embed, depth, heads, window, neck, c0, c1, patch, sam_eps, clip_h, clip_layers, clip_heads, clip_ffn,
               clip_eps, n_embed, in_dim, {}};
    for (int i = 0; i < depth; ++i)
        if (global_flags[i]) g_v.global.push_back(i);
    if (threads > 0) omp_set_num_threads(threads);
    return (embed % 16 || clip_h % 16 || in_dim % 16) ? 1 : 0;
}

// one batch of B same-size views [B][3][H][W] -> the projected tokens post [B][G][n_embed] (G = (H/64)(W/64)),
// the pre-projection rows pre [B][G][in_dim] when non-null; ms = {sam, clip, projector}
int cv_features(const float* img, int B, int H, int Wd, float* post, float* pre_out, double* ms) {
    try {
        const VCfg& v = g_v;
        auto t0 = std::chrono::steady_clock::now();
        std::vector<float> sam;
        int oh, ow;
        sam_forward(img, B, H, Wd, sam, oh, ow);
        auto t1 = std::chrono::steady_clock::now();
        if (oh != ow || v.c1 != v.clip_h) return 2;
        const int G = oh * ow;
        std::vector<float> clip;
        clip_forward(sam.data(), B, G, clip);
        auto t2 = std::chrono::steady_clock::now();
        std::vector<float> pre((size_t)B * G * v.in_dim);
        for (int b = 0; b < B; ++b)
            for (int t = 0; t < G; ++t) {
                float* r = pre.data() + ((size_t)b * G + t) * v.in_dim;
                memcpy(r, clip.data() + ((size_t)b * (G + 1) + t + 1) * v.clip_h, (size_t)v.clip_h * 4);
                memcpy(r + v.clip_h, sam.data() + ((size_t)b * G + t) * v.c1, (size_t)v.c1 * 4);
            }
        linear(pre.data(), B * G, v.in_dim, W("model.projector.layers.weight"), opt("model.projector.layers.bias"), post,
               v.n_embed);
        if (pre_out) memcpy(pre_out, pre.data(), pre.size() * 4);
        if (getenv("DSOCR_CV_PROF")) {
            fprintf(stderr, "[cv] ln %.0f act %.0f im2col %.0f ms\n", g_vis_prof[0], g_vis_prof[1], g_vis_prof[2]);
            for (double& d : g_vis_prof) d = 0;
        }
        auto t3 = std::chrono::steady_clock::now();
        ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
        ms[1] = std::chrono::duration<double, std::milli>(t2 - t1).count();
        ms[2] = std::chrono::duration<double, std::milli>(t3 - t2).count();
        return 0;
    } catch (...) {
        return 3;
    }
}

void cr_free() {
    g_w.clear();
    g_kv.clear();
}

int cr_threads() { return omp_get_max_threads(); }

// the OpenMP team size of every later parallel region (the bench times the same page at two thread counts)
void cr_set_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
}

// Y = X . W^T for a tensor set with cr_set (micro-benchmark of the linear kernel)
int cr_linear(const char* wname, const float* X, int M, int K, float* Y, int N) {
    try {
        linear(X, M, K, W(wname), nullptr, Y, N);
        return 0;
    } catch (...) {
        return 3;
    }
}

// stage clocks since the last call (ms): linears, attention core
void cr_profile(double* out) {
    out[0] = g_lin_ms;
    out[1] = g_att_ms;
    g_lin_ms = g_att_ms = 0;
}

}  // extern "C"
