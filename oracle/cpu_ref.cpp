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

double g_lin_ms = 0, g_att_ms = 0;  // stage clocks (cr_profile)

void linear(const float* X, int M, int K, const Tensor& w, const Tensor* b, float* Y, int N) {
    if (K % 16) throw std::runtime_error("cpu_ref: K % 16 != 0");
    struct Clk {
        std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
        ~Clk() { g_lin_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count(); }
    } clk;
    if (w.kind == 1) linear_t<1>(X, M, K, w, b, Y, N);
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

// kind: 0 keep f32, 1 store f16 (values already f16-rounded), 2 store bf16 (values already bf16)
int cr_set(const char* name, const float* data, long rows, long cols, int kind) {
    Tensor t;
    t.kind = kind;
    t.rows = rows;
    t.cols = cols;
    const long n = rows * cols;
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

void cr_free() {
    g_w.clear();
    g_kv.clear();
}

int cr_threads() { return omp_get_max_threads(); }

// stage clocks since the last call (ms): linears, attention core
void cr_profile(double* out) {
    out[0] = g_lin_ms;
    out[1] = g_att_ms;
    g_lin_ms = g_att_ms = 0;
}

}  // extern "C"
