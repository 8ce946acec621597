// Host-side launch API for the gfx950 kernels.  All pointers are device pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsocr {

enum WDType : int { WDT_BF16 = 0, WDT_F16 = 1 };
// Activation epilogues (reference: candle gelu_erf, quick_gelu clip.rs:413-416, silu).
enum Act : int { ACT_NONE = 0, ACT_GELU_ERF = 1, ACT_QUICK_GELU = 2, ACT_SILU = 3 };

// ------------------------------------------------------------------ GEMM (gemm.hip)
struct GemmArgs {
    int M = 0, N = 0, K = 0;
    const float* A = nullptr;
    int lda = 0;
    const int* a_rows = nullptr;  // optional row gather for A
    const void* W = nullptr;      // [N][K] 16-bit weights
    int ldw = 0;
    int wdtype = WDT_BF16;
    long w_group_stride = 0;      // elements between group slabs
    const float* bias = nullptr;  // [N] (f32)
    long bias_group_stride = 0;
    float* C = nullptr;
    int ldc = 0;
    const int* c_rows = nullptr;  // optional row scatter for C (-1 drops the row)
    int act = 0;
    int accumulate = 0;           // C = C + result (residual add)
    const int* group_off = nullptr;  // [groups+1] device offsets into the gathered row list
    int groups = 1;
    int max_group_rows = 0;
};
void launch_gemm(const GemmArgs& g, hipStream_t s);

// ------------------------------------------------------------------ skinny linear (gemv.hip)
// y[m][n] = act(sum_k x[m][k] W[n][k] + bias[n]) (+ y) for M <= 16 rows.
struct GemvArgs {
    int M = 0, N = 0, K = 0;
    const float* x = nullptr;
    int ldx = 0;
    const void* W = nullptr;
    int ldw = 0;
    int wdtype = WDT_F16;
    const float* bias = nullptr;
    float* y = nullptr;
    int ldy = 0;
    int act = 0;
    int accumulate = 0;
};
void launch_gemv(const GemvArgs& a, hipStream_t s);

// Grouped SwiGLU experts for decode (moe.hip).  Assignment list sorted by expert:
// expert e owns sorted positions [eoff[e], eoff[e+1]); arow[p] = token row of x.
//   h[p][i] = silu(x[arow[p]] . Wg_e[i]) * (x[arow[p]] . Wu_e[i])     (W_gu_e = [gate; up], [2I][K])
//   y[p][j] = h[p] . Wd_e[j]                                           (W_d_e = [Hout][I])
struct MoeDecodeArgs {
    int T = 0, topk = 0, E = 0, K = 0, I = 0, Hout = 0;
    const float* x = nullptr;  // [T][K]
    const int* eoff = nullptr; // [E+1]
    const int* arow = nullptr; // [T*topk]
    const void* Wgu = nullptr; // E x [2I][K]
    const void* Wd = nullptr;  // E x [Hout][I]
    int wdtype = WDT_F16;
    float* h = nullptr;        // [T*topk][I]
    float* y = nullptr;        // [T*topk][Hout]
    int max_rows_per_expert = 16;
};
void launch_moe_gateup_gemv(const MoeDecodeArgs& a, hipStream_t s);
void launch_moe_down_gemv(const MoeDecodeArgs& a, hipStream_t s);

// Router: scores = softmax(logits) (or sigmoid), greedy top-k (descending, stable),
// optional renormalise + scaling (block.rs:1254-1301).
void launch_router_topk(const float* logits, int T, int E, int topk, int softmax_scoring, int norm_topk,
                        float scaling, int* topk_ids, float* topk_w, hipStream_t s);
// Group assignments by expert: eoff[E+1], arow[sorted] = token, apos[t*topk+k] = sorted position.
void launch_moe_group(const int* topk_ids, int T, int topk, int E, int* eoff, int* arow, int* apos, int* scratch,
                      hipStream_t s);
// out[t] (+)= sum_k w[t][k] * y[apos[t*topk+k]] (+ shared[t])
void launch_moe_combine(const float* y, const int* apos, const float* topk_w, const float* shared, int T, int topk,
                        int H, float* out, int accumulate, hipStream_t s);
void launch_silu_mul(const float* g, int ldg, int I, int rows, float* h, int ldh, hipStream_t s);

// ------------------------------------------------------------------ norms (norm.hip)
void launch_layernorm(const float* x, int ldx, float* y, int ldy, const int* out_rows, int rows, int cols,
                      const float* w, const float* b, float eps, hipStream_t s);
void launch_rmsnorm(const float* x, int ldx, float* y, int ldy, int rows, int cols, const float* w, float eps,
                    hipStream_t s);

// ------------------------------------------------------------------ attention (attention.hip)
struct AttnView {
    const float* ptr = nullptr;
    long row_stride = 0, head_stride = 0;
    const long* seq_off = nullptr;  // element offset of row 0 of sequence s (device); null -> s*L*row_stride
};
struct AttnArgs {
    AttnView q, k, v;
    float* o = nullptr;
    long o_row_stride = 0, o_head_stride = 0;
    const long* o_seq_off = nullptr;
    int n_seq = 0, L = 0;            // uniform length L unless seq_len given
    const int* seq_len = nullptr;
    int heads = 0, kv_heads = 0, hd = 0;
    float scale = 1.f;
    int causal = 0;
    const float* relbias = nullptr;  // [seq][head][L][rel_h + rel_w]
    int rel_h = 0, rel_w = 0;
};
void launch_attention(const AttnArgs& a, hipStream_t s);
// SAM decomposed rel-pos: out[s][h][q][kh] = q . Rh[qh-kh+gh-1], out[..][gh+kw] = q . Rw[qw-kw+gw-1]
void launch_sam_relbias(const float* q, long q_row_stride, int n_seq, int gh, int gw, int heads, int hd,
                        const float* Rh, const float* Rw, float* out, hipStream_t s);
// Decode attention over the per-page f32 KV cache (flash-decoding, split over keys).
struct DecodeAttnArgs {
    const float* q = nullptr;  long q_row_stride = 0;   // [B][heads*hd]
    const float* kc = nullptr; const float* vc = nullptr;
    long page_stride = 0, head_stride = 0;              // cache [B][H][Lmax][hd]
    const int* lens = nullptr;                          // keys per page (device)
    int B = 0, heads = 0, hd = 0, max_len = 0;
    float scale = 1.f;
    float* part = nullptr;                              // workspace
    float* o = nullptr; long o_row_stride = 0;
};
void launch_decode_attention(const DecodeAttnArgs& a, hipStream_t s);
size_t decode_attention_workspace(int B, int heads, int hd, int max_len);

// RoPE (rotate_half, optional MLA reorder) on q,k inside a fused qkv buffer and KV-cache append.
struct RopeKvArgs {
    float* qkv = nullptr; long ld = 0; int rows = 0;
    const int* row_page = nullptr; const int* row_pos = nullptr;  // per row (device)
    int heads = 0, kv_heads = 0, hd = 0, rope_dim = 0, use_mla = 0;
    const float* cos = nullptr; const float* sin = nullptr;       // [Lmax][rope_dim]
    float* kc = nullptr; float* vc = nullptr; long page_stride = 0, head_stride = 0;
};
void launch_rope_kv(const RopeKvArgs& a, hipStream_t s);

// ------------------------------------------------------------------ misc (misc.hip)
void launch_patch_im2col(const float* img, int n, int H, int W, int ps, float* cols, hipStream_t s);
void launch_conv_im2col_nhwc(const float* x, int n, int H, int W, int C, int kh, int kw, int stride, int pad,
                             float* cols, hipStream_t s);
void launch_add_broadcast(float* x, const float* t, long rows_per_rep, int cols, int reps, hipStream_t s);
void launch_clip_embed(const float* sam, const float* cls, const float* pos, int n, int S, int C, float* out,
                       hipStream_t s);
void launch_concat_clip_sam(const float* clip, const float* sam, int n, int S, int C1, int C2, float* out,
                            hipStream_t s);
// dst[r] = source per (kind, index): 0 = table row (16-bit, widened), 1 = srcA row, 2 = srcB row, 3 = vecA, 4 = vecB
void launch_assemble_rows(const int* kind, const int* index, int rows, int H, const void* table, int table_dt,
                          const float* srcA, const float* srcB, const float* vecA, const float* vecB, float* dst,
                          long ld_dst, hipStream_t s);
void launch_embed_tokens(const void* table, int table_dt, const int* ids, int n, int H, float* out, long ld,
                         hipStream_t s);
// Greedy token selection with repetition penalty + no-repeat-ngram ban (sampling.rs:34-158).
struct SampleArgs {
    float* logits = nullptr; int B = 0, V = 0; long ld = 0;
    const int* ctx = nullptr; long ctx_cap = 0; const int* ctx_len = nullptr;
    int ngram = 0; float rep_penalty = 1.f;
    int* banned = nullptr; int* banned_cnt = nullptr; int banned_cap = 0;
    float* red_val = nullptr; int* red_idx = nullptr; int red_blocks = 0;
    int* out_tok = nullptr;
};
void launch_sample_greedy(const SampleArgs& a, hipStream_t s);
size_t sample_workspace_blocks(int V);
// Per-step bookkeeping: record the token (EOS finishes the page), grow the
// context, embed it as the next step's input; then advance KV positions.
void launch_step_update(const int* tok, int B, int* ctx, long ctx_cap, int* ctx_len, int* out_ids, int* out_len,
                        long out_cap, int* done, int eos, const void* table, int table_dt, int H, float* x_next,
                        hipStream_t s);
void launch_step_advance(int* kv_pos, int* kv_len, int B, hipStream_t s);

}  // namespace dsocr
