// Host-side launch API for the gfx950 kernels.  All pointers are device pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsocr {

enum WDType : int { WDT_BF16 = 0, WDT_F16 = 1 };

// Profiling hook: while prof_events() holds a (start, stop) pair, the next kernel launched through
// DSOCR_LAUNCH (decode.hip, lmhead.hip) records its own dispatch begin / end into the two events
// (hipExtLaunchKernelGGL: the dispatch-packet timestamps rocprofv3's kernel trace reports) and the
// pair is cleared.  Host-side, per thread; never set while a stream is being captured.
// In-context launch spans (dev_common.hpp WaveSpan): per-wave (entry, exit) slots of one launch,
// folded by launch_span_reduce into rec[min(*step, cap - 1)] = {first entry, last exit, distinct ids
// among ids[0..n_ids) (0 if none), waves seen} (100 MHz wall clock) and cleared for the next launch.
constexpr long SPAN_SLOTS = 16384;
// Chain spans (Engine::set_spans bit 4): every stamped launch of a decode step writes its waves' slots into its
// own region of SPAN_SLOTS pairs; one fold at the end of the step writes rec[step][region] = {first entry, last
// exit, waves, 0} over the slots stamped since the previous fold (tmark: two words, alternated by step parity).
void launch_span_chain_fold(const unsigned long long* slots, int nreg, unsigned long long* rec, const int* step, int cap,
                            unsigned long long* tmark, hipStream_t s);
void launch_span_reduce(unsigned long long* slots, unsigned long long* rec, const int* step, int cap, const int* ids,
                        int n_ids, hipStream_t s);
struct ProfEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
ProfEvents& prof_events();
// Activation epilogues (reference: candle gelu_erf, quick_gelu clip.rs:413-416, silu).
enum Act : int { ACT_NONE = 0, ACT_GELU_ERF = 1, ACT_QUICK_GELU = 2, ACT_SILU = 3 };

// ------------------------------------------------------------------ GEMM (gemm.hip)
// bf16 NT GEMM C[M][N] (+)= act(A[M][K] . W[N][K]^T + bias) with f32 accumulate (gemm_bf16.hip):
// the split-plane form of the f32 vision linears (A = [lo|mid|hi] planes, W = [W|W|W]).
struct GemmBf16Args {
    int M = 0, N = 0, K = 0;          // K % 64 == 0
    const void* A = nullptr; long lda = 0;
    const void* W = nullptr; long ldw = 0;
    const float* bias = nullptr;
    float* C = nullptr; long ldc = 0;
    const int* c_rows = nullptr;      // optional row scatter for C (-1 drops the row)
    int act = 0, accumulate = 0;
    int splits = 1; float* part = nullptr;  // split-K: [splits][M][N] f32 partials (reduced in order)
    // bf16 output (the dots.ocr tower's bf16 tensors): C is then uint16_t [M][ldc] and every op of the
    // epilogue rounds to bf16 as the reference's separate bf16 ops do (quant.rs:141-150):
    // v = rnd(acc); bias: v = rnd(v + b); act: v = rnd(act(v)); accumulate: v = rnd(C + v)
    int out_bf16 = 0;
    int w_f16 = 0;  // gemm_f32a only: W holds f16 values (split into hi / lo bf16 in registers)
    int variant = 0;  // gemm_f32a bf16 weights: 0 = default (one LDS stage), 2 = two stages (tools/kbench A/B)
    // tile raster: consecutive tiles (of one XCD) walk group_m M row bands down one N column, then the next
    // column (grouped order: ~group_m bands x (resident / group_m) columns live at once share their A and W
    // k-slices in the XCD's L2); 1 = one band across all N tiles (the round-3 order); -1 = the default
    // (DSOCR_GEMM_GROUP_M, else 8)
    int group_m = -1;
    // SwiGLU pair epilogue (dots.ocr fc1|fc3, ping-pong kernel only): W rows interleaved per 32 (fc1 rows
    // 32b..32b+31, then fc3 rows 32b..32b+31), N = 2I; C is bf16 [M][ldc] of h = rnd(silu(g) * u), I columns
    int swiglu = 0;
    // 2-D rotary of the q / k columns in the epilogue (dots.ocr q|k|v GEMM, ping-pong kernel only): columns
    // below rope_cols (a multiple of 256) are heads of 128 dims rotated with the [M][128] f32 cos / sin tables
    // exactly as dots_rope8_kernel does
    const float* rope_cos = nullptr;
    const float* rope_sin = nullptr;
    int rope_cols = 0;
    unsigned long long* stamps = nullptr;  // ping-pong kernel diagnostic build: per-wave segment cycle sums (tools/kbench)
};
void launch_gemm_bf16(const GemmBf16Args& g, hipStream_t s);
int gemm_bf16_splits(int M, int N, int K);  // K slices that fill the chip (>= 8 K steps each)
// f32 A x bf16 W^T with the exact 3-plane split fused into the fragment loads (K % 32 == 0, f32 out)
bool gemm_f32a_ok(const GemmBf16Args& g);
int gemm_f32a_splits(int M, int N, int K);
void launch_gemm_f32a(const GemmBf16Args& g, hipStream_t s);

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
// Grouped routed-expert GEMM (gemm_bf16.hip): 32-row tiles mapped to (group, row tile) on the device,
// A rows gathered by the LDS DMA, exact-f32 planes split in registers.  launch_gemm routes here.
bool gemm_f32a_grouped_ok(const GemmArgs& g);
void launch_gemm_f32a_grouped(const GemmArgs& g, hipStream_t s, int tile_rows = 0);  // 0: by rows per group

// ------------------------------------------------------------------ MoE prefill helpers (moe.hip)
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
    // causal (prefill): workspace for the key-piece partials (attention_causal_part_floats); without it
    // one block walks all of a query block's keys
    float* part = nullptr;
    size_t part_floats = 0;
};
void launch_attention(const AttnArgs& a, hipStream_t s);
size_t attention_causal_part_floats(int n_seq, int heads, int L, int hd);
// Bidirectional attention on bf16-valued q / k / v with f32 math on the bf16 matrix cores
// (attention_bf16.hip): n_seq uniform sequences of L rows; element (seq, row, head, d) of q at
// q + seq*L*q_rs + row*q_rs + head*q_hs + d (likewise k, v with kv heads); o f32 or bf16 (o_bf16).
struct AttnBf16Args {
    const uint16_t* q = nullptr; const uint16_t* k = nullptr; const uint16_t* v = nullptr;
    long q_rs = 0, q_hs = 0, k_rs = 0, k_hs = 0, v_rs = 0, v_hs = 0;
    void* o = nullptr; long o_rs = 0, o_hs = 0; int o_bf16 = 0;
    int n_seq = 0, L = 0, heads = 0, kv_heads = 0, hd = 0;
    float scale = 1.f;
    // P.V passes: 3 = p split exactly into three bf16 planes (f32 products); 2 = hi + mid planes, p to 16
    // significant bits (each plane round-to-nearest: relative error <= 2^-17 per probability)
    int pv_planes = 3;
};
void launch_attention_bf16(const AttnBf16Args& a, hipStream_t s);
// SAM decomposed rel-pos: out[s][h][q][kh] = q . Rh[qh-kh+gh-1], out[..][gh+kw] = q . Rw[qw-kw+gw-1]
void launch_sam_relbias(const float* q, long q_row_stride, int n_seq, int gh, int gw, int heads, int hd,
                        const float* Rh, const float* Rw, float* out, hipStream_t s);
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
// logits [B][ld] -> trace[b][out_len[b]][V] for pages not done (out_len < steps): the parity trace
void launch_trace_logits(const float* logits, int B, int V, long ld, const int* out_len, const int* done, float* trace,
                         long steps, hipStream_t s);
void launch_embed_tokens(const void* table, int table_dt, const int* ids, int n, int H, float* out, long ld,
                         hipStream_t s);
// Repetition penalty over the context tokens (sampling.rs:34-96), in place on the logits.
struct SampleArgs {
    float* logits = nullptr; int B = 0, V = 0; long ld = 0;
    const int* ctx = nullptr; long ctx_cap = 0; const int* ctx_len = nullptr;
    float rep_penalty = 1.f;
};
void launch_rep_penalty(const SampleArgs& a, hipStream_t s);

// ------------------------------------------------------------------ fused decode step (decode.hip)
// Skinny linear with the preceding RMSNorm fused (norm_w != null: x is normalised on the fly).
struct DecGemvArgs {
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
    const float* norm_w = nullptr;
    float eps = 0.f;
    float* xn_out = nullptr;  // optional: block 0 writes the staged (normalised) rows [M][K] here
    const void* w_swz = nullptr;  // optional: W in dec_mm's fragment order (launch_mm_swizzle), M = 3..8
    unsigned long long* span = nullptr;  // launch-span slots (dec_gemv, dec_mm, dec_route_grp) or null
};
void launch_dec_gemv(const DecGemvArgs& a, hipStream_t s);
// 3..8 tokens on the matrix cores (decode_mm.hip): weight rows as MFMA A operands, the (optionally
// RMS-normalised) activation rows as three exact 16-bit planes (f16: per-row power-of-two scaled)
bool dec_mm_ok(const DecGemvArgs& a);
void launch_dec_mm(const DecGemvArgs& a, hipStream_t s);
// W [N][K] -> dec_mm fragment order ([N/16][K/32][64][8] 16-bit): every wave weight load one 1 KiB block
size_t mm_swizzle_elems(int N, int K);
// long-K form (K % 64 == 0, any length; the dense layer-0 down projection): split-K over pieces of 512
// with write-through partial tiles and an in-launch last-arriver sum; part / tick sized below, tick
// zero between launches (the last arriver resets it)
bool dec_mm_splitk_ok(const DecGemvArgs& a);
size_t dec_mm_splitk_part_floats(int N, int K);
size_t dec_mm_splitk_ticks(int N);
void launch_dec_mm_splitk(const DecGemvArgs& a, float* part, int* tick, hipStream_t s);
void launch_mm_swizzle(const void* w, int N, int K, void* out, hipStream_t s);
// Router GEMV whose last-arriving block writes the greedy top-k of every token (T <= 8).
struct DecRouteEpi {
    int topk = 0, softmax_scoring = 1, norm_topk = 0;
    float scaling = 1.f;
    int* ids = nullptr; float* w = nullptr;   // [T][topk]
    int* counter = nullptr;                   // zero between launches
    // optional: the picks grouped by expert (MOE_GRP_* layout below) for the grouped decode kernels
    int* grp = nullptr;
    unsigned long long* stamps = nullptr;  // dev: wall clock at dec_route_grp's phase points (profile only)
};
// Expert groups of one decode MoE layer (T <= 8 tokens): grp[0] = number of distinct experts picked,
// record s (s < grp[0]) at grp + MOE_GRP_REC * (1 + s): [0] expert id, [1] picks (tokens) n,
// [2 .. 2+n) the h rows t*topk + k in increasing token order, [10 .. 10+n) their routing weights
// (f32 bits).  Records are in increasing expert order.
constexpr int MOE_GRP_REC = 32;
inline size_t moe_grp_ints(int E, int T, int topk) {
    const int slots = E < T * topk ? E : T * topk;
    return (size_t)MOE_GRP_REC * (1 + slots);
}
void launch_dec_router(const DecGemvArgs& a, const DecRouteEpi& r, hipStream_t s);
bool dec_router_ok(int T, int E, int K, int topk);
// One-block router for T <= 8 tokens, E <= 64 experts: [RMSNorm of x (rows -> a.xn_out)] + logits
// (-> a.y when set) + greedy top-k (-> r.ids / r.w) + expert records (-> r.grp when set).
bool dec_route_grp_ok(int T, int E, int K, int topk);
void launch_dec_route_grp(const DecGemvArgs& a, const DecRouteEpi& r, hipStream_t s);
// RoPE on q / new k + KV-cache append + flash-decoding over 64-key chunks + combine.
struct DecAttn2Args {
    const float* qkv = nullptr; long ld = 0;           // [B][(heads + 2 kv_heads) * hd]
    const int* kv_pos = nullptr;                        // position of the token being decoded
    int B = 0, heads = 0, kv_heads = 0, hd = 0, rope_dim = 0, use_mla = 0, max_len = 0;
    const float* cos = nullptr; const float* sin = nullptr;
    float* kc = nullptr; float* vc = nullptr; long page_stride = 0, head_stride = 0;
    float scale = 1.f;
    float* part = nullptr;
    int* counters = nullptr;                            // [B][heads] arrival tickets, zero between launches
    float* o = nullptr; long o_ld = 0;
    int* err = nullptr;                                 // polled merge: give-up flag (set instead of hanging)
    unsigned long long* span = nullptr;                 // launch-span slots (SPAN_SLOTS pairs) or null
    int prerot = 0;                                     // q / k rows already rotated (dec_qkv_rope)
    // phase clocks (tools/kbench qkvattn1 / attn8; null in the engine): per block (linear index) 8 words,
    // s_memrealtime (100 MHz) at [0] entry, [1] projection rows stored (fused), [2] q polled (fused) /
    // softmax done (standalone), [3] chunk record stored, [4] merge poll done, [5] exit
    unsigned long long* stamps = nullptr;
    int kv_delay = 0;  // fused q/k/v + attention: ticks (10 ns) the K / V cache loads wait behind the projection
};
void launch_dec_attn(const DecAttn2Args& a, hipStream_t s);
// q/k/v projection of one token with RoPE applied in the epilogue (rows < rot_rows rotated at
// position kv_pos[0]; table layout [pos][hd], rope on the full head dim, rotate_half pairing).
struct DecRopeEpi {
    const int* kv_pos = nullptr;
    const float* cos = nullptr; const float* sin = nullptr;
    int hd = 0, rot_rows = 0;
};
bool dec_qkv_rope_ok(const DecGemvArgs& a, const DecRopeEpi& r);
void launch_dec_qkv_rope(const DecGemvArgs& a, const DecRopeEpi& r, hipStream_t s);
// One page: q/k/v projection + RoPE and the decode attention in one launch (the attention blocks stream
// their K / V chunk while the projection runs, then poll for q / k / v); the q/k/v row g.y == a.qkv must
// enter the first launch sentinel-filled (dec_qkv_sentinel_init), every launch leaves it so
// (includes the residency rule below: the launch is refused - the engine then takes the two-launch form -
// when the polling attention blocks could fill every slot the device has for the kernel)
bool dec_qkv_attn_ok(const DecGemvArgs& g, const DecRopeEpi& r, const DecAttn2Args& a);
// Residency rule of the in-launch polled hand-offs: waiting_blocks (the blocks that may spin on other
// blocks of the same grid) < usable slots (min(api, 8), one fewer where the API may over-admit, x CUs).
// Pure host decision (no device call); dec_qkv_attn_ok / dec_attn_polled apply it with the kernel's
// occupancy query.
bool poll_wait_fits(long waiting_blocks, int api_blocks_per_cu, int cus);
// dec_attn takes the polling merge (else the arrival ticket)
bool dec_attn_polled(const DecAttn2Args& a);
void launch_dec_qkv_attn(const DecGemvArgs& g, const DecRopeEpi& r, const DecAttn2Args& a, hipStream_t s);
void dec_qkv_sentinel_init(float* qkv, size_t floats, hipStream_t s);
size_t dec_attn_workspace(int B, int heads, int hd, int max_len);
// the record buffer enters every dec_attn launch sentinel-filled (the polling merge refills what it reads)
void dec_attn_part_init(float* part, size_t bytes, hipStream_t s);
// Router top-k + grouping by expert in one block (T <= 64, E <= 256, top_k <= 8).
struct MoeRouteArgs {
    const float* logits = nullptr;
    int T = 0, E = 0, topk = 0, softmax_scoring = 1, norm_topk = 0;
    float scaling = 1.f;
    int* ids = nullptr; float* w = nullptr;
    int* eoff = nullptr; int* arow = nullptr; int* apos = nullptr;
    float* aw = nullptr;            // routing weight by sorted position
    int* active = nullptr; int* n_active = nullptr;
};
void launch_moe_route(const MoeRouteArgs& a, hipStream_t s);
// Routed experts + shared experts (gate/up: one launch; down + weighted combine + residual: one launch).
struct MoeDec2Args {
    int T = 0, topk = 0, E = 0, K = 0, I = 0, Is = 0, Hout = 0, slots = 0;
    const float* x = nullptr;       // [T][K] (pre-norm residual stream if norm_w)
    const float* norm_w = nullptr; float eps = 0.f;
    const int* eoff = nullptr; const int* arow = nullptr; const int* apos = nullptr; const int* ids = nullptr;
    const int* active = nullptr; const int* n_active = nullptr;
    const float* aw = nullptr;      // routing weight by sorted position (folded into h)
    const void* Wgu = nullptr; const void* Wd = nullptr;    // routed: E x [2I][K], E x [Hout][I]
    const void* sWgu = nullptr; const void* sWd = nullptr;  // shared / dense: [2Is][K], [Hout][Is]
    int wdtype = WDT_F16;
    float* h = nullptr; float* hs = nullptr;
    float* out = nullptr;           // [T][Hout], += combined
    // slot mode (T <= 8): h row of (token t, pick k) = t*topk + k (apos must be null).  With
    // `logits` set the gate/up blocks route themselves (ids_out / w_out receive the picks);
    // with logits == null the picks come from dec_router in ids / aw.
    int slot_mode = 0;
    const float* logits = nullptr;
    int softmax_scoring = 1, norm_topk = 0;
    float scaling = 1.f;
    int* ids_out = nullptr; float* w_out = nullptr;
    unsigned long long* span = nullptr;    // launch-span slots (SPAN_SLOTS pairs) or null
    // grouped mode (3 <= T <= 8): expert groups written by the router epilogue (MOE_GRP_* layout);
    // h rows stay in slot order (t*topk + k)
    const int* grp = nullptr;
    // optional fragment-ordered copies (launch_mm_swizzle) for the matrix-core grouped kernels:
    // routed [E * 2I][K], shared [2 Is][K]; routed down [E * H][I], shared down [H][Is]
    const void* Wgu_swz = nullptr; const void* sWgu_swz = nullptr;
    const void* Wd_swz = nullptr; const void* sWd_swz = nullptr;
    // matrix-core grouped down: per-segment partial tiles [segments][8][Hout] and per-128-row
    // arrival tickets [Hout / 128] (zero between launches; the last arriver resets them)
    float* dn_part = nullptr; int* dn_tick = nullptr;
    // grouped gate/up with the routing inside (moe_gateup_mm_route_ok): the router rows [E][K] (wdtype), an
    // optional logit bias; x is then the raw residual stream, normalised with norm_w in every block
    const void* router = nullptr; const float* router_bias = nullptr;
    const void* router_swz = nullptr;  // ... optional fragment-ordered copy of the router rows (launch_mm_swizzle)
    unsigned long long* stamps = nullptr;  // dev (tools/kbench moe8): per block 8 words of s_memrealtime at phase points
};
// Decode gate/up for one token (T = 1, E <= 64): every wave is independent — 1 of 4 streams
// shared-expert rows from its first instruction, 3 of 4 route themselves (rank-based top-k of
// the router logits) and stream their routed expert's rows; activations = the normalised row
// the router kernel wrote (xn).
bool moe_gateup_mix_ok(const MoeDec2Args& a);
void launch_moe_gateup_mix(const MoeDec2Args& a, const float* xn, hipStream_t s);
// Decode down + combine + residual for one token: split-K over each block's waves.
bool moe_down_mix_ok(const MoeDec2Args& a);
void launch_moe_down_mix(const MoeDec2Args& a, hipStream_t s);
void launch_moe_gateup2(const MoeDec2Args& a, hipStream_t s);
void launch_moe_down2(const MoeDec2Args& a, hipStream_t s);
// Grouped decode MoE (3 <= T <= 8): every distinct routed expert's rows are streamed once per layer
// (gate/up: routed groups + the shared expert in one launch; down: per output row over the
// concatenated [active experts | shared] K axis, per-token accumulators).
bool moe_grp_ok(const MoeDec2Args& a);
void launch_moe_gateup_grp(const MoeDec2Args& a, hipStream_t s);
void launch_moe_down_grp(const MoeDec2Args& a, hipStream_t s);
// the grouped gate/up on the matrix cores (decode_mm.hip): expert rows as MFMA A fragments, the
// token rows as three exact f16 planes
bool moe_gateup_mm_ok(const MoeDec2Args& a);
// the same with the router in every block (no dec_route_grp launch before it): RMSNorm of x with norm_w
// (x / den * w, as dec_route_grp), the E <= 64 router logits on the matrix cores, greedy top-k per token,
// the expert records (block 0 also writes them to grp, with the picks to ids_out / w_out, for the down launch)
bool moe_gateup_mm_route_ok(const MoeDec2Args& a);
void launch_moe_gateup_mm(const MoeDec2Args& a, hipStream_t s);
bool moe_down_mm_ok(const MoeDec2Args& a);
size_t moe_down_mm_part_floats(int E, int T, int topk, int I, int Is, int H);
void launch_moe_down_mm(const MoeDec2Args& a, hipStream_t s);

// One decode MoE layer for T tokens (block.rs:1215-1395): [RMSNorm] -> router GEMV (+ routing /
// grouping) -> gate/up -> down + weighted combine + shared experts + residual:
// out[T][H] += moe(rmsnorm(x)).  The single dispatch shared by Engine::decode_step and the
// kernel-level entry dsocr_k_moe.  Workspaces are device buffers sized as commented.
struct MoeDecodeArgs {
    int T = 0, H = 0, E = 0, topk = 0, I = 0, Is = 0;
    const float* x = nullptr; const float* norm_w = nullptr; float eps = 0.f;  // x: [T][H] (may equal out)
    const void* router = nullptr; int router_wdt = WDT_F16; const float* router_bias = nullptr;
    const void* Wgu = nullptr; const void* Wd = nullptr;    // [E][2I][H], [E][H][I]
    const void* sWgu = nullptr; const void* sWd = nullptr;  // [2Is][H], [H][Is] (or null)
    const void* Wgu_swz = nullptr; const void* sWgu_swz = nullptr;  // optional fragment-ordered copies
    const void* Wd_swz = nullptr; const void* sWd_swz = nullptr;
    const void* router_swz = nullptr;  // optional fragment-ordered router rows (the routing inside gate/up)
    int wdtype = WDT_F16;
    int softmax_scoring = 1, norm_topk = 0; float scaling = 1.f;
    float* out = nullptr;
    // workspaces
    float* xn = nullptr;        // [T][H]     normalised rows (T > 2)
    float* xn_router = nullptr; // [T][H]     normalised row handed from the router to gate/up (T = 1)
    float* logits = nullptr;    // [T][E]
    int* ids = nullptr; float* wts = nullptr;   // [T*topk] picks (outputs)
    float* h = nullptr;         // [T*topk][I]
    float* hs = nullptr;        // [T][Is]
    int* grp = nullptr;         // moe_grp_ints(E, T, topk)
    int* route_cnt = nullptr;   // [16], zero between launches (router epilogue ticket)
    float* dn_part = nullptr;   // moe_down_mm_part_floats(...)  (grouped matrix-core down)
    int* dn_tick = nullptr;     // [H / 128], zero between launches
    int* eoff = nullptr; int* arow = nullptr; int* apos = nullptr; int* active = nullptr;  // T > 8:
    int* n_active = nullptr; float* aw = nullptr;                                          // [E+1],[TK],[TK],[E],[1],[TK]
    unsigned long long* span = nullptr;  // launch-span slots for the gate/up and down launches (or null)
    unsigned long long* route_span = nullptr;  // launch-span slots for the router launch (or null)
    unsigned long long* stamps = nullptr;      // dev: the grouped gate/up's phase clocks (MoeDec2Args::stamps)
};
// ---- one-page decode step as ONE persistent launch (decode_persist.hip): every decoder layer inside 256 resident
// workgroups handing their vectors over as {f32, tag} granules (tag = the decode position; the granule buffer is
// reset to all-ones before a generate's first step and after the dry step)
constexpr int PK_G = 256;                 // workgroups, one per CU
constexpr int PK_CPH = 25;                // attention chunks per head
constexpr int PK_STAMPS = 9;              // phase clocks per (workgroup, layer) when DecPersistArgs::stamps is set
constexpr long PK_SPIN_TICKS = 5000000;   // one hand-off gives up after 50 ms (s_memrealtime, 100 MHz): *err = 2
struct PersistLayerW {
    const uint16_t* qkv = nullptr;        // f16 [3 heads hd][H] (q | k | v)
    const uint16_t* o = nullptr;          // f16 [H][heads hd]
    const float* in_w = nullptr;          // input RMSNorm weight [H]
    const float* post_w = nullptr;        // post-attention RMSNorm weight [H]
    const uint16_t* router = nullptr;     // f16 [E][H] (MoE layers)
    const float* router_bias = nullptr;   // [E] or null
    const uint16_t* e_gu = nullptr;       // routed f16 [E][2I][H] (gate rows, then up rows)
    const uint16_t* e_dT = nullptr;       // routed down TRANSPOSED f16 [E][I][H]
    const uint16_t* s_gu = nullptr;       // shared (MoE) / dense f16 [2 inter][H]
    const uint16_t* s_dT = nullptr;       // shared / dense down TRANSPOSED f16 [inter][H]
    int moe = 0;
    int inter = 0;                        // MoE: shared inter (n_shared * moe_inter); dense: intermediate_size
};
struct DecPersistArgs {
    int layers = 0;
    const PersistLayerW* lw = nullptr;    // device array [layers]
    float* x = nullptr;                   // s_x [H]: layer 0's input (plain loads), the last layer's output
    const int* kv_pos = nullptr;          // decode position (the tag of every granule of this step)
    const float* cos = nullptr; const float* sin = nullptr;  // rope tables [pos][hd]
    float* kc = nullptr; float* vc = nullptr;                // f32 cache, + l * layer_kv + head * head_stride + pos * hd
    long layer_kv = 0, head_stride = 0;
    float scale = 1.f, eps = 0.f;
    int softmax_scoring = 1, norm_topk = 0;
    float scaling = 1.f;
    unsigned long long* g = nullptr;      // granules [dec_persist_granules(layers)]
    int* err = nullptr;                   // a hand-off that gave up sets 2
    unsigned long long* stamps = nullptr; // optional [stamp_cap][PK_G][layers][PK_STAMPS] s_memrealtime phase clocks,
    int stamp_pos0 = 0, stamp_cap = 0;    // ... of the step at position stamp_pos0 + i, i < stamp_cap
};
size_t dec_persist_granules(int layers);
size_t dec_persist_lds_bytes();
// the decoder shape the launch is written for (DeepSeek-OCR: H 1280, 10 x 128 MHA, 64 experts top-6 of 896, 2
// shared, dense 6848), max_len <= 25 chunks x 64 keys
bool dec_persist_shape_ok(int hidden, int heads, int kv_heads, int head_dim, int n_routed, int topk, int moe_inter,
                          int shared_inter, int dense_inter, int max_len);
int dec_persist_resident();  // 1: all PK_G workgroups are resident at once on this device
void launch_dec_persist(const DecPersistArgs& a, hipStream_t s);
void launch_transpose16(const void* in, void* out, int N, int K, hipStream_t s);  // out[k][n] = in[n][k], 16-bit

enum MoeParts : int { MOE_ROUTE = 1, MOE_GATEUP = 2, MOE_DOWN = 4, MOE_ALL = 7 };
// kernel names of the gate/up and down launches the dispatch picks for these arguments
// false when the routing runs inside the gate/up launch (3..8 tokens, DSOCR_ROUTE_FUSED): MOE_ROUTE launches nothing
bool moe_decode_route_launch(const MoeDecodeArgs& a);
void moe_decode_kernel_names(const MoeDecodeArgs& a, const char** gateup, const char** down);
void launch_moe_decode(const MoeDecodeArgs& a, hipStream_t s, int parts = MOE_ALL);
// Greedy selection (ngram ban evaluated in-kernel) + step bookkeeping + KV advance.
struct DecSampleArgs {
    const float* logits = nullptr; int B = 0, V = 0; long ld = 0;
    int* ctx = nullptr; long ctx_cap = 0; int* ctx_len = nullptr;
    int ngram = 0;
    float* red_val = nullptr; int* red_idx = nullptr; int red_blocks = 0;
    int* out_tok = nullptr; int* out_ids = nullptr; int* out_len = nullptr; long out_cap = 0;
    int* done = nullptr; int eos = -1;
    const void* table = nullptr; int table_dt = 0; int H = 0; float* x_next = nullptr;
    int* kv_pos = nullptr; int* kv_len = nullptr;
    // n-gram ban list for the NEXT step ([count | tokens], ban_ld ints per page), written by the
    // final kernel after the context update when set (read by the screened lm_head)
    int* ban_out = nullptr; long ban_ld = 0;
    // screened selection (lmhead.hip): the candidate rows the int8 lm_head kept, the running
    // threshold key, exact rescoring from the bf16 rows and the normalised row xn
    // per lm_head block: kept-row count, best lower bound, and up to `slot` (row, hi) entries stored
    // entry-major ([page][entry][block]: the final kernel reads one entry of every block per load)
    const int* blk_cnt = nullptr; const float* blk_t = nullptr; const int* cand = nullptr; const float* cand_hi = nullptr;
    int nblk = 0; long slot = 0;
    const void* w_exact = nullptr; const float* xn = nullptr; int K = 0;
    int w_exact_wdt = WDT_BF16;  // the exact rows' storage (bf16, or f16 from a snapshot's dequantised lm_head)
    unsigned long long* stats = nullptr;  // [steps, kept rows, survivors] accumulated (diagnostics)
    // stochastic selection (sampling.hip; do_sample && temperature > 0): per-page rand StdRng state
    // ([B][RNG_WORDS]), top-k (0: off), top-p (active in [0, 1)), scratch of st_ld >= V entries
    // per page (keys / indices double-buffered: [B][2][st_ld]; f64 weights [B][st_ld])
    int do_sample = 0; double temperature = 0.0, top_p = -1.0; long top_k = 0;
    uint32_t* rng = nullptr; uint32_t* st_key = nullptr; int* st_idx = nullptr; double* st_w = nullptr; long st_ld = 0;
    unsigned long long* st_stamps = nullptr;  // diagnostics: shader clock at the sampler's phase points (page 0)
};
// rand StdRng state words per page: ChaCha12 key, 64-bit block counter, buffer index, 64-word buffer
constexpr int RNG_KEY = 0, RNG_CTR = 8, RNG_IDX = 10, RNG_BUF = 16, RNG_WORDS = 80;
void launch_dec_sample(const DecSampleArgs& a, hipStream_t s);
void launch_dec_stoch_select(const DecSampleArgs& a, hipStream_t s);
size_t dec_sample_blocks(int V);
// Screened lm_head (lmhead.hip): int8 rows + per-row scale / error bound give every row an
// interval [lo, hi] that provably contains the exact kernel's logit; each block keeps the best
// lower bound of its unbanned rows and the rows whose hi reached its running threshold (its own
// slot: no cross-block atomics); block 0 writes the normalised row.
struct LmHeadQ8Args {
    const float* x = nullptr; long ldx = 0; const float* norm_w = nullptr; float eps = 0.f;
    const void* q = nullptr; const float* scale = nullptr; const float* bound = nullptr;
    int B = 0, N = 0, K = 0;
    const int* ban = nullptr; long ban_ld = 0;
    int* blk_cnt = nullptr; float* blk_t = nullptr; int* cand = nullptr; float* cand_hi = nullptr;
    int nblk = 0; long slot = 0;  // from lmhead_q8_grid
    float* xn_out = nullptr;  // [B][K]
    // B = 3..8 (lmhead_q8mm): the fragment-ordered int8 copy and s_v ||Q_v|| per row (scale / bound / qnorm
    // padded to whole 16-row tiles); the grid from lmhead_q8mm_grid
    const void* qfrag = nullptr; const float* qnorm = nullptr;
};
void launch_lmhead_q8(const LmHeadQ8Args& a, hipStream_t s);
// grid of the screened lm_head for B pages: blocks per page and the per-block slot length
void lmhead_q8_grid(int N, int K, int B, int* nblk, long* slot);
// B = 3..8: one int8 stream for every token on the int8 matrix cores (K % 64 == 0, K <= 1536)
bool lmhead_q8mm_ok(int B, int N, int K);
void lmhead_q8mm_grid(int N, int K, int B, int* nblk, long* slot);
size_t lmhead_qfrag_bytes(int V, int K);
// load time: int8 rows + scale + bound (+ optional s ||Q|| and the fragment-ordered copy for B = 3..8);
// w: bf16 or f16 rows (wdtype)
void launch_lmhead_quantize(const void* w, int V, int K, void* q, float* scale, float* bound, hipStream_t s,
                            float* qnorm = nullptr, void* qfrag = nullptr, int wdtype = WDT_BF16);

// DSQ snapshot tensors (dsq.hip): dtype codes of crates/dsq/src/lib.rs:60-110; decode a record's
// payload ([out][in], row-major blocks) into fp16 on the device
constexpr int DSQ_F32 = 0, DSQ_F16 = 1, DSQ_Q8_0 = 8, DSQ_Q4K = 12, DSQ_Q6K = 14, DSQ_BF16 = 16;
size_t dsq_payload_bytes(int qtype, long out_dim, long in_dim);
void launch_dsq_dequant(int qtype, const void* src, long out_dim, long in_dim, void* out_f16, hipStream_t s);

// Page preprocessing on the GPU (preprocess.hip): Pillow 22-bit bicubic (tap tables from the host),
// then a vertical pass fused with canvas placement / tile cropping and the CHW normalisation
struct PpOut {
    const uint8_t* hz = nullptr; int dw = 0;                          // horizontal-pass rows [*][dw][3]
    const int* bounds = nullptr; const int* coeffs = nullptr; int ksize = 0;  // vertical taps
    int mode = 0;            // 0 global canvas, 1 tiles
    int size = 0;            // G or T
    int n_out = 1;           // 1 (global) or number of tiles
    int ox = 0, oy = 0, nw = 0, nh = 0;  // global: resized image placement
    int grid_w = 1;          // tiles per row
    float* out = nullptr;    // [n_out][3][size][size]
};
void launch_pp_resize_h(const uint8_t* src, int sw, int sh, const int* bounds, const int* coeffs, int ksize, int dw,
                        uint8_t* hz, hipStream_t s);
void launch_pp_resize_v_chw(const PpOut& a, hipStream_t s);

}  // namespace dsocr
