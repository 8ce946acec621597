// One-page decode step as ONE persistent launch (T = 1, DeepSeek-OCR's decoder shape): every decoder layer of a
// step runs inside 256 resident workgroups (one per CU) that hand each layer-internal vector to each other as
// 8-byte {f32 value, u32 tag} granules (MI355X_MICROARCH.md price list rows handoff-1to1 / allgather /
// transport-variants: one write-through `sc1` store per granule, `sc1` loads polled until the tag matches: no
// flag, no fence, no grid barrier).  What the launch chain cannot do and this launch does: every workgroup issues
// the weight rows of its NEXT piece of work (and its K / V cache chunk) before that piece's input exists, so the
// HBM stream of a phase overlaps the hand-off in front of it instead of starting after a kernel boundary.
//
// Reference: TransformerBlock::forward_internal (crates/infer-deepseek/src/transformer/block.rs:124-191) per
// layer — attention_forward (:446-804: q/k/v, rotate_half RoPE :1403-1471, f32 KV cache :776-789, softmax
// attention), o_proj + residual, post-attention RMSNorm, run_moe (:1215-1395: softmax router, greedy top-k,
// per-expert SwiGLU :1326-1351, shared experts, combine :1357-1389) or run_dense_mlp (:1179-1213) + residual.
//
// Wave roles (MI355X_MICROARCH.md rows polling-cost / gather-pass): vector-memory loads return in issue order, so
// a wave that polls a hand-off also waits for every prefetch it has in flight.  Hence waves 0..6 ("workers") issue
// every weight / cache stream and compute, and never poll; wave 7 (the "poller") has nothing in flight when it
// polls: it gathers every hand-off into LDS, loads the small per-layer vectors (norm weights, rope row, router
// bias), runs the RMSNorms, the attention merge and the top-k.  Workgroup barriers are raw s_barrier (no vmcnt
// drain: the workers' prefetches stay in flight across them).  The K / V chunk and the down rows land in LDS by
// LDS-DMA (global_load_lds, 16 bytes per lane), the q/k/v, o_proj, router and gate/up rows in worker registers.
//
// Work of workgroup c per layer (G = 256; dec_persist_shape_ok checks the shape):
//   x      : x_l (1280 granules; layer 0: s_x, plain) -> RMSNorm (poller)
//   q/k/v  : rows [15 c, 15 c + 15) of the fused [3840][1280] projection -> QKV granules
//   attn   : c < 250: head c / 25, key chunk c % 25 of ceil(L / 25) keys (LDS-DMA'd during the previous layer):
//            q (and, owning the new position, k / v) gathered, RoPE, k / v appended to the f32 cache, scores /
//            softmax / P.V over the chunk -> partial record {m, l, o[128]} granules
//   merge  : dims [5 c, 5 c + 5): the 25 records of the dim's head (flash-decoding merge) -> CTX granules
//   o_proj : rows [5 c, 5 c + 5) over the gathered ctx, + residual -> XN granules (x_new)
//   mlp    : x_new -> RMSNorm (poller); MoE: c < 64 computes router logit c -> LG granules; the poller gathers
//            the 64 logits and ranks the top-6 (topk_wave64); the workers compute h for 28 (gate, up) row pairs
//            (4 per worker): 7 of the shared expert, 21 of the routed picks (routed h index 21 c .. 21 c + 20 of
//            6 x 896); dense layer 0: 26-27 of the 6848.  Each h scales its row of the TRANSPOSED down matrix
//            (split-K: the workgroup's partial of all 1280 outputs); the 7 workers' partials meet in LDS ->
//            DP granules, 5 rows per owner workgroup
//   reduce : owner c sums the 256 partials of rows [5 c, 5 c + 5), + x_new -> x_{l+1} granules (last layer:
//            s_x, plain, for the head launch that follows)
// Numerics: f32 everywhere with the reference's formulas (x / den * w RMSNorm, x / (1 + e^-x) SiLU, softmax with
// the maximum subtracted, stable-descending top-k, routing weight folded into h as in the launch chain); the
// summation orders differ from the launch chain (split-K down, per-dim attention merge): covered by the
// full-length greedy-id / logit parity tests (tests/test_persist.py, tests/test_full_parity.py).
#include "dev_common.hpp"

#include <type_traits>

namespace dsocr {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void pk_lds_void;

namespace {
constexpr int NT = 512, NW = 8, NWK = 7;  // threads, waves, worker waves (wave 7 polls)
constexpr int G = PK_G;                   // workgroups (one per CU)
constexpr int H = 1280, HC = H / 8;       // hidden, 16-byte chunks of an f16 row
constexpr int HD = 128, NH = 10, QKVN = 3 * NH * HD;
constexpr int QR = QKVN / G;              // 15 q/k/v rows per workgroup
constexpr int OR = H / G;                 // 5 owner rows per workgroup
constexpr int E = 64, TOPK = 6, I = 896, IS = 1792;
constexpr int SH_PER = IS / G;            // 7 shared h per workgroup (one per worker)
constexpr int RT_PER = TOPK * I / G;      // 21 routed h per workgroup (three per worker)
constexpr int CPH = PK_CPH;               // attention chunks per head
constexpr int KPW = 8;                    // keys per worker wave
constexpr int CHMAX = KPW * NWK;          // 56 keys per chunk
constexpr int PR = 132;                   // partial record granules: m, l, -, -, o[128]
constexpr int DPR = 6;                    // owner staging per source: the 3 granule pairs that hold its 5 rows
constexpr int SLOTS = 4;                  // MLP h slots per worker
static_assert(QR * G == QKVN && OR * G == H && SH_PER * G == IS && RT_PER * G == TOPK * I, "exact split");
static_assert(SH_PER == NWK && RT_PER == 3 * NWK && QR <= 3 * NWK && OR <= NWK - 2, "worker roles");

// granule offsets inside one layer's region (all even: 16-byte aligned pairs)
constexpr long O_EX = 0;                  // x_{l+1} (written by layer l)
constexpr long O_QKV = O_EX + H;
constexpr long O_PART = O_QKV + QKVN;
constexpr long O_CTX = O_PART + (long)NH * CPH * PR;
constexpr long O_XN = O_CTX + H;
constexpr long O_LG = O_XN + H;
constexpr long O_DP = O_LG + E;
constexpr long O_LAYER = O_DP + (long)G * H;  // DP: [source workgroup][H] (contiguous per producer)
static_assert(O_LAYER % 2 == 0 && O_DP % 2 == 0 && O_PART % 2 == 0 && O_LG % 2 == 0 && PR % 2 == 0, "pairs");

// LDS (floats; every region 16-byte aligned)
constexpr int L_XA = 0;                     // [H] normalised x_l, then ctx
constexpr int L_XB = L_XA + H;              // [H] normalised x_new, then the workgroup's summed down partial
constexpr int L_WN = L_XB + H;              // [H] input RMSNorm weight
constexpr int L_WN2 = L_WN + H;             // [H] post-attention RMSNorm weight
constexpr int L_CS = L_WN2 + H;             // [HD] rope cos at the position
constexpr int L_SN = L_CS + HD;             // [HD] rope sin
constexpr int L_RAW = L_SN + HD;            // [3 HD] gathered q / k / v
constexpr int L_QS = L_RAW + 3 * HD;        // [HD] rotated q
constexpr int L_KS = L_QS + HD;             // [HD] rotated new k
constexpr int L_VS = L_KS + HD;             // [HD] new v
constexpr int L_RED = L_VS + HD;            // [64]
constexpr int L_OW = L_RED + 64;            // [2 NWK][HD] attention o per half-wave
constexpr int L_LG = L_OW + 2 * NWK * HD;   // [64] logits
constexpr int L_RK = L_LG + 64;             // [128] rank scratch
constexpr int L_IDS = L_RK + 128;           // [8] picks (int)
constexpr int L_WTS = L_IDS + 8;            // [8] pick weights
constexpr int L_XRES = L_WTS + 8;           // [8] x_l of the owner rows
constexpr int L_XNEW = L_XRES + 8;          // [8] x_new of the owner rows
constexpr int L_MISC = L_XNEW + 8;          // [8] router bias of this workgroup's expert
constexpr int L_MST = L_MISC + 8;           // [5][32][4] merge staging (m, l, o)
constexpr int L_YS = L_MST + OR * 32 * 4;   // [NWK][H] worker partials / owner-gather staging [G][DPR]
constexpr int L_R = L_YS + NWK * H;         // K [56][HD] + V [56][HD] during attention; down rows [28][H/2 f32]
constexpr int R_ROW = H / 2;                // one f16 row of 1280 in floats
constexpr int R_FLOATS = (NWK * SLOTS * R_ROW > 2 * CHMAX * HD) ? NWK * SLOTS * R_ROW : 2 * CHMAX * HD;
constexpr int L_END = L_R + R_FLOATS;
static_assert(L_R % 4 == 0 && L_YS % 4 == 0 && L_MST % 4 == 0, "aligned");
static_assert(G * DPR <= NWK * H, "owner staging");
}  // namespace

size_t dec_persist_granules(int layers) { return (size_t)layers * O_LAYER; }
size_t dec_persist_lds_bytes() { return (size_t)L_END * 4; }  // > 80 KiB: one workgroup per CU
static_assert(L_END * 4 <= 160 * 1024 && L_END * 4 > 80 * 1024, "lds");

// 16-byte nontemporal load through a GLOBAL pointer: the weight pointers come from the per-layer table in memory,
// so the compiler cannot infer their address space and would emit flat loads (counted in lgkmcnt too)
typedef const __attribute__((address_space(1))) u32x4* pk_gptr16;
__device__ __forceinline__ uint4 pk_ld16(const void* p) {
    const u32x4 v = __builtin_nontemporal_load((pk_gptr16)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 pk_ldf4(const float* p) {  // plain 16-byte load of a small per-layer vector
    const u32x4 v = *(pk_gptr16)p;
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
// LDS-DMA: 16 bytes per active lane to lds_base + lane * 16 (lds_base wave-uniform), nontemporal
__device__ __forceinline__ void pk_dma16(const void* src, float* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src, (pk_lds_void*)lds_base, 16, 0, 2);
}

// raw workgroup barrier: LDS stores of this wave complete, then s_barrier (no vmcnt drain: prefetches stay in
// flight across it; __syncthreads' release fence would wait for them)
__device__ __forceinline__ void pk_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void pk_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// this wave's LDS stores visible to its own later LDS loads by other lanes
__device__ __forceinline__ void pk_wave_lds() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ float pk_half_sum(float v) {  // sum over the 32 lanes of a half-wave
    v += dpp_f<DPP_QUAD_XOR1>(0.f, v);
    v += dpp_f<DPP_QUAD_XOR2>(0.f, v);
    v += dpp_f<DPP_ROW_HALF_MIRROR>(0.f, v);
    v += dpp_f<DPP_ROW_MIRROR>(0.f, v);
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1f | (16 << 10)));
    return v;
}

__device__ __forceinline__ void ld_x8l(const float* p, float* o) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// one 1280-long f16 row as 3 x 16 bytes per lane (chunks lane, 64 + lane, 128 + lane; the third only lanes < 32)
__device__ __forceinline__ void pk_row_issue(const uint16_t* row, uint4 (&w)[3]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < 3; ++u) w[u] = pk_ld16(row + (min(u * 64 + lane, HC - 1) << 3));
}
// the same row into LDS (R_ROW floats at dst) by LDS-DMA
__device__ __forceinline__ void pk_row_dma(const uint16_t* row, float* dst) {
    const int lane = threadIdx.x & 63;
    pk_dma16(row + lane * 8, dst);
    pk_dma16(row + 512 + lane * 8, dst + 256);
    if (lane < 32) pk_dma16(row + 1024 + lane * 8, dst + 512);
}
// dot of a register row with the LDS row xs, summed over the wave (every lane gets it)
__device__ __forceinline__ float pk_row_dot(const uint4 (&w)[3], const float* xs) {
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int cc = u * 64 + lane;
        if (cc < HC) {
            float w8[8], x8[8];
            unpack8<f16_t>(w[u], w8);
            ld_x8l(xs + (cc << 3), x8);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc = fmaf(x8[j], w8[j], acc);
        }
    }
    return wave_sum(acc);
}

template <bool STAMP>
__global__ __launch_bounds__(NT, 1) void dec_persist_kernel(DecPersistArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* xa = sm + L_XA;
    float* xb = sm + L_XB;
    float* wn = sm + L_WN;
    float* wn2 = sm + L_WN2;
    float* cs = sm + L_CS;
    float* sn = sm + L_SN;
    float* raw = sm + L_RAW;
    float* qs = sm + L_QS;
    float* ks = sm + L_KS;
    float* vs = sm + L_VS;
    float* red = sm + L_RED;
    float* ow = sm + L_OW;
    float* lgs = sm + L_LG;
    float* rks = sm + L_RK;
    int* ids = reinterpret_cast<int*>(sm + L_IDS);
    float* wts = sm + L_WTS;
    float* xres = sm + L_XRES;
    float* xnew = sm + L_XNEW;
    float* misc = sm + L_MISC;
    float* mst = sm + L_MST;
    float* ys = sm + L_YS;
    float* rr = sm + L_R;
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool poller = wave == NW - 1;
    const auto gr = __builtin_amdgcn_make_buffer_rsrc(a.g, (short)0, (int)((long)a.layers * O_LAYER * 8), 0x00020000);
    const int pos = a.kv_pos[0];
    const unsigned tag = (unsigned)pos;
    const int Lk = pos + 1;                      // keys attended (the new one included)
    const int CH = (Lk + CPH - 1) / CPH;         // keys per chunk (<= CHMAX: dec_persist_shape_ok's max_len)
    const bool att = c < NH * CPH;
    const int ah = att ? c / CPH : 0, aj = att ? c % CPH : 0;
    const int k0 = aj * CH;
    const int kn = att ? max(0, min(CH, Lk - k0)) : 0;
    const bool own = att && pos >= k0 && pos < k0 + kn;
    bool dead = false;                           // a hand-off gave up (error flag set): stop waiting
    unsigned long long stp[PK_STAMPS];
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if (STAMP) stp[i] = __builtin_amdgcn_s_memrealtime();
    };

    // ---- granule hand-offs (stores: any wave; loads: the poller)
    auto put1 = [&](long gi, float v) __attribute__((always_inline)) {
        const u32x2 w = {__float_as_uint(v), tag};
        __builtin_amdgcn_raw_buffer_store_b64(w, gr, (int)(gi * 8), 0, 16);  // sc1: write-through
    };
    auto put2 = [&](long gi, float v0, float v1) __attribute__((always_inline)) {
        const u32x4 w = {__float_as_uint(v0), tag, __float_as_uint(v1), tag};
        __builtin_amdgcn_raw_buffer_store_b128(w, gr, (int)(gi * 8), 0, 16);
    };
    auto give_up = [&](unsigned long long t0) __attribute__((always_inline)) {
        if (dead) return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)PK_SPIN_TICKS) {
            dead = true;
            if (a.err) __hip_atomic_store(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return true;
        }
        return false;
    };
    // poller: pairs lane, lane + 64, ... (< np, at most MAXP per lane) of the granules from gi0 (even) into
    // dst[2 p], dst[2 p + 1]; every load of a pass in flight at once
    auto gather = [&](auto maxp_tag, long gi0, int np, float* dst, int pmap = 0) __attribute__((always_inline)) {
        // pmap = 0: pair p at granule gi0 + 2 p; pmap = 1 (owner reduction): pair p = 3 s + k at gi0 + s H + 2 k
        constexpr int MAXP = decltype(maxp_tag)::value;
        unsigned pend = 0;
#pragma unroll
        for (int k = 0; k < MAXP; ++k)
            if (lane + 64 * k < np) pend |= 1u << k;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        u32x4 v[MAXP];
        while (pend) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < MAXP; ++k)
                if ((pend >> k) & 1u) {
                    const int pp = lane + 64 * k;
                    const long gi = pmap ? gi0 + (long)(pp / 3) * H + 2 * (pp % 3) : gi0 + 2 * pp;
                    v[k] = __builtin_amdgcn_raw_buffer_load_b128(gr, (int)(gi * 8), 0, 16);
                }
#pragma unroll
            for (int k = 0; k < MAXP; ++k)
                if (((pend >> k) & 1u) && v[k].y == tag && v[k].w == tag) {
                    const int p = lane + 64 * k;
                    dst[2 * p] = __uint_as_float(v[k].x);
                    dst[2 * p + 1] = __uint_as_float(v[k].z);
                    pend &= ~(1u << k);
                }
            if (!pend) break;
            if (give_up(t0)) {
#pragma unroll
                for (int k = 0; k < MAXP; ++k)
                    if ((pend >> k) & 1u) {
                        const int p = lane + 64 * k;
                        dst[2 * p] = 0.f;
                        dst[2 * p + 1] = 0.f;
                    }
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // poller: a 1280-float vector from global memory into LDS (plain loads, five 16-byte loads per lane)
    auto load_vec = [&](const float* src, float* dst) __attribute__((always_inline)) {
        float4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = pk_ldf4(src + (k * 64 + lane) * 4);
#pragma unroll
        for (int k = 0; k < 5; ++k) *reinterpret_cast<float4*>(dst + (k * 64 + lane) * 4) = v[k];
    };
    // poller: RMSNorm of the LDS row x in place, x / sqrt(mean(x^2) + eps) * w
    auto norm_row = [&](float* x, const float* w) __attribute__((always_inline)) {
        float4 v[5];
        float q = 0.f;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            v[k] = *reinterpret_cast<const float4*>(x + (k * 64 + lane) * 4);
            q += (v[k].x * v[k].x + v[k].y * v[k].y) + (v[k].z * v[k].z + v[k].w * v[k].w);
        }
        const float den = sqrtf(wave_sum(q) / (float)H + a.eps);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const float4 w4 = *reinterpret_cast<const float4*>(w + (k * 64 + lane) * 4);
            v[k].x = (v[k].x / den) * w4.x;
            v[k].y = (v[k].y / den) * w4.y;
            v[k].z = (v[k].z / den) * w4.z;
            v[k].w = (v[k].w / den) * w4.w;
            *reinterpret_cast<float4*>(x + (k * 64 + lane) * 4) = v[k];
        }
    };

    // ---- worker prefetch of a layer's q/k/v rows (wave w: rows 15 c + w + 7 r) and K / V chunk (LDS-DMA)
    uint4 wq[3][3];
    auto issue_qkv_kv = [&](int l) __attribute__((always_inline)) {
        const PersistLayerW& W = a.lw[l];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            if (wave + NWK * r < QR) pk_row_issue(W.qkv + (long)(QR * c + wave + NWK * r) * H, wq[r]);
        if (att) {
            const float* Kc = a.kc + (long)l * a.layer_kv + (long)ah * a.head_stride;
            const float* Vc = a.vc + (long)l * a.layer_kv + (long)ah * a.head_stride;
            const int d4 = (lane & 31) * 4;
#pragma unroll
            for (int i = 0; i < KPW / 2; ++i) {
                const int kk = wave * KPW + 2 * i;                  // keys kk (lanes 0..31), kk + 1 (32..63)
                const int key = min(k0 + kk + (lane >> 5), Lk - 1); // clamped: a key past the chunk is masked
                pk_dma16(Kc + (long)key * HD + d4, rr + kk * HD);
                pk_dma16(Vc + (long)key * HD + d4, rr + CHMAX * HD + kk * HD);
            }
        }
    };
    // The two roles run separate layer loops (disjoint register live ranges: a worker's prefetched rows are not
    // live in the poller's code and the reverse); both meet at the same nine raw barriers per layer.
    if (poller) {
        // the rope row of this step's position (every layer rotates at it)
        if (lane < HD / 4) {
            *reinterpret_cast<float4*>(cs + lane * 4) = pk_ldf4(a.cos + (long)pos * HD + lane * 4);
            *reinterpret_cast<float4*>(sn + lane * 4) = pk_ldf4(a.sin + (long)pos * HD + lane * 4);
        }
        for (int l = 0; l < a.layers; ++l) {
            const PersistLayerW& W = a.lw[l];
            const long gl = (long)l * O_LAYER;
            const bool moe = W.moe != 0;
            // ======== x_l: gather, keep the owner rows, RMSNorm
            stamp(0);
            load_vec(W.in_w, wn);
            if (moe && c < E && lane == 0) misc[0] = W.router_bias ? W.router_bias[c] : 0.f;
            if (l == 0) load_vec(a.x, xa);
            else gather(std::integral_constant<int, 10>(), gl - O_LAYER + O_EX, H / 2, xa);
            pk_wave_lds();
            if (lane < OR) xres[lane] = xa[OR * c + lane];
            norm_row(xa, wn);
            load_vec(W.post_w, wn2);
            stamp(1);
            pk_sync();  // #1: normalised x_l
            // ======== q / k / v of this chunk's head
            if (att) {
                const long qb = gl + O_QKV + (long)ah * HD;
                gather(std::integral_constant<int, 1>(), qb, HD / 2, raw);
                if (own) {
                    gather(std::integral_constant<int, 1>(), qb + H, HD / 2, raw + HD);
                    gather(std::integral_constant<int, 1>(), qb + 2 * H, HD / 2, raw + 2 * HD);
                }
                pk_wave_lds();
                // rotate_half RoPE at the position (block.rs:1403-1471): x cos + (-x[d + 64] | x[d - 64]) sin
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const int d = lane + 64 * h2;
                    const float pq = d < HD / 2 ? -1.f * raw[d + HD / 2] : raw[d - HD / 2];
                    qs[d] = raw[d] * cs[d] + pq * sn[d];
                    if (own) {
                        const float* kr = raw + HD;
                        const float pk = d < HD / 2 ? -1.f * kr[d + HD / 2] : kr[d - HD / 2];
                        ks[d] = kr[d] * cs[d] + pk * sn[d];
                        vs[d] = raw[2 * HD + d];
                    }
                }
            }
            stamp(2);
            pk_sync();  // #2: q (k, v) rotated in LDS
            pk_sync();  // #3: chunk maximum (workers)
            pk_sync();  // #4: chunk partials (workers)
            stamp(3);
            // ======== merge: dims d_t = 5 c + t; (t, chunk j) for q = lane, lane + 64 < 125
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int q = lane + 64 * k;
                if (q < OR * CPH) {
                    const int t = q / CPH, j = q % CPH;
                    const int d = OR * c + t, h = d / HD, dd = d % HD;
                    const long rec = gl + O_PART + (long)(h * CPH + j) * PR;
                    float mv = -INFINITY, lv = 0.f, ov = 0.f;
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    for (;;) {
                        asm volatile("" ::: "memory");
                        const u32x4 ml = __builtin_amdgcn_raw_buffer_load_b128(gr, (int)(rec * 8), 0, 16);
                        const u32x2 o2 = __builtin_amdgcn_raw_buffer_load_b64(gr, (int)((rec + 4 + dd) * 8), 0, 16);
                        if (ml.y == tag && ml.w == tag && o2.y == tag) {
                            mv = __uint_as_float(ml.x);
                            lv = __uint_as_float(ml.z);
                            ov = __uint_as_float(o2.x);
                            break;
                        }
                        if (give_up(t0)) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                    *reinterpret_cast<float4*>(mst + (t * 32 + j) * 4) = make_float4(mv, lv, ov, 0.f);
                }
            }
            pk_wave_lds();
#pragma unroll
            for (int t = 0; t < OR; ++t) {
                const float4 r4 = lane < CPH ? *reinterpret_cast<const float4*>(mst + (t * 32 + lane) * 4)
                                             : make_float4(-INFINITY, 0.f, 0.f, 0.f);
                const float M = wave_max(r4.x);
                const float w = r4.x != -INFINITY ? expf(r4.x - M) : 0.f;
                const float ls = wave_sum(r4.y * w);
                const float os = wave_sum(r4.z * w);
                if (lane == 0) put1(gl + O_CTX + OR * c + t, os / ls);
            }
            stamp(4);
            // ======== ctx for o_proj
            gather(std::integral_constant<int, 10>(), gl + O_CTX, H / 2, xa);
            pk_sync();  // #5: ctx in LDS
            // ======== x_new -> RMSNorm
            stamp(5);
            gather(std::integral_constant<int, 10>(), gl + O_XN, H / 2, xb);
            pk_wave_lds();
            norm_row(xb, wn2);
            pk_sync();  // #6: normalised x_new
            if (moe) {
                // the 64 logits (lanes 0..31 poll a pair each), then the reference router's greedy top-k
                gather(std::integral_constant<int, 1>(), gl + O_LG, E / 2, lgs);
                pk_wave_lds();
                topk_wave64(lgs[lane], E, TOPK, a.softmax_scoring, a.norm_topk, a.scaling, rks, ids, wts);
            }
            stamp(6);
            pk_sync();  // #7: picks
            pk_sync();  // #8: worker partials
            for (int j = tid; j < H; j += NT) {
                float v = ys[j];
#pragma unroll
                for (int w = 1; w < NWK; ++w) v += ys[w * H + j];
                xb[j] = v;
            }
            pk_sync();  // #9: the workgroup's partial; ys free
            stamp(7);
            // ======== owner reduction: rows [5 c, 5 c + 5) over the 256 partials, + x_new
            // every source's partial is contiguous: rows 5 c .. 5 c + 4 sit in the 3 pairs from granule 5 c & ~1
            const int odd = (OR * c) & 1;
            gather(std::integral_constant<int, 12>(), gl + O_DP + ((OR * c) & ~1), G * 3, ys, 1);
            pk_wave_lds();
#pragma unroll
            for (int r = 0; r < OR; ++r) {
                float s = ys[lane * DPR + odd + r] + ys[(lane + 64) * DPR + odd + r];
                s += ys[(lane + 128) * DPR + odd + r] + ys[(lane + 192) * DPR + odd + r];
                s = wave_sum(s);
                const float xo = xnew[r] + s;
                if (lane == 0) {
                    if (l + 1 < a.layers) put1(gl + O_EX + OR * c + r, xo);
                    else a.x[OR * c + r] = xo;
                }
            }
            stamp(8);
            if (STAMP && lane == 0 && a.stamps && pos - a.stamp_pos0 >= 0 && pos - a.stamp_pos0 < a.stamp_cap) {
                unsigned long long* sp =
                    a.stamps + (((long)(pos - a.stamp_pos0) * G + c) * a.layers + l) * PK_STAMPS;
#pragma unroll
                for (int i = 0; i < PK_STAMPS; ++i) sp[i] = stp[i];
            }
        }
        return;
    }

    // ---- workers
    issue_qkv_kv(0);
    const int kq = wave * KPW + (lane >> 5);  // key of instruction i: kq + 2 i
    const int d4 = (lane & 31) * 4;
    for (int l = 0; l < a.layers; ++l) {
        const PersistLayerW& W = a.lw[l];
        const long gl = (long)l * O_LAYER;
        const bool moe = W.moe != 0;
        pk_sync();  // #1: normalised x_l
        // ======== q/k/v rows
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            if (wave + NWK * r < QR) {
                const float y = pk_row_dot(wq[r], xa);
                if (lane == 0) put1(gl + O_QKV + QR * c + wave + NWK * r, y);
            }
        }
        pk_sync();  // #2: q (k, v) rotated in LDS
        // ======== attention chunk
        float sc[KPW / 2];
        if (att) {
            if (own && wave == 0) {  // the new key / value into the f32 cache (block.rs:776-789)
                float* Kc = a.kc + (long)l * a.layer_kv + (long)ah * a.head_stride + (long)pos * HD;
                float* Vc = a.vc + (long)l * a.layer_kv + (long)ah * a.head_stride + (long)pos * HD;
                if (lane < 32) *reinterpret_cast<float4*>(Kc + d4) = *reinterpret_cast<const float4*>(ks + d4);
                else *reinterpret_cast<float4*>(Vc + d4) = *reinterpret_cast<const float4*>(vs + d4);
            }
            pk_wait_all();  // this wave's K / V DMA landed
            const float4 q4 = *reinterpret_cast<const float4*>(qs + d4);
            float mloc = -INFINITY;
#pragma unroll
            for (int i = 0; i < KPW / 2; ++i) {
                const int kk = kq + 2 * i;
                const float4 k4 = k0 + kk == pos ? *reinterpret_cast<const float4*>(ks + d4)
                                                 : *reinterpret_cast<const float4*>(rr + kk * HD + d4);
                float v = fmaf(q4.w, k4.w, fmaf(q4.z, k4.z, fmaf(q4.y, k4.y, q4.x * k4.x)));
                v = pk_half_sum(v);
                sc[i] = kk < kn ? v * a.scale : -INFINITY;
                mloc = fmaxf(mloc, sc[i]);
            }
            const float mw = wave_max(mloc);
            if (lane == 0) red[wave] = mw;
        }
        pk_sync();  // #3: chunk maximum
        if (att) {
            float am = -INFINITY;
#pragma unroll
            for (int i = 0; i < NWK; ++i) am = fmaxf(am, red[i]);
            float ls = 0.f;
            float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i = 0; i < KPW / 2; ++i) {
                const int kk = kq + 2 * i;
                const float p = kk < kn ? expf(sc[i] - am) : 0.f;
                // never p * (stale cache bits): a key past the chunk reads as 0, the new key from the hand-off
                const float4 v4 = kk >= kn ? make_float4(0.f, 0.f, 0.f, 0.f)
                                           : (k0 + kk == pos ? *reinterpret_cast<const float4*>(vs + d4)
                                                             : *reinterpret_cast<const float4*>(rr + CHMAX * HD + kk * HD + d4));
                ls += p;
                o.x = fmaf(p, v4.x, o.x);
                o.y = fmaf(p, v4.y, o.y);
                o.z = fmaf(p, v4.z, o.z);
                o.w = fmaf(p, v4.w, o.w);
            }
            *reinterpret_cast<float4*>(ow + (2 * wave + (lane >> 5)) * HD + d4) = o;
            if ((lane & 31) == 0) red[16 + 2 * wave + (lane >> 5)] = ls;
        }
        pk_sync();  // #4: chunk partials in LDS; R (K / V) free
        // ======== the record (workers 0, 1), then the prefetch for o_proj / router / MLP
        if (att) {
            const long rec = gl + O_PART + (long)(ah * CPH + aj) * PR;
            if (tid < HD / 2) {
                float o0 = 0.f, o1 = 0.f;
#pragma unroll
                for (int hw = 0; hw < 2 * NWK; ++hw) {
                    o0 += ow[hw * HD + 2 * tid];
                    o1 += ow[hw * HD + 2 * tid + 1];
                }
                put2(rec + 4 + 2 * tid, o0, o1);
            } else if (tid == HD / 2) {
                float m = -INFINITY, ls = 0.f;
#pragma unroll
                for (int i = 0; i < NWK; ++i) m = fmaxf(m, red[i]);
#pragma unroll
                for (int hw = 0; hw < 2 * NWK; ++hw) ls += red[16 + hw];
                put2(rec, m, ls);
            }
        }
        uint4 wo[3], wr[3];
        uint4 gu[SLOTS][2][3];
        float swt[SLOTS];
        int nslot_dense = 0, dbase = 0;
        if (!moe) {
            const int per = W.inter / G, rem = W.inter % G;
            nslot_dense = per + (c < rem ? 1 : 0);
            dbase = c * per + min(c, rem);
        }
        if (wave < OR) pk_row_issue(W.o + (long)(OR * c + wave) * H, wo);
        if (moe && c < E && wave == OR) pk_row_issue(W.router + (long)c * H, wr);
        // MLP slot 0 prefetched now (MoE: shared h 7 c + w; dense: h dbase + w), slots 1..3 after the picks
        // (MoE: routed h 21 c + 3 w + j - 1; dense: h dbase + w + 7 j)
        {
            const int i = moe ? SH_PER * c + wave : dbase + wave;
            const int inter = moe ? IS : W.inter;
            pk_row_issue(W.s_gu + (long)i * H, gu[0][0]);
            pk_row_issue(W.s_gu + (long)(inter + i) * H, gu[0][1]);
            pk_row_dma(W.s_dT + (long)i * H, rr + (wave * SLOTS) * R_ROW);
            swt[0] = 1.f;
        }
        pk_sync();  // #5: ctx in LDS
        // ======== o_proj rows [5 c, 5 c + 5) + residual
        if (wave < OR) {
            const float y = pk_row_dot(wo, xa);
            const float xn = xres[wave] + y;
            if (lane == 0) {
                put1(gl + O_XN + OR * c + wave, xn);
                xnew[wave] = xn;
            }
        }
        pk_sync();  // #6: normalised x_new
        float yacc[3][8];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) yacc[u][k] = 0.f;
        float hv[SLOTS];
        // h = silu(g) u (w_k folded in for a routed pick; candle: x / (1 + exp(-x)))
        auto slot_h = [&](int j) __attribute__((always_inline)) {
            float ag = 0.f, au = 0.f;
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int cc = u * 64 + lane;
                if (cc < HC) {
                    float g8[8], u8[8], x8[8];
                    unpack8<f16_t>(gu[j][0][u], g8);
                    unpack8<f16_t>(gu[j][1][u], u8);
                    ld_x8l(xb + (cc << 3), x8);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        ag = fmaf(x8[k], g8[k], ag);
                        au = fmaf(x8[k], u8[k], au);
                    }
                }
            }
            const float gs = wave_sum(ag), us = wave_sum(au);
            hv[j] = ((gs / (1.0f + expf(-gs))) * us) * swt[j];
        };
        // its down row (LDS) scaled by h into the partial
        auto slot_down = [&](int j) __attribute__((always_inline)) {
            const float* dr = rr + (wave * SLOTS + j) * R_ROW;
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int cc = u * 64 + lane;
                if (cc < HC) {
                    const float4 q = *reinterpret_cast<const float4*>(dr + cc * 4);
                    uint4 bits;
                    __builtin_memcpy(&bits, &q, 16);
                    float d8[8];
                    unpack8<f16_t>(bits, d8);
#pragma unroll
                    for (int k = 0; k < 8; ++k) yacc[u][k] = fmaf(hv[j], d8[k], yacc[u][k]);
                }
            }
        };
        if (moe && c < E && wave == OR) {  // router logit c
            const float v = pk_row_dot(wr, xb) + misc[0];
            if (lane == 0) put1(gl + O_LG + c, v);
        }
        slot_h(0);
        pk_sync();  // #7: picks
        auto slot_ok = [&](int j) __attribute__((always_inline)) { return moe || wave + NWK * j < nslot_dense; };
#pragma unroll
        for (int j = 1; j < SLOTS; ++j) {
            if (!slot_ok(j)) continue;
            if (moe) {
                const int g = RT_PER * c + 3 * wave + j - 1;
                const int k = g / I, i = g % I;
                const int e = min(max(ids[k], 0), E - 1);  // (a pick is always < E; clamped: no stray stream)
                const uint16_t* gp = W.e_gu + ((long)e * 2 * I + i) * H;
                pk_row_issue(gp, gu[j][0]);
                pk_row_issue(gp + (long)I * H, gu[j][1]);
                pk_row_dma(W.e_dT + ((long)e * I + i) * H, rr + (wave * SLOTS + j) * R_ROW);
                swt[j] = wts[k];
            } else {
                const int i = dbase + wave + NWK * j;
                pk_row_issue(W.s_gu + (long)i * H, gu[j][0]);
                pk_row_issue(W.s_gu + (long)(W.inter + i) * H, gu[j][1]);
                pk_row_dma(W.s_dT + (long)i * H, rr + (wave * SLOTS + j) * R_ROW);
                swt[j] = 1.f;
            }
        }
#pragma unroll
        for (int j = 1; j < SLOTS; ++j)
            if (slot_ok(j)) slot_h(j);
        pk_wait_all();  // every down row landed
#pragma unroll
        for (int j = 0; j < SLOTS; ++j)
            if (slot_ok(j)) slot_down(j);
        // ======== the workgroup's partial of all 1280 outputs: 7 workers met in LDS, 5 rows per owner
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int cc = u * 64 + lane;
            if (cc < HC) {
                *reinterpret_cast<float4*>(ys + wave * H + (cc << 3)) = make_float4(yacc[u][0], yacc[u][1], yacc[u][2], yacc[u][3]);
                *reinterpret_cast<float4*>(ys + wave * H + (cc << 3) + 4) = make_float4(yacc[u][4], yacc[u][5], yacc[u][6], yacc[u][7]);
            }
        }
        pk_sync();  // #8: worker partials
        for (int j = tid; j < H; j += NT) {
            float v = ys[j];
#pragma unroll
            for (int w = 1; w < NWK; ++w) v += ys[w * H + j];
            xb[j] = v;
        }
        pk_sync();  // #9: the workgroup's partial; ys free
        // this workgroup's partial of all 1280 outputs, contiguous (coalesced 16-byte write-through stores)
        for (int pp = tid; pp < H / 2; pp += NWK * 64) put2(gl + O_DP + (long)c * H + 2 * pp, xb[2 * pp], xb[2 * pp + 1]);
        // the next layer's q/k/v rows and K / V chunk stream during the reduction hand-off
        if (l + 1 < a.layers) issue_qkv_kv(l + 1);
    }
}

// ------------------------------------------------------------------ f16 transpose (load time)
// out[k][n] = in[n][k] for a [N][K] 16-bit matrix: the down projections as [inter][hidden] rows for the split-K
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* in, uint16_t* out, int N, int K) {
    __shared__ uint16_t t[64][66];
    const int n0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int n = n0 + r, k = k0 + tx;
        if (n < N && k < K) t[r][tx] = in[(long)n * K + k];
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int k = k0 + r, n = n0 + tx;
        if (n < N && k < K) out[(long)k * N + n] = t[tx][r];
    }
}

void launch_transpose16(const void* in, void* out, int N, int K, hipStream_t s) {
    const dim3 grid((K + 63) / 64, (N + 63) / 64);
    hipLaunchKernelGGL(transpose16_kernel, grid, dim3(256), 0, s, reinterpret_cast<const uint16_t*>(in),
                       reinterpret_cast<uint16_t*>(out), N, K);
}

bool dec_persist_shape_ok(int hidden, int heads, int kv_heads, int head_dim, int n_routed, int topk, int moe_inter,
                          int shared_inter, int dense_inter, int max_len) {
    return hidden == H && heads == NH && kv_heads == NH && head_dim == HD && n_routed == E && topk == TOPK &&
           moe_inter == I && shared_inter == IS && dense_inter > 0 && (dense_inter + G - 1) / G <= SLOTS * NWK &&
           max_len >= 1 && max_len <= CPH * CHMAX;
}

int dec_persist_resident() {
    static int ok = -1;
    if (ok < 0) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
        const size_t lds = dec_persist_lds_bytes();
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(dec_persist_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(dec_persist_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, dec_persist_kernel<false>, NT, lds) != hipSuccess)
            per = 0;
        (void)hipGetLastError();
        // every workgroup waits on others: all G must be resident at once (one per CU)
        ok = (per >= 1 && cus >= G) ? 1 : 0;
    }
    return ok;
}

void launch_dec_persist(const DecPersistArgs& a, hipStream_t s) {
    if (!dec_persist_resident()) throw std::runtime_error("EINVAL: dec_persist needs 256 resident workgroups");
    if (!a.lw || !a.g || !a.x || !a.kv_pos || !a.cos || !a.sin || !a.kc || !a.vc || a.layers <= 0)
        throw std::runtime_error("EINVAL: dec_persist arguments");
    if (a.stamps) DSOCR_LAUNCH((dec_persist_kernel<true>), dim3(G), dim3(NT), dec_persist_lds_bytes(), s, a);
    else DSOCR_LAUNCH((dec_persist_kernel<false>), dim3(G), dim3(NT), dec_persist_lds_bytes(), s, a);
}

}  // namespace dsocr
