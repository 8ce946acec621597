// Device-side helpers shared by the gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <hip/hip_ext.h>

#include "kernels.hpp"

// hipLaunchKernelGGL, or hipExtLaunchKernelGGL with the pending profiling events (prof_events())
#define DSOCR_LAUNCH(K, G, B, S, ST, ...)                                                             \
    do {                                                                                             \
        ::dsocr::ProfEvents& _pe = ::dsocr::prof_events();                                           \
        if (_pe.start) {                                                                             \
            const ::dsocr::ProfEvents _ev = _pe;                                                     \
            _pe = ::dsocr::ProfEvents();                                                             \
            hipExtLaunchKernelGGL(K, G, B, S, ST, _ev.start, _ev.stop, 0, __VA_ARGS__);              \
        } else {                                                                                     \
            hipLaunchKernelGGL(K, G, B, S, ST, __VA_ARGS__);                                         \
        }                                                                                            \
    } while (0)

namespace dsocr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte streaming load (weights read once per decode step: nontemporal, see
// MI355X_MICROARCH.md price list row nt-weights).
__device__ __forceinline__ uint4 ldg_nt16(const void* p) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// 16-byte streaming f32 load (the decode attention's K / V cache: read once per step)
__device__ __forceinline__ float4 ldg_nt_f4(const float* p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
}

// Weight element types: checkpoints are bf16; the decoder keeps the reference's
// `--dtype f16` rounding (fp16 storage).  Both widen exactly to f32.
struct bf16_t { uint16_t v; };
struct f16_t { uint16_t v; };

__device__ __forceinline__ float to_f32(bf16_t x) { return __uint_as_float((uint32_t)x.v << 16); }
__device__ __forceinline__ float to_f32(f16_t x) {
    _Float16 h;
    __builtin_memcpy(&h, &x.v, 2);
    return (float)h;
}
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t bits16) { return __uint_as_float(bits16 << 16); }
__device__ __forceinline__ float f16_bits_to_f32(uint32_t bits16) {
    uint16_t b = (uint16_t)bits16;
    _Float16 h;
    __builtin_memcpy(&h, &b, 2);
    return (float)h;
}

template <typename WT>
__device__ __forceinline__ float wbits_to_f32(uint32_t bits16);
template <>
__device__ __forceinline__ float wbits_to_f32<bf16_t>(uint32_t b) { return bf16_bits_to_f32(b & 0xffffu); }
template <>
__device__ __forceinline__ float wbits_to_f32<f16_t>(uint32_t b) { return f16_bits_to_f32(b & 0xffffu); }

// Unpack 8 packed 16-bit weights (one 16-byte load) to f32.
template <typename WT>
__device__ __forceinline__ void unpack8(const uint4 q, float* o) {
    o[0] = wbits_to_f32<WT>(q.x); o[1] = wbits_to_f32<WT>(q.x >> 16);
    o[2] = wbits_to_f32<WT>(q.y); o[3] = wbits_to_f32<WT>(q.y >> 16);
    o[4] = wbits_to_f32<WT>(q.z); o[5] = wbits_to_f32<WT>(q.z >> 16);
    o[6] = wbits_to_f32<WT>(q.w); o[7] = wbits_to_f32<WT>(q.w >> 16);
}

// Wave64 reductions on DPP row operations (a few cycles each) instead of __shfl_xor, which
// lowers to ds_bpermute (an LDS-crossbar round trip, ~120 cycles) — a 6-step butterfly of
// those dominated the small decode kernels.  Pattern: quad xor 1, quad xor 2, row half
// mirror, row mirror (every lane of a 16-lane row now holds the row total), then
// row_bcast15 / row_bcast31 fold the rows into lane 63, which is broadcast.  Requires all
// 64 lanes active (every call site is in wave-uniform control flow).
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dpp_f(float old, float src) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, ROWMASK, 0xf, false));
}
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ int dpp_i(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, CTRL, ROWMASK, 0xf, false);
}
constexpr int DPP_QUAD_XOR1 = 0xB1, DPP_QUAD_XOR2 = 0x4E, DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_MIRROR = 0x140,
              DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143;

__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<DPP_QUAD_XOR1>(0.f, v);
    v += dpp_f<DPP_QUAD_XOR2>(0.f, v);
    v += dpp_f<DPP_ROW_HALF_MIRROR>(0.f, v);
    v += dpp_f<DPP_ROW_MIRROR>(0.f, v);
    v += dpp_f<DPP_ROW_BCAST15, 0xA>(0.f, v);
    v += dpp_f<DPP_ROW_BCAST31, 0xC>(0.f, v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f<DPP_QUAD_XOR1>(-INFINITY, v));
    v = fmaxf(v, dpp_f<DPP_QUAD_XOR2>(-INFINITY, v));
    v = fmaxf(v, dpp_f<DPP_ROW_HALF_MIRROR>(-INFINITY, v));
    v = fmaxf(v, dpp_f<DPP_ROW_MIRROR>(-INFINITY, v));
    v = fmaxf(v, dpp_f<DPP_ROW_BCAST15, 0xA>(-INFINITY, v));
    v = fmaxf(v, dpp_f<DPP_ROW_BCAST31, 0xC>(-INFINITY, v));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// (value, index) argmax over the wave, ties -> lower index; result broadcast to all lanes
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ void argmax_step(float& bv, int& bi) {
    const float ov = dpp_f<CTRL, ROWMASK>(-INFINITY, bv);
    const int oi = dpp_i<CTRL, ROWMASK>(0x7fffffff, bi);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
}
__device__ __forceinline__ void wave_argmax(float& bv, int& bi) {
    argmax_step<DPP_QUAD_XOR1>(bv, bi);
    argmax_step<DPP_QUAD_XOR2>(bv, bi);
    argmax_step<DPP_ROW_HALF_MIRROR>(bv, bi);
    argmax_step<DPP_ROW_MIRROR>(bv, bi);
    argmax_step<DPP_ROW_BCAST15, 0xA>(bv, bi);
    argmax_step<DPP_ROW_BCAST31, 0xC>(bv, bi);
    bv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv), 63));
    bi = __builtin_amdgcn_readlane(bi, 63);
}
// sum over the 4 lanes of a quad (lanes 4q .. 4q+3), result in every lane of the quad
__device__ __forceinline__ float quad_sum(float v) {
    v += dpp_f<DPP_QUAD_XOR1>(0.f, v);
    v += dpp_f<DPP_QUAD_XOR2>(0.f, v);
    return v;
}

// Activation epilogues (reference: candle gelu_erf, quick_gelu clip.rs:413-416, silu).

__device__ __forceinline__ float apply_act(float x, int act) {
    switch (act) {
        case ACT_GELU_ERF: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
        case ACT_QUICK_GELU: return (1.0f / (1.0f + expf(-(1.702f * x)))) * x;
        case ACT_SILU: return x / (1.0f + expf(-x));
        default: return x;
    }
}

// In-context launch spans (Engine::set_spans, off by default): a kernel whose args carry a slot
// array opens a WaveSpan first thing; every wave then writes (entry, exit) wall clock (s_memrealtime,
// 100 MHz) to its own slot, exit being the destructor, i.e. after the wave's last store is issued on
// whichever path it leaves by.  span_reduce_kernel (misc.hip), launched right after on the same
// stream, folds the slots to the launch's (first entry, last exit) and clears them.
struct WaveSpan {
    unsigned long long* s;
    unsigned long long t0 = 0;
    __device__ __forceinline__ explicit WaveSpan(unsigned long long* slots) : s(slots) {
        if (s) t0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ ~WaveSpan() {
        if (!s) return;
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const long gw = ((long)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) +
                        (threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0 && gw < SPAN_SLOTS) {
            s[2 * gw] = t0;
            s[2 * gw + 1] = t1;
        }
    }
};

// order-preserving float <-> unsigned key (atomicMax over floats); key 0 sorts below every
// float and decodes to -inf
__device__ __forceinline__ unsigned fkey(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_dec(unsigned k) {
    if (k == 0u) return -INFINITY;
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Rank of the lane's score among the wave's 64, descending, ties -> lower lane: #{j : s_j > s_e or (s_j == s_e and
// j < e)}.  Each score becomes a 64-bit key (order-preserving score bits, then 63 - lane), so the rank is a count of
// keys above the lane's own: one 64-bit vector compare and one carry-add per key, from a 64-key LDS copy (32
// broadcast 16-byte reads).  The float-compare form (a > b || (a == b && j < e)) compiles to scalar mask
// arithmetic between vector compares and measured 1.9 us per call on gfx950 (tools/mb_topk.hip).  Same order for
// the scores top-k sees (no NaN; -inf pads lanes >= E; +0 only).  lds: 128 floats (64 keys) private to the wave.
template <bool LOWREG = false>
__device__ __forceinline__ int wave_rank64(float sc, float* lds) {
    const int lane = threadIdx.x & 63;
    const unsigned long long key = ((unsigned long long)fkey(sc) << 32) | (unsigned)(63 - lane);
    unsigned long long* kl = reinterpret_cast<unsigned long long*>(lds);
    kl[lane] = key;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    int r0 = 0, r1 = 0;
    if constexpr (LOWREG) {
        // four passes of 16 keys (32 VGPRs of keys in flight, not 128: for callers that keep a token row live)
#pragma unroll 1
        for (int g = 0; g < 4; ++g) {
#pragma unroll
            for (int j2 = 0; j2 < 8; ++j2) {
                const ulonglong2 o = reinterpret_cast<const ulonglong2*>(kl)[8 * g + j2];
                r0 += o.x > key ? 1 : 0;
                r1 += o.y > key ? 1 : 0;
            }
        }
    } else {
#pragma unroll
        for (int j2 = 0; j2 < 32; ++j2) {
            const ulonglong2 o = reinterpret_cast<const ulonglong2*>(kl)[j2];
            r0 += o.x > key ? 1 : 0;
            r1 += o.y > key ? 1 : 0;
        }
    }
    return r0 + r1;
}

// Greedy top-k of one token by one wave, lane e holding expert e's logit (E <= 64): the picks of
// topk_write (softmax / sigmoid scores, descending, ties -> lower expert id, weights summed in
// pick order, optional renormalise + scaling), by rank (wave_rank64).  lds: 128 floats private to the wave.  Lane 0
// writes ids[k], w[k].
__device__ __forceinline__ void topk_wave64(float logit, int E, int K, int softmax_scoring, int norm_topk, float scaling,
                                            float* lds, int* ids, float* w) {
    const int lane = threadIdx.x & 63;
    float sc;
    if (softmax_scoring) {
        const float v = lane < E ? logit : -INFINITY;
        const float mx = wave_max(v);
        const float ex = lane < E ? expf(v - mx) : 0.f;
        const float sum = wave_sum(ex);
        sc = lane < E ? ex / sum : -INFINITY;
    } else {
        sc = lane < E ? 1.0f / (1.0f + expf(-logit)) : -INFINITY;
    }
    int rank = wave_rank64(sc, lds);
    if (lane >= E) rank = 1 << 20;
    float wsum = 0.f;
    int pe[8];
    float pv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        pe[k] = 0;
        pv[k] = 0.f;
        if (k < K) {
            const unsigned long long bm = __ballot(rank == k);
            pe[k] = __builtin_ctzll(bm);
            pv[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), pe[k]));
            wsum += pv[k];
        }
    }
    if (lane < K) {
        float v = pv[0];
        int e = pe[0];
#pragma unroll
        for (int k = 1; k < 8; ++k)
            if (lane == k) { v = pv[k]; e = pe[k]; }
        if (K > 1 && norm_topk) v = v / (wsum + 1e-20f);
        if (scaling != 1.0f) v = v * scaling;
        ids[lane] = e;
        w[lane] = v;
    }
}

// The expert records of one step's picks (MOE_GRP_* layout, kernels.hpp) on one wave: lane e collects the tokens
// that picked expert e (a token's picks are distinct, so at most one per token) in increasing token order; record
// s = the number of picked experts below e.  ids / w: token t's picks at P t + k, P = PITCH (0: topk), T <= 8,
// P t + k < 64.  Scatter, not search: lane P t + k ORs bit t into its expert's token mask and notes k (LDS, tmp:
// 576 ints private to the wave), then lane e reads its mask and its 8 slots back — a few dozen instructions where
// comparing every lane with all 64 picks costs ~200 (measured 1.5 us, tools/mb_topk.hip).  grp[0] = record count.
template <int PITCH>
__device__ __forceinline__ void group_picks_wave64(const int* ids, const float* w, int T, int K, int E, int* grp,
                                                   int* tmp) {
    const int lane = threadIdx.x & 63;
    const int P = PITCH ? PITCH : K;
    int* tok = tmp;       // [64 experts] token bit masks
    int* kof = tmp + 64;  // [64 experts][8 tokens] the pick's k
    tok[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int t = lane / P, k = lane - t * P;
    const int v = ids[lane];
    if (t < T && k < K && v >= 0 && v < 64) {
        __hip_atomic_fetch_or(tok + v, 1 << t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        kof[v * 8 + t] = k;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int msk = tok[lane];
    const int4 ka = reinterpret_cast<const int4*>(kof + lane * 8)[0], kb = reinterpret_cast<const int4*>(kof + lane * 8)[1];
    const int kk[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
    float hw[8];  // read for every token (stale slots clamped in range), used for the hits only
#pragma unroll
    for (int u = 0; u < 8; ++u) hw[u] = w[min(P * u + (kk[u] & 7), 63)];
    const int cnt = __popc(msk);
    const bool act = cnt > 0 && lane < E;
    const unsigned long long bm = __ballot(act);
    const int sidx = __popcll(bm & ((1ull << lane) - 1ull));
    if (act) {
        int* rec = grp + MOE_GRP_REC * (1 + sidx);
        rec[0] = lane;
        rec[1] = cnt;
        int q = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if ((msk >> u) & 1) {
                rec[2 + q] = u * K + kk[u];
                rec[10 + q] = __float_as_int(hw[u]);
                ++q;
            }
    }
    if (lane == 0) grp[0] = __popcll(bm);
}


}  // namespace dsocr
