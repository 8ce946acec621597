// Multi-token decode projections on the matrix cores (3..8 pages decoding together: BASELINE
// configs[2], 8 pages per GPU).  The reference computes every projection as an f32 matmul of f32
// activations with the model's 16-bit weights widened to f32 (transformer/block.rs attention / MLP
// linears at seq_len 1 per page); here the 16-bit weight rows go straight from HBM into
// v_mfma_f32_16x16x32_{f16,bf16} as the A operand (16 output rows x 32 k per step), and the f32
// activation rows become the B operand as three 16-bit planes x = p0 + p1 + p2:
//   * bf16 weights: three bf16 planes represent every f32 exactly (8 + 8 + 8 significand bits);
//   * f16 weights: each token row is first scaled by a power of two 2^s that puts its largest
//     magnitude in [2^14, 2^15) (exact), then split into three f16 planes; the split leaves an
//     absolute error below 2^-25 in scaled units (f16's subnormal half-step), i.e. 2^-39 of the row
//     maximum — far below the f32 rounding of the dot product itself — and the result is scaled back
//     by 2^-s (exact).
// Every product is then exact in the f32 accumulator (16-bit x 16-bit significands) and only the
// summation order differs from an f32 matmul.  The VALU does no per-weight work at all (the decode
// GEMV spent a convert and M FMAs per weight plus one wave reduction per output), so the launch is
// bound by the weight stream.
//
// Fragment maps (cdna_hip_programming.md §3, gfx950 16x16x32): lane l holds A[row l&15][k 8(l>>4)+j]
// and B[k 8(l>>4)+j][col l&15], j < 8; C[row 4(l>>4)+i][col l&15], i < 4.  Columns are tokens
// (8 staged; lanes of columns 8..15 read the rows of columns 0..7 and their results are dropped).
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

typedef _Float16 mm_f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 mm_b16x8 __attribute__((ext_vector_type(8)));

constexpr int MM_MT = 8;  // token rows staged (M <= 8)

template <typename WT>
struct MmT;
template <>
struct MmT<f16_t> {
    typedef mm_f16x8 frag;
    static constexpr bool scaled = true;
    __device__ static uint16_t to_bits(float v, float& back) {
        const _Float16 h = (_Float16)v;
        back = (float)h;
        uint16_t b;
        __builtin_memcpy(&b, &h, 2);
        return b;
    }
    __device__ static f32x4 mfma(const frag& a, const frag& b, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};
template <>
struct MmT<bf16_t> {
    typedef mm_b16x8 frag;
    static constexpr bool scaled = false;
    __device__ static uint16_t to_bits(float v, float& back) {
        const __bf16 h = (__bf16)v;
        back = (float)h;
        uint16_t b;
        __builtin_memcpy(&b, &h, 2);
        return b;
    }
    __device__ static f32x4 mfma(const frag& a, const frag& b, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};

// LDS row pitch of a plane row (16-bit elements): K + 16 puts consecutive rows 8 banks apart, which
// makes the B-operand ds_read_b128 (rows l&7, k groups l>>4) conflict-free.
__host__ __device__ inline int mm_pitch(int K) { return K + 16; }

// Wave-level staging of token row m of x (f32, K <= 1536) as 3 planes in LDS (xp[(p * MT + m) * KP +
// k]) with its inverse scale scl[m], in two halves so that the row's loads can be issued BEFORE the
// weight stream (vmcnt retires in issue order: loads issued after a weight batch wait for it).
// NORM: RMS-normalised first — the lane's chunks (lane, lane+64, lane+128; 8 floats each) squared and
// summed u-major then j, one wave sum, x * (1 / den) * w.
template <int U>
struct MmRowU {
    float v[U][8];
    float w[U][8];
};
typedef MmRowU<3> MmRow;  // K <= 1536

template <bool NORM, int U = 3>
__device__ __forceinline__ void mm_row_load(MmRowU<U>& r, const float* xr, int K, const float* nw) {
    const int lane = threadIdx.x & 63;
    const int chunks = K >> 3;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int cc = min(u * 64 + lane, chunks - 1);
        const float4 lo = *reinterpret_cast<const float4*>(xr + (cc << 3));
        const float4 hi = *reinterpret_cast<const float4*>(xr + (cc << 3) + 4);
        r.v[u][0] = lo.x; r.v[u][1] = lo.y; r.v[u][2] = lo.z; r.v[u][3] = lo.w;
        r.v[u][4] = hi.x; r.v[u][5] = hi.y; r.v[u][6] = hi.z; r.v[u][7] = hi.w;
        if (NORM) {
            const float4 wl = *reinterpret_cast<const float4*>(nw + (cc << 3));
            const float4 wh = *reinterpret_cast<const float4*>(nw + (cc << 3) + 4);
            r.w[u][0] = wl.x; r.w[u][1] = wl.y; r.w[u][2] = wl.z; r.w[u][3] = wl.w;
            r.w[u][4] = wh.x; r.w[u][5] = wh.y; r.w[u][6] = wh.z; r.w[u][7] = wh.w;
        }
    }
}

template <typename WT, bool NORM, int U = 3, bool DIVNORM = false>
__device__ __forceinline__ void mm_row_store(MmRowU<U>& r, int K, float eps, uint16_t* xp, int KP, float* scl, int m) {
    const int lane = threadIdx.x & 63;
    const int chunks = K >> 3;
    if (NORM) {
        float q = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u * 64 + lane < chunks)
#pragma unroll
                for (int j = 0; j < 8; ++j) q += r.v[u][j] * r.v[u][j];
        // one division per row: x * (1 / den) is within an ulp of the reference's x / den (the planes
        // below are exact, the GEMM sums in its own order: this path is tolerance-pinned, not bitwise)
        if (DIVNORM) {  // x / den * w: dec_route_grp's (and the reference's) form, bit for bit
            const float den = sqrtf(wave_sum(q) / (float)K + eps);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) r.v[u][j] = (r.v[u][j] / den) * r.w[u][j];
        } else {
            const float inv = 1.0f / sqrtf(wave_sum(q) / (float)K + eps);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) r.v[u][j] = (r.v[u][j] * inv) * r.w[u][j];
        }
    }
    float s_inv = 1.f;
    if (MmT<WT>::scaled) {
        float mx = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u * 64 + lane < chunks)
#pragma unroll
                for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(r.v[u][j]));
        mx = wave_max(mx);
        int s = 0;
        if (mx > 0.f) {
            int e;
            (void)frexpf(mx, &e);  // mx < 2^e
            s = 15 - e;            // mx * 2^s < 2^15
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) r.v[u][j] = ldexpf(r.v[u][j], s);
        s_inv = ldexpf(1.f, -s);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
        if (c < chunks) {
            uint16_t pb[3][8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float b0, b1, b2;
                pb[0][j] = MmT<WT>::to_bits(r.v[u][j], b0);
                const float r1 = r.v[u][j] - b0;
                pb[1][j] = MmT<WT>::to_bits(r1, b1);
                const float r2 = r1 - b1;
                pb[2][j] = MmT<WT>::to_bits(r2, b2);
            }
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                uint4 q;
                q.x = pb[p][0] | ((uint32_t)pb[p][1] << 16);
                q.y = pb[p][2] | ((uint32_t)pb[p][3] << 16);
                q.z = pb[p][4] | ((uint32_t)pb[p][5] << 16);
                q.w = pb[p][6] | ((uint32_t)pb[p][7] << 16);
                *reinterpret_cast<uint4*>(xp + ((long)(p * MM_MT + m) * KP + (c << 3))) = q;
            }
        }
    }
    if (lane == 0) scl[m] = s_inv;
}

// Y[m][n] (+)= act((norm?(X) . W^T)[m][n] * 1 + bias[n]) for m < M <= 8.  Block: WR x WK waves —
// WR 16-row tiles side by side, each tile's K split in WK contiguous ranges whose partial tiles meet
// once in LDS (summed in range order).  The block stages the planes once, then walks row tiles
// blockIdx.x, blockIdx.x + gridDim.x, ... (a persistent grid for the lm_head).  A fragments are
// 16-byte nontemporal loads straight into registers, PF k-steps per batch, double-buffered.
template <typename WT, int WR, int WK, int PF, int Q, bool NORM, bool SWZ>
__global__ __launch_bounds__(64 * WR * WK) void dec_mm_kernel(DecGemvArgs a) {
    WaveSpan span_(a.span);
    typedef typename MmT<WT>::frag frag;
    static_assert(PF % Q == 0, "a batch holds whole k groups");
    // k order inside each group of Q steps: step Q T + s gives lane group g the 8 k's
    // 32 Q T + 8 Q g + 8 s + j, so a lane's Q fragments of a group are 16 Q contiguous bytes of its row
    auto koff = [](int i) { return 32 * Q * (i / Q) + 8 * (i % Q); };
    extern __shared__ __attribute__((aligned(16))) uint16_t xp[];  // [3][MT][KP]
    __shared__ float scl[MM_MT];
    __shared__ f32x4 red[WK > 1 ? WK - 1 : 1][WR][64];
    __shared__ float res_s[WR == 1 ? MM_MT : 1][16];  // one tile per block: its residual rows, loaded up front
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int KP = mm_pitch(a.K);
    constexpr int NW = WR * WK;
    const int wr = wave % WR, wk = wave / WR;
    const int steps = a.K >> 5, per = steps / WK, t0 = wk * per;
    const int nch = per / PF;  // host guarantees per % PF == 0 (and an even nch for several tiles per block)
    const int ntiles = (a.N + 15) >> 4;
    const int col = lane & 15, g = lane >> 4;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    auto rowp = [&](int bt) {
        if (SWZ) {  // fragment-ordered copy: [tile][step][lane][8], one 1 KiB block per wave load
            const int tile = min(bt * WR + wr, ntiles - 1);
            return W + ((long)tile * steps + t0) * 512 + lane * 8;
        }
        const int n = min((bt * WR + wr) * 16 + col, a.N - 1);
        return W + (long)n * a.ldw + 8 * Q * g + 32 * t0;
    };
    frag fa[PF], fb[PF];
    auto load = [&](frag(&f)[PF], const WT* wrow, int c) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const uint4 q = ldg_nt16(SWZ ? wrow + (long)(c * PF + i) * 512 : wrow + 32 * c * PF + koff(i));
            __builtin_memcpy(&f[i], &q, 16);
        }
    };
    // this wave's activation rows are loaded first, then the first weight batch goes out, then the rows
    // are normalised / split into the LDS planes while the weights are in flight
    static_assert(NW >= 4, "staging: at most two rows per wave");
    MmRow r0, r1;
    const int m0 = wave, m1 = wave + NW;
    if (m0 < a.M) mm_row_load<NORM>(r0, a.x + (long)m0 * a.ldx, a.K, a.norm_w);
    if (NW < MM_MT && m1 < a.M) mm_row_load<NORM>(r1, a.x + (long)m1 * a.ldx, a.K, a.norm_w);
    int bt = blockIdx.x;
    const WT* cur = rowp(bt);
    // the residual rows of the block's one tile (WR == 1), with the first loads: the staging barrier waits
    // for them together, and the epilogue reads LDS instead of a dependent global round trip (8 text pages:
    // decode 638.8-639.2 -> 636.2-636.5 ms, `profiles/r04_bench8t_mm_respre{0,1}*.log`; held in LDS, not
    // registers: the register version cost occupancy)
    float rv = 0.f;
    if (WR == 1 && a.accumulate && tid < 16 * MM_MT && (tid >> 4) < a.M)
        rv = a.y[(long)(tid >> 4) * a.ldy + min(bt * 16 + (tid & 15), a.N - 1)];
    load(fa, cur, 0);
    if (m0 < a.M) mm_row_store<WT, NORM>(r0, a.K, a.eps, xp, KP, scl, m0);
    if (NW < MM_MT && m1 < a.M) mm_row_store<WT, NORM>(r1, a.K, a.eps, xp, KP, scl, m1);
    if (WR == 1 && a.accumulate && tid < 16 * MM_MT) res_s[WR == 1 ? tid >> 4 : 0][tid & 15] = rv;
    __syncthreads();
    const uint16_t* bbase = xp + (long)(col & 7) * KP + 8 * Q * g;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const frag(&f)[PF], int c) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int k = 32 * (t0 + c * PF) + koff(i);
#pragma unroll
            for (int p = 2; p >= 0; --p) {
                const frag b = *reinterpret_cast<const frag*>(bbase + (long)p * MM_MT * KP + k);
                acc = MmT<WT>::mfma(f[i], b, acc);
            }
        }
    };
    auto finish = [&](int btile) {
        const int tile = btile * WR + wr;
        if (WK > 1) {
            if (wk > 0) red[wk - 1][wr][lane] = acc;
            __syncthreads();
            if (wk == 0) {
#pragma unroll
                for (int q = 0; q < WK - 1; ++q) {
                    const f32x4 o = red[q][wr][lane];
                    acc[0] += o[0]; acc[1] += o[1]; acc[2] += o[2]; acc[3] += o[3];
                }
            }
            __syncthreads();  // red reused by the next tile
        }
        if (wk == 0 && col < a.M && tile < ntiles) {
            const float s = scl[col];
            float* yr = a.y + (long)col * a.ldy;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int nn = tile * 16 + 4 * g + i;
                if (nn < a.N) {
                    float v = apply_act(acc[i] * s + (a.bias ? a.bias[nn] : 0.f), a.act);
                    if (a.accumulate) v = (WR == 1 ? res_s[WR == 1 ? col : 0][4 * g + i] : yr[nn]) + v;
                    yr[nn] = v;
                }
            }
        }
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    // one stream over (tile, chunk): the next batch (the next chunk, or the next tile's first) is
    // always in flight while the current one is consumed
    for (;;) {
        const int nbt = bt + gridDim.x;
        const bool more = nbt * WR < ntiles;
        const WT* nxt = more ? rowp(nbt) : cur;
        for (int c = 0; c < nch; c += 2) {
            if (c + 1 < nch) load(fb, cur, c + 1);
            else if (more) load(fb, nxt, 0);
            compute(fa, c);
            if (c + 1 >= nch) break;
            if (c + 2 < nch) load(fa, cur, c + 2);
            else if (more) load(fa, nxt, 0);
            compute(fb, c + 1);
        }
        finish(bt);
        if (!more) break;
        bt = nbt;
        cur = nxt;
        if (nch & 1) {  // odd batch count: the next tile's first batch landed in fb
#pragma unroll
            for (int i = 0; i < PF; ++i) fa[i] = fb[i];
        }
    }
}

bool dec_mm_ok(const DecGemvArgs& a) {
    return a.M >= 1 && a.M <= MM_MT && a.K % 32 == 0 && a.K <= 1536 && (a.K >> 5) % 40 == 0 && a.N >= 16 &&
           !a.xn_out && a.ldw >= a.K && a.ldw % 8 == 0;
}

static int mm_resident_blocks(const void* kernel, int threads, size_t lds) {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(1, per_cu) * std::max(1, cus);
}

template <typename WT, int WR, int WK, int PF, int Q, bool NORM, bool SWZ = false>
static void mm_launch(const DecGemvArgs& a, hipStream_t s) {
    const size_t lds = sizeof(uint16_t) * 3 * MM_MT * (size_t)mm_pitch(a.K);
    const int ntiles = (a.N + 15) / 16;
    int blocks = (ntiles + WR - 1) / WR;
    if (WR > 1) {  // persistent: at most one resident round
        static int resident = 0;
        if (!resident) resident = mm_resident_blocks((const void*)dec_mm_kernel<WT, WR, WK, PF, Q, NORM, SWZ>, 64 * WR * WK, lds);
        blocks = std::min(blocks, resident);
    }
    DSOCR_LAUNCH((dec_mm_kernel<WT, WR, WK, PF, Q, NORM, SWZ>), dim3(blocks), dim3(64 * WR * WK), lds, s, a);
}

// block shapes (K steps of 32 a multiple of 40: per-wave batches divide evenly): WR 8 persistent for the
// large-N head, WK 8 (K split over 8 waves) otherwise (measured: WK 4, WR 4 persistent and a k-permuted A
// fragment order were slower)
template <typename WT, bool NORM>
static void mm_dispatch(const DecGemvArgs& a, hipStream_t s) {
    if (a.w_swz) {  // fragment-ordered weights (3..8 pages: the lm_head's copy, q/k/v, o_proj, dense gate|up)
        DecGemvArgs b = a;
        b.W = a.w_swz;
        if (a.N >= 16384) mm_launch<WT, 8, 1, 10, 1, NORM, true>(b, s);
        else mm_launch<WT, 1, 8, 5, 1, NORM, true>(b, s);
        return;
    }
    if (a.N >= 16384) mm_launch<WT, 8, 1, 10, 1, NORM>(a, s);
    else mm_launch<WT, 1, 8, 5, 1, NORM>(a, s);
}

// W [N][K] row-major -> fragment order [N/16 tiles][K/32 steps][64 lanes][8]: lane l of step t of tile
// T holds W[16 T + (l & 15)][32 t + 8 (l >> 4) .. + 7] (rows past N repeat row N-1)
__global__ void mm_swizzle_kernel(const uint16_t* w, int N, int K, uint16_t* out) {
    const int steps = K >> 5;
    const long total = (long)((N + 15) >> 4) * steps * 64;
    for (long f = blockIdx.x * (long)blockDim.x + threadIdx.x; f < total; f += (long)gridDim.x * blockDim.x) {
        const int lane = (int)(f & 63);
        const long ts = f >> 6;
        const int t = (int)(ts % steps);
        const long tile = ts / steps;
        const int n = (int)std::min<long>(tile * 16 + (lane & 15), N - 1);
        const uint4 q = *reinterpret_cast<const uint4*>(w + (long)n * K + 32 * t + 8 * (lane >> 4));
        *reinterpret_cast<uint4*>(out + f * 8) = q;
    }
}

size_t mm_swizzle_elems(int N, int K) { return (size_t)((N + 15) / 16) * 16 * (size_t)K; }

void launch_mm_swizzle(const void* w, int N, int K, void* out, hipStream_t s) {
    if (K % 32) throw std::runtime_error("EINVAL: mm_swizzle needs K % 32 == 0");
    hipLaunchKernelGGL(mm_swizzle_kernel, dim3(2048), dim3(256), 0, s, (const uint16_t*)w, N, K, (uint16_t*)out);
}

void launch_dec_mm(const DecGemvArgs& a, hipStream_t s) {
    if (!dec_mm_ok(a)) throw std::runtime_error("EINVAL: dec_mm outside its range");
    if (a.wdtype == WDT_BF16) {
        if (a.norm_w) mm_dispatch<bf16_t, true>(a, s); else mm_dispatch<bf16_t, false>(a, s);
    } else {
        if (a.norm_w) mm_dispatch<f16_t, true>(a, s); else mm_dispatch<f16_t, false>(a, s);
    }
}

// ------------------------------------------------------------------ grouped decode MoE gate/up (3..8 tokens)
// Work units of 16 intermediate rows: the shared expert's Is/16 units first, then (record s, tile t)
// for the router's records (MOE_GRP_*: each distinct routed expert once, with its tokens).  A unit is
// the 16 gate rows and the 16 up rows over the full K, streamed as MFMA A fragments (PF k-steps of
// both per batch, double-buffered, the next unit's first batch in flight behind the current one's
// last); the 8 normalised token rows (xn) are the B operand as three f16 planes staged once per
// block.  KS waves share a unit, each streaming K / KS of it (more, shorter streams: one wave per
// 80 KB unit left CUs idle at 16 experts and drew 5.1 TB/s at 32, `tools/mb_units.hip`); the pieces
// meet in LDS, summed in piece order by the unit's first wave, which runs the epilogue.  The waves of
// a unit hand over through two LDS counters (pieces posted, pieces consumed) instead of a block
// barrier: a barrier would wait for the next unit's loads already in flight.  Persistent grid
// (resident blocks only): block b takes units b NU + w / KS, then + grid NU, ... (NU = 8 / KS).
// Epilogue per (row, token): g, u scaled back, h = silu(g) * u (candle silu: x / (1 + exp(-x))),
// times the pick's routing weight for routed experts, to h[slot row] (slot = t * topk + k) or hs[t];
// tokens outside a record are computed (a 16-column tile costs the same) and dropped.
__device__ __forceinline__ int lds_load_relaxed(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <typename WT, int PF, bool SWZ, int KS, bool ROUTE>
__global__ __launch_bounds__(512, 2) void moe_gateup_mm_kernel(MoeDec2Args a) {
    WaveSpan span_(a.span);
    typedef typename MmT<WT>::frag frag;
    constexpr int NWV = 8, NU = NWV / KS;
    static_assert(NWV % KS == 0, "whole units per block");
    constexpr int GREC = 65 * MOE_GRP_REC;  // the layer's expert records (count + <= 64 records) kept in LDS
    extern __shared__ __attribute__((aligned(16))) uint16_t xp[];  // [3][MT][KP]
    __shared__ float scl[MM_MT];
    // pieces 1.. of each unit (gate, up partial tiles) at [us * (KS - 1) + piece - 1]; ROUTE: the prologue's router
    // k-half partials [4][64] f32x4, logits [8][64] and rank scratch [8][64] share the same LDS
    constexpr int RED = NU * (KS - 1) * 2 * 64 * 4;
    constexpr int SCR = ROUTE ? (RED > 2048 ? RED : 2048) : (RED > 4 ? RED : 4);
    __shared__ __attribute__((aligned(16))) float scr[SCR];
    f32x4(*red)[2][64] = reinterpret_cast<f32x4(*)[2][64]>(scr);
    __shared__ int hand[2 * NU];  // [us]: pieces posted, [NU + us]: units consumed
    // Every record word the unit loop reads comes from LDS (ds_read: lgkmcnt).  A global load there would be
    // waited on with vmcnt, i.e. behind every weight load in flight (the double-buffered stream drained at each
    // unit: measured in the round-4 kernel's ISA, `s_waitcnt vmcnt(0)` after each record load).
    __shared__ __attribute__((aligned(16))) int grp_s[GREC];
    __shared__ __attribute__((aligned(16))) int ids_s[ROUTE ? 64 : 4];
    __shared__ float w_s[ROUTE ? 64 : 1];  // ROUTE: [8 tokens][8 picks], like ids_s
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the hand-off branches are scalar
    const int col = lane & 15, g = lane >> 4;
    const int piece = wave % KS, us = wave / KS;
    const int tiles_r = a.I >> 4, tiles_s = a.sWgu ? a.Is >> 4 : 0;
    const int steps = a.K >> 5, nch = steps / PF, nb = nch / KS, c0 = piece * nb;
    const int stride = gridDim.x * NU;
    const int KP = mm_pitch(a.K);
    const uint16_t* bbase = xp + (long)(col & 7) * KP + 8 * g;
    // phase clocks kept in LDS and written out at the end (a global store before a barrier would make the barrier
    // wait for its acknowledgement and stretch the phase it measures)
    __shared__ unsigned long long st_s[8];
#define GU_STAMP(i) \
    if (a.stamps && tid == 0) st_s[i] = __builtin_amdgcn_s_memrealtime();
    GU_STAMP(0);
    if constexpr (ROUTE) {
        // ---- the router of dec_route_grp, in every block: token row w normalised on wave w (x / den * w) and
        // staged as the B planes (the gate/up below uses the same rows); the 64 x K router matrix from L2 as MFMA
        // A fragments (wave w: rows 16 (w & 3) .., k-steps of half w >> 2), halves met in LDS; top-k per token
        // (topk_wave64) and the expert records (wave 0), so no router launch runs before this one
        constexpr int RB = 10;  // router k-steps per register batch (the router_ok range: two batches per half)
        const int half = steps >> 1, nrb = half / RB;
        const int tile = wave & 3, kh = wave >> 2;
        // row-major: lane (col, g) reads 64 bytes of 16 rows per load; the fragment-ordered copy (E % 16 == 0):
        // one contiguous 1 KiB per load, 20 KiB per wave (tools/mb_bcast.hip: 160 KiB into one CU in 1.4 vs
        // 3.8 us)
        const WT* R = a.router_swz
                          ? reinterpret_cast<const WT*>(a.router_swz) +
                                ((long)(min(tile, a.E / 16 - 1) * steps + kh * half) * 64 + lane) * 8  // E % 16 == 0 copy
                          : reinterpret_cast<const WT*>(a.router) + (long)min(16 * tile + col, a.E - 1) * a.K + 8 * g +
                                32L * kh * half;
        const long RS = a.router_swz ? 512 : 32;  // elements between a lane's consecutive k-steps
        frag ra[RB], rb[RB];
        auto rload = [&](frag(&f)[RB], int bi) {
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                const uint4 q = *reinterpret_cast<const uint4*>(R + RS * (bi * RB + i));
                __builtin_memcpy(&f[i], &q, 16);
            }
        };
        // both router batches go out first (L2-resident after the first blocks of an XCD touch them), then the
        // token rows; the staging barrier below waits for all of them, so the MFMAs run without a load wait
        rload(ra, 0);
        if (nrb > 1) rload(rb, 1);
        MmRow xr;
        if (wave < a.T) mm_row_load<true>(xr, a.x + (long)wave * a.K, a.K, a.norm_w);
        if (wave < a.T)
            mm_row_store<WT, true, 3, true>(xr, a.K, a.eps, xp, KP, scl, wave);
        if (KS > 1 && tid < 2 * NU) hand[tid] = 0;
        __syncthreads();
        GU_STAMP(1);
        f32x4 racc = {0.f, 0.f, 0.f, 0.f};
        auto rcompute = [&](const frag(&f)[RB], int bi) {
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                const int k = 32 * (kh * half + bi * RB + i);
#pragma unroll
                for (int p = 2; p >= 0; --p) {
                    const frag b = *reinterpret_cast<const frag*>(bbase + (long)p * MM_MT * KP + k);
                    racc = MmT<WT>::mfma(f[i], b, racc);
                }
            }
        };
        for (int bi = 0; bi < nrb; bi += 2) {
            rcompute(ra, bi);
            if (bi + 2 < nrb) rload(ra, bi + 2);
            if (bi + 1 >= nrb) break;
            rcompute(rb, bi + 1);
            if (bi + 3 < nrb) rload(rb, bi + 3);
        }
        GU_STAMP(2);
        f32x4* rpart = reinterpret_cast<f32x4*>(scr);  // [4 tiles][64 lanes]
        float* lg_s = scr + 1024;                       // [8 tokens][64 experts]
        float* rank_s = scr;                            // [8][128] (64-bit keys; the halves are read by then)
        if (kh == 1) rpart[tile * 64 + lane] = racc;
        __syncthreads();
        if (kh == 0) {
            const f32x4 o = rpart[tile * 64 + lane];
            const float sc = scl[col & 7];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int e = 16 * tile + 4 * g + i;
                if (col < a.T && e < a.E) lg_s[col * 64 + e] = (racc[i] + o[i]) * sc + (a.router_bias ? a.router_bias[e] : 0.f);
            }
        }
        __syncthreads();
        if (wave < a.T)
            topk_wave64(lg_s[wave * 64 + lane], a.E, a.topk, a.softmax_scoring, a.norm_topk, a.scaling, rank_s + wave * 128,
                        ids_s + wave * 8, w_s + wave * 8);  // token t's picks at 8 t ..
        __syncthreads();
        GU_STAMP(3);
        // wave 0, lane e: the tokens that picked expert e (a token's picks are distinct), in increasing token
        // order -> record sidx = number of picked experts below e (dec_route_grp's records); block 0 also writes
        // them, the picks and the logits to global memory (for the down launch and the tools), after its last
        // barrier
        if (wave == 0) group_picks_wave64<8>(ids_s, w_s, a.T, a.topk, a.E, grp_s, reinterpret_cast<int*>(rank_s));
        // block 0's logits copy (for the tools) read before the last prologue barrier: the unit loop's split-K
        // partials reuse this LDS (scr) without another barrier
        const float lg_copy = (blockIdx.x == 0 && (tid >> 6) < a.T) ? lg_s[(tid >> 6) * 64 + (tid & 63)] : 0.f;
        __syncthreads();
        GU_STAMP(4);
        if (blockIdx.x == 0) {
            const int TK = a.T * a.topk;
            if (tid < TK) {
                const int t = tid / a.topk, l = 8 * t + tid - t * a.topk;
                a.ids_out[tid] = ids_s[l];
                a.w_out[tid] = w_s[l];
            }
            if (a.logits && (tid >> 6) < a.T && (tid & 63) < a.E)
                const_cast<float*>(a.logits)[(tid >> 6) * a.E + (tid & 63)] = lg_copy;
            int* gg = const_cast<int*>(a.grp);
            const int nw = MOE_GRP_REC * (1 + grp_s[0]);
            for (int i = tid; i < nw; i += 512) gg[i] = grp_s[i];
        }
    }
    // ---- the records (ROUTE: in LDS already; else copied from the router's global records once, behind the
    // x loads and ahead of the weight stream) and the first unit's stream
    MmRow xr;  // non-ROUTE: wave w stages token row w: its loads go out before the weight batch
    if constexpr (!ROUTE) {
        if (wave < a.T) mm_row_load<false>(xr, a.x + (long)wave * a.K, a.K, nullptr);
        static_assert(GREC / 4 <= 2 * 512, "two int4 per thread cover the records");
        const int4* gsrc = reinterpret_cast<const int4*>(a.grp);
        const int n4 = min(GREC / 4, MOE_GRP_REC / 4 * (1 + min(min(a.E, a.slots), 64)));  // moe_grp_ints' records
        const int i0 = tid, i1 = tid + 512;
        int4 r0 = {0, 0, 0, 0}, r1 = {0, 0, 0, 0};
        if (i0 < n4) r0 = gsrc[i0];
        if (i1 < n4) r1 = gsrc[i1];
        if (i0 < n4) reinterpret_cast<int4*>(grp_s)[i0] = r0;
        if (i1 < n4) reinterpret_cast<int4*>(grp_s)[i1] = r1;
        if (KS > 1 && tid < 2 * NU) hand[tid] = 0;
        if (wave < a.T) mm_row_store<WT, false>(xr, a.K, 0.f, xp, KP, scl, wave);
        __syncthreads();
    }
    const int n_units = tiles_s + grp_s[0] * tiles_r;
    int unit = blockIdx.x * NU + us;
    // unit -> the lane's two fragment streams (gate, up), first row, record, shared?  Kept as plain variables
    // (a struct select between the current and the next unit went through scratch, i.e. through vmcnt)
    constexpr long FS = SWZ ? 512 : 32;  // elements between a lane's consecutive k-step fragments
    auto src = [&](int uu, const WT*& pg, const WT*& pu, int& i0, int& rs, int& sh) {
        sh = uu < tiles_s ? 1 : 0;
        int t = uu;
        rs = 0;
        if (!sh) {
            rs = (uu - tiles_s) / tiles_r;
            t = (uu - tiles_s) % tiles_r;
        }
        i0 = t * 16;
        const int rows_I = sh ? a.Is : a.I;
        const int e = sh ? 0 : grp_s[MOE_GRP_REC * (1 + rs)];
        if (SWZ) {
            const WT* base = sh ? reinterpret_cast<const WT*>(a.sWgu_swz) : reinterpret_cast<const WT*>(a.Wgu_swz);
            const long tg = (sh ? 0L : (long)e * (2 * a.I / 16)) + t;
            pg = base + (tg * steps) * 512 + lane * 8;
            pu = base + ((tg + rows_I / 16) * steps) * 512 + lane * 8;
        } else {
            const WT* Wg = sh ? reinterpret_cast<const WT*>(a.sWgu)
                              : reinterpret_cast<const WT*>(a.Wgu) + (long)e * 2 * a.I * a.K;
            pg = Wg + (long)(i0 + col) * a.K + 8 * g;
            pu = pg + (long)rows_I * a.K;
        }
    };
    frag ga[PF], ua[PF], gb[PF], ub[PF];
    auto load = [&](frag(&fg)[PF], frag(&fu)[PF], const WT* pg, const WT* pu, int c) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const uint4 q0 = ldg_nt16(pg + FS * (c * PF + i));
            const uint4 q1 = ldg_nt16(pu + FS * (c * PF + i));
            __builtin_memcpy(&fg[i], &q0, 16);
            __builtin_memcpy(&fu[i], &q1, 16);
        }
    };
    const WT *cpg, *cpu;
    int ci0, crs, csh;
    src(min(unit, max(n_units - 1, 0)), cpg, cpu, ci0, crs, csh);
    if (unit < n_units) {
        load(ga, ua, cpg, cpu, c0);
        if (nb > 1) load(gb, ub, cpg, cpu, c0 + 1);
    }
    f32x4 accg = {0.f, 0.f, 0.f, 0.f}, accu = {0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const frag(&fg)[PF], const frag(&fu)[PF], int c) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int k = 32 * (c * PF + i);
#pragma unroll
            for (int p = 2; p >= 0; --p) {
                const frag b = *reinterpret_cast<const frag*>(bbase + (long)p * MM_MT * KP + k);
                accg = MmT<WT>::mfma(fg[i], b, accg);
                accu = MmT<WT>::mfma(fu[i], b, accu);
            }
        }
    };
    bool first = true;
    GU_STAMP(5);
    for (int n = 0; unit < n_units; unit += stride, ++n) {
        const int nu = unit + stride;
        const bool more = nu < n_units;
        const WT *npg = cpg, *npu = cpu;
        int ni0 = ci0, nrs = crs, nsh = csh;
        if (more) src(nu, npg, npu, ni0, nrs, nsh);
        for (int c = 0; c < nb; c += 2) {
            if (c + 1 < nb) { if (!(first && c == 0)) load(gb, ub, cpg, cpu, c0 + c + 1); }
            else if (more) load(gb, ub, npg, npu, c0);
            compute(ga, ua, c0 + c);
            if (first && c == 0) GU_STAMP(6);
            if (c + 1 >= nb) break;
            if (c + 2 < nb) load(ga, ua, cpg, cpu, c0 + c + 2);
            else if (more) load(ga, ua, npg, npu, c0);
            compute(gb, ub, c0 + c + 1);
        }
        if (KS > 1) {
            if (piece > 0) {
                const int ri = us * (KS - 1) + piece - 1;
                // the unit's first wave has read this slot's previous partials (almost never waits)
                while (lds_load_relaxed(&hand[NU + us]) < n) __builtin_amdgcn_s_sleep(1);
                red[ri][0][lane] = accg;
                red[ri][1][lane] = accu;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the partials are in LDS before the count
                if (lane == 0) __hip_atomic_fetch_add(&hand[us], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                while (lds_load_relaxed(&hand[us]) < (n + 1) * (KS - 1)) __builtin_amdgcn_s_sleep(1);
                asm volatile("" ::: "memory");
#pragma unroll
                for (int q = 1; q < KS; ++q) {
                    const int ri = us * (KS - 1) + q - 1;
                    const f32x4 pg = red[ri][0][lane], pu = red[ri][1][lane];
                    accg[0] += pg[0]; accg[1] += pg[1]; accg[2] += pg[2]; accg[3] += pg[3];
                    accu[0] += pu[0]; accu[1] += pu[1]; accu[2] += pu[2]; accu[3] += pu[3];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before the slot is released
                if (lane == 0) __hip_atomic_fetch_add(&hand[NU + us], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (piece == 0) {
            // token col's slot row (routed: -1 when the token did not pick this expert) and weight
            int slot = -1;
            float wk = 1.f;
            if (csh) {
                slot = col < a.T ? col : -1;
            } else {
                const int rb = MOE_GRP_REC * (1 + crs);
                const int cnt = grp_s[rb + 1];
                for (int q = 0; q < cnt; ++q) {
                    const int r = grp_s[rb + 2 + q];
                    if (r / a.topk == col) { slot = r; wk = __int_as_float(grp_s[rb + 10 + q]); }
                }
            }
            if (slot >= 0) {
                const float sc = scl[col];
                float hv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float gs = accg[i] * sc, us_ = accu[i] * sc;
                    const float h = (gs / (1.0f + expf(-gs))) * us_;
                    hv[i] = csh ? h : h * wk;
                }
                float* dst = csh ? a.hs + (long)slot * a.Is : a.h + (long)slot * a.I;
                *reinterpret_cast<float4*>(dst + ci0 + 4 * g) = make_float4(hv[0], hv[1], hv[2], hv[3]);
            }
        }
        accg = f32x4{0.f, 0.f, 0.f, 0.f};
        accu = f32x4{0.f, 0.f, 0.f, 0.f};
        cpg = npg; cpu = npu; ci0 = ni0; crs = nrs; csh = nsh;
        if (nb & 1) {  // odd batch count: the next unit's first batch landed in the b buffers
#pragma unroll
            for (int i = 0; i < PF; ++i) { ga[i] = gb[i]; ua[i] = ub[i]; }
        }
        first = false;
    }
    GU_STAMP(7);
    if (a.stamps && tid == 0)
        for (int i = 0; i < 8; ++i) a.stamps[blockIdx.x * 8 + i] = (!ROUTE && i >= 1 && i <= 4) ? 0ull : st_s[i];
#undef GU_STAMP
}

// waves per unit: DSOCR_GU_KS = 1 / 2 / 4 (default 2; K / 32 / PF batches must divide by it).  Measured at
// 8 pages (`profiles/r04_bench8*_gu_ks*.log`): 2 beats 1 (16 experts: 19.5 -> 15.6 us wave span, 30: 34.3 ->
// 32.9) and 4 (one block per CU at this register count: 3.5 rounds of pieces); a 128-register budget (two
// blocks per CU) spilled and ran 1.6x slower
static int gu_ks() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("DSOCR_GU_KS");
        v = e ? atoi(e) : 2;
        if (v != 1 && v != 2 && v != 4) v = 2;
    }
    return v;
}


bool moe_gateup_mm_ok(const MoeDec2Args& a) {
    const bool swz_ok = !a.Wgu_swz || !a.sWgu || a.sWgu_swz;
    return a.grp && a.T >= 1 && a.T <= MM_MT && a.topk >= 1 && a.K % 32 == 0 && a.K <= 1536 && ((a.K >> 5) % 5) == 0 &&
           a.I % 16 == 0 && (!a.sWgu || a.Is % 16 == 0) && !a.norm_w && a.x && swz_ok;
}

// the routing inside (see the kernel): E <= 64 experts, T * topk <= 64, topk <= 8, K / 32 k-steps split in two halves
// of whole 10-step register batches; the picks and records also go to ids_out / w_out / grp for the down launch
bool moe_gateup_mm_route_ok(const MoeDec2Args& a) {
    MoeDec2Args b = a;
    b.norm_w = nullptr;
    return moe_gateup_mm_ok(b) && a.norm_w && a.router && a.E >= a.topk && a.E <= 64 && a.topk <= 8 &&
           a.T * a.topk <= 64 && ((a.K >> 5) % 20) == 0 && a.ids_out && a.w_out && (!a.router_swz || a.E % 16 == 0);
}

void launch_moe_gateup_mm(const MoeDec2Args& a, hipStream_t s) {
    const bool route = a.router != nullptr;
    if (route ? !moe_gateup_mm_route_ok(a) : !moe_gateup_mm_ok(a))
        throw std::runtime_error("EINVAL: grouped decode gate/up (matrix cores) outside its range");
    const size_t lds = sizeof(uint16_t) * 3 * MM_MT * (size_t)mm_pitch(a.K);
    const int slots = std::min(a.E, a.T * a.topk);
    const int max_units = (a.sWgu ? a.Is / 16 : 0) + slots * (a.I / 16);
    int ks = gu_ks();
    while (ks > 1 && ((a.K >> 5) / 5) % ks) ks >>= 1;
#define DSOCR_GM(WTY, SW, KS, RT)                                                                                      \
    do {                                                                                                            \
        static int resident = 0;                                                                                    \
        if (!resident) {                                                                                            \
            /* the pieces' LDS takes the block past 64 KB: allowed per kernel */                                    \
            (void)hipFuncSetAttribute((const void*)moe_gateup_mm_kernel<WTY, 5, SW, KS, RT>,                        \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);                       \
            resident = mm_resident_blocks((const void*)moe_gateup_mm_kernel<WTY, 5, SW, KS, RT>, 512, lds);         \
        }                                                                                                           \
        const int blocks = std::max(1, std::min(resident, (max_units + 8 / KS - 1) / (8 / KS)));                   \
        DSOCR_LAUNCH((moe_gateup_mm_kernel<WTY, 5, SW, KS, RT>), dim3(blocks), dim3(512), lds, s, a);                \
        static bool checked = false;                                                                                \
        if (!checked) {                                                                                             \
            const hipError_t e = hipPeekAtLastError();                                                              \
            if (e != hipSuccess)                                                                                    \
                throw std::runtime_error(std::string("EINTERNAL: moe_gateup_mm launch: ") + hipGetErrorString(e)); \
            checked = true;                                                                                         \
        }                                                                                                           \
    } while (0)
#define DSOCR_GMK(WTY, SW)                                                  \
    do {                                                                    \
        if (route) {                                                        \
            if (ks == 4) DSOCR_GM(WTY, SW, 4, true);                        \
            else if (ks == 2) DSOCR_GM(WTY, SW, 2, true);                   \
            else DSOCR_GM(WTY, SW, 1, true);                                \
        } else {                                                            \
            if (ks == 4) DSOCR_GM(WTY, SW, 4, false);                       \
            else if (ks == 2) DSOCR_GM(WTY, SW, 2, false);                  \
            else DSOCR_GM(WTY, SW, 1, false);                               \
        }                                                                   \
    } while (0)
    if (a.wdtype == WDT_BF16) { if (a.Wgu_swz) DSOCR_GMK(bf16_t, true); else DSOCR_GMK(bf16_t, false); }
    else { if (a.Wgu_swz) DSOCR_GMK(f16_t, true); else DSOCR_GMK(f16_t, false); }
#undef DSOCR_GMK
#undef DSOCR_GM
}

// ------------------------------------------------------------------ grouped decode MoE down (3..8 tokens)
// out[t][j] += sum over the routed records s of Wd[e_s][j] . h~[slot(s, t)] + Wds[j] . hs[t] (h~ carries
// the routing weight).  Segments: the n_act records, then the shared expert's K cut into Is / I
// pseudo-experts of I.  Work unit = (segment, 128 output rows); a block streams its unit's 8 x 16 rows
// as MFMA A fragments against the segment's token columns staged as three f16 planes (column t = the
// h~ row of the token's pick, zero when the token did not pick the expert), stores the partial tile
// write-through (sc1) to part[segment][t][j], and takes a ticket on the row tile; the block whose
// ticket completes the tile (every segment stored) sums the segments in order (records by expert id,
// then the shared pieces) with sc1 loads and adds to out (split-K seam: MI355X_MICROARCH.md price list
// 'splitk-seam'; hand-off: the sc1-load table's first row).
template <typename WT, int PF, bool SWZ, int NWV, int KS>
__global__ __launch_bounds__(64 * NWV * KS, KS == 2 ? 6 : 4) void moe_down_mm_kernel(MoeDec2Args a) {
    WaveSpan span_(a.span);
    typedef typename MmT<WT>::frag frag;
    constexpr int RT = 16 * NWV, U = 2;  // rows per unit (16 per wave), chunks per lane (I <= 1024)
    extern __shared__ __attribute__((aligned(16))) uint16_t xp[];  // [3][MT][KP]
    __shared__ float scl[MM_MT];
    __shared__ int last_s;
    constexpr int NW = NWV * KS;  // KS waves per 16-row tile, each a K / KS piece (met in LDS)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rw = wave % NWV, piece = wave / NWV;
    const int col = lane & 15, g = lane >> 4;
    // phase clocks (dev, tools/kbench moe8 KB_STAMPS): kept in LDS, written at the block's exit
    __shared__ unsigned long long dst_s[8];
#define DN_STAMP(i) \
    if (a.stamps && tid == 0) dst_s[i] = __builtin_amdgcn_s_memrealtime();
#define DN_FLUSH(n)                                                                             \
    if (a.stamps && tid == 0)                                                                   \
        for (int i_ = 0; i_ < (n); ++i_) a.stamps[(long)blockIdx.x * 8 + i_] = dst_s[i_];
    DN_STAMP(0);
    const int n_sh = a.sWd ? a.Is / a.I : 0;
    const int tiles = a.Hout / RT;
    const int unit = blockIdx.x;
    const int seg = unit / tiles, tile = unit % tiles;
    // the record count and this segment's record (expert, picks, their h rows) in ONE round trip: the record is
    // read as if the segment were routed (in bounds either way) and dropped when it is a shared piece
    int rw_[10];
    {
        const int* recg = a.grp + MOE_GRP_REC * (1 + min(seg, min(min(a.E, a.slots), 64) - 1));  // allocated records only
        const int4 q0 = *reinterpret_cast<const int4*>(recg), q1 = *reinterpret_cast<const int4*>(recg + 4);
        const int2 q2 = *reinterpret_cast<const int2*>(recg + 8);
        rw_[0] = q0.x; rw_[1] = q0.y; rw_[2] = q0.z; rw_[3] = q0.w;
        rw_[4] = q1.x; rw_[5] = q1.y; rw_[6] = q1.z; rw_[7] = q1.w; rw_[8] = q2.x; rw_[9] = q2.y;
    }
    const int n_act = a.grp[0];
    const int n_seg = n_act + n_sh;
    if (unit >= n_seg * tiles) return;  // block-uniform, before any barrier
    const bool shared = seg >= n_act;
    const int hpiece = seg - n_act;
    const int e = shared ? 0 : rw_[0];
    const int steps = a.I >> 5, nch = steps / PF / KS, c0 = piece * nch;  // nch: batches of this piece
    const int j0 = tile * RT + 16 * rw;
    // A stream: rows j0 .. j0 + 15 of the segment's down matrix over its I columns
    const WT* pa;
    long fs = 32;
    if (SWZ) {
        if (shared) {
            const int steps_s = a.Is >> 5;
            pa = reinterpret_cast<const WT*>(a.sWd_swz) + ((long)(j0 >> 4) * steps_s + hpiece * steps) * 512 + lane * 8;
        } else {
            pa = reinterpret_cast<const WT*>(a.Wd_swz) + (((long)e * a.Hout + j0) / 16 * steps) * 512 + lane * 8;
        }
        fs = 512;
    } else if (shared) {
        pa = reinterpret_cast<const WT*>(a.sWd) + (long)(j0 + col) * a.Is + (long)hpiece * a.I + 8 * g;
    } else {
        pa = reinterpret_cast<const WT*>(a.Wd) + ((long)e * a.Hout + j0 + col) * a.I + 8 * g;
    }
    frag fa[PF], fb[PF];
    auto load = [&](frag(&f)[PF], int c) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const uint4 q = ldg_nt16(pa + fs * (c * PF + i));
            __builtin_memcpy(&f[i], &q, 16);
        }
    };
    // wave w stages token columns w (and w + NWV when NWV < 8): the h~ row of the token's pick of this
    // expert (shared: hs[t] piece), zero when the token did not pick it
    auto src_of = [&](int t) -> const float* {
        if (t >= a.T) return nullptr;
        if (shared) return a.hs + (long)t * a.Is + (long)hpiece * a.I;
        const float* p = nullptr;
        const int cnt = rw_[1];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int r = rw_[2 + q];
            if (q < cnt && r / a.topk == t) p = a.h + (long)r * a.I;
        }
        return p;
    };
    constexpr int SPW = MM_MT / NW;  // token columns staged per wave
    static_assert(SPW >= 1 && MM_MT % NW == 0, "whole token columns per wave");
    const float* srcrow[SPW];
    MmRowU<U> xr[SPW];
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        srcrow[q] = src_of(wave + q * NW);
        if (srcrow[q]) mm_row_load<false, U>(xr[q], srcrow[q], a.I, nullptr);
    }
    load(fa, c0);
    // KS = 2: the second batch goes out after the token planes are staged, so its registers are not live
    // beside the token rows: 80 VGPRs, 6 waves per SIMD, three 8-wave blocks per CU, and the 640 units of
    // 30 experts at 8 pages resident in one round (104 VGPRs held two blocks per CU: 128 units started a
    // second round at ~12 us).  The first batch alone keeps ~29 MB in flight chip-wide.
    if (KS == 1 && nch > 1) load(fb, c0 + 1);
    const int KP = mm_pitch(a.I);
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        if (!srcrow[q]) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) xr[q].v[u][j] = 0.f;
        }
        mm_row_store<WT, false, U>(xr[q], a.I, 0.f, xp, KP, scl, wave + q * NW);
    }
    if (KS > 1 && nch > 1) load(fb, c0 + 1);
    __syncthreads();
    DN_STAMP(1);
    const uint16_t* bbase = xp + (long)(col & 7) * KP + 8 * g;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const frag(&f)[PF], int c) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int k = 32 * (c * PF + i);
#pragma unroll
            for (int p = 2; p >= 0; --p) {
                const frag b = *reinterpret_cast<const frag*>(bbase + (long)p * MM_MT * KP + k);
                acc = MmT<WT>::mfma(f[i], b, acc);
            }
        }
    };
    for (int c = 0; c < nch; c += 2) {
        if (c + 1 < nch && c > 0) load(fb, c0 + c + 1);
        compute(fa, c0 + c);
        if (c + 1 >= nch) break;
        if (c + 2 < nch) load(fa, c0 + c + 2);
        compute(fb, c0 + c + 1);
    }
    DN_STAMP(2);
    if (KS > 1) {  // the pieces of a row tile meet in LDS, summed in piece order by piece 0
        __shared__ f32x4 red[KS > 1 ? KS - 1 : 1][NWV][64];
        if (piece > 0) red[piece - 1][rw][lane] = acc;
        __syncthreads();
        if (piece == 0)
#pragma unroll
            for (int q = 0; q < KS - 1; ++q) {
                const f32x4 o = red[q][rw][lane];
                acc[0] += o[0]; acc[1] += o[1]; acc[2] += o[2]; acc[3] += o[3];
            }
    }
    // partial tile -> part[seg][t][j]: one 16-byte write-through (sc1) store per lane (rows 4g .. 4g + 3
    // of token column col); tokens outside the segment are zero columns
    const auto prs = __builtin_amdgcn_make_buffer_rsrc(a.dn_part, (short)0, 0x7fffffff, 0x00020000);
    if (piece == 0 && col < a.T) {
        const float sc = scl[col];
        const float v4[4] = {acc[0] * sc, acc[1] * sc, acc[2] * sc, acc[3] * sc};
        u32x4 bits;
        __builtin_memcpy(&bits, v4, 16);
        __builtin_amdgcn_raw_buffer_store_b128(bits, prs, (int)((((long)seg * MM_MT + col) * a.Hout + j0 + 4 * g) * 4), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        int* tk = a.dn_tick + tile;
        const int old = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == n_seg - 1;
        if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = last;
    }
    __syncthreads();
    DN_STAMP(3);
    if (!last_s) {
        DN_FLUSH(4);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below
    // the last arriver: the ordered sum over segments.  A token's column of a segment it does not
    // belong to was computed from a zero B column, so it holds exact zeros and adding it leaves every
    // partial sum unchanged; all segments are therefore summed unconditionally.  Thread = (4 rows of one
    // token, one of NQ contiguous segment ranges): 16-byte sc1 loads of every segment of its range issued
    // together (one L2 round trip; a per-segment test, or batches of scalar loads, made each batch its own
    // round trip), summed in segment order; the ranges meet through LDS (the staging planes, dead here):
    // NQ = 2 (256 threads): r_0 + r_1; NQ = 4 (512 threads, KS = 2): (r_0 + r_1) + (r_2 + r_3), a fixed order.
    // Four ranges at KS = 2 keep the loads in flight per thread at 13 (52 VGPRs; the kernel is held to 80).
    constexpr int NQ = 64 * NWV * KS / 128;
    static_assert(NWV == 4 && RT * MM_MT / 4 == 128 && (NQ == 2 || NQ == 4), "tail layout: 128 row quads x NQ ranges");
    float4* rng_s = reinterpret_cast<float4*>(xp);  // [NQ - 1][128]
    const int q4 = tid & 127, hf = tid >> 7;
    const int t = q4 / (RT / 4), j = tile * RT + (q4 % (RT / 4)) * 4;
    const int nh = (n_seg + NQ - 1) / NQ;
    const int sb = min(hf * nh, n_seg), se = min(sb + nh, n_seg);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    // the residual quad, loaded with the segments (not after the ranges meet: one round trip fewer)
    float4* op = reinterpret_cast<float4*>(a.out + (long)min(t, a.T - 1) * a.Hout + j);
    const float4 o_in = hf ? make_float4(0.f, 0.f, 0.f, 0.f) : *op;
    if (t < a.T) {
        constexpr int SB = NQ == 4 ? 13 : 18;  // segments in flight per batch (n_seg <= 50 at 8 pages: one batch)
        const long sstride = (long)MM_MT * a.Hout * 4;
        const int base = (int)(((long)t * a.Hout + j) * 4);
        for (int s0 = sb; s0 < se; s0 += SB) {
            u32x4 pv[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q)
                pv[q] = __builtin_amdgcn_raw_buffer_load_b128(prs, base + (int)(min(s0 + q, se - 1) * sstride), 0, 16);
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                if (s0 + q < se) {
                    v.x += __uint_as_float(pv[q][0]);
                    v.y += __uint_as_float(pv[q][1]);
                    v.z += __uint_as_float(pv[q][2]);
                    v.w += __uint_as_float(pv[q][3]);
                }
            }
        }
    }
    if (hf > 0) rng_s[(hf - 1) * 128 + q4] = v;
    __syncthreads();
    if (!hf && t < a.T) {
        float4 u = rng_s[q4];
        float4 s = make_float4(v.x + u.x, v.y + u.y, v.z + u.z, v.w + u.w);
        if (NQ == 4) {
            const float4 u2 = rng_s[128 + q4], u3 = rng_s[256 + q4];
            s = make_float4(s.x + (u2.x + u3.x), s.y + (u2.y + u3.y), s.z + (u2.z + u3.z), s.w + (u2.w + u3.w));
        }
        float4 o = o_in;
        o.x = o.x + s.x;
        o.y = o.y + s.y;
        o.z = o.z + s.z;
        o.w = o.w + s.w;
        *op = o;
    }
    DN_STAMP(4);
    DN_FLUSH(5);
#undef DN_STAMP
#undef DN_FLUSH
}

bool moe_down_mm_ok(const MoeDec2Args& a) {
    const bool swz_ok = !a.Wd_swz || !a.sWd || a.sWd_swz;
    return a.grp && a.dn_part && a.dn_tick && a.T >= 1 && a.T <= MM_MT && a.I % 32 == 0 && a.I <= 1024 &&
           ((a.I >> 5) % 7) == 0 && a.Hout % 128 == 0 && (!a.sWd || (a.Is % a.I == 0 && a.Is / a.I <= 8)) &&
           std::min(a.E, a.T * a.topk) + (a.sWd ? a.Is / a.I : 0) <= 72 && swz_ok;
}

size_t moe_down_mm_part_floats(int E, int T, int topk, int I, int Is, int H) {
    return (size_t)(std::min(E, T * topk) + (I > 0 && Is > 0 ? Is / I : 0)) * MM_MT * H;
}

// Units of 64 output rows (4 waves): 17 segments x 20 row tiles = 340 blocks at 8 pages, where 128-row
// units (8 waves) left a third of the CUs idle (170 blocks).  Two waves per 16-row tile, each half of K (8
// waves per block; DSOCR_DN_KS = 1 for one): 16 experts 12.9 -> 12.0 us wave span, 30 unchanged (21.0 / 21.3:
// 680 blocks of 512 threads take 1.3 residency rounds), `profiles/r04_bench8{t,i}_dn_ks{1,2}.log`.
static int dn_ks() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("DSOCR_DN_KS");
        v = e && atoi(e) == 1 ? 1 : 2;
    }
    return v;
}

void launch_moe_down_mm(const MoeDec2Args& a, hipStream_t s) {
    if (!moe_down_mm_ok(a)) throw std::runtime_error("EINVAL: grouped decode down (matrix cores) outside its range");
    const size_t lds = sizeof(uint16_t) * 3 * MM_MT * (size_t)mm_pitch(a.I);
    const int max_seg = std::min(a.E, a.T * a.topk) + (a.sWd ? a.Is / a.I : 0);
    dim3 grid(max_seg * (a.Hout / 64));
#define DSOCR_DM(WTY, SW)                                                                              \
    do {                                                                                               \
        if (dn_ks() == 2 && ((a.I >> 5) / 7) % 2 == 0) DSOCR_LAUNCH((moe_down_mm_kernel<WTY, 7, SW, 4, 2>), grid, dim3(512), lds, s, a); \
        else DSOCR_LAUNCH((moe_down_mm_kernel<WTY, 7, SW, 4, 1>), grid, dim3(256), lds, s, a);          \
    } while (0)
    if (a.wdtype == WDT_BF16) { if (a.Wd_swz) DSOCR_DM(bf16_t, true); else DSOCR_DM(bf16_t, false); }
    else { if (a.Wd_swz) DSOCR_DM(f16_t, true); else DSOCR_DM(f16_t, false); }
#undef DSOCR_DM
}


// ------------------------------------------------------------------ long-K projection, 3..8 tokens
// Y[m][n] (+)= X[m] . W[n]^T (+ bias) for K too long to stage whole (the dense layer-0 down
// projection, K = 6848): K is cut in pieces of MMK_PIECE; unit = (piece, 64 output rows); a block
// stages its piece of the token rows as three planes (one power-of-two scale per (row, piece)),
// streams its 4 waves x 16 rows, stores the scaled partial tile write-through and takes a ticket on
// its row tile; the last arriver sums the pieces in order, adds the bias and (+=) the output.
constexpr int MMK_PIECE = 512;

template <typename WT>
__global__ __launch_bounds__(256) void dec_mm_splitk_kernel(DecGemvArgs a, float* part, int* tick) {
    typedef typename MmT<WT>::frag frag;
    constexpr int NWV = 4, RW = 64, U = 1;  // waves, rows per unit, chunks per lane (piece <= 512)
    __shared__ __attribute__((aligned(16))) uint16_t xp[3 * MM_MT * (MMK_PIECE + 16)];
    __shared__ float scl[MM_MT];
    __shared__ int last_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int n_pieces = (a.K + MMK_PIECE - 1) / MMK_PIECE;
    const int tiles = (a.N + RW - 1) / RW;
    const int piece = blockIdx.x % n_pieces, tile = blockIdx.x / n_pieces;
    const int k0 = piece * MMK_PIECE, klen = min(MMK_PIECE, a.K - k0);
    const int steps = klen >> 5;  // host: every piece a multiple of 64
    const int KP = MMK_PIECE + 16;
    const int j0 = tile * RW + 16 * wave;
    const WT* pa = reinterpret_cast<const WT*>(a.W) + (long)min(j0 + col, a.N - 1) * a.ldw + k0 + 8 * g;
    // token rows of this piece: wave w stages rows w and w + 4 (loads before the weight stream)
    MmRowU<U> r0, r1;
    const int m0 = wave, m1 = wave + NWV;
    if (m0 < a.M) mm_row_load<false, U>(r0, a.x + (long)m0 * a.ldx + k0, klen, nullptr);
    if (m1 < a.M) mm_row_load<false, U>(r1, a.x + (long)m1 * a.ldx + k0, klen, nullptr);
    frag fa[2], fb[2];
    auto load = [&](frag(&f)[2], int c) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint4 q = ldg_nt16(pa + 32 * (2 * c + i));
            __builtin_memcpy(&f[i], &q, 16);
        }
    };
    const int nch = steps / 2;
    load(fa, 0);
    if (nch > 1) load(fb, 1);
    if (m0 < a.M) mm_row_store<WT, false, U>(r0, klen, 0.f, xp, KP, scl, m0);
    if (m1 < a.M) mm_row_store<WT, false, U>(r1, klen, 0.f, xp, KP, scl, m1);
    __syncthreads();
    const uint16_t* bbase = xp + (long)(col & 7) * KP + 8 * g;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const frag(&f)[2], int c) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int k = 32 * (2 * c + i);
#pragma unroll
            for (int p = 2; p >= 0; --p) {
                const frag b = *reinterpret_cast<const frag*>(bbase + (long)p * MM_MT * KP + k);
                acc = MmT<WT>::mfma(f[i], b, acc);
            }
        }
    };
    for (int c = 0; c < nch; c += 2) {
        if (c + 1 < nch && c > 0) load(fb, c + 1);
        compute(fa, c);
        if (c + 1 >= nch) break;
        if (c + 2 < nch) load(fa, c + 2);
        compute(fb, c + 1);
    }
    if (col < a.M && j0 < a.N) {
        const float sc = scl[col];
        float* dst = part + ((long)piece * MM_MT + col) * a.N + j0 + 4 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (j0 + 4 * g + i < a.N) __hip_atomic_store(dst + i, acc[i] * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int old = __hip_atomic_fetch_add(tick + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == n_pieces - 1;
        if (last) __hip_atomic_store(tick + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below
    for (int i = tid; i < RW * MM_MT; i += NWV * 64) {
        const int m = i / RW, n = tile * RW + i % RW;
        if (m >= a.M || n >= a.N) continue;
        float v = 0.f;
        constexpr int SB = 16;  // pieces in flight together (one L2 round trip per batch, in order)
        for (int p0 = 0; p0 < n_pieces; p0 += SB) {
            float pv[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q)
                pv[q] = __hip_atomic_load(part + ((long)min(p0 + q, n_pieces - 1) * MM_MT + m) * a.N + n,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int q = 0; q < SB; ++q)
                if (p0 + q < n_pieces) v += pv[q];
        }
        v = apply_act(v + (a.bias ? a.bias[n] : 0.f), a.act);
        float* yp = a.y + (long)m * a.ldy + n;
        if (a.accumulate) v = *yp + v;
        *yp = v;
    }
    (void)tiles;
}

bool dec_mm_splitk_ok(const DecGemvArgs& a) {
    return a.M >= 1 && a.M <= MM_MT && a.K % 64 == 0 && a.N >= 16 && !a.norm_w && !a.xn_out && a.ldw % 8 == 0 &&
           a.ldx % 4 == 0;
}

size_t dec_mm_splitk_part_floats(int N, int K) { return (size_t)((K + MMK_PIECE - 1) / MMK_PIECE) * MM_MT * N; }
size_t dec_mm_splitk_ticks(int N) { return (size_t)(N + 63) / 64; }

void launch_dec_mm_splitk(const DecGemvArgs& a, float* part, int* tick, hipStream_t s) {
    if (!dec_mm_splitk_ok(a) || !part || !tick) throw std::runtime_error("EINVAL: dec_mm_splitk outside its range");
    const int n_pieces = (a.K + MMK_PIECE - 1) / MMK_PIECE, tiles = (a.N + 63) / 64;
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((dec_mm_splitk_kernel<bf16_t>), dim3(n_pieces * tiles), dim3(256), 0, s, a, part, tick);
    else DSOCR_LAUNCH((dec_mm_splitk_kernel<f16_t>), dim3(n_pieces * tiles), dim3(256), 0, s, a, part, tick);
}

}  // namespace dsocr
