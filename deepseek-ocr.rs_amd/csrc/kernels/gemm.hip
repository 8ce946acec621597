// f32-exact GEMM on the gfx950 matrix cores: C = act(A . W^T + bias) (+ C).
//
// Reference semantics: every linear of the DeepSeek-OCR page path is an f32
// matmul (sam.rs:656-701 linear_forward, clip.rs:418-447 apply_linear,
// block.rs:1085-1134 apply_linear_f32_keep) with weights widened from bf16/f16.
// We keep the weights in their 16-bit storage type and widen while staging into
// LDS, then run v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate;
// cdna_hip_programming.md §3 "FP32-input MFMA").
//
// Tile: 128x128 per 256-thread workgroup (4 waves as 2x2, 64x64 per wave =
// 2x2 MFMA 32x32 tiles), BK = 16, LDS k-major so fragment reads are
// conflict-free, register prefetch of the next K tile (T14-style split).
// Optional row gather for A (a_rows), row scatter for C (c_rows, -1 = drop),
// and grouping (blockIdx.z = group, rows [goff[g], goff[g+1]) of the gathered
// list, weight slab g) for the MoE prefill grouped GEMM.
#include <cstdint>
#include <cstdlib>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

constexpr int GB_M = 128, GB_N = 128, GB_K = 16, G_PAD = 4;

template <typename WT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
    __shared__ float As[GB_K][GB_M + G_PAD];
    __shared__ float Bs[GB_K][GB_N + G_PAD];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;

    // ---- group resolution
    int grp = blockIdx.z;
    int m_begin = 0, m_count = g.M;
    const WT* W = reinterpret_cast<const WT*>(g.W);
    const float* bias = g.bias;
    if (g.group_off) {
        m_begin = g.group_off[grp];
        m_count = g.group_off[grp + 1] - m_begin;
        W += (size_t)grp * g.w_group_stride;
        if (bias) bias += (size_t)grp * g.bias_group_stride;
    }
    const int m0 = blockIdx.y * GB_M;
    if (m0 >= m_count) return;
    const int n0 = blockIdx.x * GB_N;

    // ---- per-thread global load coordinates
    // A: 128 rows x 16 k = 512 float4; thread t -> rows (t>>2) and (t>>2)+64, k quad (t&3)*4
    const int a_r0 = tid >> 2, a_kq = (tid & 3) * 4;
    long a_src[2];
    bool a_ok[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int r = m0 + a_r0 + 64 * i;
        a_ok[i] = r < m_count;
        int rr = a_ok[i] ? (m_begin + r) : m_begin;
        long row = g.a_rows ? (long)g.a_rows[rr] : (long)rr;
        a_src[i] = row * (long)g.lda;
    }
    // W: 128 n x 16 k halves = 256 x 8; thread t -> n = t>>1, k oct (t&1)*8
    const int b_n = tid >> 1, b_k8 = (tid & 1) * 8;
    const bool b_ok = (n0 + b_n) < g.N;
    const long b_src = (long)(b_ok ? (n0 + b_n) : 0) * (long)g.ldw;

    float4 ra[2];
    uint4 rb;
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int k = k0 + a_kq;
            if (a_ok[i] && k < g.K) {
                ra[i] = *reinterpret_cast<const float4*>(g.A + a_src[i] + k);
            } else {
                ra[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        int k = k0 + b_k8;
        if (b_ok && k < g.K) {
            rb = *reinterpret_cast<const uint4*>(W + b_src + k);
        } else {
            rb = make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            As[a_kq + 0][a_r0 + 64 * i] = ra[i].x;
            As[a_kq + 1][a_r0 + 64 * i] = ra[i].y;
            As[a_kq + 2][a_r0 + 64 * i] = ra[i].z;
            As[a_kq + 3][a_r0 + 64 * i] = ra[i].w;
        }
        float w8[8];
        unpack8<WT>(rb, w8);
#pragma unroll
        for (int j = 0; j < 8; ++j) Bs[b_k8 + j][b_n] = w8[j];
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int ksteps = (g.K + GB_K - 1) / GB_K;
    gload(0);
    for (int kt = 0; kt < ksteps; ++kt) {
        lstore();
        __syncthreads();
        if (kt + 1 < ksteps) gload((kt + 1) * GB_K);
        const int half = lane >> 5, l32 = lane & 31;
#pragma unroll
        for (int kk = 0; kk < GB_K / 2; ++kk) {
            const int kr = kk * 2 + half;
            float a0 = As[kr][wm * 64 + l32];
            float a1 = As[kr][wm * 64 + 32 + l32];
            float b0 = Bs[kr][wn * 64 + l32];
            float b1 = Bs[kr][wn * 64 + 32 + l32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }

    // ---- epilogue: D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const int half = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int col = n0 + wn * 64 + ni * 32 + l32;
            if (col >= g.N) continue;
            const float bv = bias ? bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (row >= m_count) continue;
                long orow = g.c_rows ? (long)g.c_rows[m_begin + row] : (long)(m_begin + row);
                if (orow < 0) continue;
                float v = apply_act(acc[mi][ni][r] + bv, g.act);
                float* cp = g.C + orow * (long)g.ldc + col;
                if (g.accumulate) v += *cp;
                *cp = v;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 GEMM (same contract, same result to f32 rounding): every f32 activation is
// split exactly into three bf16 terms a = hi + mid + lo (RNE at each step; the residuals
// are exact in f32 by Sterbenz), weights are bf16 (vision: one exact plane) or f16 (decoder:
// hi + lo bf16 planes, exact since f16 has an 11-bit significand).  A.W^T is then the sum
// of 3 (bf16 W) or 5 (f16 W; the lo x lo term is below f32 rounding) products on
// v_mfma_f32_32x32x16_bf16 — bf16 x bf16 products are exact in the f32 accumulator — at
// 16x the per-instruction rate of the f32-input MFMA (MI355X_MICROARCH.md constants).
// Tile 128x128x32, 4 waves as 2x2 of 64x64 (2x2 MFMA 32x32 tiles each); LDS holds the
// bf16 planes row-major with k contiguous (row stride 80 B: conflict-free fragment reads).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int XB_M = 128, XB_N = 128, XB_K = 32, XB_KP = 40;

__device__ __forceinline__ void split3(float a, __bf16& hi, __bf16& mid, __bf16& lo) {
    hi = (__bf16)a;
    const float r1 = a - (float)hi;
    mid = (__bf16)r1;
    const float r2 = r1 - (float)mid;
    lo = (__bf16)r2;
}

template <typename WT>
__global__ __launch_bounds__(256) void gemm_x3_kernel(GemmArgs g) {
    constexpr int WP = sizeof(WT) == 2 && __is_same(WT, bf16_t) ? 1 : 2;
    __shared__ __attribute__((aligned(16))) __bf16 As[3][XB_M][XB_KP];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[WP][XB_N][XB_KP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int m_begin = 0, m_count = g.M;
    const WT* W = reinterpret_cast<const WT*>(g.W);
    const float* bias = g.bias;
    if (g.group_off) {
        const int grp = blockIdx.z;
        m_begin = g.group_off[grp];
        m_count = g.group_off[grp + 1] - m_begin;
        W += (size_t)grp * g.w_group_stride;
        if (bias) bias += (size_t)grp * g.bias_group_stride;
    }
    const int m0 = blockIdx.y * XB_M;
    if (m0 >= m_count) return;
    const int n0 = blockIdx.x * XB_N;
    // staging coordinates: thread -> (row tid>>1, 16 consecutive k at (tid&1)*16)
    const int s_r = tid >> 1, s_k = (tid & 1) * 16;
    const bool a_ok = m0 + s_r < m_count;
    const int arr = m_begin + (a_ok ? m0 + s_r : 0);
    const float* a_ptr = g.A + (long)(g.a_rows ? g.a_rows[arr] : arr) * g.lda + s_k;
    const bool b_ok = n0 + s_r < g.N;
    const WT* w_ptr = W + (long)(b_ok ? n0 + s_r : 0) * g.ldw + s_k;
    float4 ra[4];
    uint4 rb[2];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[i] = *reinterpret_cast<const float4*>(a_ptr + k0 + 4 * i);
#pragma unroll
        for (int i = 0; i < 2; ++i) rb[i] = *reinterpret_cast<const uint4*>(w_ptr + k0 + 8 * i);
    };
    auto lstore = [&]() {
        __bf16 h[16], m[16], l[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float v[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) split3(a_ok ? v[j] : 0.f, h[4 * i + j], m[4 * i + j], l[4 * i + j]);
        }
        bf16x8_t* ah = reinterpret_cast<bf16x8_t*>(&As[0][s_r][s_k]);
        bf16x8_t* am = reinterpret_cast<bf16x8_t*>(&As[1][s_r][s_k]);
        bf16x8_t* al = reinterpret_cast<bf16x8_t*>(&As[2][s_r][s_k]);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            bf16x8_t vh, vm, vl;
#pragma unroll
            for (int j = 0; j < 8; ++j) { vh[j] = h[8 * q + j]; vm[j] = m[8 * q + j]; vl[j] = l[8 * q + j]; }
            ah[q] = vh;
            am[q] = vm;
            al[q] = vl;
        }
        if constexpr (WP == 1) {
            bf16x8_t* bp = reinterpret_cast<bf16x8_t*>(&Bs[0][s_r][s_k]);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint4 u = b_ok ? rb[q] : make_uint4(0u, 0u, 0u, 0u);
                bf16x8_t v;
                __builtin_memcpy(&v, &u, 16);
                bp[q] = v;
            }
        } else {
            bf16x8_t* bh = reinterpret_cast<bf16x8_t*>(&Bs[0][s_r][s_k]);
            bf16x8_t* bl = reinterpret_cast<bf16x8_t*>(&Bs[1][s_r][s_k]);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                float w8[8];
                unpack8<WT>(rb[q], w8);
                bf16x8_t vh, vl;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float w = b_ok ? w8[j] : 0.f;
                    const __bf16 wh = (__bf16)w;
                    vh[j] = wh;
                    vl[j] = (__bf16)(w - (float)wh);
                }
                bh[q] = vh;
                bl[q] = vl;
            }
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int half = lane >> 5, l32 = lane & 31;
    const int ksteps = g.K / XB_K;
    gload(0);
    for (int kt = 0; kt < ksteps; ++kt) {
        lstore();
        __syncthreads();
        if (kt + 1 < ksteps) gload((kt + 1) * XB_K);
#pragma unroll
        for (int ks = 0; ks < XB_K / 16; ++ks) {
            const int kb = ks * 16 + 8 * half;
            bf16x8_t af[2][3], bfr[2][WP];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    af[mi][p] = *reinterpret_cast<const bf16x8_t*>(&As[p][wm * 64 + mi * 32 + l32][kb]);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int q = 0; q < WP; ++q)
                    bfr[ni][q] = *reinterpret_cast<const bf16x8_t*>(&Bs[q][wn * 64 + ni * 32 + l32][kb]);
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    // small terms first, the dominant hi x hi product last
                    if constexpr (WP == 2) {
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][1], bfr[ni][1], acc[mi][ni], 0, 0, 0);
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][0], bfr[ni][1], acc[mi][ni], 0, 0, 0);
                    }
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][2], bfr[ni][0], acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][1], bfr[ni][0], acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][0], bfr[ni][0], acc[mi][ni], 0, 0, 0);
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int col = n0 + wn * 64 + ni * 32 + l32;
            if (col >= g.N) continue;
            const float bv = bias ? bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (row >= m_count) continue;
                const long orow = g.c_rows ? (long)g.c_rows[m_begin + row] : (long)(m_begin + row);
                if (orow < 0) continue;
                float v = apply_act(acc[mi][ni][r] + bv, g.act);
                float* cp = g.C + orow * (long)g.ldc + col;
                if (g.accumulate) v += *cp;
                *cp = v;
            }
        }
    }
}

void launch_gemm(const GemmArgs& g, hipStream_t s) {
    dim3 block(256);
    int mtiles = (g.group_off ? g.max_group_rows : g.M);
    dim3 grid((g.N + GB_N - 1) / GB_N, (mtiles + GB_M - 1) / GB_M, g.group_off ? g.groups : 1);
    if (grid.y == 0 || grid.x == 0) return;
    // grouped (MoE prefill): the exact-f32 grouped kernel (gemm_bf16.hip) — 32-row tiles up to 256 mean
    // rows per expert (1 page: prefill 10.1 -> 9.4 ms, 2 pages 13.4 -> 13.1), 128-row tiles above
    if (g.group_off && gemm_f32a_grouped_ok(g)) {
        launch_gemm_f32a_grouped(g, s);
        return;
    }
    // split-bf16 MFMA path when the tiles are whole along K and the rows 16-byte aligned; else the
    // f32-input kernel
    const bool x3 = g.K % XB_K == 0 && g.lda % 4 == 0 && g.ldw % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(g.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.W) & 15) == 0;
    if (x3) {
        dim3 gx((g.N + XB_N - 1) / XB_N, (mtiles + XB_M - 1) / XB_M, g.group_off ? g.groups : 1);
        if (g.wdtype == WDT_BF16) hipLaunchKernelGGL(gemm_x3_kernel<bf16_t>, gx, block, 0, s, g);
        else hipLaunchKernelGGL(gemm_x3_kernel<f16_t>, gx, block, 0, s, g);
        return;
    }
    if (g.wdtype == WDT_BF16)
        hipLaunchKernelGGL(gemm_f32_kernel<bf16_t>, grid, block, 0, s, g);
    else
        hipLaunchKernelGGL(gemm_f32_kernel<f16_t>, grid, block, 0, s, g);
}

}  // namespace dsocr
