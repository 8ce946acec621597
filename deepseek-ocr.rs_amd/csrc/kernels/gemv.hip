// Decode-phase linears (M = pages in flight, <= 16 rows per pass): HBM-bound
// weight streaming.  One wave owns RB output rows and walks K with 16-byte
// weight loads (8 x 16-bit) per lane; activations are tiny and L1/L2 resident.
// f32 FMA on widened weights == the reference's f32 matmul on the f16/bf16
// weights (block.rs:1085-1134, transformer/model.rs:243-270).
//
// Also the decode MoE grouped GEMV (the north-star kernel): one launch covers
// every routed expert; a wave owns RB rows of one expert and reuses each
// weight load for all tokens routed to that expert (run_moe, block.rs:1326-1351).
#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

template <typename WT, int MT, int RB>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int n0 = (blockIdx.x * 4 + wave) * RB;
    if (n0 >= a.N) return;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    const int chunks = a.K >> 3;
    float acc[RB][MT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;

    for (int c = lane; c < chunks; c += 64) {
        const int k = c << 3;
        uint4 wq[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int n = min(n0 + r, a.N - 1);
            wq[r] = ldg_nt16(W + (long)n * a.ldw + k);
        }
        float xv[MT][8];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            if (m < a.M) {
                const float4* xp = reinterpret_cast<const float4*>(a.x + (long)m * a.ldx + k);
                float4 x0 = xp[0], x1 = xp[1];
                xv[m][0] = x0.x; xv[m][1] = x0.y; xv[m][2] = x0.z; xv[m][3] = x0.w;
                xv[m][4] = x1.x; xv[m][5] = x1.y; xv[m][6] = x1.z; xv[m][7] = x1.w;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[m][j] = 0.f;
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float w8[8];
            unpack8<WT>(wq[r], w8);
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[r][m] = fmaf(xv[m][j], w8[j], acc[r][m]);
        }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            float v = wave_sum(acc[r][m]);
            const int n = n0 + r;
            if (lane == 0 && m < a.M && n < a.N) {
                v = apply_act(v + (a.bias ? a.bias[n] : 0.f), a.act);
                float* yp = a.y + (long)m * a.ldy + n;
                if (a.accumulate) v += *yp;
                *yp = v;
            }
        }
    }
}

template <typename WT, int MT>
static void gemv_dispatch_rb(const GemvArgs& a, hipStream_t s) {
    constexpr int RB = (MT <= 2) ? 4 : 2;
    dim3 grid((a.N + 4 * RB - 1) / (4 * RB));
    hipLaunchKernelGGL((gemv_kernel<WT, MT, RB>), grid, dim3(256), 0, s, a);
}

template <typename WT>
static void gemv_dispatch(const GemvArgs& a, hipStream_t s) {
    if (a.M <= 1) gemv_dispatch_rb<WT, 1>(a, s);
    else if (a.M <= 2) gemv_dispatch_rb<WT, 2>(a, s);
    else if (a.M <= 4) gemv_dispatch_rb<WT, 4>(a, s);
    else if (a.M <= 8) gemv_dispatch_rb<WT, 8>(a, s);
    else gemv_dispatch_rb<WT, 16>(a, s);
}

void launch_gemv(const GemvArgs& a, hipStream_t s) {
    if (a.N == 0 || a.M == 0) return;
    // rows beyond 16 are processed in passes of 16
    for (int m0 = 0; m0 < a.M; m0 += 16) {
        GemvArgs p = a;
        p.M = a.M - m0 < 16 ? a.M - m0 : 16;
        p.x = a.x + (long)m0 * a.ldx;
        p.y = a.y + (long)m0 * a.ldy;
        if (a.wdtype == WDT_BF16) gemv_dispatch<bf16_t>(p, s);
        else gemv_dispatch<f16_t>(p, s);
    }
}

// ------------------------------------------------------------------ MoE decode (grouped GEMV)
// grid.x = E * ceil(I / (4*RB)); wave owns RB intermediate rows i of expert e and
// computes gate_i and up_i for every token routed to e (chunks of MT tokens).
// ROUTED only distinguishes the routed-expert instantiation from the dense / shared-expert one
// (E = 1) in profiles; the code is identical.
template <typename WT, int MT, int RB, bool ROUTED>
__global__ __launch_bounds__(256) void moe_gateup_kernel(MoeDecodeArgs a) {
    const int units_per_e = (a.I + 4 * RB - 1) / (4 * RB);
    const int e = blockIdx.x / units_per_e;
    const int u = blockIdx.x % units_per_e;
    const int p0 = a.eoff[e], cnt = a.eoff[e + 1] - p0;
    if (cnt == 0) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i0 = (u * 4 + wave) * RB;
    if (i0 >= a.I) return;
    const WT* Wg = reinterpret_cast<const WT*>(a.Wgu) + (long)e * 2 * a.I * a.K;
    const WT* Wu = Wg + (long)a.I * a.K;
    const int chunks = a.K >> 3;
    for (int t0 = 0; t0 < cnt; t0 += MT) {
        const int tn = min(MT, cnt - t0);
        int rows[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) rows[m] = a.arow[p0 + t0 + min(m, tn - 1)];
        float ag[RB][MT], au[RB][MT];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m) { ag[r][m] = 0.f; au[r][m] = 0.f; }
        for (int c = lane; c < chunks; c += 64) {
            const int k = c << 3;
            uint4 qg[RB], qu[RB];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int i = min(i0 + r, a.I - 1);
                qg[r] = ldg_nt16(Wg + (long)i * a.K + k);
                qu[r] = ldg_nt16(Wu + (long)i * a.K + k);
            }
            float xv[MT][8];
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const float4* xp = reinterpret_cast<const float4*>(a.x + (long)rows[m] * a.K + k);
                float4 x0 = xp[0], x1 = xp[1];
                xv[m][0] = x0.x; xv[m][1] = x0.y; xv[m][2] = x0.z; xv[m][3] = x0.w;
                xv[m][4] = x1.x; xv[m][5] = x1.y; xv[m][6] = x1.z; xv[m][7] = x1.w;
            }
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                float wg[8], wu[8];
                unpack8<WT>(qg[r], wg);
                unpack8<WT>(qu[r], wu);
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        ag[r][m] = fmaf(xv[m][j], wg[j], ag[r][m]);
                        au[r][m] = fmaf(xv[m][j], wu[j], au[r][m]);
                    }
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                float gs = wave_sum(ag[r][m]);
                float us = wave_sum(au[r][m]);
                const int i = i0 + r;
                if (lane == 0 && m < tn && i < a.I) {
                    float sg = gs / (1.0f + expf(-gs));  // silu (candle: x / (1 + exp(-x)))
                    a.h[(long)(p0 + t0 + m) * a.I + i] = sg * us;
                }
            }
    }
}

template <typename WT, int MT, int RB, bool ROUTED>
__global__ __launch_bounds__(256) void moe_down_kernel(MoeDecodeArgs a) {
    const int units_per_e = (a.Hout + 4 * RB - 1) / (4 * RB);
    const int e = blockIdx.x / units_per_e;
    const int u = blockIdx.x % units_per_e;
    const int p0 = a.eoff[e], cnt = a.eoff[e + 1] - p0;
    if (cnt == 0) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j0 = (u * 4 + wave) * RB;
    if (j0 >= a.Hout) return;
    const WT* Wd = reinterpret_cast<const WT*>(a.Wd) + (long)e * a.Hout * a.I;
    const int chunks = a.I >> 3;
    for (int t0 = 0; t0 < cnt; t0 += MT) {
        const int tn = min(MT, cnt - t0);
        float acc[RB][MT];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
        for (int c = lane; c < chunks; c += 64) {
            const int k = c << 3;
            uint4 q[RB];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int j = min(j0 + r, a.Hout - 1);
                q[r] = ldg_nt16(Wd + (long)j * a.I + k);
            }
            float hv[MT][8];
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const int p = p0 + t0 + min(m, tn - 1);
                const float4* hp = reinterpret_cast<const float4*>(a.h + (long)p * a.I + k);
                float4 h0 = hp[0], h1 = hp[1];
                hv[m][0] = h0.x; hv[m][1] = h0.y; hv[m][2] = h0.z; hv[m][3] = h0.w;
                hv[m][4] = h1.x; hv[m][5] = h1.y; hv[m][6] = h1.z; hv[m][7] = h1.w;
            }
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                float w8[8];
                unpack8<WT>(q[r], w8);
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) acc[r][m] = fmaf(hv[m][jj], w8[jj], acc[r][m]);
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                float v = wave_sum(acc[r][m]);
                const int j = j0 + r;
                if (lane == 0 && m < tn && j < a.Hout) a.y[(long)(p0 + t0 + m) * a.Hout + j] = v;
            }
    }
}

template <typename WT, int MT, bool ROUTED>
static void moe_launch_pair_gateup(const MoeDecodeArgs& a, hipStream_t s) {
    constexpr int RB = 2;
    const int units = (a.I + 4 * RB - 1) / (4 * RB);
    hipLaunchKernelGGL((moe_gateup_kernel<WT, MT, RB, ROUTED>), dim3(a.E * units), dim3(256), 0, s, a);
}
template <typename WT, int MT, bool ROUTED>
static void moe_launch_pair_down(const MoeDecodeArgs& a, hipStream_t s) {
    constexpr int RB = 2;
    const int units = (a.Hout + 4 * RB - 1) / (4 * RB);
    hipLaunchKernelGGL((moe_down_kernel<WT, MT, RB, ROUTED>), dim3(a.E * units), dim3(256), 0, s, a);
}

template <typename WT, bool ROUTED>
static void moe_dispatch(const MoeDecodeArgs& a, hipStream_t s, bool gateup) {
    if (a.max_rows_per_expert <= 1) {
        gateup ? moe_launch_pair_gateup<WT, 1, ROUTED>(a, s) : moe_launch_pair_down<WT, 1, ROUTED>(a, s);
    } else if (a.max_rows_per_expert <= 4) {
        gateup ? moe_launch_pair_gateup<WT, 4, ROUTED>(a, s) : moe_launch_pair_down<WT, 4, ROUTED>(a, s);
    } else {
        gateup ? moe_launch_pair_gateup<WT, 8, ROUTED>(a, s) : moe_launch_pair_down<WT, 8, ROUTED>(a, s);
    }
}

static void moe_dispatch_all(const MoeDecodeArgs& a, hipStream_t s, bool gateup) {
    const bool routed = a.E > 1;
    if (a.wdtype == WDT_BF16) {
        routed ? moe_dispatch<bf16_t, true>(a, s, gateup) : moe_dispatch<bf16_t, false>(a, s, gateup);
    } else {
        routed ? moe_dispatch<f16_t, true>(a, s, gateup) : moe_dispatch<f16_t, false>(a, s, gateup);
    }
}

void launch_moe_gateup_gemv(const MoeDecodeArgs& a, hipStream_t s) { moe_dispatch_all(a, s, true); }
void launch_moe_down_gemv(const MoeDecodeArgs& a, hipStream_t s) { moe_dispatch_all(a, s, false); }

}  // namespace dsocr
