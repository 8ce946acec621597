// Fused decode-step kernels (B pages x 1 token).  One decode step of the reference
// (model/mod.rs:1977-2034 -> block.rs:124-191 x 12 -> lm_head -> select_token_id)
// becomes 7 launches per layer instead of 15:
//   dec_gemv (RMSNorm fused) -> dec_attn (RoPE + KV append + flash-decoding + combine)
//   -> dec_gemv (o_proj + residual) -> dec_gemv (router, norm fused)
//   -> moe_route (softmax top-k + grouping, one block) -> moe_gateup2 (routed + shared)
//   -> moe_down2 (routed + shared + weighted combine + residual)
// Every reduction keeps the reference's f32 order where it is observable
// (top-k weighted sum in top-k order, then + shared, then the residual add).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

ProfEvents& prof_events() {
    static thread_local ProfEvents p;
    return p;
}

// ------------------------------------------------------------------ helpers
// Dynamic LDS of the GEMV-type kernels: [XS_RED floats of row partial sums][M][K staged rows].
constexpr int XS_RED = 128;  // >= M * (blockDim / 64)

// Block-wide: stage M rows of x (row m = rows ? rows[m] : m, stride ldx) into LDS, RMS-normalised
// when nw != null (rms_norm_slow, block.rs:24-29: x / sqrt(mean(x^2) + eps) * w).  Every
// thread of the block must call it (two barriers).
__device__ __forceinline__ void stage_rows(const float* x, long ldx, const int* rows, int M, int K, const float* nw,
                                           float eps, float* smem) {
    float* red = smem;
    float* xs = smem + XS_RED;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwv = blockDim.x >> 6;
    const int step = blockDim.x * 4;
    if (nw) {
        for (int m = 0; m < M; ++m) {
            const float* xr = x + (long)(rows ? rows[m] : m) * ldx;
            float q = 0.f;
            for (int k = tid * 4; k < K; k += step) {
                const float4 v = *reinterpret_cast<const float4*>(xr + k);
                q += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
            }
            q = wave_sum(q);
            if (lane == 0) red[m * nwv + wave] = q;
        }
        __syncthreads();
    }
    for (int m = 0; m < M; ++m) {
        const float* xr = x + (long)(rows ? rows[m] : m) * ldx;
        float den = 1.f;
        if (nw) {
            float q = 0.f;
            for (int w = 0; w < nwv; ++w) q += red[m * nwv + w];
            den = sqrtf(q / (float)K + eps);
        }
        for (int k = tid * 4; k < K; k += step) {
            float4 v = *reinterpret_cast<const float4*>(xr + k);
            if (nw) {
                const float4 w = *reinterpret_cast<const float4*>(nw + k);
                v.x = (v.x / den) * w.x;
                v.y = (v.y / den) * w.y;
                v.z = (v.z / den) * w.z;
                v.w = (v.w / den) * w.w;
            }
            *reinterpret_cast<float4*>(xs + m * K + k) = v;
        }
    }
    __syncthreads();
}

// Two-phase staging for the hot kernels.  vmcnt is in-order on CDNA: a load issued after
// the weight stream can only be consumed once every weight load has landed.  So the
// activation rows (and the norm weight) are loaded into registers FIRST (xload), the weight
// stream is issued next, and xstage then normalises / writes LDS waiting only for the
// activation loads.  XR float4 per thread per row covers K <= XR * 4 * blockDim.
template <int MT, int XR>
struct XRegs {
    float4 v[MT][XR];
    float4 w[XR];
};

template <int MT, int XR>
__device__ __forceinline__ void xload(XRegs<MT, XR>& r, const float* x, long ldx, const int* rows, int M, int K,
                                      const float* nw) {
    const int tid = threadIdx.x, nt = blockDim.x;
    // unconditional loads from clamped addresses (a predicated load becomes an exec-masked
    // branch plus a vmcnt(0) drain in hipcc's output); lanes past K / M are ignored by xstage
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int mm = min(m, M - 1);
        const float* xr = x + (long)(rows ? rows[mm] : mm) * ldx;
#pragma unroll
        for (int i = 0; i < XR; ++i) {
            const int k = min((tid + i * nt) * 4, K - 4);
            r.v[m][i] = *reinterpret_cast<const float4*>(xr + k);
        }
    }
    const float* nwp = nw ? nw : x;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const int k = min((tid + i * nt) * 4, K - 4);
        r.w[i] = *reinterpret_cast<const float4*>(nwp + k);
    }
}

template <int MT, int XR>
__device__ __forceinline__ void xstage(const XRegs<MT, XR>& r, int M, int K, bool norm, float eps, float* smem) {
    float* red = smem;
    float* xs = smem + XS_RED;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nt = blockDim.x, nwv = nt >> 6;
    if (norm) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            if (m < M) {
                float q = 0.f;
#pragma unroll
                for (int i = 0; i < XR; ++i) {
                    const float4 v = r.v[m][i];
                    if ((tid + i * nt) * 4 < K) q += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
                }
                q = wave_sum(q);
                if (lane == 0) red[m * nwv + wave] = q;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        if (m < M) {
            float den = 1.f;
            if (norm) {
                float q = 0.f;
                for (int w = 0; w < nwv; ++w) q += red[m * nwv + w];
                den = sqrtf(q / (float)K + eps);
            }
#pragma unroll
            for (int i = 0; i < XR; ++i) {
                const int k = (tid + i * nt) * 4;
                if (k < K) {
                    float4 v = r.v[m][i];
                    if (norm) {
                        const float4 w = r.w[i];
                        v.x = (v.x / den) * w.x;
                        v.y = (v.y / den) * w.y;
                        v.z = (v.z / den) * w.z;
                        v.w = (v.w / den) * w.w;
                    }
                    *reinterpret_cast<float4*>(xs + m * K + k) = v;
                }
            }
        }
    }
    __syncthreads();
}

// 8 consecutive f32 (LDS or global) into registers
__device__ __forceinline__ void ld_x8(const float* xs, float* o) {
    const float4 a = *reinterpret_cast<const float4*>(xs);
    const float4 b = *reinterpret_cast<const float4*>(xs + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

static size_t stage_bytes(int M, int K) { return sizeof(float) * (XS_RED + (size_t)M * K); }
constexpr size_t STAGE_LDS_MAX = 64 * 1024;

// ------------------------------------------------------------------ dec_gemv
// y[m][n] (+)= act(sum_k xn[m][k] W[n][k] + b[n]); xn = rmsnorm(x) if norm_w else x.
// A wave owns RB rows.  Every lane issues its 16-byte weight loads for the first U*64
// chunks BEFORE the block stages x through LDS, so the HBM latency of the weight
// stream overlaps the norm prologue; K <= 64*U*8 is a single batch.
template <typename WT, int MT, int RB, int U>
__global__ __launch_bounds__(256) void dec_gemv_kernel(DecGemvArgs a) {
    WaveSpan span_(a.span);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = (blockIdx.x * 4 + wave) * RB;
    const bool active = n0 < a.N;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    const int chunks = a.K >> 3;
    constexpr int XR = 2;
    const bool fast = a.K <= XR * 4 * 256;
    XRegs<MT, XR> xr;
    if (fast) xload<MT, XR>(xr, a.x, a.ldx, nullptr, a.M, a.K, a.norm_w);
    // accumulate (residual) rows of one or two tokens: loaded now, with x, instead of after the wave sums
    // (one dependent round trip fewer at the end of o_proj)
    constexpr bool YPRE = MT <= 2;
    float ypre[YPRE ? RB : 1][YPRE ? MT : 1];
    if constexpr (YPRE) {
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m)
                ypre[r][m] = a.accumulate ? a.y[(long)min(m, a.M - 1) * a.ldy + min(n0 + r, a.N - 1)] : 0.f;
    }
    uint4 wq[U][RB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int n = min(n0 + r, a.N - 1);
            wq[u][r] = ldg_nt16(W + (long)n * a.ldw + (min(c, chunks - 1) << 3));
        }
    }
    if (fast) xstage<MT, XR>(xr, a.M, a.K, a.norm_w != nullptr, a.eps, smem);
    else stage_rows(a.x, a.ldx, nullptr, a.M, a.K, a.norm_w, a.eps, smem);
    const float* xs = smem + XS_RED;
    if (a.xn_out && blockIdx.x == 0)  // hand the normalised rows to the next kernel
        for (int i = threadIdx.x * 4; i < a.M * a.K; i += blockDim.x * 4)
            *reinterpret_cast<float4*>(a.xn_out + i) = *reinterpret_cast<const float4*>(xs + i);
    if (!active) return;
    float acc[RB][MT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
    for (int base = 0;;) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = base + u * 64 + lane;
            if (c < chunks) {
                float w8[RB][8];
#pragma unroll
                for (int r = 0; r < RB; ++r) unpack8<WT>(wq[u][r], w8[r]);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < a.M) {
                        float xv[8];
                        ld_x8(xs + m * a.K + (c << 3), xv);
#pragma unroll
                        for (int r = 0; r < RB; ++r)
#pragma unroll
                            for (int j = 0; j < 8; ++j) acc[r][m] = fmaf(xv[j], w8[r][j], acc[r][m]);
                    }
                }
            }
        }
        base += 64 * U;
        if (base >= chunks) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = base + u * 64 + lane;
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int n = min(n0 + r, a.N - 1);
                wq[u][r] = ldg_nt16(W + (long)n * a.ldw + (min(c, chunks - 1) << 3));
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            float v = wave_sum(acc[r][m]);
            const int n = n0 + r;
            if (lane == 0 && m < a.M && n < a.N) {
                v = apply_act(v + (a.bias ? a.bias[n] : 0.f), a.act);
                float* yp = a.y + (long)m * a.ldy + n;
                if (a.accumulate) {
                    if constexpr (YPRE) v = ypre[r][m] + v;
                    else v = *yp + v;
                }
                *yp = v;
            }
        }
}

// Several tokens (M = 3..8): blocks of 4 waves, RB weight rows per wave (issued first), the M
// activation rows staged once per block in LDS — wave w stages rows w and w + 4 in the GEMV chunk
// layout (lane: chunks lane, lane+64, lane+128), RMS-normalising them when NORM (its squares summed
// u-major then j, one wave sum, x / den * w: dec_route_grp's form), so the standalone RMSNorm
// launch disappears.  Per-row arithmetic that of dec_gemv (chunk u-major, then j; wave sum; + bias,
// act, y); rows past M are clamped to row M-1 and discarded, so the MT x RB FMA chains interleave.
template <typename WT, int MT, int RB, bool NORM>
__global__ __launch_bounds__(256) void dec_gemv_lds_kernel(DecGemvArgs a) {
    constexpr int U = 3;
    extern __shared__ __attribute__((aligned(16))) float xs[];  // [MT][K]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = (blockIdx.x * 4 + wave) * RB;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    const int chunks = a.K >> 3;
    uint4 wq[U][RB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int cc = min(u * 64 + lane, chunks - 1);
#pragma unroll
        for (int r = 0; r < RB; ++r) wq[u][r] = ldg_nt16(W + (long)min(n0 + r, a.N - 1) * a.ldw + (cc << 3));
    }
#pragma unroll
    for (int h = 0; h < (MT + 3) / 4; ++h) {
        const int m = wave + 4 * h;
        if (m < a.M) {
            float xv[U][8], nw[U][8];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int cc = min(u * 64 + lane, chunks - 1);
                ld_x8(a.x + (long)m * a.ldx + (cc << 3), xv[u]);
                if (NORM) ld_x8(a.norm_w + (cc << 3), nw[u]);
            }
            if (NORM) {
                float q = 0.f;
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (u * 64 + lane < chunks)
#pragma unroll
                        for (int j = 0; j < 8; ++j) q += xv[u][j] * xv[u][j];
                const float den = sqrtf(wave_sum(q) / (float)a.K + a.eps);
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int j = 0; j < 8; ++j) xv[u][j] = (xv[u][j] / den) * nw[u][j];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = u * 64 + lane;
                if (c < chunks) {
                    float* d = xs + (long)m * a.K + (c << 3);
                    *reinterpret_cast<float4*>(d) = make_float4(xv[u][0], xv[u][1], xv[u][2], xv[u][3]);
                    *reinterpret_cast<float4*>(d + 4) = make_float4(xv[u][4], xv[u][5], xv[u][6], xv[u][7]);
                }
            }
        }
    }
    __syncthreads();
    if (n0 >= a.N) return;
    float acc[RB][MT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
        if (c < chunks) {
            float w8[RB][8];
#pragma unroll
            for (int r = 0; r < RB; ++r) unpack8<WT>(wq[u][r], w8[r]);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                float xv[8];
                ld_x8(xs + (long)min(m, a.M - 1) * a.K + (c << 3), xv);
#pragma unroll
                for (int r = 0; r < RB; ++r)
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[r][m] = fmaf(xv[j], w8[r][j], acc[r][m]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            float v = wave_sum(acc[r][m]);
            const int n = n0 + r;
            if (lane == 0 && m < a.M && n < a.N) {
                v = apply_act(v + (a.bias ? a.bias[n] : 0.f), a.act);
                float* yp = a.y + (long)m * a.ldy + n;
                if (a.accumulate) v = *yp + v;
                *yp = v;
            }
        }
}

// Large-N variant (lm_head: 129280 rows): a fixed grid of waves walks the row groups with a
// two-deep register pipeline (the loads of group i+1 are in flight while group i is
// reduced), so the per-block x staging / norm prologue is paid once per ~8 row groups.
template <typename WT, int U, int RB>
__device__ __forceinline__ void gemv_issue(uint4 (&q)[U][RB], const WT* W, int n0, int N, long ldw, int chunks,
                                           int lane, bool ok) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int n = min(n0 + r, N - 1);
            q[u][r] = ldg_nt16(W + (long)n * ldw + (min(c, chunks - 1) << 3));
            (void)ok;
        }
    }
}

template <typename WT, int MT, int U, int RB>
__device__ __forceinline__ void gemv_finish(const uint4 (&q)[U][RB], const float* xs, const DecGemvArgs& a, int n0,
                                            int chunks, int lane) {
    float acc[RB][MT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
        if (c < chunks) {
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                float w8[8];
                unpack8<WT>(q[u][r], w8);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < a.M) {
                        float xv[8];
                        ld_x8(xs + m * a.K + (c << 3), xv);
#pragma unroll
                        for (int j = 0; j < 8; ++j) acc[r][m] = fmaf(xv[j], w8[j], acc[r][m]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            float v = wave_sum(acc[r][m]);
            const int n = n0 + r;
            if (lane == 0 && m < a.M && n < a.N) {
                v = apply_act(v + (a.bias ? a.bias[n] : 0.f), a.act);
                float* yp = a.y + (long)m * a.ldy + n;
                if (a.accumulate) v = *yp + v;
                *yp = v;
            }
        }
}

template <typename WT, int MT, int RB>
__global__ __launch_bounds__(256) void dec_gemv_stream_kernel(DecGemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int U = 3;  // K <= 1536: one batch per row
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    const int chunks = a.K >> 3;
    const int ngroups = (a.N + RB - 1) / RB;
    const int stride = gridDim.x * 4;
    int g = blockIdx.x * 4 + wave;
    uint4 qa[U][RB], qb[U][RB];
    XRegs<MT, 2> xr;  // K <= 1536 here
    xload<MT, 2>(xr, a.x, a.ldx, nullptr, a.M, a.K, a.norm_w);
    gemv_issue<WT, U, RB>(qa, W, g * RB, a.N, a.ldw, chunks, lane, g < ngroups);
    xstage<MT, 2>(xr, a.M, a.K, a.norm_w != nullptr, a.eps, smem);
    const float* xs = smem + XS_RED;
    for (; g < ngroups; g += 2 * stride) {
        const int g2 = g + stride, g3 = g2 + stride;
        gemv_issue<WT, U, RB>(qb, W, g2 * RB, a.N, a.ldw, chunks, lane, g2 < ngroups);
        gemv_finish<WT, MT, U, RB>(qa, xs, a, g * RB, chunks, lane);
        if (g2 >= ngroups) break;
        gemv_issue<WT, U, RB>(qa, W, g3 * RB, a.N, a.ldw, chunks, lane, g3 < ngroups);
        gemv_finish<WT, MT, U, RB>(qb, xs, a, g2 * RB, chunks, lane);
    }
}

template <typename WT, int MT>
static void dec_gemv_rb(const DecGemvArgs& a, hipStream_t s) {
    const size_t lds = stage_bytes(a.M, a.K);
    if constexpr (MT >= 4 && MT <= 8) {  // several tokens: no LDS staging
        // matrix-core form (decode_mm.hip): weights straight into MFMA, activations as 16-bit planes
        if (dec_mm_ok(a)) {
            launch_dec_mm(a, s);
            return;
        }
        // rows per wave of dec_gemv_lds, measured on MI355X at M = 8, K = 1280 (tools/kbench gemv8): 2 for
        // N = 3840 (8.4 us, 11.1 with the norm fused vs 5 + 10.6 for a separate RMSNorm), 1 for N = 1280 (5.9)
        const int rows_rb = a.N >= 2560 ? 2 : 1;
        if (a.N <= 16384 && !a.xn_out && a.K <= 64 * 3 * 8 && a.K % 8 == 0) {
            const size_t xl = sizeof(float) * MT * (size_t)a.K;
#define DSOCR_GR(R)                                                                                                   \
    do {                                                                                                              \
        const dim3 g((a.N + 4 * R - 1) / (4 * R));                                                                    \
        if (a.norm_w) DSOCR_LAUNCH((dec_gemv_lds_kernel<WT, MT, R, true>), g, dim3(256), xl, s, a);                   \
        else DSOCR_LAUNCH((dec_gemv_lds_kernel<WT, MT, R, false>), g, dim3(256), xl, s, a);                           \
    } while (0)
            if (rows_rb == 1) DSOCR_GR(1); else DSOCR_GR(2);
#undef DSOCR_GR
            return;
        }
    }
    // small N: one row per wave so the whole matrix is in flight at once; large N: RB rows per wave
    if (a.N <= 16384) {
        constexpr int RB = 1;
        DSOCR_LAUNCH((dec_gemv_kernel<WT, MT, RB, 3>), dim3((a.N + 4 * RB - 1) / (4 * RB)), dim3(256), lds, s, a);
    } else if (a.K <= 64 * 3 * 8 && MT <= 2) {
        constexpr int RB = 4;
        // exactly one resident wave of blocks (no tail of late-starting blocks)
        static int resident = 0;
        if (!resident) {
            int per_cu = 0, dev = 0, cus = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dec_gemv_stream_kernel<WT, MT, RB>, 256, lds);
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            resident = std::max(1, per_cu) * std::max(1, cus);
        }
        const int groups = (a.N + RB - 1) / RB;
        const int blocks = std::min((groups + 3) / 4, resident);
        DSOCR_LAUNCH((dec_gemv_stream_kernel<WT, MT, RB>), dim3(blocks), dim3(256), lds, s, a);
    } else {
        constexpr int RB = MT <= 2 ? 4 : 2;
        DSOCR_LAUNCH((dec_gemv_kernel<WT, MT, RB, 3>), dim3((a.N + 4 * RB - 1) / (4 * RB)), dim3(256), lds, s, a);
    }
}
template <typename WT>
static void dec_gemv_dispatch(const DecGemvArgs& a, hipStream_t s) {
    if (a.M <= 1) dec_gemv_rb<WT, 1>(a, s);
    else if (a.M <= 2) dec_gemv_rb<WT, 2>(a, s);
    else if (a.M <= 4) dec_gemv_rb<WT, 4>(a, s);
    else if (a.M <= 8) dec_gemv_rb<WT, 8>(a, s);
    else dec_gemv_rb<WT, 16>(a, s);
}
void launch_dec_gemv(const DecGemvArgs& a, hipStream_t s) {
    if (a.M == 0 || a.N == 0) return;
    // rows per launch: <= 16 and the staged rows must fit the 64 KB dynamic LDS window
    const int per = (int)std::min<size_t>(16, (STAGE_LDS_MAX - sizeof(float) * XS_RED) / (sizeof(float) * a.K));
    if (per < 1) throw std::runtime_error("EINVAL: dec_gemv K too large for LDS staging");
    for (int m0 = 0; m0 < a.M; m0 += per) {
        DecGemvArgs p = a;
        p.M = std::min(per, a.M - m0);
        p.x = a.x + (long)m0 * a.ldx;
        p.y = a.y + (long)m0 * a.ldy;
        if (a.wdtype == WDT_BF16) dec_gemv_dispatch<bf16_t>(p, s);
        else dec_gemv_dispatch<f16_t>(p, s);
    }
}

// ------------------------------------------------------------------ q/k/v projection + RoPE
// dec_gemv for the fused q/k/v rows with the rotation (rotate_half RoPE, block.rs:1403-1471) in
// the epilogue: a wave owns the row pair (d, d + HD/2) of one head segment, so both halves of
// the rotation meet in one lane; q and k segments are rotated at the decode position, v rows pass
// through.  The per-row arithmetic is dec_gemv's (chunk u-major, then j), the rotation is the
// attention kernel's formula x*cos + sign*partner*sin.  One token (M = 1).
// (Every wave normalising the row itself, without LDS or a block barrier, measured +0.75 us per layer:
// the block-staged row is read from LDS, not re-read from L2 by each wave.)
// SC1: the rows are handed to attention blocks of the same launch (dec_qkv_attn): stored write-through
template <typename WT, bool SC1>
__device__ __forceinline__ void qkv_rope_body(const DecGemvArgs& a, const DecRopeEpi& r, int bid) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int U = 3, XR = 2;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int half = r.hd / 2;
    const int p = bid * 4 + wave;                        // pair index
    const int npairs = a.N / 2;
    const bool active = p < npairs;
    const int pp = min(p, npairs - 1);
    const int n0 = (pp / half) * r.hd + pp % half, n1 = n0 + half;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    const int chunks = a.K >> 3;
    XRegs<1, XR> xr;
    xload<1, XR>(xr, a.x, a.ldx, nullptr, 1, a.K, a.norm_w);
    const int pos = r.kv_pos[0];
    uint4 w0[U], w1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int cc = min(u * 64 + lane, chunks - 1);
        w0[u] = ldg_nt16(W + (long)n0 * a.ldw + (cc << 3));
        w1[u] = ldg_nt16(W + (long)n1 * a.ldw + (cc << 3));
    }
    const int d = n0 % r.hd;
    const bool rot = n0 < r.rot_rows;
    const float c0 = rot ? r.cos[(long)pos * r.hd + d] : 1.f, s0 = rot ? r.sin[(long)pos * r.hd + d] : 0.f;
    const float c1 = rot ? r.cos[(long)pos * r.hd + d + half] : 1.f, s1 = rot ? r.sin[(long)pos * r.hd + d + half] : 0.f;
    xstage<1, XR>(xr, 1, a.K, a.norm_w != nullptr, a.eps, smem);
    if (!active) return;
    const float* xs = smem + XS_RED;
    float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int cc = u * 64 + lane;
        if (cc < chunks) {
            float f0[8], f1[8], xv[8];
            unpack8<WT>(w0[u], f0);
            unpack8<WT>(w1[u], f1);
            ld_x8(xs + (cc << 3), xv);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc0 = fmaf(xv[j], f0[j], acc0);
                acc1 = fmaf(xv[j], f1[j], acc1);
            }
        }
    }
    float y0 = wave_sum(acc0), y1 = wave_sum(acc1);
    if (lane == 0) {
        y0 = y0 + (a.bias ? a.bias[n0] : 0.f);
        y1 = y1 + (a.bias ? a.bias[n1] : 0.f);
        if (rot) {
            const float o0 = y0 * c0 + (-1.f * y1) * s0;
            const float o1 = y1 * c1 + (1.f * y0) * s1;
            y0 = o0;
            y1 = o1;
        }
        if (SC1) {
            __hip_atomic_store(a.y + n0, y0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.y + n1, y1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            a.y[n0] = y0;
            a.y[n1] = y1;
        }
    }
}

template <typename WT>
__global__ __launch_bounds__(256) void dec_qkv_rope_kernel(DecGemvArgs a, DecRopeEpi r) {
    qkv_rope_body<WT, false>(a, r, blockIdx.x);
}

bool dec_qkv_rope_ok(const DecGemvArgs& a, const DecRopeEpi& r) {
    return a.M == 1 && r.hd % 2 == 0 && a.N % r.hd == 0 && a.K % 8 == 0 && a.K <= 64 * 3 * 8 && r.kv_pos && r.cos &&
           r.sin;
}

void launch_dec_qkv_rope(const DecGemvArgs& a, const DecRopeEpi& r, hipStream_t s) {
    if (!dec_qkv_rope_ok(a, r)) throw std::runtime_error("EINVAL: dec_qkv_rope outside its range");
    const size_t lds = stage_bytes(1, a.K);
    dim3 grid((a.N / 2 + 3) / 4);
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((dec_qkv_rope_kernel<bf16_t>), grid, dim3(256), lds, s, a, r);
    else DSOCR_LAUNCH((dec_qkv_rope_kernel<f16_t>), grid, dim3(256), lds, s, a, r);
}

// ------------------------------------------------------------------ router + top-k
// MoE router logits (E x K GEMV, norm fused) whose LAST-arriving block routes every token:
// softmax (or sigmoid) + greedy top-k (block.rs:1254-1301) -> ids[t*topk+k], w[t*topk+k].
// Logits are stored write-through (sc1 atomics) so the hand-off needs only the arrival
// ticket and one agent acquire in the last block (cdna_hip_programming.md Guideline 16 R1).
__device__ __forceinline__ void topk_write(const float* lg, int E, int K, int softmax_scoring, int norm_topk,
                                           float scaling, int* ids, float* w, bool sc1 = false) {
    const int lane = threadIdx.x & 63;
    float sc[4];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = min(lane + 64 * j, E - 1);
        // sc1: logits handed over inside the launch (stored sc1 by other blocks)
        sc[j] = sc1 ? __hip_atomic_load(lg + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : lg[e];
        if (lane + 64 * j >= E) sc[j] = -INFINITY;
        mx = fmaxf(mx, sc[j]);
    }
    if (softmax_scoring) {
        mx = wave_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sc[j] = (lane + 64 * j) < E ? expf(sc[j] - mx) : 0.f;
            sum += sc[j];
        }
        sum = wave_sum(sum);
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[j] = (lane + 64 * j) < E ? sc[j] / sum : -INFINITY;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[j] = (lane + 64 * j) < E ? 1.0f / (1.0f + expf(-sc[j])) : -INFINITY;
    }
    float picked[8];
    int pid[8];
    float wsum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        picked[k] = 0.f;
        pid[k] = 0;
        if (k < K) {
            float bv = -INFINITY;
            int bi = 0x7fffffff;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int e = lane + 64 * j;
                if (e < E && (sc[j] > bv || (sc[j] == bv && e < bi))) { bv = sc[j]; bi = e; }
            }
            wave_argmax(bv, bi);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (lane + 64 * j == bi) sc[j] = -INFINITY;
            picked[k] = bv;
            pid[k] = bi;
            wsum += bv;
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k < K) {
                float v = picked[k];
                if (K > 1 && norm_topk) v = v / (wsum + 1e-20f);
                if (scaling != 1.0f) v = v * scaling;
                ids[k] = pid[k];
                w[k] = v;
            }
        }
    }
}

template <typename WT, int MT>
__global__ __launch_bounds__(256) void dec_router_kernel(DecGemvArgs a, DecRouteEpi r) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ int last_s;
    constexpr int U = 3, XR = 2;  // K <= 1536
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = blockIdx.x * 4 + wave;
    const bool active = n < a.N;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    const int chunks = a.K >> 3;
    XRegs<MT, XR> xr;
    xload<MT, XR>(xr, a.x, a.ldx, nullptr, a.M, a.K, a.norm_w);
    uint4 wq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) wq[u] = ldg_nt16(W + (long)min(n, a.N - 1) * a.ldw + (min(u * 64 + lane, chunks - 1) << 3));
    xstage<MT, XR>(xr, a.M, a.K, a.norm_w != nullptr, a.eps, smem);
    const float* xs = smem + XS_RED;
    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
        if (c < chunks) {
            float w8[8];
            unpack8<WT>(wq[u], w8);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < a.M) {
                    float xv[8];
                    ld_x8(xs + m * a.K + (c << 3), xv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[m] = fmaf(xv[j], w8[j], acc[m]);
                }
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const float v = wave_sum(acc[m]) + (a.bias ? a.bias[min(n, a.N - 1)] : 0.f);
        if (lane == 0 && active && m < a.M)
            __hip_atomic_store(a.y + (long)m * a.ldy + n, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(r.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (int)gridDim.x - 1;
        if (last) __hip_atomic_store(r.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
    // every logit was stored sc1 and is read back with sc1 loads: no acquire fence needed
    // (MI355X_MICROARCH.md, hand-offs with sc1 loads in place of the acquire, first row)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!r.grp) {
        for (int t = wave; t < a.M; t += 4)
            topk_write(a.y + (long)t * a.ldy, a.N, r.topk, r.softmax_scoring, r.norm_topk, r.scaling,
                       r.ids + t * r.topk, r.w + t * r.topk, true);
        return;
    }
    // picks into LDS, then wave 0 groups them by expert (records in increasing expert order, the
    // tokens of a record in increasing order: the h rows t*topk + k are scanned in order)
    __shared__ int ids_s[64];
    __shared__ float w_s[64];
    for (int t = wave; t < a.M; t += 4)
        topk_write(a.y + (long)t * a.ldy, a.N, r.topk, r.softmax_scoring, r.norm_topk, r.scaling, ids_s + t * r.topk,
                   w_s + t * r.topk, true);
    __syncthreads();
    const int TK = a.M * r.topk;
    if (threadIdx.x < TK) {
        r.ids[threadIdx.x] = ids_s[threadIdx.x];
        r.w[threadIdx.x] = w_s[threadIdx.x];
    }
    if (wave == 0) {
        int base = 0;
        for (int e0 = 0; e0 < a.N; e0 += 64) {
            const int e = e0 + lane;
            int cnt = 0;
            for (int i = 0; i < TK; ++i) cnt += ids_s[i] == e ? 1 : 0;
            const unsigned long long act = __ballot(cnt > 0 && e < a.N);
            const int s = base + __popcll(act & ((1ull << lane) - 1ull));
            if (cnt > 0 && e < a.N) {
                int* rec = r.grp + MOE_GRP_REC * (1 + s);
                rec[0] = e;
                rec[1] = cnt;
                int n = 0;
                for (int i = 0; i < TK; ++i)
                    if (ids_s[i] == e) {
                        rec[2 + n] = i;
                        rec[10 + n] = __float_as_int(w_s[i]);
                        ++n;
                    }
            }
            base += __popcll(act);
        }
        if (lane == 0) r.grp[0] = base;
    }
}

bool dec_router_ok(int T, int E, int K, int topk) {
    return T <= 8 && E <= 256 && K <= 64 * 3 * 8 && topk <= 8 && T * topk <= 64;
}

// Decode router for T <= 8 tokens, E <= 64 experts: RMSNorm + router logits + greedy top-k +
// expert records in one launch.  Blocks of 8 waves and 8 expert rows.  Wave w normalises token row w
// in the GEMV chunk layout (lane: chunks lane, lane+64, lane+128; its squares summed u-major then j,
// one wave sum, x / den * w — dec_gemv_rows' NORM form) in registers and puts expert row w of the
// block into LDS; then wave w dots its token row with the block's 8 expert rows (dec_gemv's per-row
// arithmetic; the last block also hands the rows to the expert kernels: xn_out).  Logits are stored write-through (sc1); the last block to
// take its ticket reads them back with sc1 loads (MI355X_MICROARCH.md hand-offs, first row), routes
// token w on wave w (topk_wave64) and wave 0 groups the picks by expert (MOE_GRP_* records).
template <typename WT>
__global__ __launch_bounds__(512) void dec_route_grp_kernel(DecGemvArgs a, DecRouteEpi r) {
    WaveSpan span_(a.span);
    constexpr int U = 3, MT = 8;  // K <= 1536, T <= 8
    extern __shared__ __attribute__((aligned(16))) uint4 ws[];  // [8 experts][K / 8] 16-bit weight chunks
    __shared__ float lg_s[MT][64];
    __shared__ __attribute__((aligned(16))) float rank_s[MT][128];
    __shared__ int ids_s[64];
    __shared__ float w_s[64];
    __shared__ int last_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#define RG_STAMP(i)                                                      \
    if (r.stamps && tid == 0 && (blockIdx.x == 0 || (i) >= 5)) r.stamps[i] = __builtin_amdgcn_s_memrealtime();
    RG_STAMP(0);
    const int n0 = blockIdx.x * MT;
    const int chunks = a.K >> 3;
    const WT* W = reinterpret_cast<const WT*>(a.W);
    // wave w: expert row n0 + w into LDS (16-bit, as stored) and token row w normalised in registers; then
    // every wave dots its token row with the block's 8 expert rows.  The products and their order per
    // (token, expert) are dec_gemv's (lane chunks u-major, then j; one wave sum); the LDS traffic is the
    // 16-bit weights once per wave instead of the f32 token rows once per expert (half the bytes)
    uint4 wq[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        wq[u] = ldg_nt16(W + (long)min(n0 + wave, a.N - 1) * a.ldw + (min(u * 64 + lane, chunks - 1) << 3));
    float xv[U][8];
    if (wave < a.M) {
        float nw[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int cc = min(u * 64 + lane, chunks - 1);
            ld_x8(a.x + (long)wave * a.ldx + (cc << 3), xv[u]);
            if (a.norm_w) ld_x8(a.norm_w + (cc << 3), nw[u]);
        }
        if (a.norm_w) {
            float q = 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u * 64 + lane < chunks)
#pragma unroll
                    for (int j = 0; j < 8; ++j) q += xv[u][j] * xv[u][j];
            const float den = sqrtf(wave_sum(q) / (float)a.K + a.eps);
            RG_STAMP(1);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[u][j] = (xv[u][j] / den) * nw[u][j];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u * 64 + lane;
        if (c < chunks) ws[wave * chunks + c] = wq[u];
    }
    __syncthreads();
    RG_STAMP(2);
    RG_STAMP(3);
    float mine = 0.f;  // lane e keeps expert n0 + e's logit for token `wave`
    if (wave < a.M) {
        float acc[MT];
#pragma unroll
        for (int e = 0; e < MT; ++e) acc[e] = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = u * 64 + lane;
            if (c < chunks) {
#pragma unroll
                for (int e = 0; e < MT; ++e) {
                    float w8[8];
                    unpack8<WT>(ws[e * chunks + c], w8);
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[e] = fmaf(xv[u][j], w8[j], acc[e]);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < MT; ++e) {
            const float v = wave_sum(acc[e]) + (a.bias ? a.bias[min(n0 + e, a.N - 1)] : 0.f);
            if (lane == e) mine = v;
        }
    }
    RG_STAMP(4);
    if (wave < a.M && lane < MT && n0 + lane < a.N)
        __hip_atomic_store(a.y + (long)wave * a.ldy + n0 + lane, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int old = __hip_atomic_fetch_add(r.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (int)gridDim.x - 1;
        if (last) __hip_atomic_store(r.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below
    RG_STAMP(5);
    {
        const int m = tid >> 6, e = tid & 63;  // 512 threads: one logit each
        lg_s[m][e] = (m < a.M && e < a.N)
                         ? __hip_atomic_load(a.y + (long)m * a.ldy + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : -INFINITY;
    }
    __syncthreads();
    if (wave < a.M)
        topk_wave64(lg_s[wave][lane], a.N, r.topk, r.softmax_scoring, r.norm_topk, r.scaling, rank_s[wave],
                    ids_s + wave * r.topk, w_s + wave * r.topk);
    __syncthreads();
    RG_STAMP(6);
    const int TK = a.M * r.topk;
    if (tid < TK) {
        r.ids[tid] = ids_s[tid];
        r.w[tid] = w_s[tid];
    }
    // wave 0, lane e: the tokens that picked expert e (a token's picks are distinct, so at most one
    // per token), in increasing token order -> record s = number of picked experts below e
    if (wave == 0 && r.grp)  // scratch: wave 0's rank keys (read by now)
        group_picks_wave64<0>(ids_s, w_s, a.M, r.topk, a.N, r.grp, reinterpret_cast<int*>(&rank_s[0][0]));
    // the normalised rows for the expert kernels, from this (last) block's registers after its last barrier: a
    // global store before a barrier makes the barrier wait for its acknowledgement
    if (a.xn_out && wave < a.M)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = u * 64 + lane;
            if (c < chunks) {
                float* g = a.xn_out + (long)wave * a.K + (c << 3);
                *reinterpret_cast<float4*>(g) = make_float4(xv[u][0], xv[u][1], xv[u][2], xv[u][3]);
                *reinterpret_cast<float4*>(g + 4) = make_float4(xv[u][4], xv[u][5], xv[u][6], xv[u][7]);
            }
        }
    RG_STAMP(7);
#undef RG_STAMP
}

bool dec_route_grp_ok(int T, int E, int K, int topk) {
    return T >= 1 && T <= 8 && E >= 1 && E <= 64 && K % 8 == 0 && K <= 64 * 3 * 8 && topk >= 1 && topk <= 8 &&
           topk <= E && T * topk <= 64;
}

void launch_dec_route_grp(const DecGemvArgs& a, const DecRouteEpi& r, hipStream_t s) {
    if (!dec_route_grp_ok(a.M, a.N, a.K, r.topk) || !r.ids || !r.w || !r.counter || !a.y)
        throw std::runtime_error("EINVAL: decode router (grouped) outside its range");
    dim3 grid((a.N + 7) / 8);
    const size_t lds = sizeof(uint16_t) * 8 * (size_t)a.K;
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((dec_route_grp_kernel<bf16_t>), grid, dim3(512), lds, s, a, r);
    else DSOCR_LAUNCH((dec_route_grp_kernel<f16_t>), grid, dim3(512), lds, s, a, r);
}

void launch_dec_router(const DecGemvArgs& a, const DecRouteEpi& r, hipStream_t s) {
    if (!dec_router_ok(a.M, a.N, a.K, r.topk) || !r.counter) throw std::runtime_error("EINVAL: dec_router out of range");
    const int mt = a.M == 1 ? 1 : (a.M <= 2 ? 2 : (a.M <= 4 ? 4 : 8));
    const size_t lds = stage_bytes(mt, a.K);
    dim3 grid((a.N + 3) / 4);
#define DSOCR_RT(WTY, MTV) DSOCR_LAUNCH((dec_router_kernel<WTY, MTV>), grid, dim3(256), lds, s, a, r)
    if (a.wdtype == WDT_BF16) {
        if (mt == 1) DSOCR_RT(bf16_t, 1); else if (mt == 2) DSOCR_RT(bf16_t, 2);
        else if (mt == 4) DSOCR_RT(bf16_t, 4); else DSOCR_RT(bf16_t, 8);
    } else {
        if (mt == 1) DSOCR_RT(f16_t, 1); else if (mt == 2) DSOCR_RT(f16_t, 2);
        else if (mt == 4) DSOCR_RT(f16_t, 4); else DSOCR_RT(f16_t, 8);
    }
#undef DSOCR_RT
}

// ------------------------------------------------------------------ decode attention
// grid (chunks of 64 keys, heads, B).  The token being decoded sits at pos = kv_pos[b]: q and the new
// k are rotated here (rotate_half RoPE, block.rs:1403-1471) unless the projection's epilogue already
// did (PREROT, one page: dec_qkv_rope); the block owning chunk pos/64 appends k, v to the f32 cache
// (block.rs:776-789) and uses them directly.  Each block issues its K and V cache loads first, then
// builds q; the chunk partials of a (page, head) are merged by chunk 0's block polling them (POLL, <= 24
// chunks of 128-dim heads) or by the last arriver of a ticket (flash-decoding combine).
// phase clock (DecAttn2Args::stamps): thread 0 of each block stores s_memrealtime into the block's own
// 8-word record (no atomics: 680 blocks on one word serialised the launch)
__device__ __forceinline__ void da_stamp(unsigned long long* st, int slot) {
    if (!st || threadIdx.x != 0) return;
    const long blk = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
    st[blk * 8 + slot] = __builtin_amdgcn_s_memrealtime();
}

constexpr int DA_CH = 64;       // keys per block
constexpr int DA2_CH_MIN = DA_CH;
constexpr uint32_t DA_SENT = 0x7FBADBADu;  // "record word not written yet" (a NaN payload no arithmetic produces)

// sum over aligned groups of N lanes (N = 4 or 8), result in every lane of the group
template <int N>
__device__ __forceinline__ float group_sum(float v) {
    v += dpp_f<DPP_QUAD_XOR1>(0.f, v);
    v += dpp_f<DPP_QUAD_XOR2>(0.f, v);
    if (N == 8) v += dpp_f<DPP_ROW_HALF_MIRROR>(0.f, v);
    return v;
}

// FUSED (dec_qkv_attn, one page, PREROT + POLL): q and the new k / v come from q/k/v blocks of the
// same launch, stored write-through into a row that enters the launch sentinel-filled; this block
// issues its K / V cache loads first, then polls its rows until no word holds the sentinel, and the
// merging block (chunk 0) refills them once every chunk of the head has read them (its record is
// written after that read).  The cache stream overlaps the projection's weight stream.
template <int HD, bool PREROT, bool POLL, bool FUSED>
__device__ __forceinline__ void dec_attn_body(const DecAttn2Args& a, const int c, const int h, const int b) {
    constexpr int CH = DA_CH;
    constexpr int LPK = 256 / CH;                                // lanes per key when scoring
    constexpr int DPL = HD / LPK;                                // dims per lane when scoring
    constexpr int DG = HD / 4, KG = 256 / DG, KPG = CH / KG;     // PV: float4 dim groups x key groups
    static_assert(KPG >= 1 && DPL % 4 == 0, "unsupported head_dim");
    __shared__ float qs[HD];
    __shared__ float knew[HD];
    __shared__ float vnew[HD];
    __shared__ float p_s[CH];
    __shared__ float red[8];
    __shared__ int last_s;
    __shared__ float4 o_s[384];  // P.V partials; reused by the combine (m, l per chunk + per-group sums)
    const int k0 = c * CH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kvh = h / (a.heads / a.kv_heads);
    float* Kc = a.kc + (long)b * a.page_stride + (long)kvh * a.head_stride;
    float* Vc = a.vc + (long)b * a.page_stride + (long)kvh * a.head_stride;
    // 1. the chunk's K / V cache loads (keys clamped to the position: keys past it are masked at use)
    const int key = tid / LPK, sub = tid % LPK;
    const int dg = tid % DG, kg = tid / DG;
    float4 kreg[DPL / 4];
    float4 vreg[KPG];
    // TK (128-dim heads): K is loaded like V, instruction i of wave w reading keys w*16 + 2i and
    // w*16 + 2i + 1 whole (1 KiB contiguous per instruction: 8 L2 lines, where one key per 4 lanes touched
    // 64 lines per instruction); lane l holds dims 4 (l & 31) .. + 3 of key tk_key(i) = w*16 + 2i + (l >> 5),
    // and the q.k dot products are finished by a transposing butterfly over the 32 lanes of a key
    // (9 swizzle / DPP adds for 8 keys).
    constexpr bool TK = HD == 128;
    const int tk_half = lane >> 5, tk_d4 = (lane & 31) * 4;
    auto tk_key = [&](int i) { return wave * 16 + 2 * i + tk_half; };
    auto issue_k = [&](int kb, int klim) {
        if constexpr (TK) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                kreg[i] = ldg_nt_f4(Kc + (long)min(kb + tk_key(i), klim) * HD + tk_d4);
        } else {
            const float4* kp = reinterpret_cast<const float4*>(Kc + (long)min(kb + key, klim) * HD + sub * DPL);
#pragma unroll
            for (int i = 0; i < DPL / 4; ++i) kreg[i] = kp[i];
        }
    };
    auto issue_v = [&](int kb, int klim) {
#pragma unroll
        for (int j = 0; j < KPG; ++j) {
            const int kk = min(kb + (TK ? tk_key(j) : kg * KPG + j), klim);
            vreg[j] = ldg_nt_f4(Vc + (long)kk * HD + dg * 4);
        }
    };
    const float* row = a.qkv + (long)b * a.ld;
    float q_pre = 0.f, k_pre = 0.f, v_pre = 0.f;
    if (PREROT && !FUSED) {  // unconditional (every thread loads a valid element): one round trip with pos
        const int td = tid & (HD - 1);
        q_pre = row[h * HD + td];
        k_pre = row[a.heads * HD + kvh * HD + td];
        v_pre = row[(a.heads + a.kv_heads) * HD + kvh * HD + td];
    }
    const int pos = a.kv_pos[b];
    const int len = pos + 1;
    if (k0 >= len) return;
    if (FUSED && a.kv_delay > 0) {
        // the projection blocks' weight stream first: this block's K / V cache loads wait kv_delay ticks
        // (s_memrealtime, 10 ns) so the two streams do not share HBM while q is still being computed
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)a.kv_delay) __builtin_amdgcn_s_sleep(2);
    }
    issue_k(k0, min(k0 + CH, len) - 1);
    issue_v(k0, min(k0 + CH, len) - 1);
    const bool own = pos >= k0 && pos < k0 + CH;
    bool gave_up = false;
    if constexpr (FUSED) {
        // the head's q (and, owning the position, the new k / v) from this launch's projection blocks
        const int td = tid & (HD - 1);
        const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), (short)0,
                                                          (a.heads + 2 * a.kv_heads) * HD * 4, 0x00020000);
        const int oq = (h * HD + td) * 4, ok = ((a.heads + kvh) * HD + td) * 4,
                  ov = ((a.heads + a.kv_heads + kvh) * HD + td) * 4;
        for (unsigned it = 0;; ++it) {
            asm volatile("" ::: "memory");
            bool pend = false;
            if (tid < HD) {  // waves 0..HD/64-1 poll (the others only join the vote): half the polling traffic
                q_pre = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, oq, 0, 16));
                k_pre = own ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, ok, 0, 16)) : 0.f;
                v_pre = own ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, ov, 0, 16)) : 0.f;
                pend = __float_as_uint(q_pre) == DA_SENT || __float_as_uint(k_pre) == DA_SENT ||
                       __float_as_uint(v_pre) == DA_SENT;
            }
            if (!__syncthreads_or(pend)) break;
            if (it > (1u << 20)) {
                if (tid == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gave_up = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        da_stamp(a.stamps, 2);
    }
    // a block that gave up (the error flag is set; the host raises after the step) leaves the K / V cache
    // untouched: sentinel q / k / v never enter the cache.  It still writes its record so the merge of its
    // head does not wait out a second bounded spin.
    const bool write_kv = own && !gave_up;
    const int nc = (len + CH - 1) / CH;
    // 2. RoPE inputs
    const float* krow = row + a.heads * HD + kvh * HD;
    const float* vrow = row + (a.heads + a.kv_heads) * HD + kvh * HD;
    float qx = 0.f, qr = 0.f, kx = 0.f, kr = 0.f, vx = 0.f, cs = 1.f, sn = 0.f, sg = 0.f;
    if (PREROT) {
        if (tid < HD) {
            qs[tid] = q_pre;
            if (own) {
                knew[tid] = k_pre;
                vnew[tid] = v_pre;
                if (write_kv && h == kvh * (a.heads / a.kv_heads)) {  // one writer per kv head
                    Kc[(long)pos * HD + tid] = k_pre;
                    Vc[(long)pos * HD + tid] = v_pre;
                }
            }
        }
    } else if (tid < HD) {
        int ix = tid, ir = tid;
        if (tid < a.rope_dim) {
            const int half = a.rope_dim / 2;
            auto map = [&](int i) { return !a.use_mla ? i : (i < half ? 2 * i : 2 * (i - half) + 1); };
            ix = map(tid);
            ir = tid < half ? map(tid + half) : map(tid - half);
            sg = tid < half ? -1.f : 1.f;
            cs = a.cos[(long)pos * a.rope_dim + tid];
            sn = a.sin[(long)pos * a.rope_dim + tid];
        }
        qx = row[h * HD + ix];
        qr = row[h * HD + ir];
        if (own) {
            kx = krow[ix];
            kr = krow[ir];
            vx = vrow[tid];
        }
    }
    // 3. rotated q (and the new k, v in the owning chunk): x*cos + sign*partner*sin
    if (!PREROT && tid < HD) {
        qs[tid] = qx * cs + (sg * qr) * sn;
        if (own) {
            const float kv = kx * cs + (sg * kr) * sn;
            knew[tid] = kv;
            vnew[tid] = vx;
            if (h == kvh * (a.heads / a.kv_heads)) {  // one writer per kv head
                Kc[(long)pos * HD + tid] = kv;
                Vc[(long)pos * HD + tid] = vx;
            }
        }
    }
    __syncthreads();
    const int kn = min(CH, len - k0);
    // 4. scores: LPK lanes per key, wave w owns keys w*CH/4 .. (w+1)*CH/4 - 1
    if constexpr (TK) {
        const float4 q4 = *reinterpret_cast<const float4*>(qs + tk_d4);
        const float4 kn4 = *reinterpret_cast<const float4*>(knew + tk_d4);
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 k4 = k0 + tk_key(i) == pos ? kn4 : kreg[i];
            v[i] = fmaf(q4.w, k4.w, fmaf(q4.z, k4.z, fmaf(q4.y, k4.y, q4.x * k4.x)));
        }
        // butterfly: after the xor-16 / 8 / 4 steps lane l holds key i = b2 + 2 b3 + 4 b4 (bits of l)
        // summed over its 8 lanes of that bit pattern; the quad sum finishes the 32 lanes
        const int b4 = (lane >> 4) & 1, b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1;
        float u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float keep = b4 ? v[j + 4] : v[j], send = b4 ? v[j] : v[j + 4];
            u[j] = keep + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), 0x1f | (16 << 10)));
        }
        float t[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float keep = b3 ? u[j + 2] : u[j], send = b3 ? u[j] : u[j + 2];
            t[j] = keep + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), 0x1f | (8 << 10)));
        }
        float r;
        {
            const float keep = b2 ? t[1] : t[0], send = b2 ? t[0] : t[1];
            r = keep + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), 0x1f | (4 << 10)));
        }
        r = group_sum<4>(r);
        const int kk = tk_key(b2 + 2 * b3 + 4 * b4);
        const float sc = kk < kn ? r * a.scale : -INFINITY;
        if ((lane & 3) == 0) p_s[kk] = sc;
        const float mw = wave_max(sc);
        if (lane == 0) red[wave] = mw;
    } else {
        float acc = 0.f;
        if (key < kn) {
            if (k0 + key == pos) {
#pragma unroll
                for (int i = 0; i < DPL; ++i) acc = fmaf(qs[sub * DPL + i], knew[sub * DPL + i], acc);
            } else {
#pragma unroll
                for (int i = 0; i < DPL / 4; ++i) {
                    acc = fmaf(qs[sub * DPL + 4 * i + 0], kreg[i].x, acc);
                    acc = fmaf(qs[sub * DPL + 4 * i + 1], kreg[i].y, acc);
                    acc = fmaf(qs[sub * DPL + 4 * i + 2], kreg[i].z, acc);
                    acc = fmaf(qs[sub * DPL + 4 * i + 3], kreg[i].w, acc);
                }
            }
        }
        acc = group_sum<LPK>(acc);
        const float sc = key < kn ? acc * a.scale : -INFINITY;
        if (sub == 0) p_s[key] = sc;
        const float mw = wave_max(sc);
        if (lane == 0) red[wave] = mw;
    }
    __syncthreads();
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (wave == 0) {  // whole wave active for the DPP reduction
        const float p = (tid < CH && tid < kn) ? expf(p_s[tid] - m) : 0.f;
        if (tid < CH) p_s[tid] = p;
        const float l = wave_sum(p);
        if (tid == 0) red[4] = l;
    }
    __syncthreads();
    if (!FUSED) da_stamp(a.stamps, 2);  // standalone: the chunk's scores and softmax done (K landed)
    // 5. P.V over this thread's KPG keys
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < KPG; ++j) {
        const int key2 = TK ? tk_key(j) : kg * KPG + j;
        if (key2 >= kn) vreg[j] = make_float4(0.f, 0.f, 0.f, 0.f);  // never 0 * (stale cache bits)
        else if (k0 + key2 == pos) vreg[j] = *reinterpret_cast<const float4*>(vnew + dg * 4);
    }
#pragma unroll
    for (int j = 0; j < KPG; ++j) {
        const float p = p_s[TK ? tk_key(j) : kg * KPG + j];
        o.x = fmaf(p, vreg[j].x, o.x);
        o.y = fmaf(p, vreg[j].y, o.y);
        o.z = fmaf(p, vreg[j].z, o.z);
        o.w = fmaf(p, vreg[j].w, o.w);
    }
    const float l_run = red[4];
    o_s[tid] = o;
    __syncthreads();
    // partial record of chunk c: [m, l, -, -, o[HD]] (16-byte aligned), stored WRITE-THROUGH (sc1)
    // so the hand-off needs no L2-writeback release fence (cdna_hip_programming.md Guideline 16 R1)
    constexpr int PR = HD + 4;
    const int chunks = (a.max_len + CH - 1) / CH;
    float* part0 = a.part + ((long)b * a.heads + h) * chunks * PR;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(part0, (short)0, chunks * PR * 4, 0x00020000);
    if (tid < DG) {
        float4 t = o_s[tid];
        for (int g = 1; g < KG; ++g) {
            const float4 u = o_s[g * DG + tid];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        u32x4 bits;
        __builtin_memcpy(&bits, &t, 16);
        __builtin_amdgcn_raw_buffer_store_b128(bits, rsrc, (c * PR + 4 + tid * 4) * 4, 0, 16);
    }
    if (tid == 0) {
        const float ml[4] = {m, l_run, 0.f, 0.f};
        u32x4 bits;
        __builtin_memcpy(&bits, ml, 16);
        __builtin_amdgcn_raw_buffer_store_b128(bits, rsrc, c * PR * 4, 0, 16);
    }
    da_stamp(a.stamps, 3);
    // 6. POLL: no ticket.  Chunk 0's block merges: it polls the records of the other chunks until
    //    none of the words it needs still holds the sentinel (the record buffer enters every launch
    //    filled with it: dec_attn_part_init, then each merge refills what it read), so a writer
    //    neither waits for its stores' acknowledgement nor takes an atomic round trip.  A word is
    //    written once per launch and read with sc1 loads; a value is never the sentinel's NaN
    //    payload (arithmetic produces the canonical NaN).  Bounded spin: a give-up sets *err.
    //    Otherwise: arrival ticket (every storing wave drains, then one relaxed agent add); the last
    //    chunk block of (b, h) merges every partial.  Every partial byte was stored sc1 and
    //    every load of it below is an sc1 buffer load, so no acquire fence is needed
    //    (MI355X_MICROARCH.md, hand-offs with sc1 loads in place of the acquire, first row).
    if constexpr (POLL) {
        if (c != 0) return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (POLL) {
        last_s = 1;
    } else if (tid == 0) {
        int* cnt = a.counters + (long)b * a.heads + h;
        const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == nc - 1;
        if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    auto ld1 = [&](int idx) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, idx * 4, 0, 16)); };
    // chunk maxima / sums into LDS, then each of the 256/HD thread groups folds a strided
    // subset of the chunks for its dim (unconditional loads: a predicated load becomes an
    // exec-masked branch with a vmcnt(0) drain)
    float* ms = reinterpret_cast<float*>(o_s);
    float* ls = ms + 512;
    float* accp = ms + 1024;
    float* lp = ms + 1280;
    constexpr int KS = 256 / HD;
    const int dim = tid % HD, grp = tid / HD;
    float l = 0.f, acc = 0.f;
    bool refill = false;
    constexpr int NJ = 12;  // o partials per thread held in registers (nc <= KS * NJ)
    if (nc <= KS * NJ && nc <= 64) {
        // ONE round trip: (m, l) of chunk `lane` (every wave holds all of them) and this thread's o partials
        // (clamped indices, weight 0 past nc by a select) are all in flight together
        float ov[NJ];
        const int tc = min(lane, nc - 1);
        float mt, lt0;
        for (unsigned it = 0;; ++it) {
            asm volatile("" ::: "memory");  // the records change under us: re-load them every pass
#pragma unroll
            for (int j = 0; j < NJ; ++j) ov[j] = ld1(min(grp + KS * j, nc - 1) * PR + 4 + dim);
            mt = ld1(tc * PR);
            lt0 = ld1(tc * PR + 1);
            if (!POLL) break;
            bool pend = __float_as_uint(mt) == DA_SENT || __float_as_uint(lt0) == DA_SENT;
#pragma unroll
            for (int j = 0; j < NJ; ++j) pend = pend || __float_as_uint(ov[j]) == DA_SENT;
            if (!__syncthreads_or(pend)) break;
            if (it > (1u << 20)) {
                if (tid == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        da_stamp(a.stamps, 4);
        refill = POLL;  // the words this thread read are refilled at the very end (after the last barrier)
        // chunk maxima / sums straight from the lanes that hold them: a wave max and lane reads, no LDS round
        // trips or barrier (kbench attn stamps: the LDS form took ~2.5 us from the last poll to the exit)
        const float mm = wave_max(lane < nc ? mt : -INFINITY);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int cc = grp + KS * j;
            const float mc = __shfl(mt, min(cc, 63)), lc = __shfl(lt0, min(cc, 63));
            if (cc < nc) {
                const float w = expf(mc - mm);
                l += lc * w;
                acc += ov[j] * w;
            }
        }
    } else {
        for (int cc = tid; cc < nc; cc += 256) {
            ms[cc] = ld1(cc * PR);
            ls[cc] = ld1(cc * PR + 1);
        }
        __syncthreads();
        float mm = -INFINITY;
        for (int cc = 0; cc < nc; ++cc) mm = fmaxf(mm, ms[cc]);
#pragma unroll 4
        for (int cc = grp; cc < nc; cc += KS) {
            const float w = expf(ms[cc] - mm);
            l += ls[cc] * w;
            acc += ld1(cc * PR + 4 + dim) * w;
        }
    }
    accp[grp * HD + dim] = acc;
    lp[grp * HD + dim] = l;
    __syncthreads();
    if (tid < HD) {
        float at = 0.f, lt = 0.f;
#pragma unroll
        for (int g = 0; g < KS; ++g) { at += accp[g * HD + tid]; lt += lp[g * HD + tid]; }
        a.o[(long)b * a.o_ld + (long)h * HD + tid] = at / lt;
    }
    if constexpr (FUSED) {
        // every chunk of this head has read its q / k / v (its record, merged above, came after): refill
        if (tid < HD) {
            const uint32_t sent = DA_SENT;
            const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), (short)0,
                                                              (a.heads + 2 * a.kv_heads) * HD * 4, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(sent, rr, (h * HD + tid) * 4, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b32(sent, rr, ((a.heads + kvh) * HD + tid) * 4, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b32(sent, rr, ((a.heads + a.kv_heads + kvh) * HD + tid) * 4, 0, 16);
        }
    }
    if (POLL && refill) {
        // refill the record words this thread read (each word by exactly one thread) for the next launch.
        // Here, after the block's last barrier: a __syncthreads waits for the write-through acknowledgements
        // of every store before it (kbench attn stamps: merge poll -> exit 2.5-3 us with the refill before
        // the combine's barriers)
        const uint32_t sent = DA_SENT;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (grp + KS * j < nc) __builtin_amdgcn_raw_buffer_store_b32(sent, rsrc, ((grp + KS * j) * PR + 4 + dim) * 4, 0, 16);
        if (tid < nc) {
            __builtin_amdgcn_raw_buffer_store_b32(sent, rsrc, (tid * PR) * 4, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b32(sent, rsrc, (tid * PR + 1) * 4, 0, 16);
        }
    }
    da_stamp(a.stamps, 5);
}

template <int HD, bool PREROT, bool POLL>
__global__ __launch_bounds__(256) void dec_attn_kernel(DecAttn2Args a) {
    WaveSpan span_(a.span);
    da_stamp(a.stamps, 0);
    dec_attn_body<HD, PREROT, POLL, false>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// One page (MHA, 128-dim heads, <= 24 chunks): the q/k/v projection (qkv_rope_body, blocks [0, nq)) and
// the decode attention (blocks nq + h * chunks + c) in ONE launch: the attention blocks stream their K / V
// cache chunk while the projection blocks stream the q/k/v weights, then take q / k / v by polling
// (FUSED above) - the kernel boundary between the two and the attention's load latency leave the chain.
template <typename WT>
__global__ __launch_bounds__(256) void dec_qkv_attn_kernel(DecGemvArgs g, DecRopeEpi r, DecAttn2Args a, int nq) {
    WaveSpan span_(a.span);
    da_stamp(a.stamps, 0);
    if ((int)blockIdx.x < nq) {
        qkv_rope_body<WT, true>(g, r, blockIdx.x);
        da_stamp(a.stamps, 1);
        return;
    }
    const int chunks = (a.max_len + DA_CH - 1) / DA_CH;
    const int i = (int)blockIdx.x - nq;
    dec_attn_body<128, true, true, true>(a, i % chunks, i / chunks, 0);
}

// ------------------------------------------------------------------ residency of the polled hand-offs
// A polling block waits on blocks of its own grid.  HIP promises no dispatch order (MI355X_MICROARCH.md,
// "Contract"), so such a launch is deadlock-free only if the blocks that can wait never hold every slot the
// device has for the kernel: then a block that never waits always finds a slot, runs to completion, and
// every producer eventually runs.  Rule: waiting < usable slots, with usable slots per CU =
// min(API answer, 8) less one where the API may over-admit (the guide's residency note: at 82-98 SGPRs
// the API reports one block per CU more than the hardware admits).  Blocks that can wait:
//   dec_qkv_attn: every attention block (each polls its head's q / k / v row) = chunks * heads;
//   dec_attn (POLL): the merging block of each (page, head) = B * heads.
bool poll_wait_fits(long waiting_blocks, int api_blocks_per_cu, int cus) {
    if (waiting_blocks <= 0) return true;
    int per_cu = std::min(api_blocks_per_cu, 8);
    if (per_cu >= 6) per_cu -= 1;
    return per_cu > 0 && cus > 0 && waiting_blocks < (long)per_cu * cus;
}

namespace {
int device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
    }
    return cus;
}
template <typename K>
int blocks_per_cu(K kernel, size_t lds) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds) != hipSuccess) return 0;
    return per_cu;
}
int qkv_attn_blocks_per_cu(int wdtype, size_t lds) {
    static int bf = -1, f16 = -1;  // the dynamic LDS is stage_bytes(1, K): one model per process
    int& v = wdtype == WDT_BF16 ? bf : f16;
    if (v < 0) v = wdtype == WDT_BF16 ? blocks_per_cu(dec_qkv_attn_kernel<bf16_t>, lds) : blocks_per_cu(dec_qkv_attn_kernel<f16_t>, lds);
    return v;
}
int attn_poll_blocks_per_cu(bool prerot) {
    static int pr = -1, npr = -1;
    int& v = prerot ? pr : npr;
    if (v < 0) v = prerot ? blocks_per_cu(dec_attn_kernel<128, true, true>, 0) : blocks_per_cu(dec_attn_kernel<128, false, true>, 0);
    return v;
}
}  // namespace

bool dec_qkv_attn_ok(const DecGemvArgs& g, const DecRopeEpi& r, const DecAttn2Args& a) {
    const int chunks = (a.max_len + DA_CH - 1) / DA_CH;
    if (!(dec_qkv_rope_ok(g, r) && a.B == 1 && a.hd == 128 && r.hd == 128 && a.heads == a.kv_heads && a.err &&
          chunks <= 24 && a.max_len <= 512 * DA_CH && g.y == a.qkv && g.N == (a.heads + 2 * a.kv_heads) * a.hd &&
          r.rot_rows == (a.heads + a.kv_heads) * a.hd))
        return false;
    return poll_wait_fits((long)chunks * a.heads, qkv_attn_blocks_per_cu(g.wdtype, stage_bytes(1, g.K)), device_cus());
}

bool dec_attn_polled(const DecAttn2Args& a) {
    const int chunks = (a.max_len + DA_CH - 1) / DA_CH;
    return a.err && a.hd == 128 && chunks <= 24 &&
           poll_wait_fits((long)a.B * a.heads, attn_poll_blocks_per_cu(a.prerot != 0), device_cus());
}

void launch_dec_qkv_attn(const DecGemvArgs& g, const DecRopeEpi& r, const DecAttn2Args& a, hipStream_t s) {
    if (!dec_qkv_attn_ok(g, r, a)) throw std::runtime_error("EINVAL: dec_qkv_attn outside its range");
    const int nq = (g.N / 2 + 3) / 4;
    const int chunks = (a.max_len + DA_CH - 1) / DA_CH;
    const size_t lds = stage_bytes(1, g.K);
    dim3 grid(nq + chunks * a.heads);
    if (g.wdtype == WDT_BF16) DSOCR_LAUNCH((dec_qkv_attn_kernel<bf16_t>), grid, dim3(256), lds, s, g, r, a, nq);
    else DSOCR_LAUNCH((dec_qkv_attn_kernel<f16_t>), grid, dim3(256), lds, s, g, r, a, nq);
}

void dec_qkv_sentinel_init(float* qkv, size_t floats, hipStream_t s) {
    if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(qkv), (int)DA_SENT, floats, s) != hipSuccess)
        throw std::runtime_error("EINTERNAL: hipMemsetD32Async (q/k/v hand-off row)");
}

void dec_attn_part_init(float* part, size_t bytes, hipStream_t s) {
    if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(part), (int)DA_SENT, bytes / 4, s) != hipSuccess)
        throw std::runtime_error("EINTERNAL: hipMemsetD32Async (attention records)");
}

size_t dec_attn_workspace(int B, int heads, int hd, int max_len) {
    return (size_t)B * heads * ((max_len + DA2_CH_MIN - 1) / DA2_CH_MIN) * (hd + 4) * sizeof(float);
}

void launch_dec_attn(const DecAttn2Args& a, hipStream_t s) {
    if (!a.counters) throw std::runtime_error("EINTERNAL: dec_attn needs a zeroed counter array");
    if (a.max_len > 512 * DA_CH) throw std::runtime_error("EINVAL: decode context too long for the attention combine");
    if (a.hd != 128 && a.hd != 64 && a.hd != 32) throw std::runtime_error("EINVAL: decode attention supports head_dim 32 / 64 / 128");
    const int chunks = (a.max_len + DA_CH - 1) / DA_CH;
    const bool prerot = a.prerot != 0;
    dim3 g1(chunks, a.heads, a.B);
    // polling merge (no ticket): 128-dim heads, <= 24 chunks (one load round trip in the merge), a
    // give-up flag, a sentinel-filled record buffer, the merging blocks within the residency rule;
    // otherwise the arrival ticket (no block waits)
    if (dec_attn_polled(a)) {
        if (prerot) DSOCR_LAUNCH((dec_attn_kernel<128, true, true>), g1, dim3(256), 0, s, a);
        else DSOCR_LAUNCH((dec_attn_kernel<128, false, true>), g1, dim3(256), 0, s, a);
        return;
    }
#define DSOCR_DA(HDV)                                                                                         \
    do {                                                                                                       \
        if (prerot) DSOCR_LAUNCH((dec_attn_kernel<HDV, true, false>), g1, dim3(256), 0, s, a);                \
        else DSOCR_LAUNCH((dec_attn_kernel<HDV, false, false>), g1, dim3(256), 0, s, a);                      \
    } while (0)
    if (a.hd == 128) DSOCR_DA(128); else if (a.hd == 64) DSOCR_DA(64); else DSOCR_DA(32);
#undef DSOCR_DA
}

// ------------------------------------------------------------------ MoE routing (one block)
// softmax (or sigmoid) + greedy top-k (stable, block.rs:1271-1301) per token, then
// grouping: eoff[E+1], arow/apos/aw by sorted position, and the compact list of active
// experts (block.rs:1303-1324 sorts on the host; here one block does it in LDS).
constexpr int RT_MAXT = 64;  // tokens per routing block

struct RouteLds {
    int ids[RT_MAXT * 8];
    float w[RT_MAXT * 8];
    int cnt[257];
    int cur[257];
};

// top-k of one token's E logits (lg in LDS or global) by one wave
__device__ __forceinline__ void route_token(const MoeRouteArgs& a, const float* lg, int t, RouteLds& L) {
    const int lane = threadIdx.x & 63, E = a.E, K = a.topk;
    float sc[4];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = lane + 64 * j;
        sc[j] = e < E ? lg[e] : -INFINITY;
        mx = fmaxf(mx, sc[j]);
    }
    if (a.softmax_scoring) {
        mx = wave_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = lane + 64 * j;
            sc[j] = e < E ? expf(sc[j] - mx) : 0.f;
            sum += sc[j];
        }
        sum = wave_sum(sum);
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[j] = (lane + 64 * j) < E ? sc[j] / sum : -INFINITY;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[j] = (lane + 64 * j) < E ? 1.0f / (1.0f + expf(-sc[j])) : -INFINITY;
    }
    float picked[8];
    float wsum = 0.f;
    for (int k = 0; k < K; ++k) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = lane + 64 * j;
            if (e < E && (sc[j] > bv || (sc[j] == bv && e < bi))) { bv = sc[j]; bi = e; }
        }
        wave_argmax(bv, bi);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (lane + 64 * j == bi) sc[j] = -INFINITY;
        picked[k] = bv;
        wsum += bv;
        if (lane == 0) { L.ids[t * K + k] = bi; a.ids[t * K + k] = bi; }
    }
    if (lane == 0)
        for (int k = 0; k < K; ++k) {
            float v = picked[k];
            if (K > 1 && a.norm_topk) v = v / (wsum + 1e-20f);
            if (a.scaling != 1.0f) v = v * a.scaling;
            a.w[t * K + k] = v;
            L.w[t * K + k] = v;
        }
}

// block-wide grouping of L.ids (T*topk assignments) by expert; call after a barrier
__device__ __forceinline__ void group_assignments(const MoeRouteArgs& a, RouteLds& L) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nt = blockDim.x;
    const int E = a.E, n = a.T * a.topk;
    for (int i = tid; i < n; i += nt) atomicAdd(&L.cnt[L.ids[i]], 1);
    __syncthreads();
    if (wave == 0) {  // exclusive scan of the E counts + active-expert compaction, 4 experts per lane
        int c[4], local = 0, al = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = lane * 4 + j;
            c[j] = e < E ? L.cnt[e] : 0;
            local += c[j];
            al += c[j] > 0;
        }
        int incl = local, ai = al;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64), z = __shfl_up(ai, o, 64);
            if (lane >= o) { incl += y; ai += z; }
        }
        int acc = incl - local, ap = ai - al;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = lane * 4 + j;
            if (e < E) {
                L.cnt[e] = acc;
                acc += c[j];
                if (c[j] > 0) a.active[ap++] = e;
            }
        }
        if (lane == 63) { L.cnt[E] = incl; *a.n_active = ai; }
    }
    __syncthreads();
    for (int e = tid; e <= E; e += nt) a.eoff[e] = L.cnt[e];
    for (int i = tid; i < n; i += nt) {
        const int e = L.ids[i];
        const int p = L.cnt[e] + atomicAdd(&L.cur[e], 1);
        a.arow[p] = i / a.topk;
        a.apos[i] = p;
        a.aw[p] = L.w[i];
    }
}

__global__ __launch_bounds__(256) void moe_route_kernel(MoeRouteArgs a) {
    __shared__ RouteLds L;
    const int wave = threadIdx.x >> 6;
    for (int e = threadIdx.x; e <= a.E; e += 256) { L.cnt[e] = 0; L.cur[e] = 0; }
    for (int t = wave; t < a.T; t += 4) route_token(a, a.logits + (long)t * a.E, t, L);
    __syncthreads();
    group_assignments(a, L);
}

void launch_moe_route(const MoeRouteArgs& a, hipStream_t s) {
    if (a.T > RT_MAXT || a.E > 256 || a.topk > 8) throw std::runtime_error("EINVAL: routing supports T <= 64, E <= 256, top_k <= 8");
    DSOCR_LAUNCH(moe_route_kernel, dim3(1), dim3(256), 0, s, a);
}

// One wave: greedy top-k of E router logits (softmax or sigmoid scores, stable: ties -> lower
// expert id, block.rs:1271-1301); returns the `want`-th pick (e, its score) and the sum of the
// top-k scores (for norm_topk_prob).  Results are wave-uniform.
__device__ __forceinline__ void topk_select(const float* lg, int E, int K, int softmax_scoring, int want, int& e_out,
                                            float& v_out, float& wsum) {
    const int lane = threadIdx.x & 63;
    float sc[4];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = lane + 64 * j;
        sc[j] = e < E ? lg[e] : -INFINITY;
        mx = fmaxf(mx, sc[j]);
    }
    if (softmax_scoring) {
        mx = wave_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = lane + 64 * j;
            sc[j] = e < E ? expf(sc[j] - mx) : 0.f;
            sum += sc[j];
        }
        sum = wave_sum(sum);
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[j] = (lane + 64 * j) < E ? sc[j] / sum : -INFINITY;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[j] = (lane + 64 * j) < E ? 1.0f / (1.0f + expf(-sc[j])) : -INFINITY;
    }
    wsum = 0.f;
    e_out = 0;
    v_out = 0.f;
    for (int k = 0; k < K; ++k) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = lane + 64 * j;
            if (e < E && (sc[j] > bv || (sc[j] == bv && e < bi))) { bv = sc[j]; bi = e; }
        }
        wave_argmax(bv, bi);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (lane + 64 * j == bi) sc[j] = -INFINITY;
        wsum += bv;
        if (k == want) { e_out = bi; v_out = bv; }
    }
}

// ------------------------------------------------------------------ MoE gate/up (routed + shared)
// blocks [0, slots*units_r): routed expert active[s] (rows I); the rest: the shared
// experts (rows Is, all T tokens).  h = silu(x.Wg) * (x.Wu) with x = rmsnorm(X) staged in
// LDS; routed rows are pre-multiplied by their routing weight (aw, sorted order) so that
// the down kernel reduces every expert of a token into ONE accumulator.
template <typename WT, int MT>
__global__ __launch_bounds__(256) void moe_gateup2_kernel(MoeDec2Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int RB = 2, U = 3;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int units_r = (a.I + 4 * RB - 1) / (4 * RB);
    const int bid = blockIdx.x;
    __shared__ int sel_e;
    __shared__ float sel_w;
    const WT* Wg;
    const WT* Wu;
    int rows_I, u, p0, cnt;
    float* hout;
    const int* rowmap;
    const float* xb = a.x;    // rows come from xb[rowmap[p]] (grouped) or xb[t0 + m]
    float slot_w = 1.f;       // slot mode: routing weight of this (token, k) slot
    constexpr int XR = 2;
    const bool fast = a.K <= XR * 4 * 256;
    XRegs<MT, XR> xr;
    bool xpre = false;        // slot mode loads its activation row before routing itself
    if (bid < a.slots * units_r && a.slot_mode) {
        // slot mode (T <= 8): block (s = t*topk + k, unit) picks its own expert from the router
        // logits (the same greedy top-k as moe_route), no grouping pass
        const int sl = bid / units_r, t = sl / a.topk, k = sl % a.topk;
        u = bid % units_r;
        if (fast) {
            xload<MT, XR>(xr, a.x + (long)t * a.K, a.K, nullptr, 1, a.K, a.norm_w);
            xpre = true;
        }
        if (wave == 0) {
            int e;
            float v, wsum;
            topk_select(a.logits + (long)t * a.E, a.E, a.topk, a.softmax_scoring, k, e, v, wsum);
            if (a.topk > 1 && a.norm_topk) v = v / (wsum + 1e-20f);
            if (a.scaling != 1.0f) v = v * a.scaling;
            if (lane == 0) {
                sel_e = e;
                sel_w = v;
                if (u == 0) { a.ids_out[sl] = e; a.w_out[sl] = v; }
            }
        }
        __syncthreads();
        const int e = sel_e;
        slot_w = sel_w;
        rows_I = a.I;
        Wg = reinterpret_cast<const WT*>(a.Wgu) + (long)e * 2 * a.I * a.K;
        Wu = Wg + (long)a.I * a.K;
        p0 = sl;
        cnt = 1;
        hout = a.h;
        rowmap = nullptr;
        xb = a.x + (long)t * a.K;
    } else if (bid < a.slots * units_r) {
        const int s = bid / units_r;
        if (s >= *a.n_active) return;
        const int e = a.active[s];
        u = bid % units_r;
        rows_I = a.I;
        Wg = reinterpret_cast<const WT*>(a.Wgu) + (long)e * 2 * a.I * a.K;
        Wu = Wg + (long)a.I * a.K;
        p0 = a.eoff[e];
        cnt = a.eoff[e + 1] - p0;
        hout = a.h;
        rowmap = a.arow;
    } else {
        if (!a.sWgu) return;
        u = bid - a.slots * units_r;
        rows_I = a.Is;
        Wg = reinterpret_cast<const WT*>(a.sWgu);
        Wu = Wg + (long)a.Is * a.K;
        p0 = 0;
        cnt = a.T;
        hout = a.hs;
        rowmap = nullptr;
    }
    const int i0 = (u * 4 + wave) * RB;
    const bool active = i0 < rows_I;
    const int chunks = a.K >> 3;
    const float* xs = smem + XS_RED;
    for (int t0 = 0; t0 < cnt; t0 += MT) {
        const int tn = min(MT, cnt - t0);
        if (fast && !xpre) {
            if (rowmap) xload<MT, XR>(xr, xb, a.K, rowmap + p0 + t0, tn, a.K, a.norm_w);
            else xload<MT, XR>(xr, xb + (long)t0 * a.K, a.K, nullptr, tn, a.K, a.norm_w);
        }
        xpre = false;
        uint4 qg[U][RB], qu[U][RB];
#pragma unroll
        for (int uu = 0; uu < U; ++uu) {
            const int c = uu * 64 + lane;
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int i = min(i0 + r, rows_I - 1);
                const int cc = min(c, chunks - 1);
                qg[uu][r] = ldg_nt16(Wg + (long)i * a.K + (cc << 3));
                qu[uu][r] = ldg_nt16(Wu + (long)i * a.K + (cc << 3));
            }
        }
        if (t0 > 0) __syncthreads();  // previous group's LDS rows fully consumed
        if (fast) xstage<MT, XR>(xr, tn, a.K, a.norm_w != nullptr, a.eps, smem);
        else if (rowmap) stage_rows(xb, a.K, rowmap + p0 + t0, tn, a.K, a.norm_w, a.eps, smem);
        else stage_rows(xb + (long)t0 * a.K, a.K, nullptr, tn, a.K, a.norm_w, a.eps, smem);
        if (!active) continue;
        float ag[RB][MT], au[RB][MT];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m) { ag[r][m] = 0.f; au[r][m] = 0.f; }
        for (int base = 0;;) {
#pragma unroll
            for (int uu = 0; uu < U; ++uu) {
                const int c = base + uu * 64 + lane;
                if (c >= chunks) continue;
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    float wg[8], wu[8];
                    unpack8<WT>(qg[uu][r], wg);
                    unpack8<WT>(qu[uu][r], wu);
#pragma unroll
                    for (int m = 0; m < MT; ++m) {
                        if (m < tn) {
                            float xv[8];
                            ld_x8(xs + m * a.K + (c << 3), xv);
#pragma unroll
                            for (int j = 0; j < 8; ++j) {
                                ag[r][m] = fmaf(xv[j], wg[j], ag[r][m]);
                                au[r][m] = fmaf(xv[j], wu[j], au[r][m]);
                            }
                        }
                    }
                }
            }
            base += 64 * U;
            if (base >= chunks) break;
#pragma unroll
            for (int uu = 0; uu < U; ++uu) {
                const int c = base + uu * 64 + lane;
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int i = min(i0 + r, rows_I - 1);
                    const int cc = min(c, chunks - 1);
                    qg[uu][r] = ldg_nt16(Wg + (long)i * a.K + (cc << 3));
                    qu[uu][r] = ldg_nt16(Wu + (long)i * a.K + (cc << 3));
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const float gs = wave_sum(ag[r][m]);
                const float us = wave_sum(au[r][m]);
                const int i = i0 + r;
                if (lane == 0 && m < tn && i < rows_I) {
                    float hv = (gs / (1.0f + expf(-gs))) * us;  // silu (candle: x / (1 + exp(-x)))
                    if (rowmap) hv = hv * a.aw[p0 + t0 + m];
                    else if (hout == a.h) hv = hv * slot_w;
                    hout[(long)(p0 + t0 + m) * rows_I + i] = hv;
                }
            }
    }
}

// Slot-mode gate/up (T <= 8, the decode configurations): straight-line code so that the
// in-order vmcnt accounting stays exact (activation loads -> [routing] -> weight stream ->
// stage -> FMA).  Blocks [0, T*topk*units_r) are (token, pick) slots that route themselves;
// the rest are the shared experts over all T tokens (MT >= T).
template <typename WT, int MT, int RB = 2>
__device__ __forceinline__ void gateup_slot_body(const MoeDec2Args& a, const int bid, float* smem) {
    __shared__ int sel_e;
    __shared__ float sel_w;
    constexpr int U = 3, XR = 2;  // K <= 1536
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int units_r = (a.I + 4 * RB - 1) / (4 * RB);
    const bool routed = bid < a.slots * units_r;
    if (!routed && !a.sWgu) return;
    const int sl = routed ? bid / units_r : 0;
    const int t = sl / max(1, a.topk), k = sl % max(1, a.topk);
    const int u = routed ? bid % units_r : bid - a.slots * units_r;
    const int M = routed ? 1 : a.T;
    XRegs<MT, XR> xr;
    xload<MT, XR>(xr, a.x + (routed ? (long)t * a.K : 0L), a.K, nullptr, M, a.K, a.norm_w);
    if (routed) {
        if (wave == 0) {
            int e;
            float v, wsum;
            topk_select(a.logits + (long)t * a.E, a.E, a.topk, a.softmax_scoring, k, e, v, wsum);
            if (a.topk > 1 && a.norm_topk) v = v / (wsum + 1e-20f);
            if (a.scaling != 1.0f) v = v * a.scaling;
            if (lane == 0) {
                sel_e = e;
                sel_w = v;
                if (u == 0) {
                    a.ids_out[sl] = e;
                    a.w_out[sl] = v;
                }
            }
        }
        __syncthreads();
    }
    const int rows_I = routed ? a.I : a.Is;
    const int e_sel = sel_e;
    const WT* Wg = routed ? reinterpret_cast<const WT*>(a.Wgu) + (long)e_sel * 2 * a.I * a.K
                          : reinterpret_cast<const WT*>(a.sWgu);
    const WT* Wu = Wg + (long)rows_I * a.K;
    const int i0 = (u * 4 + wave) * RB;
    const bool active = i0 < rows_I;
    const int chunks = a.K >> 3;
    uint4 qg[U][RB], qu[U][RB];
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
        const int c = uu * 64 + lane;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int i = min(i0 + r, rows_I - 1);
            const int cc = min(c, chunks - 1);
            qg[uu][r] = ldg_nt16(Wg + (long)i * a.K + (cc << 3));
            qu[uu][r] = ldg_nt16(Wu + (long)i * a.K + (cc << 3));
        }
    }
    xstage<MT, XR>(xr, M, a.K, a.norm_w != nullptr, a.eps, smem);
    if (!active) return;
    const float* xs = smem + XS_RED;
    float ag[RB][MT], au[RB][MT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) { ag[r][m] = 0.f; au[r][m] = 0.f; }
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
        const int c = uu * 64 + lane;
        if (c >= chunks) continue;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float wg[8], wu[8];
            unpack8<WT>(qg[uu][r], wg);
            unpack8<WT>(qu[uu][r], wu);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < M) {
                    float xv[8];
                    ld_x8(xs + m * a.K + (c << 3), xv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        ag[r][m] = fmaf(xv[j], wg[j], ag[r][m]);
                        au[r][m] = fmaf(xv[j], wu[j], au[r][m]);
                    }
                }
            }
        }
    }
    const float scale = routed ? sel_w : 1.f;
    float* hout = routed ? a.h + (long)sl * a.I : a.hs;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const float gs = wave_sum(ag[r][m]);
            const float us = wave_sum(au[r][m]);
            const int i = i0 + r;
            if (lane == 0 && m < M && i < rows_I) {
                float hv = (gs / (1.0f + expf(-gs))) * us;  // silu (candle: x / (1 + exp(-x)))
                if (routed) hv = hv * scale;
                hout[(long)m * rows_I + i] = hv;
            }
        }
}

template <typename WT, int MT>
__global__ __launch_bounds__(256) void moe_gateup_slot_kernel(MoeDec2Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    gateup_slot_body<WT, MT>(a, blockIdx.x, smem);
}
// the shared-expert blocks of the slot grid on their own (bid offset past the routed slots), so the
// routed launch carries single-token registers and LDS (B > 1: MT = T only where it is needed)
template <typename WT, int MT, int RB>
__global__ __launch_bounds__(256) void moe_gateup_shared_kernel(MoeDec2Args a, int bid0) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    gateup_slot_body<WT, MT, RB>(a, bid0 + blockIdx.x, smem);
}

// ------------------------------------------------------------------ MoE down + combine + residual
// A wave owns output row j of every token: v = sum_k h~[row(t,k)] . Wd_{e_k}[j]
// (h~ already carries w_k) + hs[t] . Wsd[j];  X[t][j] += v.  Per token the block first
// loads the activations it needs ([topk x I] routed rows + [Is] shared row) into registers,
// then issues every weight load, then stages the activations through LDS (STAGE: when
// they fit in 64 KB), so that no activation load queues behind the weight stream.
constexpr int DN_HREG = 8;  // float4 activation registers per thread (topk*I + Is <= 8192)

template <typename WT, bool STAGE>
__global__ __launch_bounds__(256) void moe_down2_kernel(MoeDec2Args a) {
    extern __shared__ __attribute__((aligned(16))) float hsm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j = blockIdx.x * 4 + wave;
    const bool active = j < a.Hout;
    if (!STAGE && !active) return;
    const int K = a.topk;
    const int ch_r = K > 0 ? (a.I >> 3) : 0, ch_s = a.sWd ? (a.Is >> 3) : 0;
    const int jj0 = min(j, a.Hout - 1);
    const WT* Ws = reinterpret_cast<const WT*>(a.sWd) + (long)jj0 * a.Is;
    const int nr4 = K * (a.I >> 2), ns4 = ch_s ? (a.Is >> 2) : 0;  // float4 counts (routed, shared)
    for (int t = 0; t < a.T; ++t) {
        float4 hreg[DN_HREG];
        if (STAGE) {
#pragma unroll
            for (int r = 0; r < DN_HREG; ++r) {
                const int f = tid + r * 256;
                const float* src = nullptr;
                if (f < nr4) {
                    const int k = f / (a.I >> 2), off = f - k * (a.I >> 2);
                    const int row = a.apos ? a.apos[t * K + k] : t * K + k;
                    src = a.h + (long)row * a.I + off * 4;
                } else if (f < nr4 + ns4) {
                    src = a.hs + (long)t * a.Is + (f - nr4) * 4;
                }
                hreg[r] = src ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        float acc = 0.f;
        for (int br = 0, bs = 0; br < ch_r || bs < ch_s; br += 128, bs += 256) {
            uint4 qr[8][2], qs[4];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k < K) {
                    const int e = a.ids[t * K + k];
                    const WT* Wd = reinterpret_cast<const WT*>(a.Wd) + ((long)e * a.Hout + jj0) * a.I;
#pragma unroll
                    for (int uu = 0; uu < 2; ++uu) {
                        const int c = br + uu * 64 + lane;
                        qr[k][uu] = ldg_nt16(Wd + (min(c, ch_r - 1) << 3));
                    }
                }
            }
#pragma unroll
            for (int uu = 0; uu < 4; ++uu) {
                const int c = bs + uu * 64 + lane;
                qs[uu] = ch_s ? ldg_nt16(Ws + (min(c, ch_s - 1) << 3)) : make_uint4(0u, 0u, 0u, 0u);
            }
            if (STAGE && br == 0) {
                if (t > 0) __syncthreads();  // previous token's rows consumed
#pragma unroll
                for (int r = 0; r < DN_HREG; ++r) {
                    const int f = tid + r * 256;
                    if (f < nr4 + ns4) *reinterpret_cast<float4*>(hsm + f * 4) = hreg[r];
                }
                __syncthreads();
            }
            if (!active) continue;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k < K) {
                    const float* hp = STAGE ? hsm + (long)k * a.I
                                            : a.h + (long)(a.apos ? a.apos[t * K + k] : t * K + k) * a.I;
#pragma unroll
                    for (int uu = 0; uu < 2; ++uu) {
                        const int c = br + uu * 64 + lane;
                        if (c < ch_r) {
                            float hv[8], w8[8];
                            ld_x8(hp + (c << 3), hv);
                            unpack8<WT>(qr[k][uu], w8);
#pragma unroll
                            for (int q = 0; q < 8; ++q) acc = fmaf(hv[q], w8[q], acc);
                        }
                    }
                }
            }
            const float* hs = STAGE ? hsm + (long)K * a.I : a.hs + (long)t * a.Is;
#pragma unroll
            for (int uu = 0; uu < 4; ++uu) {
                const int c = bs + uu * 64 + lane;
                if (c < ch_s) {
                    float hv[8], w8[8];
                    ld_x8(hs + (c << 3), hv);
                    unpack8<WT>(qs[uu], w8);
#pragma unroll
                    for (int q = 0; q < 8; ++q) acc = fmaf(hv[q], w8[q], acc);
                }
            }
        }
        if (active) {
            const float v = wave_sum(acc);
            if (lane == 0) {
                float* xp = a.out + (long)t * a.Hout + j;
                *xp = *xp + v;
            }
        }
    }
}

// Slot-mode down (T <= 8, topk = KT at compile time, I <= 1024, Is <= 2048): per token,
// activations -> registers, every routed + shared weight load, then LDS staging and FMAs;
// straight-line so each consumer waits only for the loads it needs.
template <typename WT, int KT>
__device__ __forceinline__ void down_slot_body(const MoeDec2Args& a, const int bid, float* hsm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j = bid * 4 + wave;
    const bool active = j < a.Hout;
    const int jj = min(j, a.Hout - 1);
    const int ch_r = a.I >> 3, ch_s = a.sWd ? (a.Is >> 3) : 0;
    const int nr4 = KT * (a.I >> 2), ns4 = a.sWd ? (a.Is >> 2) : 0, n4 = nr4 + ns4;
    const WT* Ws = a.sWd ? reinterpret_cast<const WT*>(a.sWd) + (long)jj * a.Is
                         : reinterpret_cast<const WT*>(a.Wd) + (long)jj * a.I;
    const int cs_max = a.sWd ? ch_s - 1 : ch_r - 1;
    for (int t = 0; t < a.T; ++t) {
        // slot rows t*KT .. t*KT+KT-1 of h are contiguous: [KT*I routed | Is shared] as one vector
        const float* hr = a.h + (long)t * KT * a.I;
        const float* hsh = a.sWd ? a.hs + (long)t * a.Is : hr;
        f32x4 hreg[DN_HREG];  // native vector type: a float4 struct array stays in scratch here
#pragma unroll
        for (int r = 0; r < DN_HREG; ++r) {
            const int f = min(tid + r * 256, n4 - 1);
            const float* src = f < nr4 ? hr + f * 4 : hsh + (f - nr4) * 4;
            hreg[r] = *reinterpret_cast<const f32x4*>(src);
        }
        uint4 qr[KT][2], qs[4];
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            const int e = a.ids[t * KT + k];
            const WT* Wd = reinterpret_cast<const WT*>(a.Wd) + ((long)e * a.Hout + jj) * a.I;
#pragma unroll
            for (int uu = 0; uu < 2; ++uu) qr[k][uu] = ldg_nt16(Wd + (min(uu * 64 + lane, ch_r - 1) << 3));
        }
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) qs[uu] = ldg_nt16(Ws + (min(uu * 64 + lane, cs_max) << 3));
        __syncthreads();  // previous token's rows consumed (unconditional: keeps hreg in VGPRs)
#pragma unroll
        for (int r = 0; r < DN_HREG; ++r)  // LDS holds 256*DN_HREG float4: no bounds branch
            *reinterpret_cast<f32x4*>(hsm + (tid + r * 256) * 4) = hreg[r];
        __syncthreads();
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < KT; ++k) {
#pragma unroll
            for (int uu = 0; uu < 2; ++uu) {
                const int c = uu * 64 + lane;
                if (c < ch_r) {
                    float hv[8], w8[8];
                    ld_x8(hsm + k * a.I + (c << 3), hv);
                    unpack8<WT>(qr[k][uu], w8);
#pragma unroll
                    for (int q = 0; q < 8; ++q) acc = fmaf(hv[q], w8[q], acc);
                }
            }
        }
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) {
            const int c = uu * 64 + lane;
            if (c < ch_s) {
                float hv[8], w8[8];
                ld_x8(hsm + nr4 * 4 + (c << 3), hv);
                unpack8<WT>(qs[uu], w8);
#pragma unroll
                for (int q = 0; q < 8; ++q) acc = fmaf(hv[q], w8[q], acc);
            }
        }
        const float v = wave_sum(acc);
        if (active && lane == 0) {
            float* xp = a.out + (long)t * a.Hout + j;
            *xp = *xp + v;
        }
    }
}

template <typename WT, int KT>
__global__ __launch_bounds__(256) void moe_down_slot_kernel(MoeDec2Args a) {
    extern __shared__ __attribute__((aligned(16))) float hsm[];
    down_slot_body<WT, KT>(a, blockIdx.x, hsm);
}

// ------------------------------------------------------------------ decode gate/up, T = 1 (mix)
// Rank form of the greedy top-k (block.rs:1254-1301: softmax, stable descending sort, ties ->
// lower expert id): lane e holds score s_e; rank_e = #{j : s_j > s_e or (s_j == s_e and j < e)};
// pick k is the lane whose rank is k.  Identical picks to topk_select, no serial argmax rounds.
// lds: 128 floats private to the calling wave (wave_rank64).  Returns (expert, weight) of pick `want`.
// coop: the four waves of a block all call this (same logits), each counting the keys of one quarter and
// summing the quarters over part (4 x 64 ints, one block barrier).  At one page every routed wave ranks
// the same 64 scores, 28 waves per CU at once: the whole-rank form is bound by the CU's LDS read rate
// (32 broadcast 16-byte reads per wave), the quarter form reads a quarter of that.
__device__ __forceinline__ void topk_rank_pick(float logit, int E, int K, int softmax_scoring, int norm_topk,
                                               float scaling, int want, float* lds, int* part, bool coop,
                                               int& e_out, float& w_out) {
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
    int rank;
    if (coop) {
        const int wave = threadIdx.x >> 6;
        const unsigned long long key = ((unsigned long long)fkey(sc) << 32) | (unsigned)(63 - lane);
        unsigned long long* kl = reinterpret_cast<unsigned long long*>(lds);
        kl[lane] = key;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        int r0 = 0, r1 = 0;
#pragma unroll
        for (int j2 = 0; j2 < 8; ++j2) {
            const ulonglong2 o = reinterpret_cast<const ulonglong2*>(kl)[8 * wave + j2];
            r0 += o.x > key ? 1 : 0;
            r1 += o.y > key ? 1 : 0;
        }
        part[wave * 64 + lane] = r0 + r1;
        __syncthreads();
        rank = part[lane] + part[64 + lane] + part[128 + lane] + part[192 + lane];
    } else {
        rank = wave_rank64<true>(sc, lds);
    }
    if (lane >= E) rank = 1 << 20;
    // sum of the top-k scores in pick order (topk_select adds them in rank order); the pick's lane is uniform,
    // so its score comes over with a lane read, not an LDS permute
    float wsum = 0.f;
    if (K > 1 && norm_topk) {
        for (int k = 0; k < K; ++k) {
            const unsigned long long bm = __ballot(rank == k);
            const int e = __builtin_ctzll(bm);
            wsum += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), e));
        }
    }
    const unsigned long long bm = __ballot(rank == want);
    const int e = __builtin_ctzll(bm);
    float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), e));
    if (K > 1 && norm_topk) v = v / (wsum + 1e-20f);
    if (scaling != 1.0f) v = v * scaling;
    e_out = e;
    w_out = v;
}

template <typename WT>
__global__ __launch_bounds__(256) void moe_gateup_mix_kernel(MoeDec2Args a, const float* xn, int routed_first) {
    constexpr int RB = 1;  // one gate + up row pair per wave (66 VGPRs: the 1792-block grid is resident at once)
    WaveSpan span_(a.span);
    __shared__ __attribute__((aligned(16))) float rank_lds[4][128];
    __shared__ int part_s[4 * 64];
    constexpr int U = 3;  // K <= 1536
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const int wpr = (a.I + RB - 1) / RB;                 // routed waves per pick
    const int n_sh = a.sWgu ? (a.Is + RB - 1) / RB : 0;  // shared waves
    const int n_rt = a.topk * wpr;
    // wave roles: routed_first = 0: wave 0 of every block streams the shared expert, waves 1..3 a routed
    // expert; 1: the first ceil(n_rt / 4) blocks are all routed and the shared blocks come last, so the waves
    // with the longer chain (logits -> picks -> weights) are dispatched first and the ones without it last
    const int nbr = (n_rt + 3) >> 2;
    const bool shared = routed_first ? b >= nbr : wave == 0;
    const int widx = routed_first ? (shared ? 4 * (b - nbr) + wave : 4 * b + wave) : (shared ? b : 3 * b + wave - 1);
    if (shared ? widx >= n_sh : widx >= n_rt) return;   // whole wave: no block barrier below
    const int chunks = a.K >> 3;
    const int sl = shared ? 0 : widx / wpr;
    const int i0 = (shared ? widx : widx % wpr) * RB;
    int e = 0;
    float wk = 1.f;
    uint4 qg[U][RB], qu[U][RB];
    float xr[U][8];
    auto issue = [&](const WT* Wg, const WT* Wu, int rows) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int cc = min(u * 64 + lane, chunks - 1);
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int i = min(i0 + r, rows - 1);
                qg[u][r] = ldg_nt16(Wg + (long)i * a.K + (cc << 3));
                qu[u][r] = ldg_nt16(Wu + (long)i * a.K + (cc << 3));
            }
        }
    };
    auto load_x = [&]() {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int cc = min(u * 64 + lane, chunks - 1);
            ld_x8(xn + (cc << 3), xr[u]);
        }
    };
    if (shared) {
        // the shared expert needs nothing from this step: its weight stream goes out first
        const WT* Wg = reinterpret_cast<const WT*>(a.sWgu);
        issue(Wg, Wg + (long)a.Is * a.K, a.Is);
        load_x();
    } else {
        // the token row goes out behind the pick's weight rows: its L2 latency hides under theirs, and the pick
        // runs with no row registers live (the 1792-block grid's residency is set by this kernel's VGPRs)
        const float lg = a.logits[min(lane, a.E - 1)];
        // a whole routed block (routed_first: blocks < n_rt / 4 hold four routed waves, none returned) ranks
        // cooperatively; any other routed wave alone
        const bool coop = routed_first && b < (n_rt >> 2);
        topk_rank_pick(lg, a.E, a.topk, a.softmax_scoring, a.norm_topk, a.scaling, sl, rank_lds[wave], part_s, coop, e,
                       wk);
        const WT* Wg = reinterpret_cast<const WT*>(a.Wgu) + (long)e * 2 * a.I * a.K;
        issue(Wg, Wg + (long)a.I * a.K, a.I);
        load_x();
        if (i0 == 0 && lane == 0) { a.ids_out[sl] = e; a.w_out[sl] = wk; }
    }
    const int rows = shared ? a.Is : a.I;
    float ag[RB], au[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) { ag[r] = 0.f; au[r] = 0.f; }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int cc = u * 64 + lane;
        if (cc >= chunks) continue;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float wg[8], wu[8];
            unpack8<WT>(qg[u][r], wg);
            unpack8<WT>(qu[u][r], wu);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                ag[r] = fmaf(xr[u][j], wg[j], ag[r]);
                au[r] = fmaf(xr[u][j], wu[j], au[r]);
            }
        }
    }
    float* hout = shared ? a.hs : a.h + (long)sl * a.I;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const float gs = wave_sum(ag[r]);
        const float us = wave_sum(au[r]);
        const int i = i0 + r;
        if (lane == 0 && i < rows) {
            float hv = (gs / (1.0f + expf(-gs))) * us;  // silu (candle: x / (1 + exp(-x)))
            if (!shared) hv = hv * wk;
            hout[i] = hv;
        }
    }
}

// Decode down + combine + residual for one token (T = 1), split-K over the block's NW = 8 waves:
// the K axis [topk routed h rows (I each, slot order, w_k already folded) | shared h (Is)] is
// cut in 8 contiguous chunk ranges, wave w owns one for the block's RPB = 2 output rows, its h
// values come straight from L2 into registers (no block barrier before the FMAs); the 8 wave
// partials meet once in LDS and x[j] += ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)).
template <typename WT>
__global__ __launch_bounds__(512) void moe_down_mix_kernel(MoeDec2Args a) {
    constexpr int RPB = 2, NW = 8;
    WaveSpan span_(a.span);
    __shared__ float part[NW][RPB];
    constexpr int U = 16 / NW;  // chunks per lane: (topk * I + Is) / 8 / NW waves <= 64 U (= 2)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j0 = blockIdx.x * RPB;
    const int cpi = a.I >> 3, cps = a.sWd ? (a.Is >> 3) : 0;
    const int nr = a.topk * cpi, nch = nr + cps;
    const int per = (nch + NW - 1) / NW;
    const int c0 = wave * per, c1 = min(nch, c0 + per);
    // lanes past the wave's range load its last chunk again (dropped below), so a range inside one segment
    // (the model: 6 x 112 routed + 224 shared chunks over 8 waves of 112) reads one expert id at a uniform
    // address, issued as the wave's first load: the weight addresses wait for it alone, where the per-lane
    // id loads sat behind the h loads in the in-order vmcnt.  Same process, one page, 256 tokens: 108.90 vs
    // 109.08 ms, every one of four alternating rounds (profiles/r06_ab/down_mix_uniform_id_same_process.log)
    const int glim = c1 > c0 ? c1 - 1 : nch - 1;
    const int sf = __builtin_amdgcn_readfirstlane(c0 < nr ? c0 / cpi : -1);  // (the division runs on the VALU)
    const int sl = __builtin_amdgcn_readfirstlane(glim < nr ? glim / cpi : -1);
    const bool uni = sf == sl;
    const int e_w = (uni && sf >= 0) ? a.ids[sf] : 0;
    // the residual rows, loaded first (not after the LDS combine: one dependent round trip fewer)
    const float xres = a.out[min(j0 + (int)(threadIdx.x & (RPB - 1)), a.Hout - 1)];
    // 1. h of this wave's chunks (independent of the picks)
    f32x4 hv[U][2];
    int seg[U], off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int g = min(c0 + u * 64 + lane, glim);
        const bool rt = g < nr;
        seg[u] = rt ? g / cpi : -1;
        off[u] = (rt ? g % cpi : g - nr) << 3;
        const float* src = rt ? a.h + (long)seg[u] * a.I + off[u] : a.hs + off[u];
        hv[u][0] = *reinterpret_cast<const f32x4*>(src);
        hv[u][1] = *reinterpret_cast<const f32x4*>(src + 4);
    }
    // 2. the picked experts' down rows (+ shared) for RPB output rows
    uint4 q[RPB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = uni ? e_w : (seg[u] >= 0 ? a.ids[seg[u]] : 0);  // shared chunks (all at topk 0) read no id
#pragma unroll
        for (int r = 0; r < RPB; ++r) {
            const int j = min(j0 + r, a.Hout - 1);
            const WT* W = seg[u] >= 0 ? reinterpret_cast<const WT*>(a.Wd) + ((long)e * a.Hout + j) * a.I + off[u]
                                      : reinterpret_cast<const WT*>(a.sWd) + (long)j * a.Is + off[u];
            q[r][u] = ldg_nt16(W);
        }
    }
    float acc[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) acc[r] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (c0 + u * 64 + lane < c1) {
            const float hx[8] = {hv[u][0][0], hv[u][0][1], hv[u][0][2], hv[u][0][3],
                                 hv[u][1][0], hv[u][1][1], hv[u][1][2], hv[u][1][3]};
#pragma unroll
            for (int r = 0; r < RPB; ++r) {
                float w8[8];
                unpack8<WT>(q[r][u], w8);
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[r] = fmaf(hx[k], w8[k], acc[r]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        const float v = wave_sum(acc[r]);
        if (lane == 0) part[wave][r] = v;
    }
    __syncthreads();
    if (threadIdx.x < RPB && j0 + threadIdx.x < a.Hout) {
        const int r = threadIdx.x;
        const float v = ((part[0][r] + part[1][r]) + (part[2][r] + part[3][r])) + ((part[4][r] + part[5][r]) + (part[6][r] + part[7][r]));
        a.out[j0 + r] = xres + v;
    }
}

bool moe_down_mix_ok(const MoeDec2Args& a) {
    const int nch = a.topk * (a.I >> 3) + (a.sWd ? (a.Is >> 3) : 0);
    return a.slot_mode && a.T == 1 && !a.apos && a.I % 8 == 0 && (!a.sWd || a.Is % 8 == 0) && (nch + 7) / 8 <= 128 &&
           a.ids;
}

void launch_moe_down_mix(const MoeDec2Args& a, hipStream_t s) {
    if (!moe_down_mix_ok(a)) throw std::runtime_error("EINVAL: moe_down_mix outside its range");
    // 8 waves of 2 chunks per lane (50 VGPRs, 8 waves per SIMD) beat 4 of 4 (84 VGPRs): shorter per-wave
    // load chains, 6.49 -> 6.01 us; 2 output rows per block
    const dim3 grid((a.Hout + 1) / 2);
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((moe_down_mix_kernel<bf16_t>), grid, dim3(512), 0, s, a);
    else DSOCR_LAUNCH((moe_down_mix_kernel<f16_t>), grid, dim3(512), 0, s, a);
}

bool moe_gateup_mix_ok(const MoeDec2Args& a) {
    return a.slot_mode && a.logits && a.T == 1 && a.E <= 64 && a.topk <= 8 && a.K % 8 == 0 && a.K <= 64 * 3 * 8 &&
           a.ids_out && a.w_out;
}

// DSOCR_GU_ORDER (A/B switch, read at every launch): 0 (default since round 6) = one shared wave per block; 1 =
// routed blocks first, shared blocks last.  Round 5 kept 1 from a same-process A/B under a graph-mode kernel trace
// (9.13 -> 8.77 us per launch, profiles/r05_ab_gu_order.txt); without the profiler, in separate processes on one
// box, 0 is the faster: 256-token decode 107.9 vs 109.8 ms (mean of three alternating pairs, never slower,
// profiles/r06_ab/gu_order_repeat.log).  The waves' arithmetic is unchanged.
static int gu_order() {
    const char* e = getenv("DSOCR_GU_ORDER");
    return e ? atoi(e) : 0;
}

void launch_moe_gateup_mix(const MoeDec2Args& a, const float* xn, hipStream_t s) {
    if (!moe_gateup_mix_ok(a) || !xn) throw std::runtime_error("EINVAL: moe_gateup_mix outside its range");
    // one gate + up row pair per wave: 9.46 -> 8.73 us against two (98 / 90 VGPRs), 3.47 -> 3.55 pages/s
    const int n_sh = a.sWgu ? a.Is : 0;
    const int n_rt = a.topk * a.I;
    const int rf = gu_order();
    dim3 grid(rf ? (n_rt + 3) / 4 + (n_sh + 3) / 4 : std::max(n_sh, (n_rt + 2) / 3));
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((moe_gateup_mix_kernel<bf16_t>), grid, dim3(256), 0, s, a, xn, rf);
    else DSOCR_LAUNCH((moe_gateup_mix_kernel<f16_t>), grid, dim3(256), 0, s, a, xn, rf);
}

void launch_moe_gateup2(const MoeDec2Args& a, hipStream_t s) {
    if (a.T == 1 && a.slots == 0 && a.sWgu && a.Is > 0 && a.K % 8 == 0 && a.K <= 64 * 3 * 8) {
        // one token through a dense / shared-only MLP (layer 0): one gate + up row pair per wave, 4 rows per
        // block (moe_gateup_shared_kernel, RB = 1: twice the blocks of RB = 2, half as long)
        MoeDec2Args sh = a;
        const int ns = (a.Is + 3) / 4;
        if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((moe_gateup_shared_kernel<bf16_t, 1, 1>), dim3(ns), dim3(256), stage_bytes(1, a.K), s, sh, 0);
        else DSOCR_LAUNCH((moe_gateup_shared_kernel<f16_t, 1, 1>), dim3(ns), dim3(256), stage_bytes(1, a.K), s, sh, 0);
        return;
    }
    constexpr int RB = 2;
    const int units_r = (a.I + 4 * RB - 1) / (4 * RB);
    const int units_s = a.sWgu ? (a.Is + 4 * RB - 1) / (4 * RB) : 0;
    dim3 grid(a.slots * units_r + units_s);
    if (a.slot_mode && a.K <= 64 * 3 * 8 && a.T > 2 && a.T <= 8) {
        // routed slots (one token each) with MT = 1, then the shared expert over the T tokens
        MoeDec2Args r = a;
        r.sWgu = nullptr;
        const int mt = a.T <= 4 ? 4 : 8;
        if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((moe_gateup_slot_kernel<bf16_t, 1>), dim3(a.slots * units_r), dim3(256), stage_bytes(1, a.K), s, r);
        else DSOCR_LAUNCH((moe_gateup_slot_kernel<f16_t, 1>), dim3(a.slots * units_r), dim3(256), stage_bytes(1, a.K), s, r);
        if (units_s) {
            // shared expert alone (slots = 0: every block is a shared block), one row per wave so the
            // M-token blocks are twice as many and half as long (same per-row arithmetic)
            const size_t lds = stage_bytes(mt, a.K);
            MoeDec2Args sh = a;
            sh.slots = 0;
            const int ns = (a.Is + 3) / 4;
#define DSOCR_SH(WTY, MTV) DSOCR_LAUNCH((moe_gateup_shared_kernel<WTY, MTV, 1>), dim3(ns), dim3(256), lds, s, sh, 0);
            if (a.wdtype == WDT_BF16) {
                if (mt == 4) { DSOCR_SH(bf16_t, 4) } else { DSOCR_SH(bf16_t, 8) }
            } else {
                if (mt == 4) { DSOCR_SH(f16_t, 4) } else { DSOCR_SH(f16_t, 8) }
            }
#undef DSOCR_SH
        }
        return;
    }
    if (a.slot_mode && a.K <= 64 * 3 * 8 && a.T <= 8) {
        const int mt = a.T == 1 ? 1 : (a.T <= 2 ? 2 : (a.T <= 4 ? 4 : 8));
        const size_t lds = stage_bytes(mt, a.K);
#define DSOCR_SLOT(WTY, MTV) DSOCR_LAUNCH((moe_gateup_slot_kernel<WTY, MTV>), grid, dim3(256), lds, s, a)
        if (a.wdtype == WDT_BF16) {
            if (mt == 1) DSOCR_SLOT(bf16_t, 1); else if (mt == 2) DSOCR_SLOT(bf16_t, 2);
            else if (mt == 4) DSOCR_SLOT(bf16_t, 4); else DSOCR_SLOT(bf16_t, 8);
        } else {
            if (mt == 1) DSOCR_SLOT(f16_t, 1); else if (mt == 2) DSOCR_SLOT(f16_t, 2);
            else if (mt == 4) DSOCR_SLOT(f16_t, 4); else DSOCR_SLOT(f16_t, 8);
        }
#undef DSOCR_SLOT
        return;
    }
    const int mt = a.T == 1 ? 1 : (a.T <= 4 ? 4 : 8);
    const size_t lds = stage_bytes(mt, a.K);
    if (lds > STAGE_LDS_MAX) throw std::runtime_error("EINVAL: moe_gateup2 hidden size too large for LDS staging");
    if (a.wdtype == WDT_BF16) {
        if (mt == 1) DSOCR_LAUNCH((moe_gateup2_kernel<bf16_t, 1>), grid, dim3(256), lds, s, a);
        else if (mt == 4) DSOCR_LAUNCH((moe_gateup2_kernel<bf16_t, 4>), grid, dim3(256), lds, s, a);
        else DSOCR_LAUNCH((moe_gateup2_kernel<bf16_t, 8>), grid, dim3(256), lds, s, a);
    } else {
        if (mt == 1) DSOCR_LAUNCH((moe_gateup2_kernel<f16_t, 1>), grid, dim3(256), lds, s, a);
        else if (mt == 4) DSOCR_LAUNCH((moe_gateup2_kernel<f16_t, 4>), grid, dim3(256), lds, s, a);
        else DSOCR_LAUNCH((moe_gateup2_kernel<f16_t, 8>), grid, dim3(256), lds, s, a);
    }
}
void launch_moe_down2(const MoeDec2Args& a, hipStream_t s) {
    if (a.topk > 8) throw std::runtime_error("EINVAL: moe_down2 supports top_k <= 8");
    dim3 grid((a.Hout + 3) / 4);
    const long n4 = (long)a.topk * (a.I / 4) + (a.sWd ? a.Is / 4 : 0);
    if (a.slot_mode && !a.apos && (a.topk == 6 || a.topk == 3) && a.I <= 1024 && (!a.sWd || a.Is <= 2048) &&
        n4 <= 256L * DN_HREG) {
        const size_t lds = (size_t)256 * DN_HREG * 16;
#define DSOCR_DSLOT(WTY, KTV) DSOCR_LAUNCH((moe_down_slot_kernel<WTY, KTV>), grid, dim3(256), lds, s, a)
        if (a.wdtype == WDT_BF16) { if (a.topk == 6) DSOCR_DSLOT(bf16_t, 6); else DSOCR_DSLOT(bf16_t, 3); }
        else { if (a.topk == 6) DSOCR_DSLOT(f16_t, 6); else DSOCR_DSLOT(f16_t, 3); }
#undef DSOCR_DSLOT
        return;
    }
    const long f4 = (long)a.topk * (a.I / 4) + (a.sWd ? a.Is / 4 : 0);
    const bool stage = f4 <= 256L * DN_HREG && f4 * 16 <= (long)STAGE_LDS_MAX;
    const size_t lds = stage ? (size_t)f4 * 16 : 0;
    if (a.wdtype == WDT_BF16) {
        if (stage) DSOCR_LAUNCH((moe_down2_kernel<bf16_t, true>), grid, dim3(256), lds, s, a);
        else DSOCR_LAUNCH((moe_down2_kernel<bf16_t, false>), grid, dim3(256), 0, s, a);
    } else {
        if (stage) DSOCR_LAUNCH((moe_down2_kernel<f16_t, true>), grid, dim3(256), lds, s, a);
        else DSOCR_LAUNCH((moe_down2_kernel<f16_t, false>), grid, dim3(256), 0, s, a);
    }
}

// ------------------------------------------------------------------ grouped decode MoE (3..8 tokens)
// At 3..8 pages the slot kernels stream an expert once per (token, pick): 48 picks at 8 pages read
// ~2.8x the bytes of the distinct experts.  Here the router epilogue's records (MOE_GRP_*) give each
// distinct expert once with its tokens.
//
// Gate/up: blocks [0, units_s) are the shared expert over all T tokens, then (record s, unit u)
// s-major (records past n_active exit before any barrier).  Per block: the record (one scalar round
// trip), the activation rows of its tokens into registers, the RB gate + RB up rows per wave
// (16-byte nontemporal loads), then the rows are staged in LDS and every weight chunk is FMA'd
// against each token's row — the per-row arithmetic of the slot kernels (chunk u-major, then j).
template <typename WT, int RB>
__global__ __launch_bounds__(256) void moe_gateup_grp_kernel(MoeDec2Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int U = 3, XR = 2, MT = 8;  // K <= 1536, T <= 8
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int units_r = (a.I + 4 * RB - 1) / (4 * RB);
    const int units_s = a.sWgu ? (a.Is + 4 * RB - 1) / (4 * RB) : 0;
    int bid = blockIdx.x;
    const bool shared = bid < units_s;
    int s = 0, u = bid;
    if (!shared) {
        bid -= units_s;
        s = bid / units_r;
        u = bid % units_r;
    }
    const int* rec = a.grp + MOE_GRP_REC * (1 + s);
    int e = 0, cnt = a.T;
    int rows[MT];
    float wts[MT];
    if (!shared) {
        if (s >= a.grp[0]) return;  // block-uniform, before any barrier
        e = rec[0];
        cnt = rec[1];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            rows[m] = rec[2 + min(m, cnt - 1)];
            wts[m] = __int_as_float(rec[10 + min(m, cnt - 1)]);
        }
    } else {
#pragma unroll
        for (int m = 0; m < MT; ++m) { rows[m] = min(m, cnt - 1); wts[m] = 1.f; }
    }
    // 1. activation rows (token t = row / topk for routed picks) into registers
    float4 xr[MT][XR];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int t = shared ? rows[m] : rows[m] / a.topk;
        const float* xp = a.x + (long)t * a.K;
#pragma unroll
        for (int i = 0; i < XR; ++i) xr[m][i] = *reinterpret_cast<const float4*>(xp + min((tid + i * 256) * 4, a.K - 4));
    }
    // 2. the weight stream
    const int rows_I = shared ? a.Is : a.I;
    const WT* Wg = shared ? reinterpret_cast<const WT*>(a.sWgu) : reinterpret_cast<const WT*>(a.Wgu) + (long)e * 2 * a.I * a.K;
    const WT* Wu = Wg + (long)rows_I * a.K;
    const int i0 = (u * 4 + wave) * RB;
    const int chunks = a.K >> 3;
    uint4 qg[U][RB], qu[U][RB];
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
        const int cc = min(uu * 64 + lane, chunks - 1);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int i = min(i0 + r, rows_I - 1);
            qg[uu][r] = ldg_nt16(Wg + (long)i * a.K + (cc << 3));
            qu[uu][r] = ldg_nt16(Wu + (long)i * a.K + (cc << 3));
        }
    }
    // 3. stage the rows (waits for the activation loads only)
    float* xs = smem;
#pragma unroll
    for (int m = 0; m < MT; ++m)
        if (m < cnt)
#pragma unroll
            for (int i = 0; i < XR; ++i) {
                const int k = (tid + i * 256) * 4;
                if (k < a.K) *reinterpret_cast<float4*>(xs + m * a.K + k) = xr[m][i];
            }
    __syncthreads();
    if (i0 >= rows_I) return;
    float ag[RB][MT], au[RB][MT];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) { ag[r][m] = 0.f; au[r][m] = 0.f; }
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
        const int c = uu * 64 + lane;
        if (c >= chunks) continue;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float wg[8], wu[8];
            unpack8<WT>(qg[uu][r], wg);
            unpack8<WT>(qu[uu][r], wu);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < cnt) {
                    float xv[8];
                    ld_x8(xs + m * a.K + (c << 3), xv);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        ag[r][m] = fmaf(xv[j], wg[j], ag[r][m]);
                        au[r][m] = fmaf(xv[j], wu[j], au[r][m]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            if (m < cnt) {
                const float gs = wave_sum(ag[r][m]);
                const float us = wave_sum(au[r][m]);
                const int i = i0 + r;
                if (lane == 0 && i < rows_I) {
                    float hv = (gs / (1.0f + expf(-gs))) * us;  // silu (candle: x / (1 + exp(-x)))
                    if (shared) a.hs[(long)m * a.Is + i] = hv;
                    else a.h[(long)rows[m] * a.I + i] = hv * wts[m];
                }
            }
        }
}

// Down + combine + residual: block owns RPB output rows j of every token.  The K axis is
// [I chunks of each active expert in record order | Is chunks of the shared expert], cut in 4
// contiguous ranges (one per wave); a lane FMAs each 8-weight chunk of row j against the h rows of
// the tokens that picked that expert (h~ already carries w_k), one accumulator per token; the
// 4 wave partials meet once in LDS: out[t][j] += (p0 + p1) + (p2 + p3).
template <typename WT, int RPB, int U>
__global__ __launch_bounds__(256) void moe_down_grp_kernel(MoeDec2Args a) {
    constexpr int MT = 8;
    __shared__ int exp_s[64];
    __shared__ int row_s[64][MT];  // record s: h row of token t, or -1
    __shared__ float part[4][RPB][MT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_act = a.grp[0];
    for (int i = tid; i < n_act * MT; i += 256) {
        const int s = i / MT, t = i % MT;
        const int* rec = a.grp + MOE_GRP_REC * (1 + s);
        const int cnt = rec[1];
        int row = -1;
        for (int m = 0; m < cnt; ++m) {
            const int rw = rec[2 + m];
            if (rw / a.topk == t) row = rw;
        }
        row_s[s][t] = row;
        if (t == 0) exp_s[s] = rec[0];
    }
    __syncthreads();
    const int j0 = blockIdx.x * RPB;
    const int cpi = a.I >> 3, cps = a.sWd ? (a.Is >> 3) : 0;
    const int nr = n_act * cpi, nch = nr + cps;
    const int per = (nch + 3) / 4;
    const int c0 = wave * per, c1 = min(nch, c0 + per);
    float acc[MT][RPB];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < RPB; ++r) acc[t][r] = 0.f;
    for (int base = c0; base < c1; base += 64 * U) {
        uint4 q[U][RPB];
        int seg[U], off[U];
#pragma unroll
        for (int uu = 0; uu < U; ++uu) {
            const int g = min(base + uu * 64 + lane, c1 - 1);
            const bool rt = g < nr;
            seg[uu] = rt ? g / cpi : -1;
            off[uu] = (rt ? g % cpi : g - nr) << 3;
            const int e = rt ? exp_s[seg[uu]] : 0;
#pragma unroll
            for (int r = 0; r < RPB; ++r) {
                const int j = min(j0 + r, a.Hout - 1);
                const WT* W = rt ? reinterpret_cast<const WT*>(a.Wd) + ((long)e * a.Hout + j) * a.I + off[uu]
                                 : reinterpret_cast<const WT*>(a.sWd) + (long)j * a.Is + off[uu];
                q[uu][r] = ldg_nt16(W);
            }
        }
#pragma unroll
        for (int uu = 0; uu < U; ++uu) {
            if (base + uu * 64 + lane >= c1) continue;
            float w8[RPB][8];
#pragma unroll
            for (int r = 0; r < RPB; ++r) unpack8<WT>(q[uu][r], w8[r]);
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                if (t >= a.T) continue;
                const int row = seg[uu] >= 0 ? row_s[seg[uu]][t] : t;
                if (row < 0) continue;
                const float* hp = seg[uu] >= 0 ? a.h + (long)row * a.I + off[uu] : a.hs + (long)t * a.Is + off[uu];
                float hv[8];
                ld_x8(hp, hv);
#pragma unroll
                for (int r = 0; r < RPB; ++r)
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc[t][r] = fmaf(hv[k], w8[r][k], acc[t][r]);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        if (t >= a.T) continue;
#pragma unroll
        for (int r = 0; r < RPB; ++r) {
            const float v = wave_sum(acc[t][r]);
            if (lane == 0) part[wave][r][t] = v;
        }
    }
    __syncthreads();
    if (tid < RPB * MT) {
        const int r = tid / MT, t = tid % MT;
        if (t < a.T && j0 + r < a.Hout) {
            const float v = (part[0][r][t] + part[1][r][t]) + (part[2][r][t] + part[3][r][t]);
            float* xp = a.out + (long)t * a.Hout + j0 + r;
            *xp = *xp + v;
        }
    }
}

bool moe_grp_ok(const MoeDec2Args& a) {
    return a.grp && a.T >= 1 && a.T <= 8 && a.topk <= 8 && a.T * a.topk <= 64 && a.E <= 256 && a.K % 8 == 0 &&
           a.K <= 64 * 3 * 8 && a.I % 8 == 0 && (!a.sWd || a.Is % 8 == 0) && !a.norm_w && (!a.sWgu) == (!a.sWd);
}

void launch_moe_gateup_grp(const MoeDec2Args& a, hipStream_t s) {
    if (!moe_grp_ok(a)) throw std::runtime_error("EINVAL: grouped decode gate/up outside its range");
    constexpr int RB = 2;
    const int units_r = (a.I + 4 * RB - 1) / (4 * RB);
    const int units_s = a.sWgu ? (a.Is + 4 * RB - 1) / (4 * RB) : 0;
    const int slots = std::min(a.E, a.T * a.topk);
    const size_t lds = sizeof(float) * 8 * (size_t)a.K;
    dim3 grid(units_s + slots * units_r);
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((moe_gateup_grp_kernel<bf16_t, RB>), grid, dim3(256), lds, s, a);
    else DSOCR_LAUNCH((moe_gateup_grp_kernel<f16_t, RB>), grid, dim3(256), lds, s, a);
}

void launch_moe_down_grp(const MoeDec2Args& a, hipStream_t s) {
    if (!moe_grp_ok(a)) throw std::runtime_error("EINVAL: grouped decode down outside its range");
    constexpr int RPB = 2, U = 8;
    dim3 grid((a.Hout + RPB - 1) / RPB);
    if (a.wdtype == WDT_BF16) DSOCR_LAUNCH((moe_down_grp_kernel<bf16_t, RPB, U>), grid, dim3(256), 0, s, a);
    else DSOCR_LAUNCH((moe_down_grp_kernel<f16_t, RPB, U>), grid, dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ decode MoE layer dispatch

namespace {
struct MoePlan {
    MoeDec2Args m;
    DecGemvArgs router;
    int mode = 0;  // 0 mix (T = 1), 1 slot (T <= 2), 2 grouped (3..8), 3 sorted (T > 8)
    bool mix_dn = false;  // one token: the split-K down (moe_down_mix)
    bool route1 = false;  // grouped mode: dec_route_grp (norm + router + top-k + records, one launch);
                          // else dec_router's last-block epilogue writes the records
    bool gu_mm = false;   // grouped mode: gate/up on the matrix cores (moe_gateup_mm)
    bool dn_mm = false;   // grouped mode: down on the matrix cores (moe_down_mm)
    bool route_in_gu = false;  // grouped mode: the routing runs inside the gate/up launch (no router launch)
    MoeDec2Args mr;            // ... its arguments
};

// DSOCR_ROUTE_FUSED=0 (A/B switch, read at every plan): at 3..8 tokens the dec_route_grp launch + a plain
// gate/up instead of the router inside the matrix-core gate/up launch (moe_gateup_mm_route_ok; 141.0 vs 143.9 ms
// per 128 8-page steps, profiles/r06_ab/decode8_switches.log).  Round 5's third form, the same routing as a
// one-block launch before a plain gate/up, measured slower than both (144.9) and was removed in round 6.
static bool route_fused_on() {
    const char* e = getenv("DSOCR_ROUTE_FUSED");
    return !(e && atoi(e) == 0);
}

MoePlan moe_plan(const MoeDecodeArgs& a) {
    const int T = a.T, E = a.E, K = a.topk, TK = T * K;
    if (T <= 0 || TK > 512 || E > 256 || K > 8 || K > E)
        throw std::runtime_error("EINVAL: decode MoE supports batch*top_k <= 512, <= 256 experts, top_k <= min(8, E)");
    if (a.H % 8 || a.I % 8 || (a.Is && a.Is % 8)) throw std::runtime_error("EINVAL: MoE dims must be multiples of 8");
    MoePlan p;
    const bool fuse_norm = T <= 2;  // T > 2: the rows are normalised once (by the router launch, into xn)
    const float* mx = (fuse_norm || !a.norm_w) ? a.x : a.xn;
    const float* mnorm = fuse_norm ? a.norm_w : nullptr;
    MoeDec2Args& m = p.m;
    m.T = T; m.K = a.H; m.Hout = a.H; m.x = mx; m.norm_w = mnorm; m.eps = a.eps; m.out = a.out;
    m.topk = K; m.E = E; m.I = a.I; m.Wgu = a.Wgu; m.Wd = a.Wd; m.wdtype = a.wdtype; m.h = a.h; m.ids = a.ids;
    if (a.sWgu && a.sWd && a.Is > 0) { m.Is = a.Is; m.sWgu = a.sWgu; m.sWd = a.sWd; m.hs = a.hs; }
    m.Wgu_swz = a.Wgu_swz; m.sWgu_swz = a.sWgu_swz; m.Wd_swz = a.Wd_swz; m.sWd_swz = a.sWd_swz;
    m.dn_part = a.dn_part; m.dn_tick = a.dn_tick; m.span = a.span; m.stamps = a.stamps;
    DecGemvArgs& gr = p.router;
    gr.M = T; gr.N = E; gr.K = a.H; gr.x = mx; gr.ldx = a.H; gr.W = a.router; gr.ldw = a.H; gr.wdtype = a.router_wdt;
    gr.bias = a.router_bias; gr.y = a.logits; gr.ldy = E; gr.norm_w = mnorm; gr.eps = a.eps; gr.span = a.route_span;
    if (T >= 3 && T <= 8 && dec_router_ok(T, E, a.H, K) && a.route_cnt && a.grp) {
        p.mode = 2;
        m.slot_mode = 1; m.slots = TK; m.grp = a.grp; m.aw = a.wts;
        if (!moe_grp_ok(m)) p.mode = 1;
    }
    if (p.mode == 2) {
        p.route1 = dec_route_grp_ok(T, E, a.H, K);
        p.gu_mm = moe_gateup_mm_ok(m);
        p.dn_mm = moe_down_mm_ok(m);
        if (p.route1 && p.gu_mm && a.norm_w && a.router_wdt == a.wdtype && route_fused_on()) {
            MoeDec2Args r = m;
            r.x = a.x; r.norm_w = a.norm_w; r.eps = a.eps;
            r.router = a.router; r.router_bias = a.router_bias; r.router_swz = a.router_swz;
            r.softmax_scoring = a.softmax_scoring; r.norm_topk = a.norm_topk; r.scaling = a.scaling;
            r.ids_out = a.ids; r.w_out = a.wts; r.logits = a.logits;  // (block 0 also writes the logits)
            if (moe_gateup_mm_route_ok(r)) {
                p.mr = r;
                p.route_in_gu = true;
            }
        }
    } else if (T <= 8) {
        // every gate/up block routes itself from the router logits (rank / serial greedy top-k)
        m.grp = nullptr;
        m.slot_mode = 1; m.slots = TK;
        m.logits = a.logits; m.softmax_scoring = a.softmax_scoring; m.norm_topk = a.norm_topk;
        m.scaling = a.scaling; m.ids_out = a.ids; m.w_out = a.wts;
        p.mode = (fuse_norm && moe_gateup_mix_ok(m) && a.xn_router) ? 0 : 1;
        if (p.mode == 0) gr.xn_out = a.xn_router;  // the router hands its normalised row to gate/up
        p.mix_dn = moe_down_mix_ok(m);
    } else {
        p.mode = 3;
        if (!(a.eoff && a.arow && a.apos && a.active && a.n_active && a.aw))
            throw std::runtime_error("EINVAL: decode MoE over 8 tokens needs the grouping workspaces");
        m.slots = std::min(E, TK);
        m.eoff = a.eoff; m.arow = a.arow; m.apos = a.apos; m.aw = a.aw; m.active = a.active; m.n_active = a.n_active;
    }
    return p;
}
}  // namespace

bool moe_decode_route_launch(const MoeDecodeArgs& a) {
    const MoePlan p = moe_plan(a);
    return !p.route_in_gu;
}

void moe_decode_kernel_names(const MoeDecodeArgs& a, const char** gateup, const char** down) {
    const MoePlan p = moe_plan(a);
    const char* gu = "moe_gateup2_kernel";
    const char* dn = "moe_down2_kernel";
    if (p.mode == 0) gu = "moe_gateup_mix_kernel";
    else if (p.mode == 1) gu = (a.T > 2 && a.Is) ? "moe_gateup_slot_kernel+moe_gateup_shared_kernel" : "moe_gateup_slot_kernel";
    else if (p.mode == 2) gu = p.gu_mm ? "moe_gateup_mm_kernel" : "moe_gateup_grp_kernel";
    if (p.mode == 2) dn = p.dn_mm ? "moe_down_mm_kernel" : "moe_down_grp_kernel";
    else if (p.mode <= 1) dn = p.mix_dn ? "moe_down_mix_kernel" : "moe_down_slot_kernel";
    if (gateup) *gateup = gu;
    if (down) *down = dn;
}

void launch_moe_decode(const MoeDecodeArgs& a, hipStream_t s, int parts) {
    const MoePlan p = moe_plan(a);
    const MoeDec2Args& m = p.m;
    if ((parts & MOE_ROUTE) && p.route_in_gu) {
        // (the gate/up launch routes)
    } else if ((parts & MOE_ROUTE) && p.route1) {
        // norm + logits + top-k + records in one block (the grouped kernels read a.xn)
        DecGemvArgs g = p.router;
        g.x = a.x; g.norm_w = a.norm_w; g.xn_out = a.norm_w ? a.xn : nullptr;
        DecRouteEpi re;
        re.topk = a.topk; re.softmax_scoring = a.softmax_scoring; re.norm_topk = a.norm_topk;
        re.scaling = a.scaling; re.ids = a.ids; re.w = a.wts; re.grp = a.grp; re.counter = a.route_cnt;
        launch_dec_route_grp(g, re, s);
    } else if (parts & MOE_ROUTE) {
        if (a.T > 2 && a.norm_w) launch_rmsnorm(a.x, a.H, a.xn, a.H, a.T, a.H, a.norm_w, a.eps, s);
        if (p.mode == 2) {
            DecRouteEpi re;
            re.topk = a.topk; re.softmax_scoring = a.softmax_scoring; re.norm_topk = a.norm_topk;
            re.scaling = a.scaling; re.ids = a.ids; re.w = a.wts; re.counter = a.route_cnt; re.grp = a.grp;
            launch_dec_router(p.router, re, s);
        } else {
            launch_dec_gemv(p.router, s);
        }
        if (p.mode == 3) {
            MoeRouteArgs ra;
            ra.logits = a.logits; ra.T = a.T; ra.E = a.E; ra.topk = a.topk; ra.softmax_scoring = a.softmax_scoring;
            ra.norm_topk = a.norm_topk; ra.scaling = a.scaling; ra.ids = a.ids; ra.w = a.wts; ra.eoff = a.eoff;
            ra.arow = a.arow; ra.apos = a.apos; ra.aw = a.aw; ra.active = a.active; ra.n_active = a.n_active;
            launch_moe_route(ra, s);
        }
    }
    if (parts & MOE_GATEUP) {
        if (p.mode == 0) launch_moe_gateup_mix(m, a.xn_router, s);
        else if (p.mode == 2 && p.route_in_gu) launch_moe_gateup_mm(p.mr, s);
        else if (p.mode == 2 && p.gu_mm) launch_moe_gateup_mm(m, s);
        else if (p.mode == 2) launch_moe_gateup_grp(m, s);
        else launch_moe_gateup2(m, s);
    }
    if (parts & MOE_DOWN) {
        if (p.mode == 2 && p.dn_mm) launch_moe_down_mm(m, s);
        else if (p.mode == 2) launch_moe_down_grp(m, s);
        else if (p.mix_dn) launch_moe_down_mix(m, s);
        else launch_moe_down2(m, s);
    }
}

// ------------------------------------------------------------------ sampling (fused)
// argmax over the vocabulary with the no-repeat-ngram ban evaluated inside each block
// (sampling.rs:141-158), then one block per page finalises: fallback, EOS / output /
// context bookkeeping, next-step embedding and the KV position advance.
constexpr int SP_BLOCK = 256;
constexpr int SP_PER_BLOCK = 2048;  // 8 logits per thread, all loaded before the first compare
size_t dec_sample_blocks(int V) { return (size_t)(V + SP_PER_BLOCK - 1) / SP_PER_BLOCK; }

__device__ __forceinline__ bool sp_better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

// (value, index) argmax over the block (first index on ties); result in sv[0] / si[0]
__device__ __forceinline__ void block_argmax(float bv, int bi, float* sv, int* si) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    wave_argmax(bv, bi);
    if (lane == 0) { sv[wave] = bv; si[wave] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
            if (sp_better(sv[w], si[w], bv, bi)) { bv = sv[w]; bi = si[w]; }
        sv[0] = bv;
        si[0] = bi;
    }
    __syncthreads();
}

template <bool LDSCTX>
__global__ __launch_bounds__(SP_BLOCK) void dec_argmax_partial_kernel(DecSampleArgs a) {
    extern __shared__ __attribute__((aligned(16))) int ctx_s[];  // the page's context, staged once per block (LDSCTX)
    __shared__ float sv[SP_BLOCK];
    __shared__ int si[SP_BLOCK];
    __shared__ unsigned ban[SP_PER_BLOCK / 32];  // banned-token bitmap of this block's vocab range
    const int b = blockIdx.y;
    const float* lg = a.logits + (long)b * a.ld;
    const int v0 = blockIdx.x * SP_PER_BLOCK, v1 = min(a.V, v0 + SP_PER_BLOCK);
    // this block's logits first (independent loads in flight during the n-gram scan)
    constexpr int PER = SP_PER_BLOCK / SP_BLOCK;
    float xv[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int v = v0 + threadIdx.x + j * SP_BLOCK;
        xv[j] = v < v1 ? lg[v] : -INFINITY;
    }
    for (int i = threadIdx.x; i < SP_PER_BLOCK / 32; i += SP_BLOCK) ban[i] = 0u;
    const int n = a.ctx_len[b], g = a.ngram;
    const int* ctx = a.ctx + (long)b * a.ctx_cap;
    const bool use_ban = g > 1 && n >= g - 1;
    if (LDSCTX && use_ban)
        for (int i = threadIdx.x; i < n; i += SP_BLOCK) ctx_s[i] = ctx[i];
    __syncthreads();
    const int* cx = LDSCTX ? ctx_s : ctx;
    if (use_ban) {
        for (int i = threadIdx.x; i <= n - g; i += SP_BLOCK) {
            const int t = cx[i + g - 1];
            if (t < v0 || t >= v1) continue;
            bool match = true;
            for (int jj = 0; jj < g - 1; ++jj)
                if (cx[i + jj] != cx[n - g + 1 + jj]) { match = false; break; }
            if (match) atomicOr(&ban[(t - v0) >> 5], 1u << ((t - v0) & 31));
        }
    }
    __syncthreads();
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int v = v0 + threadIdx.x + j * SP_BLOCK;
        const float x = xv[j];
        if (v >= v1 || !(x > -INFINITY) || !(x < INFINITY)) continue;
        if (ban[(v - v0) >> 5] & (1u << ((v - v0) & 31))) continue;
        if (sp_better(x, v, bv, bi)) { bv = x; bi = v; }
    }
    block_argmax(bv, bi, sv, si);
    if (threadIdx.x == 0) {
        a.red_val[(long)b * a.red_blocks + blockIdx.x] = sv[0];
        a.red_idx[(long)b * a.red_blocks + blockIdx.x] = si[0];
    }
}

// exact logit of row v: the dec_gemv_stream arithmetic (lane chunks u*64 + lane, 8 fmaf each in
// order, DPP wave sum) on the staged row xs (one wave)
template <typename WT>
__device__ __forceinline__ float exact_row_logit(const uint16_t* W, int v, int K, const float* xs) {
    const int lane = threadIdx.x & 63, chunks = K >> 3;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int c = u * 64 + lane;
        const uint4 q = ldg_nt16(W + (long)v * K + (min(c, chunks - 1) << 3));
        if (c < chunks) {
            float w8[8], xv[8];
            unpack8<WT>(q, w8);
            ld_x8(xs + (c << 3), xv);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc = fmaf(xv[j], w8[j], acc);
        }
    }
    return wave_sum(acc);
}

// (value, index) argmax over the block's waves: each wave's result to its LDS slot (sv / si must
// not be in use), one barrier, every thread reduces the slots itself; result in (bv, bi)
__device__ __forceinline__ void waves_argmax(float& bv, int& bi, float* sv, int* si) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0) { sv[wave] = bv; si[wave] = bi; }
    __syncthreads();
    bv = sv[0];
    bi = si[0];
    for (int w = 1; w < nw; ++w)
        if (sp_better(sv[w], si[w], bv, bi)) { bv = sv[w]; bi = si[w]; }
}

// Screened final selection (one block per page): T = the best lower bound over the unbanned rows
// (max of the lm_head blocks'); every kept row whose upper bound reaches T is rescored exactly
// and the first-index argmax taken — the exact path's token (sampling.rs:104-118).  If nothing
// survives (every unbanned logit non-finite) the reference's fallback runs: the argmax over every
// token, unbanned.  The kernel is a chain of dependent memory round trips, so everything that
// does not depend on the token is loaded up front: the step bookkeeping words, and the next
// step's n-gram ban as PREFIX matches (positions whose first g-2 tokens equal the known part of
// the next suffix) that only need the new token compared once it is known.
constexpr int SP_LIST = 1024;  // LDS survivor list (more: rescored straight from the block slots)
constexpr int SP_PM = 256;     // LDS prefix matches (more: the ban is rescanned after the update)

__device__ __forceinline__ void screened_rescore(const DecSampleArgs& a, const uint16_t* W, const float* xs,
                                                 const int* list, int n, float T, const int* bc, long sb,
                                                 float& bv, int& bi) {
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (n <= SP_LIST) {
        for (int c = wave; c < n; c += nw) {
            const int v = list[c];
            const float x = a.w_exact_wdt == WDT_F16 ? exact_row_logit<f16_t>(W, v, a.K, xs) : exact_row_logit<bf16_t>(W, v, a.K, xs);
            if ((x > -INFINITY) && (x < INFINITY) && sp_better(x, v, bv, bi)) { bv = x; bi = v; }
        }
        return;
    }
    for (int j = wave; j < a.nblk; j += nw) {
        const int c = bc[j];
        for (int i = 0; i < c; ++i) {
            if (!(a.cand_hi[sb + (long)i * a.nblk + j] >= T)) continue;
            const int v = a.cand[sb + (long)i * a.nblk + j];
            const float x = a.w_exact_wdt == WDT_F16 ? exact_row_logit<f16_t>(W, v, a.K, xs) : exact_row_logit<bf16_t>(W, v, a.K, xs);
            if ((x > -INFINITY) && (x < INFINITY) && sp_better(x, v, bv, bi)) { bv = x; bi = v; }
        }
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void dec_screen_final_kernel(DecSampleArgs a) {
    extern __shared__ __attribute__((aligned(16))) float dyn[];  // [K] staged row | survivor list
    __shared__ float sv[NT / 64], sv2[NT / 64];
    __shared__ int si2[NT / 64];
    __shared__ int nlist, nban_s, pm_n;
    __shared__ int pm_c1[SP_PM], pm_c2[SP_PM];
    __shared__ int banv_s[SP_PM];
    float* xs = dyn;
    int* list = reinterpret_cast<int*>(dyn + a.K);
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint16_t* W = reinterpret_cast<const uint16_t*>(a.w_exact);
    const int* bc = a.blk_cnt + (long)b * a.nblk;
    const float* bt = a.blk_t + (long)b * a.nblk;
    const long sb = (long)b * a.nblk * a.slot;
    const int* cx = a.ctx + (long)b * a.ctx_cap;
    const unsigned long long t0 = a.stats ? wall_clock64() : 0;
#define SP_STAMP(k) if (a.stats && tid == 0) a.stats[4 + (k)] += wall_clock64() - t0;
    // ---- token-independent loads
    const int n = a.ctx_len[b], g = a.ngram;
    int done0 = 0, olen0 = 0, kvp0 = 0, kvl0 = 0;
    if (tid == 0) {
        if (a.out_ids) { done0 = a.done[b]; olen0 = a.out_len[b]; }
        if (a.kv_pos) { kvp0 = a.kv_pos[b]; kvl0 = a.kv_len[b]; }
        nlist = 0;
        pm_n = 0;
        nban_s = 0;
    }
    // per-block threshold and count (thread j < nblk), the first token of the two prefix-match
    // positions this thread checks, and the staged row: all in flight before the first barrier
    const bool ban = a.ban_out && g > 1 && n + 1 >= g - 1;
    const int last_i = n + 1 - g;  // next step's positions: 0 .. n+1-g
    const int jc = min(tid, a.nblk - 1);
    float T = bt[jc];
    const int c0 = bc[jc];
    // block jc's first E kept rows: they do not depend on T, so they load in this round trip too
    constexpr int E = 16;
    float h[E];
    int v[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const long e = sb + (long)min(i, (int)a.slot - 1) * a.nblk + jc;
        h[i] = a.cand_hi[e];
        v[i] = a.cand[e];
    }
    if (tid >= a.nblk) T = -INFINITY;
    for (int j = tid + NT; j < a.nblk; j += NT) T = fmaxf(T, bt[j]);
    const int lc = max(last_i, 0);
    const int pa = cx[min(tid, lc)], pb = cx[min(tid + NT, lc)], s0 = cx[max(n + 2 - g, 0)];
    for (int k = tid * 4; k < a.K; k += NT * 4)
        *reinterpret_cast<float4*>(xs + k) = *reinterpret_cast<const float4*>(a.xn + (long)b * a.K + k);
    T = wave_max(T);
    if (lane == 0) sv[wave] = T;
    __syncthreads();
    T = sv[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) T = fmaxf(T, sv[w]);
    SP_STAMP(0)
    // ---- kept rows whose upper bound reaches T (a block's first E entries are already in registers)
    if (tid < a.nblk) {
        if (a.stats) atomicAdd(&nban_s, c0);  // (diagnostics: kept rows, reset below)
#pragma unroll
        for (int i = 0; i < E; ++i)
            if (i < c0 && h[i] >= T) {
                const int p = atomicAdd(&nlist, 1);
                if (p < SP_LIST) list[p] = v[i];
            }
        for (int i = E; i < c0; ++i) {
            const float hh = a.cand_hi[sb + (long)i * a.nblk + tid];
            const int vv = a.cand[sb + (long)i * a.nblk + tid];
            if (hh >= T) {
                const int p = atomicAdd(&nlist, 1);
                if (p < SP_LIST) list[p] = vv;
            }
        }
    }
    for (int j = tid + NT; j < a.nblk; j += NT) {  // more blocks than threads
        const int c = bc[j];
        for (int i = 0; i < c; ++i) {
            const float hh = a.cand_hi[sb + (long)i * a.nblk + j];
            const int vv = a.cand[sb + (long)i * a.nblk + j];
            if (hh >= T) {
                const int p = atomicAdd(&nlist, 1);
                if (p < SP_LIST) list[p] = vv;
            }
        }
    }
    SP_STAMP(6)
    // ---- next step's n-gram ban, prefix part: ctx'[i..i+g-3] == ctx[n+2-g..n-1] (first token
    // compared from the preloaded values; the rest only for the rare positions that pass)
    if (ban)
        for (int i = tid, r = 0; i <= last_i; i += NT, ++r) {
            const int first = r == 0 ? pa : (r == 1 ? pb : cx[i]);
            bool match = g < 3 || first == s0;
            for (int jj = 1; match && jj < g - 2; ++jj)
                if (cx[i + jj] != cx[n + 2 - g + jj]) match = false;
            if (match) {
                const int p = atomicAdd(&pm_n, 1);
                if (p < SP_PM) {
                    pm_c1[p] = cx[i + g - 2];                          // index <= n-1
                    pm_c2[p] = i + g - 1 < n ? cx[i + g - 1] : -1;     // -1: the new token
                }
            }
        }
    __syncthreads();
    SP_STAMP(1)
    const int nl = nlist;
    if (a.stats) {
        if (tid == 0) { a.stats[0] += 1; a.stats[1] += (unsigned long long)nban_s; a.stats[2] += (unsigned long long)nl; }
        __syncthreads();
        if (tid == 0) nban_s = 0;
    }
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    // at most one survivor per wave (the usual case: ~9 of 16 waves): each wave also loads its survivor's
    // embedding row now, so the next step's input row is in registers when the argmax is known (the gather
    // after the argmax was one more dependent round trip at the end of the step)
    constexpr int EU = 3;  // 16-byte chunks per lane of the embedding row (H <= 64 * 8 * EU)
    const bool emb_pre = a.table && nl <= NT / 64 && a.H % 8 == 0 && a.H <= 64 * 8 * EU;
    uint4 erow[EU];
    int ev = -1;
    if (emb_pre && wave < nl) {
        ev = list[wave];
        const uint16_t* tab = reinterpret_cast<const uint16_t*>(a.table) + (long)ev * a.H;
#pragma unroll
        for (int u = 0; u < EU; ++u) erow[u] = ldg_nt16(tab + (min(u * 64 + lane, a.H / 8 - 1) << 3));
    }
    screened_rescore(a, W, xs, list, nl, T, bc, sb, bv, bi);
    SP_STAMP(2)
    waves_argmax(bv, bi, sv2, si2);
    SP_STAMP(3)
    if (bi == 0x7fffffff) {
        // fallback (sampling.rs:34-96): argmax of every token ignoring the ban
        bv = -INFINITY;
        bi = 0x7fffffff;
        for (int v = wave; v < a.V; v += NT / 64) {
            const float x = a.w_exact_wdt == WDT_F16 ? exact_row_logit<f16_t>(W, v, a.K, xs) : exact_row_logit<bf16_t>(W, v, a.K, xs);
            if ((x > -INFINITY) && (x < INFINITY) && sp_better(x, v, bv, bi)) { bv = x; bi = v; }
        }
        __syncthreads();
        waves_argmax(bv, bi, sv2, si2);
    }
    const int t = bi == 0x7fffffff ? 0 : bi;
    // the next step's ban from the prefix matches into LDS first: the global stores below then need no barrier
    // after them (a barrier waits for the acknowledgement of every store before it)
    const bool ban_fast = a.ban_out && pm_n <= SP_PM;
    if (ban_fast) {
        for (int p = tid; p < pm_n; p += NT)
            if (pm_c1[p] == t) {
                const int q = atomicAdd(&nban_s, 1);
                banv_s[q] = pm_c2[p] < 0 ? t : pm_c2[p];  // q < pm_n <= SP_PM
            }
        __syncthreads();
    }
    if (tid == 0) {
        a.out_tok[b] = t;
        if (a.out_ids && !done0) {
            if (a.eos >= 0 && t == a.eos) {
                a.done[b] = 1;
            } else {
                if (olen0 < a.out_cap) { a.out_ids[(long)b * a.out_cap + olen0] = t; a.out_len[b] = olen0 + 1; }
                if (olen0 + 1 >= a.out_cap) a.done[b] = 1;
                if (n < a.ctx_cap) { a.ctx[(long)b * a.ctx_cap + n] = t; a.ctx_len[b] = n + 1; }
            }
        }
        if (a.kv_pos) {
            a.kv_pos[b] = kvp0 + 1;
            a.kv_len[b] = kvl0 + 1;
        }
    }
    if (a.table) {
        const bool hit = emb_pre && bi != 0x7fffffff && t == bi && __syncthreads_or(ev == t);
        if (hit) {  // the wave that holds the winner's row writes it
            if (ev == t) {
#pragma unroll
                for (int u = 0; u < EU; ++u) {
                    const int cc = u * 64 + lane;
                    if (cc < a.H / 8) {
                        float w8[8];
                        if (a.table_dt == WDT_BF16) unpack8<bf16_t>(erow[u], w8);
                        else unpack8<f16_t>(erow[u], w8);
                        float* d = a.x_next + (long)b * a.H + (cc << 3);
                        *reinterpret_cast<float4*>(d) = make_float4(w8[0], w8[1], w8[2], w8[3]);
                        *reinterpret_cast<float4*>(d + 4) = make_float4(w8[4], w8[5], w8[6], w8[7]);
                    }
                }
            }
        } else {
            const uint16_t* tab = reinterpret_cast<const uint16_t*>(a.table);
            for (int c = tid; c < a.H; c += NT) {
                const uint32_t bits = tab[(long)t * a.H + c];
                a.x_next[(long)b * a.H + c] = a.table_dt == WDT_BF16 ? bf16_bits_to_f32(bits) : f16_bits_to_f32(bits);
            }
        }
    }
    SP_STAMP(4)
    if (!a.ban_out) return;
    // (a page that did not take the token is done: its later selections are never read)
    int* out = a.ban_out + (long)b * a.ban_ld;
    if (ban_fast) {
        const int nb = nban_s;
        for (int q = tid; q < nb; q += NT)
            if (q + 1 < a.ban_ld) out[1 + q] = banv_s[q];
        if (tid == 0) out[0] = min(nb, (int)a.ban_ld - 1);
        SP_STAMP(5)
        return;
    } else {
        // too many prefix matches (tiny n-gram sizes): full scan of the updated context
        __syncthreads();
        const int n1 = n + 1;
        for (int i = tid; i <= n1 - g; i += NT) {
            bool match = true;
            for (int jj = 0; jj < g - 1; ++jj) {
                const int x0 = i + jj < n ? cx[i + jj] : t, x1 = n1 - g + 1 + jj < n ? cx[n1 - g + 1 + jj] : t;
                if (x0 != x1) { match = false; break; }
            }
            if (match) {
                const int q = atomicAdd(&nban_s, 1);
                if (q + 1 < a.ban_ld) out[1 + q] = i + g - 1 < n ? cx[i + g - 1] : t;
            }
        }
    }
    __syncthreads();
    if (tid == 0) out[0] = min(nban_s, (int)a.ban_ld - 1);
    SP_STAMP(5)
#undef SP_STAMP
}

template <int NT>
__global__ __launch_bounds__(NT) void dec_sample_final_kernel(DecSampleArgs a) {
    __shared__ float sv[SP_BLOCK];
    __shared__ int si[SP_BLOCK];
    __shared__ int tok_s, nban_s;
    const int b = blockIdx.x;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int j = threadIdx.x; j < a.red_blocks; j += NT) {
        float v = a.red_val[(long)b * a.red_blocks + j];
        int i = a.red_idx[(long)b * a.red_blocks + j];
        if (i != 0x7fffffff && sp_better(v, i, bv, bi)) { bv = v; bi = i; }
    }
    block_argmax(bv, bi, sv, si);
    const bool found = si[0] != 0x7fffffff;
    __syncthreads();
    if (!found) {  // everything banned / non-finite: argmax of the penalised logits, else 0
        const float* lg = a.logits + (long)b * a.ld;
        bv = -INFINITY;
        bi = 0x7fffffff;
        for (int v = threadIdx.x; v < a.V; v += NT) {
            float x = lg[v];
            if (!(x > -INFINITY) || !(x < INFINITY)) continue;
            if (sp_better(x, v, bv, bi)) { bv = x; bi = v; }
        }
        sv[threadIdx.x] = bv;
        si[threadIdx.x] = bi;
        __syncthreads();
        for (int o = NT / 2; o > 0; o >>= 1) {
            if (threadIdx.x < o && sp_better(sv[threadIdx.x + o], si[threadIdx.x + o], sv[threadIdx.x], si[threadIdx.x])) {
                sv[threadIdx.x] = sv[threadIdx.x + o];
                si[threadIdx.x] = si[threadIdx.x + o];
            }
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        const int t = si[0] == 0x7fffffff ? 0 : si[0];
        tok_s = t;
        nban_s = 0;
        a.out_tok[b] = t;
        if (a.out_ids && !a.done[b]) {
            if (a.eos >= 0 && t == a.eos) {
                a.done[b] = 1;
            } else {
                const int st = a.out_len[b];
                if (st < a.out_cap) { a.out_ids[(long)b * a.out_cap + st] = t; a.out_len[b] = st + 1; }
                if (st + 1 >= a.out_cap) a.done[b] = 1;
                const int n = a.ctx_len[b];
                if (n < a.ctx_cap) { a.ctx[(long)b * a.ctx_cap + n] = t; a.ctx_len[b] = n + 1; }
            }
        }
        if (a.kv_pos) {
            a.kv_pos[b] += 1;
            a.kv_len[b] += 1;
        }
    }
    __syncthreads();
    if (a.ban_out) {
        // the next step's banned tokens (sampling.rs:141-158 on the updated context)
        const int n = a.ctx_len[b], g = a.ngram;
        const int* cx = a.ctx + (long)b * a.ctx_cap;
        int* out = a.ban_out + (long)b * a.ban_ld;
        if (g > 1 && n >= g - 1)
            for (int i = threadIdx.x; i <= n - g; i += NT) {
                bool match = true;
                for (int jj = 0; jj < g - 1; ++jj)
                    if (cx[i + jj] != cx[n - g + 1 + jj]) { match = false; break; }
                if (match) {
                    const int p = atomicAdd(&nban_s, 1);
                    if (p + 1 < a.ban_ld) out[1 + p] = cx[i + g - 1];
                }
            }
        __syncthreads();
        if (threadIdx.x == 0) out[0] = min(nban_s, (int)a.ban_ld - 1);
    }
    if (!a.table) return;
    const int t = tok_s;
    const uint16_t* tab = reinterpret_cast<const uint16_t*>(a.table);
    for (int c = threadIdx.x; c < a.H; c += NT) {
        const uint32_t bits = tab[(long)t * a.H + c];
        a.x_next[(long)b * a.H + c] = a.table_dt == WDT_BF16 ? bf16_bits_to_f32(bits) : f16_bits_to_f32(bits);
    }
}

void launch_dec_sample(const DecSampleArgs& a0, hipStream_t s) {
    DecSampleArgs a = a0;
    a.red_blocks = (int)dec_sample_blocks(a.V);
    const bool screen = !a.do_sample && a.blk_cnt && a.blk_t && a.cand && a.cand_hi && a.w_exact && a.xn && a.nblk > 0;
    if (a.ban_out && a.ban_ld < a.ctx_cap + 1) throw std::runtime_error("EINVAL: ban list shorter than the context");
    if (screen) {
        if (a.K % 8 || a.K > 1536) throw std::runtime_error("EINVAL: screened selection needs K % 8 == 0, K <= 1536");
        const size_t lds = sizeof(float) * a.K + sizeof(int) * SP_LIST;
        DSOCR_LAUNCH((dec_screen_final_kernel<1024>), dim3(a.B), dim3(1024), lds, s, a);
        return;
    }
    if (a.do_sample) launch_dec_stoch_select(a, s);  // sampling.hip: the chosen id in selection slot 0
    else if (a.ctx_cap <= 16384) DSOCR_LAUNCH((dec_argmax_partial_kernel<true>), dim3(a.red_blocks, a.B), dim3(SP_BLOCK), sizeof(int) * a.ctx_cap, s, a);
    else DSOCR_LAUNCH((dec_argmax_partial_kernel<false>), dim3(a.red_blocks, a.B), dim3(SP_BLOCK), 0, s, a);
    DSOCR_LAUNCH((dec_sample_final_kernel<SP_BLOCK>), dim3(a.B), dim3(SP_BLOCK), 0, s, a);
}

}  // namespace dsocr
