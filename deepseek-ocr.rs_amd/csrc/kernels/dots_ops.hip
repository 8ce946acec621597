// dots.ocr vision tower element-wise / norm kernels (crates/infer-dots/src/vision/dots_vit.rs) in
// the reference's bf16 semantics: activations are bf16 tensors, every op computes in f32 and
// rounds its output to bf16 (RNE); the GEMMs are gemm_bf16 with the bf16-output epilogue and the
// attention is the f32 flash attention (scores / softmax / probs.V in f32, dots_vit.rs:584-589).
#include <cmath>
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

__device__ __forceinline__ float rbf(float v) { return (float)(__bf16)v; }
__device__ __forceinline__ float ld_bf(const uint16_t* p) { return __uint_as_float((uint32_t)*p << 16); }
__device__ __forceinline__ uint16_t st_bf(float v) {
    const __bf16 b = (__bf16)v;
    uint16_t u;
    __builtin_memcpy(&u, &b, 2);
    return u;
}

// one block per row: y = rnd(x / sqrt(mean(x^2) + eps) * w) (candle rms_norm on a bf16 tensor);
// x is bf16 (in_f32 = 0) or f32 rows
__global__ __launch_bounds__(256) void dots_rmsnorm_kernel(const void* x, int in_f32, int D, const float* w, float eps,
                                                           uint16_t* y) {
    __shared__ float red[4];
    const int r = blockIdx.x, tid = threadIdx.x;
    const float* xf = reinterpret_cast<const float*>(x) + (long)r * D;
    const uint16_t* xb = reinterpret_cast<const uint16_t*>(x) + (long)r * D;
    float q = 0.f;
    for (int i = tid; i < D; i += 256) {
        const float v = in_f32 ? xf[i] : ld_bf(xb + i);
        q += v * v;
    }
    q = wave_sum(q);
    if ((tid & 63) == 0) red[tid >> 6] = q;
    __syncthreads();
    const float den = sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)D + eps);
    for (int i = tid; i < D; i += 256) {
        const float v = in_f32 ? xf[i] : ld_bf(xb + i);
        y[(long)r * D + i] = st_bf((v / den) * w[i]);
    }
}

// one block per row: rnd((x - mean) / sqrt(var + eps) * w + b) (candle layer_norm, PatchMerger ln_q)
__global__ __launch_bounds__(256) void dots_layernorm_kernel(const uint16_t* x, int D, const float* w, const float* b,
                                                             float eps, uint16_t* y) {
    __shared__ float red[4];
    __shared__ float mean_s;
    const int r = blockIdx.x, tid = threadIdx.x;
    const uint16_t* xr = x + (long)r * D;
    float s = 0.f;
    for (int i = tid; i < D; i += 256) s += ld_bf(xr + i);
    s = wave_sum(s);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) mean_s = ((red[0] + red[1]) + (red[2] + red[3])) / (float)D;
    __syncthreads();
    const float mu = mean_s;
    float q = 0.f;
    for (int i = tid; i < D; i += 256) {
        const float d = ld_bf(xr + i) - mu;
        q += d * d;
    }
    q = wave_sum(q);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = q;
    __syncthreads();
    const float den = sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)D + eps);
    for (int i = tid; i < D; i += 256) y[(long)r * D + i] = st_bf((ld_bf(xr + i) - mu) / den * w[i] + b[i]);
}

// SwiGLU (DotsSwiGLUFFN::forward, dots_vit.rs:624-630): gu = [fc1 | fc3] bf16 rows [N][2I];
// h = rnd(silu(g) * u) with candle-kernels' silu_fwd in bf16 ops: rnd(g / rnd(1 + rnd(exp(-g))))
__global__ __launch_bounds__(256) void dots_swiglu_kernel(const uint16_t* gu, long N, int I, uint16_t* h) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= N * I) return;
    const long n = i / I;
    const int j = (int)(i % I);
    const float g = ld_bf(gu + n * 2 * I + j), u = ld_bf(gu + n * 2 * I + I + j);
    const float e = rbf(expf(-g));
    const float s = rbf(g / rbf(1.0f + e));
    h[i] = st_bf(s * u);
}

// gelu (tanh form) as candle-kernels' gelu_fwd computed in bf16 ops (PatchMerger, dots_vit.rs:682)
__global__ __launch_bounds__(256) void dots_gelu_kernel(uint16_t* x, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float c = rbf(0.044715f), k = rbf(0.7978845608028654f);
    const float v = ld_bf(x + i);
    const float x_sq = rbf(v * v);
    const float x_cube = rbf(x_sq * v);
    const float alpha = rbf(v + rbf(c * x_cube));
    const float t = rbf(tanhf(rbf(k * alpha)));
    x[i] = st_bf(rbf(0.5f * v) * rbf(1.0f + t));
}

// f32 rows [N][ldi] (first D columns) -> bf16 rows [N][ldo], zero padding up to ldo
__global__ __launch_bounds__(256) void dots_to_bf16_kernel(const float* x, long N, int D, long ldi, uint16_t* y, int ldo) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= N * ldo) return;
    const long n = i / ldo;
    const int c = (int)(i % ldo);
    y[i] = c < D ? st_bf(x[n * ldi + c]) : (uint16_t)0;
}

__global__ __launch_bounds__(256) void dots_bf16_to_f32_kernel(const uint16_t* x, long n, float* y) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = ld_bf(x + i);
}

// ---- 16-byte forms of the row kernels above (same per-element arithmetic; one row per grid.y, 8
// consecutive elements per thread, no 64-bit index division).  The scalar forms moved 2 bytes per lane
// through a 64-bit divide per element: rope 0.85 TB/s, SwiGLU 2.4, RMSNorm 2.1 on the 2044 px page.

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void ld_bf8(const uint16_t* p, float* v) {
    const u32x4 q = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(q[i] << 16);
        v[2 * i + 1] = __uint_as_float(q[i] & 0xffff0000u);
    }
}
__device__ __forceinline__ void st_bf8(uint16_t* p, const float* v) {
    u32x4 q;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = (uint32_t)st_bf(v[2 * i]) | ((uint32_t)st_bf(v[2 * i + 1]) << 16);
    *reinterpret_cast<u32x4*>(p) = q;
}

// RMSNorm of bf16 rows, D % 8 == 0, D <= 4096: a thread holds <= 2 chunks of 8 in registers (in place safe)
__global__ __launch_bounds__(256) void dots_rmsnorm8_kernel(const uint16_t* x, int D, const float* w, float eps, uint16_t* y) {
    __shared__ float red[4];
    const int r = blockIdx.x, tid = threadIdx.x;
    const int nch = D >> 3;
    const uint16_t* xr = x + (long)r * D;
    float v[2][8];
    float q = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int c = tid + 256 * h;
        if (c < nch) {
            ld_bf8(xr + 8 * c, v[h]);
#pragma unroll
            for (int e = 0; e < 8; ++e) q += v[h][e] * v[h][e];
        }
    }
    q = wave_sum(q);
    if ((tid & 63) == 0) red[tid >> 6] = q;
    __syncthreads();
    const float den = sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)D + eps);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int c = tid + 256 * h;
        if (c < nch) {
            const float4 w0 = *reinterpret_cast<const float4*>(w + 8 * c);
            const float4 w1 = *reinterpret_cast<const float4*>(w + 8 * c + 4);
            const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (v[h][e] / den) * wv[e];
            st_bf8(y + (long)r * D + 8 * c, o);
        }
    }
}

// rotary of the q and k columns only (v is read in place by the attention): 8 dims per thread, the
// partner half's 8 dims and the 8 cos / sin values in three 16 / 32-byte loads
__global__ __launch_bounds__(256) void dots_rope8_kernel(const uint16_t* qkv, int D, int hd, const float* cos_t,
                                                         const float* sin_t, uint16_t* out) {
#pragma clang fp contract(off)
    const int n = blockIdx.y;
    const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (c >= 2 * D) return;
    const uint16_t* row = qkv + (long)n * 3 * D;
    const int d = c % hd, half = hd / 2;
    const int pd = d < half ? d + half : d - half;
    float x[8], pt[8];
    ld_bf8(row + c, x);
    ld_bf8(row + (c - d) + pd, pt);
    const float4 c0 = *reinterpret_cast<const float4*>(cos_t + (long)n * hd + d);
    const float4 c1 = *reinterpret_cast<const float4*>(cos_t + (long)n * hd + d + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(sin_t + (long)n * hd + d);
    const float4 s1 = *reinterpret_cast<const float4*>(sin_t + (long)n * hd + d + 4);
    const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float rot = d < half ? -pt[e] : pt[e];
        const float a = x[e] * cs[e];
        const float bb = rot * sn[e];
        o[e] = a + bb;
    }
    st_bf8(out + (long)n * 3 * D + c, o);
}

// SwiGLU, 8 outputs per thread (I % 8 == 0)
__global__ __launch_bounds__(256) void dots_swiglu8_kernel(const uint16_t* gu, int I, uint16_t* h) {
    const int n = blockIdx.y;
    const int j = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (j >= I) return;
    float g[8], u[8], o[8];
    ld_bf8(gu + (long)n * 2 * I + j, g);
    ld_bf8(gu + (long)n * 2 * I + I + j, u);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float ex = rbf(expf(-g[e]));
        const float sv = rbf(g[e] / rbf(1.0f + ex));
        o[e] = sv * u[e];
    }
    st_bf8(h + (long)n * I + j, o);
}

static dim3 blocks_for(long n) { return dim3((unsigned)((n + 255) / 256)); }

void launch_dots_bf16_to_f32(const void* x, long n, float* y, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(dots_bf16_to_f32_kernel, blocks_for(n), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x), n, y);
}

void launch_dots_rmsnorm(const void* x, int in_f32, long rows, int D, const float* w, float eps, void* y, hipStream_t s) {
    if (rows <= 0) return;
    if (!in_f32 && D % 8 == 0 && D <= 4096 && (reinterpret_cast<uintptr_t>(w) & 15) == 0) {
        hipLaunchKernelGGL(dots_rmsnorm8_kernel, dim3((unsigned)rows), dim3(256), 0, s,
                           reinterpret_cast<const uint16_t*>(x), D, w, eps, reinterpret_cast<uint16_t*>(y));
        return;
    }
    hipLaunchKernelGGL(dots_rmsnorm_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, in_f32, D, w, eps,
                       reinterpret_cast<uint16_t*>(y));
}
void launch_dots_layernorm(const void* x, long rows, int D, const float* w, const float* b, float eps, void* y,
                           hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(dots_layernorm_kernel, dim3((unsigned)rows), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x),
                       D, w, b, eps, reinterpret_cast<uint16_t*>(y));
}
void launch_dots_rope_qk(const void* qkv, long N, int heads, int hd, const float* cos_t, const float* sin_t, void* out,
                         hipStream_t s) {
    if (N <= 0) return;
    const int D = heads * hd;
    if (hd % 16 || N > 65535) throw std::runtime_error("EINVAL: rope_qk needs head_dim % 16 == 0 and <= 65535 rows");
    hipLaunchKernelGGL(dots_rope8_kernel, dim3((unsigned)((2 * D / 8 + 255) / 256), (unsigned)N), dim3(256), 0, s,
                       reinterpret_cast<const uint16_t*>(qkv), D, hd, cos_t, sin_t, reinterpret_cast<uint16_t*>(out));
}
void launch_dots_swiglu(const void* gu, long N, int I, void* h, hipStream_t s) {
    if (N <= 0) return;
    if (I % 8 == 0 && N <= 65535) {
        hipLaunchKernelGGL(dots_swiglu8_kernel, dim3((unsigned)((I / 8 + 255) / 256), (unsigned)N), dim3(256), 0, s,
                           reinterpret_cast<const uint16_t*>(gu), I, reinterpret_cast<uint16_t*>(h));
        return;
    }
    hipLaunchKernelGGL(dots_swiglu_kernel, blocks_for(N * I), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(gu), N, I,
                       reinterpret_cast<uint16_t*>(h));
}
void launch_dots_gelu(void* x, long n, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(dots_gelu_kernel, blocks_for(n), dim3(256), 0, s, reinterpret_cast<uint16_t*>(x), n);
}
void launch_dots_to_bf16(const float* x, long N, int D, long ldi, void* y, int ldo, hipStream_t s) {
    if (N <= 0) return;
    hipLaunchKernelGGL(dots_to_bf16_kernel, blocks_for(N * ldo), dim3(256), 0, s, x, N, D, ldi,
                       reinterpret_cast<uint16_t*>(y), ldo);
}

}  // namespace dsocr
