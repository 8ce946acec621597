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

// 2-D rotary on q / k (apply_rotary, dots_vit.rs:507-574): the bf16 qkv row -> f32 q / k / v rows for
// the attention: q' = rnd(q*cos + rotate_half(q)*sin) (two products and a sum, no contraction), v widened.
// cos / sin: [N][hd] (the [t | t] halves already duplicated).  One thread per element pair.
__global__ __launch_bounds__(256) void dots_rope_kernel(const uint16_t* qkv, long N, int heads, int hd, const float* cos_t,
                                                        const float* sin_t, void* out, int out_bf16) {
#pragma clang fp contract(off)
    const long D = (long)heads * hd;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= N * 3 * D) return;
    const long n = i / (3 * D);
    const int c = (int)(i % (3 * D));
    const uint16_t* row = qkv + n * 3 * D;
    const float x = ld_bf(row + c);
    if (c >= 2 * D) {  // v
        if (out_bf16) reinterpret_cast<uint16_t*>(out)[i] = row[c];
        else reinterpret_cast<float*>(out)[i] = x;
        return;
    }
    const int d = c % hd, half = hd / 2;
    const int base = c - d;
    const float partner = ld_bf(row + base + (d < half ? d + half : d - half));
    const float rot = d < half ? -partner : partner;
    const float cs = cos_t[n * hd + d], sn = sin_t[n * hd + d];
    const float a = x * cs;
    const float bb = rot * sn;
    if (out_bf16) reinterpret_cast<uint16_t*>(out)[i] = st_bf(a + bb);
    else reinterpret_cast<float*>(out)[i] = rbf(a + bb);
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

static dim3 blocks_for(long n) { return dim3((unsigned)((n + 255) / 256)); }

void launch_dots_bf16_to_f32(const void* x, long n, float* y, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(dots_bf16_to_f32_kernel, blocks_for(n), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x), n, y);
}

void launch_dots_rmsnorm(const void* x, int in_f32, long rows, int D, const float* w, float eps, void* y, hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(dots_rmsnorm_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, in_f32, D, w, eps,
                       reinterpret_cast<uint16_t*>(y));
}
void launch_dots_layernorm(const void* x, long rows, int D, const float* w, const float* b, float eps, void* y,
                           hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(dots_layernorm_kernel, dim3((unsigned)rows), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x),
                       D, w, b, eps, reinterpret_cast<uint16_t*>(y));
}
void launch_dots_rope(const void* qkv, long N, int heads, int hd, const float* cos_t, const float* sin_t, void* out,
                      int out_bf16, hipStream_t s) {
    if (N <= 0) return;
    if (hd % 2) throw std::runtime_error("EINVAL: rotary needs an even head_dim");
    hipLaunchKernelGGL(dots_rope_kernel, blocks_for(N * 3 * heads * hd), dim3(256), 0, s,
                       reinterpret_cast<const uint16_t*>(qkv), N, heads, hd, cos_t, sin_t, out, out_bf16);
}
void launch_dots_swiglu(const void* gu, long N, int I, void* h, hipStream_t s) {
    if (N <= 0) return;
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
