// Row normalisations, one wave per row, f32 statistics.
//  * LayerNorm (candle_nn LayerNorm, remove_mean): SAM eps 1e-6 (sam.rs:718-720),
//    SAM neck LayerNorm2d (sam.rs:458-473, NHWC rows), CLIP eps 1e-5 (clip.rs:50).
//  * RMSNorm (candle rms_norm_slow): x / sqrt(mean(x^2) + eps) * w (block.rs:24-29).
// The LayerNorm can scatter its output rows (window_partition, sam.rs:926-955).
#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, int ldx, float* y, int ldy, const int* out_rows,
                                                        int rows, int cols, const float* w, const float* b, float eps) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* xr = x + (long)r * ldx;
    const long orow = out_rows ? (long)out_rows[r] : (long)r;
    if (orow < 0) return;
    float* yr = y + orow * ldy;
    float s = 0.f;
    for (int c = lane * 4; c < cols; c += 256) {
        float4 v = *reinterpret_cast<const float4*>(xr + c);
        s += (v.x + v.y) + (v.z + v.w);
    }
    const float mean = wave_sum(s) / (float)cols;
    float q = 0.f;
    for (int c = lane * 4; c < cols; c += 256) {
        float4 v = *reinterpret_cast<const float4*>(xr + c);
        float a0 = v.x - mean, a1 = v.y - mean, a2 = v.z - mean, a3 = v.w - mean;
        q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
    const float var = wave_sum(q) / (float)cols;
    const float denom = sqrtf(var + eps);
    for (int c = lane * 4; c < cols; c += 256) {
        float4 v = *reinterpret_cast<const float4*>(xr + c);
        float4 wv = *reinterpret_cast<const float4*>(w + c);
        float4 bv = *reinterpret_cast<const float4*>(b + c);
        float4 o;
        o.x = (v.x - mean) / denom * wv.x + bv.x;
        o.y = (v.y - mean) / denom * wv.y + bv.y;
        o.z = (v.z - mean) / denom * wv.z + bv.z;
        o.w = (v.w - mean) / denom * wv.w + bv.w;
        *reinterpret_cast<float4*>(yr + c) = o;
    }
}

void launch_layernorm(const float* x, int ldx, float* y, int ldy, const int* out_rows, int rows, int cols,
                      const float* w, const float* b, float eps, hipStream_t s) {
    if (rows == 0) return;
    hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, ldx, y, ldy, out_rows, rows, cols,
                       w, b, eps);
}

__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* x, int ldx, float* y, int ldy, int rows, int cols,
                                                      const float* w, float eps) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* xr = x + (long)r * ldx;
    float* yr = y + (long)r * ldy;
    float q = 0.f;
    for (int c = lane * 4; c < cols; c += 256) {
        float4 v = *reinterpret_cast<const float4*>(xr + c);
        q += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
    }
    const float denom = sqrtf(wave_sum(q) / (float)cols + eps);
    for (int c = lane * 4; c < cols; c += 256) {
        float4 v = *reinterpret_cast<const float4*>(xr + c);
        float4 wv = *reinterpret_cast<const float4*>(w + c);
        float4 o;
        o.x = (v.x / denom) * wv.x;
        o.y = (v.y / denom) * wv.y;
        o.z = (v.z / denom) * wv.z;
        o.w = (v.w / denom) * wv.w;
        *reinterpret_cast<float4*>(yr + c) = o;
    }
}

void launch_rmsnorm(const float* x, int ldx, float* y, int ldy, int rows, int cols, const float* w, float eps,
                    hipStream_t s) {
    if (rows == 0) return;
    hipLaunchKernelGGL(rmsnorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, ldx, y, ldy, rows, cols, w, eps);
}

}  // namespace dsocr
