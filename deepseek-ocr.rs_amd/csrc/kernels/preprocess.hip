// Page preprocessing on the GPU (a1-a3 of the page path):
//   resize_bicubic   vision/resample.rs:44-160 — Pillow's separable 22-bit fixed-point bicubic:
//                    horizontal pass into u8 rows, then vertical pass, each tap an i64 accumulate
//                    from 1<<21, >>22 and clamp to [0, 255]
//   build_global_view  model/mod.rs:2308-2330 — resized page centred on a gray(127) canvas
//   dynamic_preprocess vision/preprocess.rs:67-138 — resize to the tile grid, crop row-major tiles
//   image_to_tensor    model/mod.rs:2332-2347 — CHW f32, (v / 255 - 0.5) / 0.5
// The host computes the integer tap tables and the geometry (csrc/engine/host_ops.hpp, the same
// functions the host path uses); the GPU runs the horizontal pass, then ONE kernel per output that
// fuses the vertical pass with canvas placement / tile cropping and the normalisation, writing the
// f32 CHW tensors the vision tower reads straight into HBM (the host path uploads 32 MB of f32 per
// 1024 px page instead).  Bit-identical to the host path (integer taps, IEEE f32 division).
#include <cstdint>
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace dsocr {

__device__ __forceinline__ uint8_t pp_clip8(int64_t v) {
    const int64_t s = v >> 22;
    return (uint8_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

// src HWC RGB8 [sh][sw] -> hz [sh][dw] (horizontal taps: start / length per output column)
__global__ __launch_bounds__(256) void pp_resize_h_kernel(const uint8_t* __restrict__ src, int sw, int sh,
                                                          const int* __restrict__ bounds, const int* __restrict__ coeffs,
                                                          int ksize, int dw, uint8_t* __restrict__ hz) {
    const long n = (long)sh * dw;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const int y = (int)(i / dw), x = (int)(i % dw);
        const int start = bounds[2 * x], len = bounds[2 * x + 1];
        const int* co = coeffs + (long)x * ksize;
        const uint8_t* row = src + (long)y * sw * 3;
        int64_t a0 = (int64_t)1 << 21, a1 = a0, a2 = a0;
        for (int t = 0; t < len; ++t) {
            const uint8_t* p = row + (long)(start + t) * 3;
            const int64_t c = co[t];
            a0 += (int64_t)p[0] * c;
            a1 += (int64_t)p[1] * c;
            a2 += (int64_t)p[2] * c;
        }
        uint8_t* d = hz + i * 3;
        d[0] = pp_clip8(a0);
        d[1] = pp_clip8(a1);
        d[2] = pp_clip8(a2);
    }
}

// vertical pass at resized pixel (y, x) of hz [*][dw] -> 3 channels
__device__ __forceinline__ void pp_vertical(const uint8_t* hz, int dw, const int* bounds, const int* coeffs, int ksize,
                                            int y, int x, uint8_t (&v)[3]) {
    const int start = bounds[2 * y], len = bounds[2 * y + 1];
    const int* co = coeffs + (long)y * ksize;
    int64_t a0 = (int64_t)1 << 21, a1 = a0, a2 = a0;
    for (int t = 0; t < len; ++t) {
        const uint8_t* p = hz + ((long)(start + t) * dw + x) * 3;
        const int64_t c = co[t];
        a0 += (int64_t)p[0] * c;
        a1 += (int64_t)p[1] * c;
        a2 += (int64_t)p[2] * c;
    }
    v[0] = pp_clip8(a0);
    v[1] = pp_clip8(a1);
    v[2] = pp_clip8(a2);
}

__device__ __forceinline__ float pp_norm(uint8_t v) {
    const float f = __fdiv_rn((float)v, 255.0f);
    return __fdiv_rn(__fsub_rn(f, 0.5f), 0.5f);
}

// outputs: mode 0 = global canvas [3][G][G] (resized nw x nh at (ox, oy), gray elsewhere);
//          mode 1 = tiles [n][3][T][T] of the resized grid (tile i at column i % grid_w, row i / grid_w)
__global__ __launch_bounds__(256) void pp_resize_v_chw_kernel(PpOut a) {
    const long per = (long)a.size * a.size;
    const long n = per * a.n_out;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const int img = (int)(i / per);
        const int Y = (int)((i % per) / a.size), X = (int)(i % a.size);
        uint8_t v[3] = {127, 127, 127};  // (uint8_t)(0.5 * 255.0), model/mod.rs:2309
        if (a.mode == 0) {
            const int y = Y - a.oy, x = X - a.ox;
            if (a.hz && y >= 0 && y < a.nh && x >= 0 && x < a.nw)
                pp_vertical(a.hz, a.dw, a.bounds, a.coeffs, a.ksize, y, x, v);
        } else {
            const int y = (img / a.grid_w) * a.size + Y, x = (img % a.grid_w) * a.size + X;
            pp_vertical(a.hz, a.dw, a.bounds, a.coeffs, a.ksize, y, x, v);
        }
        float* o = a.out + (long)img * 3 * per + (long)Y * a.size + X;
        o[0] = pp_norm(v[0]);
        o[per] = pp_norm(v[1]);
        o[2 * per] = pp_norm(v[2]);
    }
}

static unsigned pp_grid(long n) { return (unsigned)std::max(1L, std::min((n + 255) / 256, 16384L)); }

void launch_pp_resize_h(const uint8_t* src, int sw, int sh, const int* bounds, const int* coeffs, int ksize, int dw,
                        uint8_t* hz, hipStream_t s) {
    if ((long)sh * dw == 0) return;
    hipLaunchKernelGGL(pp_resize_h_kernel, dim3(pp_grid((long)sh * dw)), dim3(256), 0, s, src, sw, sh, bounds, coeffs,
                       ksize, dw, hz);
}

void launch_pp_resize_v_chw(const PpOut& a, hipStream_t s) {
    const long n = (long)a.size * a.size * a.n_out;
    if (n == 0) return;
    if (a.mode == 1 && (!a.hz || a.grid_w < 1)) throw std::runtime_error("EINTERNAL: tile pass without resized rows");
    hipLaunchKernelGGL(pp_resize_v_chw_kernel, dim3(pp_grid(n)), dim3(256), 0, s, a);
}

}  // namespace dsocr
