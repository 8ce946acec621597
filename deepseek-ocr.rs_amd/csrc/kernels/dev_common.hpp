// Device-side helpers shared by the gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
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

}  // namespace dsocr
