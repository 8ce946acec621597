// DSQ snapshot dequantisation on load (BASELINE config 5: "dequant-on-load -> fp16 HIP kernels").
// The reference keeps Q4_K / Q6_K / Q8_0 linears quantised and multiplies through Candle's
// QMatMul (crates/dsq-runtime/src/lib.rs:336-356); here every snapshot linear is decoded once, on
// the GPU, into the fp16 row-major [out][in] layout the decode / prefill kernels already stream.
// Decoding follows Candle's k-quants to_float (GGML block layouts): each value is one f32
// multiply (and for Q4_K one subtract) in the source's order — no contraction into FMA — then
// rounded to fp16 (RNE), bit-identical to oracle/dsq.py.
//
// Layout: rows of in_dim / block elements; block b of the flattened [out][in] matrix covers
// elements [b*QK, (b+1)*QK).  One thread per output element, 256 threads = one Q4_K / Q6_K
// super-block (or 8 Q8_0 blocks) per workgroup; the block header bytes are read by every thread
// of the block (L1/L2 broadcast).  Load-time only: the kernel is HBM-bound and runs at
// >1 TB/s, a few ms for the whole 3B model.
#include <hip/hip_fp16.h>

#include <cstdint>
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace dsocr {

__device__ __forceinline__ float f16_at(const uint8_t* p) {
    const uint16_t bits = (uint16_t)p[0] | ((uint16_t)p[1] << 8);
    return f16_bits_to_f32(bits);
}

// the f32 value is pinned in a register first: otherwise the backend folds the last multiply and
// the conversion into v_fma_mix(a, b, +0) — one rounding straight to f16 (not f32 then f16) and
// -0 * x + 0 = +0 — which is not the reference's arithmetic
__device__ __forceinline__ uint16_t to_f16_rne(float v) {
    asm volatile("" : "+v"(v));
    return __half_as_ushort(__float2half_rn(v));
}

// get_scale_min_k4 (GGML k-quants): 6-bit scale / min codes of sub-block j from the 12 packed bytes
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t* q, int& d, int& m) {
    if (j < 4) {
        d = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

// Q4_K: 144 bytes / 256 values: d f16, dmin f16, scales[12], qs[128]; chunk c of 64 values uses
// qs[32c .. 32c+31] (low nibbles first, then high nibbles) and sub-blocks 2c, 2c+1
__global__ __launch_bounds__(256) void dsq_q4k_kernel(const uint8_t* __restrict__ src, long nblocks,
                                                      uint16_t* __restrict__ out) {
    for (long b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const uint8_t* blk = src + b * 144;
        const int e = threadIdx.x;
        const int c = e >> 6, pos = e & 63, l = pos & 31, hi = pos >> 5;
        const float d = f16_at(blk), dmin = f16_at(blk + 2);
        int sc, m;
        scale_min_k4(2 * c + hi, blk + 4, sc, m);
        const uint8_t q = blk[16 + 32 * c + l];
        const int nib = hi ? (q >> 4) : (q & 0xF);
        const float d1 = __fmul_rn(d, (float)sc);
        const float m1 = __fmul_rn(dmin, (float)m);
        const float y = __fsub_rn(__fmul_rn(d1, (float)nib), m1);
        out[b * 256 + e] = to_f16_rne(y);
    }
}

// Q6_K: 210 bytes / 256 values: ql[128], qh[64], int8 scales[16], d f16; half n of 128 values,
// quarter k of 32, lane l: 6-bit value from ql (low / high nibble) and qh (2 bits), minus 32
__global__ __launch_bounds__(256) void dsq_q6k_kernel(const uint8_t* __restrict__ src, long nblocks,
                                                      uint16_t* __restrict__ out) {
    for (long b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const uint8_t* blk = src + b * 210;
        const int e = threadIdx.x;
        const int n = e >> 7, r = e & 127, k = r >> 5, l = r & 31;
        const uint8_t* ql = blk + 64 * n;
        const uint8_t* qh = blk + 128 + 32 * n;
        const int8_t* sc = reinterpret_cast<const int8_t*>(blk + 192) + 8 * n;
        const int lo = (k & 1) ? ql[l + 32] : ql[l];
        const int low4 = (k & 2) ? (lo >> 4) : (lo & 0xF);
        const int q = (low4 | (((qh[l] >> (2 * k)) & 3) << 4)) - 32;
        const float d = f16_at(blk + 208);
        const float y = __fmul_rn(__fmul_rn(d, (float)sc[(l >> 4) + 2 * k]), (float)q);
        out[b * 256 + e] = to_f16_rne(y);
    }
}

// Q8_0: 34 bytes / 32 values: d f16, int8 qs[32]; 8 blocks per workgroup
__global__ __launch_bounds__(256) void dsq_q8_0_kernel(const uint8_t* __restrict__ src, long nblocks,
                                                       uint16_t* __restrict__ out) {
    const long ngroups = (nblocks + 7) / 8;
    for (long gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
        const long b = gi * 8 + (threadIdx.x >> 5);
        if (b >= nblocks) continue;
        const uint8_t* blk = src + b * 34;
        const int i = threadIdx.x & 31;
        const float y = __fmul_rn(f16_at(blk), (float)(int8_t)blk[2 + i]);
        out[b * 32 + i] = to_f16_rne(y);
    }
}

// F16 / BF16 / F32 records: to fp16 (bf16 -> f32 exact -> f16 RNE: the --dtype f16 load rule)
__global__ __launch_bounds__(256) void dsq_float_kernel(const uint8_t* __restrict__ src, long n, int qtype,
                                                        uint16_t* __restrict__ out) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        if (qtype == DSQ_F16) {
            out[i] = (uint16_t)src[2 * i] | ((uint16_t)src[2 * i + 1] << 8);
        } else if (qtype == DSQ_BF16) {
            const uint32_t bits = ((uint32_t)src[2 * i] | ((uint32_t)src[2 * i + 1] << 8)) << 16;
            out[i] = to_f16_rne(__uint_as_float(bits));
        } else {
            uint32_t bits = 0;
            for (int k = 0; k < 4; ++k) bits |= (uint32_t)src[4 * i + k] << (8 * k);
            out[i] = to_f16_rne(__uint_as_float(bits));
        }
    }
}

size_t dsq_payload_bytes(int qtype, long out_dim, long in_dim) {
    switch (qtype) {
        case DSQ_Q4K: return (size_t)out_dim * (in_dim / 256) * 144;
        case DSQ_Q6K: return (size_t)out_dim * (in_dim / 256) * 210;
        case DSQ_Q8_0: return (size_t)out_dim * (in_dim / 32) * 34;
        case DSQ_F16:
        case DSQ_BF16: return (size_t)out_dim * in_dim * 2;
        case DSQ_F32: return (size_t)out_dim * in_dim * 4;
        default: return 0;
    }
}

void launch_dsq_dequant(int qtype, const void* src, long out_dim, long in_dim, void* out_f16, hipStream_t s) {
    const long n = out_dim * in_dim;
    if (n == 0) return;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(src);
    uint16_t* o = reinterpret_cast<uint16_t*>(out_f16);
    const long cap = 65536;
    switch (qtype) {
        case DSQ_Q4K:
        case DSQ_Q6K: {
            if (in_dim % 256) throw std::runtime_error("EINVAL: k-quant rows must be a multiple of 256 values");
            const long nb = n / 256;
            const dim3 grid((unsigned)std::min(nb, cap));
            if (qtype == DSQ_Q4K) hipLaunchKernelGGL(dsq_q4k_kernel, grid, dim3(256), 0, s, p, nb, o);
            else hipLaunchKernelGGL(dsq_q6k_kernel, grid, dim3(256), 0, s, p, nb, o);
            return;
        }
        case DSQ_Q8_0: {
            if (in_dim % 32) throw std::runtime_error("EINVAL: Q8_0 rows must be a multiple of 32 values");
            const long nb = n / 32;
            hipLaunchKernelGGL(dsq_q8_0_kernel, dim3((unsigned)std::min((nb + 7) / 8, cap)), dim3(256), 0, s, p, nb, o);
            return;
        }
        case DSQ_F16:
        case DSQ_BF16:
        case DSQ_F32:
            hipLaunchKernelGGL(dsq_float_kernel, dim3((unsigned)std::min((n + 255) / 256, cap)), dim3(256), 0, s, p, n,
                               qtype, o);
            return;
        default: throw std::runtime_error("EINVAL: unsupported snapshot tensor dtype code " + std::to_string(qtype));
    }
}

}  // namespace dsocr
