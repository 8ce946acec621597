// Bidirectional flash attention on the bf16 matrix cores for bf16-valued q / k / v with the
// reference's f32 math (dots.ocr VisionAttention::forward_uniform, crates/infer-dots/src/vision/
// dots_vit.rs:433-498: q_heads . k^T in f32, * scale, softmax, probs . v in f32; compute_dtype_for
// 584-589 widens bf16 to f32).
//
// Exactness: q, k, v hold bf16 values, so every product of QK^T is exact in the f32 accumulator of
// v_mfma_f32_32x32x16_bf16 (only the summation order differs from an f32 matmul).  The softmax
// probabilities p are f32: each is split exactly into three bf16 planes p = hi + mid + lo (RNE at
// each step, the residuals exact), and P.V runs as three MFMA passes (lo, mid, hi) against the bf16
// V: again exact products summed in f32.  16x the f32-MFMA rate per pass (MI355X_MICROARCH.md
// Matrix cores), so the 3 + 1 passes cost a quarter of the f32-MFMA kernel's cycles.
//
// Layout: S^T = K . Q^T (the accumulator's column is the lane's own query: the online-softmax
// rescale needs no cross-lane traffic), O^T = V^T . P^T (V^T read from a row-major V image, below).
// 4 waves x 32 queries per block, 64-key tiles in LDS, the next tile's global loads in registers
// while the current one is consumed.
#include <algorithm>
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int AB_Q = 32;   // queries per wave
constexpr int AB_KT = 64;  // keys per LDS tile

__device__ __forceinline__ uint16_t bf_bits(float v) {
    const __bf16 b = (__bf16)v;
    uint16_t u;
    __builtin_memcpy(&u, &b, 2);
    return u;
}

#ifndef AB_EXP
#define AB_EXP(x) __expf(x)
#endif
#ifndef AB_PRIO
#define AB_PRIO 2  // bit 0: raised wave priority over the QK^T burst, bit 1: over the P.V burst (P.V only: 4.07 vs 4.03 both, 3.92 QK only; profiles/r05_dots/ab_setprio_placement)
#endif

// V is staged ROW-major (16-byte writes, as loaded) and read as the V^T MFMA operand through
// ds_read_b64_tr_b16 (the hardware transpose read, cdna_hip_programming.md T10): a 16-lane group reads 4
// keys x 16 dims and each lane receives its dim's 4 keys; two reads give the 8 keys of the lane's P
// registers (keys 16t + 4 half + {0..3, 8..11}: the accumulator order, no key permutation).  K and V
// double-buffered in LDS: one barrier per tile.  V row pitch HD + 32 (4 consecutive rows on 4 distinct
// 16-bank groups: the transposed reads are conflict-free).  Round 2's kernel staged V transposed with
// 16-bit writes, two barriers per tile and spilled (256 VGPRs + 144 B scratch): 9.09 -> 5.86 ms per
// layer at 2044 px (profiles/r03_bench_dots_*).
typedef short v4i16_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16_t lds_v4i16;

template <int HD, int PL>
__global__ __launch_bounds__(256, 2) void attention_bf16_tr_kernel(AttnBf16Args a) {
    constexpr int KP = HD + 8, VP = HD + 32;      // LDS row pitches (bf16 elements)
    constexpr int C8 = HD / 8;                    // 16-byte chunks per row
    constexpr int NCH = AB_KT * C8 / 256;         // chunks per thread per operand per tile
    constexpr int QS = HD / 16;                   // MFMA k-steps of the QK product
    constexpr int DC = HD / 32;                   // 32-dim output chunks
    __shared__ __attribute__((aligned(16))) uint16_t Ks[2][AB_KT][KP];
    __shared__ __attribute__((aligned(16))) uint16_t Vs[2][AB_KT][VP];
    const int s = blockIdx.z, h = blockIdx.y;
    const int len = a.L;
    const int qb0 = blockIdx.x * (4 * AB_Q);
    if (qb0 >= len) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int half = lane >> 5, l32 = lane & 31;
    const int kvh = h / (a.heads / a.kv_heads);
    const uint16_t* Q = a.q + (long)s * a.L * a.q_rs + (long)h * a.q_hs;
    const uint16_t* K = a.k + (long)s * a.L * a.k_rs + (long)kvh * a.k_hs;
    const uint16_t* V = a.v + (long)s * a.L * a.v_rs + (long)kvh * a.v_hs;
    const int q_lane = qb0 + wave * AB_Q + l32;
    const bool q_valid = q_lane < len;
    bf16x8_t qreg[QS];
    {
        const uint16_t* qr = Q + (long)(q_valid ? q_lane : 0) * a.q_rs + 8 * half;
#pragma unroll
        for (int st = 0; st < QS; ++st) qreg[st] = *reinterpret_cast<const bf16x8_t*>(qr + 16 * st);
    }
    // transposed-read lane roles: 16-lane group g16 (dims 16 (g16 & 1) + i), lane i = 4 q + p supplies
    // row (key) q, dims 4 p .. 4 p + 3 of the group's 16-dim block
    const int i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3, gd = 16 * ((lane >> 4) & 1);
    // the next tile's K and V move through ONE register block in turn (K loaded before QK^T, stored
    // before P.V; V loaded then, stored after P.V): 16 fewer live registers than both at once.  Buffer
    // loads bounded at the sequence's last key: keys past it read as zeros (K: scores masked below; V:
    // zero rows), so no tile clamps or branches; per lane one offset (row tid / C8 (+ 256 / C8 per j),
    // 16-byte chunk tid % C8) plus the tile's uniform row offset.
    u32x4 rg[NCH];
    const auto rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(K), (short)0, len * a.k_rs * 2, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(V), (short)0, len * a.v_rs * 2, 0x00020000);
    const int ko = ((tid / C8) * a.k_rs + (tid % C8) * 8) * 2;
    const int vo = ((tid / C8) * a.v_rs + (tid % C8) * 8) * 2;
#define AB_GLOAD(R, RS, OFF, K0)                                                                \
    _Pragma("unroll") for (int j = 0; j < NCH; ++j)                                             \
        rg[j] = __builtin_amdgcn_raw_buffer_load_b128((R), (OFF) + ((K0) + j * (256 / C8)) * (RS) * 2, 0, 0);
#define AB_LSTORE(T)                                                                            \
    _Pragma("unroll") for (int j = 0; j < NCH; ++j) {                                           \
        const int f = tid + 256 * j;                                                            \
        *reinterpret_cast<u32x4*>(&(T)[f / C8][(f % C8) * 8]) = rg[j];                          \
    }
    f32x16 o[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[c][r] = 0.f;
    // softmax in the log2 domain: p = 2^(s * scale * log2 e - m), m the running max of s * scale * log2 e
    // (one FMA per score before the exponential; every tile holds a valid key, so m is finite after the
    // first and alpha = 2^(m_old - m_new) = 0 there)
    const float c2 = a.scale * 1.4426950408889634f;
    float m_run = -INFINITY, l_run = 0.f;
    AB_GLOAD(rk, a.k_rs, ko, 0);
    AB_LSTORE(Ks[0]);
    AB_GLOAD(rv, a.v_rs, vo, 0);
    AB_LSTORE(Vs[0]);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < len; k0 += AB_KT, buf ^= 1) {
        AB_GLOAD(rk, a.k_rs, ko, k0 + AB_KT);  // in flight under QK^T and the softmax
        f32x16 sc[2];
        if (AB_PRIO & 1) __builtin_amdgcn_s_setprio(1);  // the matrix-core burst first, the other wave's VALU in its shadow
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[u][r] = 0.f;
#pragma unroll
            for (int st = 0; st < QS; ++st) {
                const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(&Ks[buf][u * 32 + l32][16 * st + 8 * half]);
                sc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qreg[st], sc[u], 0, 0, 0);
            }
        }
        if (AB_PRIO & 1) __builtin_amdgcn_s_setprio(0);
        if (k0 + AB_KT > len) {  // the last, partial tile: keys past the end score -inf
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (k0 + u * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= len) sc[u][r] = -INFINITY;
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sc[u][r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax * c2);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        float psum = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(fmaf(sc[u][r], c2, -m_new));
                sc[u][r] = p;
                psum += p;
            }
        psum += __shfl_xor(psum, 32, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
        if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {  // some query's max moved (rare after the first tiles)
#pragma unroll
            for (int c = 0; c < DC; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[c][r] *= alpha;
        }
        AB_LSTORE(Ks[buf ^ 1]);                // the other buffer's last readers passed the previous barrier
        AB_GLOAD(rv, a.v_rs, vo, k0 + AB_KT);   // in flight under P.V
        if (AB_PRIO & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                // p = hi + mid + lo exactly: hi = p with its low 16 bits cleared (bf16 truncation), mid the
                // same of the exact residual, lo the remaining <= 8 significant bits (a bf16 exactly); two
                // bf16 of a plane packed per register by one byte permute
                u32x4 ph, pm, pl;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float p0 = sc[u][8 * t + 2 * q], p1 = sc[u][8 * t + 2 * q + 1];
                    if constexpr (PL == 3) {
                        const uint32_t b0 = __float_as_uint(p0), b1 = __float_as_uint(p1);
                        const float r0 = p0 - __uint_as_float(b0 & 0xffff0000u), r1 = p1 - __uint_as_float(b1 & 0xffff0000u);
                        const uint32_t c0 = __float_as_uint(r0), c1 = __float_as_uint(r1);
                        const float e0 = r0 - __uint_as_float(c0 & 0xffff0000u), e1 = r1 - __uint_as_float(c1 & 0xffff0000u);
                        ph[q] = __builtin_amdgcn_perm(b1, b0, 0x07060302u);
                        pm[q] = __builtin_amdgcn_perm(c1, c0, 0x07060302u);
                        pl[q] = __builtin_amdgcn_perm(__float_as_uint(e1), __float_as_uint(e0), 0x07060302u);
                    } else {
                        // hi = RNE(p), its residual exact in f32, mid = RNE(residual): p to 16 significant bits
                        const __bf16 h0 = (__bf16)p0, h1 = (__bf16)p1;
                        const __bf16 m0 = (__bf16)(p0 - (float)h0), m1 = (__bf16)(p1 - (float)h1);
                        uint16_t x0, x1, y0, y1;
                        __builtin_memcpy(&x0, &h0, 2); __builtin_memcpy(&x1, &h1, 2);
                        __builtin_memcpy(&y0, &m0, 2); __builtin_memcpy(&y1, &m1, 2);
                        ph[q] = (uint32_t)x0 | ((uint32_t)x1 << 16);
                        pm[q] = (uint32_t)y0 | ((uint32_t)y1 << 16);
                        pl[q] = 0u;
                    }
                }
                const bf16x8_t fh = __builtin_bit_cast(bf16x8_t, ph), fm = __builtin_bit_cast(bf16x8_t, pm),
                               fl = __builtin_bit_cast(bf16x8_t, pl);
                const int kr0 = u * 32 + 16 * t + 4 * half + tq;  // this lane's supplied row (+ 8 for j = 4..7)
#pragma unroll
                for (int c = 0; c < DC; ++c) {
                    const int d0 = c * 32 + gd + 4 * tp;
                    const v4i16_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)&Vs[buf][kr0][d0]);
                    const v4i16_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)&Vs[buf][kr0 + 8][d0]);
                    bf16x8_t vf;
                    __builtin_memcpy(&vf, &lo, 8);
                    __builtin_memcpy(reinterpret_cast<char*>(&vf) + 8, &hi, 8);
                    if constexpr (PL == 3) o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, fl, o[c], 0, 0, 0);
                    o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, fm, o[c], 0, 0, 0);
                    o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, fh, o[c], 0, 0, 0);
                }
            }
        }
        if (AB_PRIO & 2) __builtin_amdgcn_s_setprio(0);
        // the next tile into the other buffer (its last readers passed the previous barrier), then one
        // barrier: the tile is visible and every wave is done with this buffer before it is refilled
        AB_LSTORE(Vs[buf ^ 1]);
        __syncthreads();
    }
    if (q_valid) {
        const long orow = (long)s * a.L * a.o_rs + (long)q_lane * a.o_rs + (long)h * a.o_hs;
#pragma unroll
        for (int c = 0; c < DC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d = c * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const float v = o[c][r] / l_run;
                if (a.o_bf16) reinterpret_cast<uint16_t*>(a.o)[orow + d] = bf_bits(v);
                else reinterpret_cast<float*>(a.o)[orow + d] = v;
            }
    }
#undef AB_GLOAD
#undef AB_LSTORE
}

// Ping-pong form (round 6; the dots.ocr tower's 128-dim heads): 8 waves per block as two groups of 4 that
// run one interval apart, so the two waves sharing a SIMD (w and w + 4, one per group) alternate between the
// matrix cores and the VALU.  A wave's work per 64-key tile t is an M phase (P.V of tile t - 1, then
// S^T = K_t . Q^T: 16 + 16 PL MFMAs) and an S phase (mask, online softmax, O rescale, P split into bf16
// planes: VALU only).  With interval I_j ending at block barrier b_j, group 0 runs M_t in I_{2t} and S_t in
// I_{2t+1}; group 1 runs M_t in I_{2t+1} and S_t in I_{2t+2}: in every interval one wave of each SIMD issues
// MFMAs while the other runs its softmax.  The 256 queries of a block (32 per wave) share every K / V tile.
// Staging: tile u = (K_u, V_u), each group writes its half of the rows during an S phase — group 1 in
// I_{2u-2}, group 0 in I_{2u-1} — from registers loaded one tile earlier (bounded buffer loads: keys past
// the sequence read as zeros).  K_u lives in Ks[u & 1] (read in I_{2u}, I_{2u+1}; its previous tile's last
// read I_{2u-3}), V_u in Vs[u % 3] (read in I_{2u+2}, I_{2u+3}; previous last read I_{2u-3}).  Every product
// and sum is the 4-wave kernel's (same tiles, same order per query), so the outputs are bitwise equal to it.
template <int HD, int PL>
__global__ __launch_bounds__(512, 1) void attention_bf16_pp_kernel(AttnBf16Args a) {
    constexpr int KP = HD + 8, VP = HD + 32;  // LDS row pitches (bf16 elements)
    constexpr int C8 = HD / 8;                // 16-byte chunks per row
    constexpr int HR = AB_KT / 2;             // rows of a tile half (one group's share)
    constexpr int NCH = HR * C8 / 256;        // chunks per thread per operand per half
    constexpr int QS = HD / 16, DC = HD / 32;
    static_assert(NCH >= 1 && HR * C8 % 256 == 0, "tile half split over a group's 256 threads");
    __shared__ __attribute__((aligned(16))) uint16_t Ks[2][AB_KT][KP];
    __shared__ __attribute__((aligned(16))) uint16_t Vs[3][AB_KT][VP];
    const int s = blockIdx.z, h = blockIdx.y;
    const int len = a.L;
    const int qb0 = blockIdx.x * (8 * AB_Q);
    if (qb0 >= len) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave >> 2, gt = tid & 255;
    const int half = lane >> 5, l32 = lane & 31;
    const int kvh = h / (a.heads / a.kv_heads);
    const uint16_t* Q = a.q + (long)s * a.L * a.q_rs + (long)h * a.q_hs;
    const uint16_t* K = a.k + (long)s * a.L * a.k_rs + (long)kvh * a.k_hs;
    const uint16_t* V = a.v + (long)s * a.L * a.v_rs + (long)kvh * a.v_hs;
    const int q_lane = qb0 + wave * AB_Q + l32;
    const bool q_valid = q_lane < len;
    bf16x8_t qreg[QS];
    {
        const uint16_t* qr = Q + (long)(q_valid ? q_lane : 0) * a.q_rs + 8 * half;
#pragma unroll
        for (int st = 0; st < QS; ++st) qreg[st] = *reinterpret_cast<const bf16x8_t*>(qr + 16 * st);
    }
    const int i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3, gd = 16 * ((lane >> 4) & 1);
    const int n = (len + AB_KT - 1) / AB_KT;  // key tiles
    // this group's half of a tile: rows HR grp + gt / C8 (+ 256 / C8 per j), chunk gt % C8
    u32x4 rk[NCH], rv[NCH];
    const auto rsk = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(K), (short)0, len * a.k_rs * 2, 0x00020000);
    const auto rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(V), (short)0, len * a.v_rs * 2, 0x00020000);
    const int hrow = HR * grp + gt / C8, hch = (gt % C8) * 8;
    const int ko = (hrow * a.k_rs + hch) * 2, vo = (hrow * a.v_rs + hch) * 2;
    auto gload = [&](int u) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int r = u * AB_KT + j * (256 / C8);
            rk[j] = __builtin_amdgcn_raw_buffer_load_b128(rsk, ko + r * a.k_rs * 2, 0, 0);
            rv[j] = __builtin_amdgcn_raw_buffer_load_b128(rsv, vo + r * a.v_rs * 2, 0, 0);
        }
    };
    auto lstore = [&](int u) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int r = hrow + j * (256 / C8);
            *reinterpret_cast<u32x4*>(&Ks[u & 1][r][hch]) = rk[j];
            *reinterpret_cast<u32x4*>(&Vs[u % 3][r][hch]) = rv[j];
        }
    };
    f32x16 o[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[c][r] = 0.f;
    f32x16 sc[2];
    u32x4 ph[2][2], pm[2][2], pl[2][2];  // P planes of the last S phase, for the next M phase's P.V
    const float c2 = a.scale * 1.4426950408889634f;
    float m_run = -INFINITY, l_run = 0.f;
    // prologue: tile 0 whole (both halves), the next half of each group in flight
    gload(0);
    lstore(0);
    if (n > 1) gload(1);
    __syncthreads();
    for (int j = 0; j < 2 * n + 2; ++j) {
        const int mj = j - grp;  // this group's own interval index
        if (mj == -1) {
            // group 1's first interval: stage its half of tile 1
            if (n > 1) {
                lstore(1);
                if (n > 2) gload(2);
            }
        } else if (mj >= 0 && mj <= 2 * n && (mj & 1) == 0) {
            // M phase of tile t: P.V of tile t - 1, then S^T = K_t . Q^T
            const int t = mj >> 1;
            if (AB_PRIO & 2) __builtin_amdgcn_s_setprio(1);
            if (t > 0) {
                const int vb = (t - 1) % 3;
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int tt = 0; tt < 2; ++tt) {
                        const bf16x8_t fh = __builtin_bit_cast(bf16x8_t, ph[u][tt]), fm = __builtin_bit_cast(bf16x8_t, pm[u][tt]),
                                       fl = __builtin_bit_cast(bf16x8_t, pl[u][tt]);
                        const int kr0 = u * 32 + 16 * tt + 4 * half + tq;
#pragma unroll
                        for (int c = 0; c < DC; ++c) {
                            const int d0 = c * 32 + gd + 4 * tp;
                            const v4i16_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)&Vs[vb][kr0][d0]);
                            const v4i16_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)&Vs[vb][kr0 + 8][d0]);
                            bf16x8_t vf;
                            __builtin_memcpy(&vf, &lo, 8);
                            __builtin_memcpy(reinterpret_cast<char*>(&vf) + 8, &hi, 8);
                            if constexpr (PL == 3) o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, fl, o[c], 0, 0, 0);
                            o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, fm, o[c], 0, 0, 0);
                            o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, fh, o[c], 0, 0, 0);
                        }
                    }
            }
            if (t < n) {
                const int kb = t & 1;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) sc[u][r] = 0.f;
#pragma unroll
                    for (int st = 0; st < QS; ++st) {
                        const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(&Ks[kb][u * 32 + l32][16 * st + 8 * half]);
                        sc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qreg[st], sc[u], 0, 0, 0);
                    }
                }
            }
            if (AB_PRIO & 2) __builtin_amdgcn_s_setprio(0);
        } else if (mj >= 1 && mj < 2 * n) {
            // S phase of tile t: the softmax of its scores, the O rescale, P's planes; then this group's staging
            const int t = mj >> 1;
            const int k0 = t * AB_KT;
            if (k0 + AB_KT > len) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (k0 + u * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= len) sc[u][r] = -INFINITY;
            }
            float tmax = -INFINITY;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sc[u][r]);
            tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
            const float m_new = fmaxf(m_run, tmax * c2);
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
            float psum = 0.f;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float pv = __builtin_amdgcn_exp2f(fmaf(sc[u][r], c2, -m_new));
                    sc[u][r] = pv;
                    psum += pv;
                }
            psum += __shfl_xor(psum, 32, 64);
            l_run = l_run * alpha + psum;
            m_run = m_new;
            if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
                for (int c = 0; c < DC; ++c)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[c][r] *= alpha;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float p0 = sc[u][8 * tt + 2 * q], p1 = sc[u][8 * tt + 2 * q + 1];
                        if constexpr (PL == 3) {
                            const uint32_t b0 = __float_as_uint(p0), b1 = __float_as_uint(p1);
                            const float r0 = p0 - __uint_as_float(b0 & 0xffff0000u), r1 = p1 - __uint_as_float(b1 & 0xffff0000u);
                            const uint32_t c0 = __float_as_uint(r0), c1 = __float_as_uint(r1);
                            const float e0 = r0 - __uint_as_float(c0 & 0xffff0000u), e1 = r1 - __uint_as_float(c1 & 0xffff0000u);
                            ph[u][tt][q] = __builtin_amdgcn_perm(b1, b0, 0x07060302u);
                            pm[u][tt][q] = __builtin_amdgcn_perm(c1, c0, 0x07060302u);
                            pl[u][tt][q] = __builtin_amdgcn_perm(__float_as_uint(e1), __float_as_uint(e0), 0x07060302u);
                        } else {
                            const __bf16 h0 = (__bf16)p0, h1 = (__bf16)p1;
                            const __bf16 m0 = (__bf16)(p0 - (float)h0), m1 = (__bf16)(p1 - (float)h1);
                            uint16_t x0, x1, y0, y1;
                            __builtin_memcpy(&x0, &h0, 2); __builtin_memcpy(&x1, &h1, 2);
                            __builtin_memcpy(&y0, &m0, 2); __builtin_memcpy(&y1, &m1, 2);
                            ph[u][tt][q] = (uint32_t)x0 | ((uint32_t)x1 << 16);
                            pm[u][tt][q] = (uint32_t)y0 | ((uint32_t)y1 << 16);
                            pl[u][tt][q] = 0u;
                        }
                    }
            // staging: group 0 writes its half of tile t + 1, group 1 of tile t + 2; then the next half's loads
            const int u = t + 1 + grp;
            if (u < n) {
                lstore(u);
                if (u + 1 < n) gload(u + 1);
            }
        }
        // every wave's staging stores and tile reads of this interval are done before the next one
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    if (q_valid) {
        const long orow = (long)s * a.L * a.o_rs + (long)q_lane * a.o_rs + (long)h * a.o_hs;
#pragma unroll
        for (int c = 0; c < DC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d = c * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const float v = o[c][r] / l_run;
                if (a.o_bf16) reinterpret_cast<uint16_t*>(a.o)[orow + d] = bf_bits(v);
                else reinterpret_cast<float*>(a.o)[orow + d] = v;
            }
    }
}

// DSOCR_DOTS_ATTN_PP=0 (A/B switch, read at every launch): the 4-wave kernel for 128-dim heads too
static bool attn_pp_on() {
    const char* e = getenv("DSOCR_DOTS_ATTN_PP");
    return !(e && atoi(e) == 0);
}

void launch_attention_bf16(const AttnBf16Args& a, hipStream_t s) {
    if (a.n_seq <= 0 || a.L <= 0) return;
    if (a.hd != 64 && a.hd != 128) throw std::runtime_error("EINVAL: attention_bf16 supports head_dim 64 / 128");
    if (a.kv_heads <= 0 || a.heads % a.kv_heads) throw std::runtime_error("EINVAL: heads must be a multiple of kv_heads");
    if ((a.q_rs | a.k_rs | a.v_rs | a.q_hs | a.k_hs | a.v_hs) % 8)
        throw std::runtime_error("EINVAL: attention_bf16 needs 16-byte aligned rows");
    if ((long)(a.L + AB_KT) * std::max(a.k_rs, a.v_rs) * 2 >= (1L << 31))
        throw std::runtime_error("EINVAL: attention_bf16 sequence slice beyond 32-bit buffer offsets");
    if (a.pv_planes != 2 && a.pv_planes != 3) throw std::runtime_error("EINVAL: attention_bf16 pv_planes is 2 or 3");
    if (a.hd == 128 && attn_pp_on()) {
        const dim3 g2((a.L + 8 * AB_Q - 1) / (8 * AB_Q), a.heads, a.n_seq);
        if (a.pv_planes == 2) DSOCR_LAUNCH((attention_bf16_pp_kernel<128, 2>), g2, dim3(512), 0, s, a);
        else DSOCR_LAUNCH((attention_bf16_pp_kernel<128, 3>), g2, dim3(512), 0, s, a);
        return;
    }
    dim3 grid((a.L + 4 * AB_Q - 1) / (4 * AB_Q), a.heads, a.n_seq);
    if (a.pv_planes == 2) {
        if (a.hd == 128) DSOCR_LAUNCH((attention_bf16_tr_kernel<128, 2>), grid, dim3(256), 0, s, a);
        else DSOCR_LAUNCH((attention_bf16_tr_kernel<64, 2>), grid, dim3(256), 0, s, a);
    } else {
        if (a.hd == 128) DSOCR_LAUNCH((attention_bf16_tr_kernel<128, 3>), grid, dim3(256), 0, s, a);
        else DSOCR_LAUNCH((attention_bf16_tr_kernel<64, 3>), grid, dim3(256), 0, s, a);
    }
}

}  // namespace dsocr
