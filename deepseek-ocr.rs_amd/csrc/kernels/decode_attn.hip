// Decode attention, one token per page (block.rs:608-789 at seq_len 1, with the RoPE of q / the new key
// (block.rs:1403-1471) and the K/V-cache append): flash decoding over the page's f32 cache.
//
// Grid (64-key chunks, heads, pages), 256 threads.  Each wave owns 16 keys and finishes them in registers:
//   * K and V are read like one contiguous stream: instruction i of a wave loads KPI whole keys (1 KiB per
//     instruction, 8 L2 lines), lane l holding dims 4 (l % LPK) .. + 3 of key i * KPI + l / LPK;
//   * the q.k sums finish in a transposing butterfly (xor LPK/2 ... 4 swizzles, then a quad sum: lane l ends
//     with the full dot product of one key), the softmax of the wave's 16 keys is a wave max / sum (DPP), and
//     P.V takes each key's probability by readlane, so a wave needs no LDS and no barrier;
//   * the 4 waves meet once in LDS (m, l, o of each) and the block writes one chunk record write-through;
//   * the chunk records of a (page, head) are merged by chunk 0's block polling them (<= 24 chunks: a
//     sentinel-filled record buffer, no atomics) or by the last arriver of a ticket (longer contexts).
// EARLY: the launch carries kv_bound >= every page's length (the decode loop re-bounds its attention nodes
// per 64-token band), so the K / V loads go out before the position is known — clamped to the bound, not
// to the position; keys past the position are masked at use.  The position is a scalar load.
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

constexpr uint32_t DA3_SENT = 0x7FBADBADu;  // "record word not written yet": a NaN payload no arithmetic produces
constexpr int DA3_CH = 64;                  // keys per block (4 waves x 16)

// transposing butterfly step: n values per lane -> n / 2; lanes with bit (lane & d) keep the upper half
template <int N, int D>
__device__ __forceinline__ void tb_step(float* u, bool hi) {
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
        const float keep = hi ? u[j + N / 2] : u[j], send = hi ? u[j] : u[j + N / 2];
        u[j] = keep + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), 0x1f | (D << 10)));
    }
}

template <int HD, bool PREROT, bool EARLY>
__global__ __launch_bounds__(256) void dec_attn3_kernel(DecAttn2Args a) {
    WaveSpan span_(a.span);
    constexpr int LPK = HD / 4;         // lanes per key (4 dims each)
    constexpr int KPI = 64 / LPK;       // keys per load instruction
    constexpr int NI = 16 / KPI;        // load instructions per operand per wave (16 keys)
    constexpr int PR = HD + 4;          // record: [m, l, -, -, o[HD]]
    static_assert(HD == 32 || HD == 64 || HD == 128, "head_dim 32 / 64 / 128");
    __shared__ float wm[4], wl[4];
    __shared__ __attribute__((aligned(16))) float wo[4][HD];
    __shared__ int last_s;
    __shared__ float mrg[2][256];  // merge: per-thread partial sums of o and l
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int group = a.heads / a.kv_heads, kvh = h / group;
    const int k0 = c * DA3_CH + wave * 16;
    const int kh = lane / LPK, d4 = (lane % LPK) * 4;
    // the position: one scalar load (constant for the launch), consumed after the K / V loads are issued
    const int pos = ((const __attribute__((address_space(4))) int*)(uintptr_t)a.kv_pos)[b];
    float* Kc = a.kc + (long)b * a.page_stride + (long)kvh * a.head_stride;
    float* Vc = a.vc + (long)b * a.page_stride + (long)kvh * a.head_stride;
    const float* row = a.qkv + (long)b * a.ld;
    const float* qrow = row + h * HD;
    const float* krow = row + (a.heads + kvh) * HD;
    const float* vrow = row + (a.heads + a.kv_heads + kvh) * HD;
    float4 kr[NI], vr[NI];
    auto key_of = [&](int i) { return k0 + i * KPI + kh; };
    auto issue = [&](int lim) {
#pragma unroll
        for (int i = 0; i < NI; ++i) kr[i] = *reinterpret_cast<const float4*>(Kc + (long)min(key_of(i), lim) * HD + d4);
#pragma unroll
        for (int i = 0; i < NI; ++i) vr[i] = *reinterpret_cast<const float4*>(Vc + (long)min(key_of(i), lim) * HD + d4);
    };
    float4 qv, kn, vn;
    if (PREROT) {  // q, the new key and value: already rotated rows, independent of the position
        qv = *reinterpret_cast<const float4*>(qrow + d4);
        kn = *reinterpret_cast<const float4*>(krow + d4);
        vn = *reinterpret_cast<const float4*>(vrow + d4);
    }
    if (EARLY) {
        issue(a.kv_bound - 1);
        // the loads above must go out before anything waits for the position: a compiler-only barrier (no
        // instruction, no wait), so they are not sunk below the position test
        asm volatile("" ::: "memory");
    }
    const int len = pos + 1;
    if (c * DA3_CH >= len) return;  // block-uniform
    if (!EARLY) issue(pos);
    if (!PREROT) {
        // RoPE (rotate_half, or the interleaved MLA order) of q and the new key at this lane's 4 dims
        float qa[4], ka[4];
        const float* cs = a.cos + (long)pos * a.rope_dim;
        const float* sn = a.sin + (long)pos * a.rope_dim;
        const int half = a.rope_dim / 2;
        auto map = [&](int i) { return !a.use_mla ? i : (i < half ? 2 * i : 2 * (i - half) + 1); };
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = d4 + j;
            if (d < a.rope_dim) {
                const int ix = map(d), ir = d < half ? map(d + half) : map(d - half);
                const float sg = d < half ? -1.f : 1.f;
                qa[j] = qrow[ix] * cs[d] + (sg * qrow[ir]) * sn[d];
                ka[j] = krow[ix] * cs[d] + (sg * krow[ir]) * sn[d];
            } else {
                qa[j] = qrow[d];
                ka[j] = krow[d];
            }
        }
        qv = make_float4(qa[0], qa[1], qa[2], qa[3]);
        kn = make_float4(ka[0], ka[1], ka[2], ka[3]);
        vn = *reinterpret_cast<const float4*>(vrow + d4);
    }
    // the new key / value: the owning lanes take them from the row and append them to the cache (one
    // writer per kv head: the first head of its group)
    const bool writer = h == kvh * group;
#pragma unroll
    for (int i = 0; i < NI; ++i)
        if (key_of(i) == pos) {
            kr[i] = kn;
            vr[i] = vn;
            if (writer) {
                *reinterpret_cast<float4*>(Kc + (long)pos * HD + d4) = kn;
                *reinterpret_cast<float4*>(Vc + (long)pos * HD + d4) = vn;
            }
        }
    // never 0 * (stale cache bits): keys past the position (loaded under EARLY) contribute exact zeros
#pragma unroll
    for (int i = 0; i < NI; ++i)
        if (key_of(i) > pos) vr[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    // scores: 4-dim partial dot per (lane, instruction), transposing butterfly, quad sum
    float u[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) u[i] = fmaf(qv.w, kr[i].w, fmaf(qv.z, kr[i].z, fmaf(qv.y, kr[i].y, qv.x * kr[i].x)));
    int ti = 0;  // this lane's key after the butterfly: instruction ti
    if constexpr (NI >= 8) { const bool hi = (lane >> 4) & 1; tb_step<8, 16>(u, hi); ti += hi ? 4 : 0; }
    if constexpr (NI >= 4) { const bool hi = (lane >> 3) & 1; tb_step<4, 8>(u, hi); ti += hi ? 2 : 0; }
    if constexpr (NI >= 2) { const bool hi = (lane >> 2) & 1; tb_step<2, 4>(u, hi); ti += hi ? 1 : 0; }
    const float dot = quad_sum(u[0]);
    const int mykey = key_of(ti);
    const bool valid = mykey <= pos;
    const float sc = valid ? dot * a.scale : -INFINITY;
    const float m = wave_max(sc);
    const float p = valid ? expf(sc - m) : 0.f;
    const float l = wave_sum((lane & 3) == 0 ? p : 0.f);
    // P.V: the probability of key (i, kh) sits in lane kh * LPK + (butterfly bits of i)
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        // butterfly bits of instruction i: NI 8 -> lane bits 4, 3, 2; NI 4 -> bits 3, 2; NI 2 -> bit 2
        int src = 0;
        if constexpr (NI == 8) src = ((i >> 2) & 1) * 16 + ((i >> 1) & 1) * 8 + (i & 1) * 4;
        if constexpr (NI == 4) src = ((i >> 1) & 1) * 8 + (i & 1) * 4;
        if constexpr (NI == 2) src = (i & 1) * 4;
        float pk = 0.f;
#pragma unroll
        for (int g = 0; g < KPI; ++g) {
            const float pg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), g * LPK + src));
            pk = kh == g ? pg : pk;
        }
        o.x = fmaf(pk, vr[i].x, o.x);
        o.y = fmaf(pk, vr[i].y, o.y);
        o.z = fmaf(pk, vr[i].z, o.z);
        o.w = fmaf(pk, vr[i].w, o.w);
    }
    // the KPI lane groups hold the same dims for different keys
#pragma unroll
    for (int d = LPK; d < 64; d <<= 1) {
        o.x += __shfl_xor(o.x, d);
        o.y += __shfl_xor(o.y, d);
        o.z += __shfl_xor(o.z, d);
        o.w += __shfl_xor(o.w, d);
    }
    if (lane == 0) { wm[wave] = m; wl[wave] = l; }
    if (lane < LPK) *reinterpret_cast<float4*>(&wo[wave][d4]) = o;
    __syncthreads();
    // chunk record: the 4 waves' partials combined (a wave with no valid key has m = -inf, weight 0)
    const int chunks = (a.max_len + DA3_CH - 1) / DA3_CH;
    float* part0 = a.part + ((long)b * a.heads + h) * chunks * PR;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(part0, (short)0, chunks * PR * 4, 0x00020000);
    const float mc = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    float ew[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) ew[w] = wm[w] == -INFINITY ? 0.f : expf(wm[w] - mc);
    if (tid < HD) {
        const float v = ((ew[0] * wo[0][tid] + ew[1] * wo[1][tid]) + (ew[2] * wo[2][tid] + ew[3] * wo[3][tid]));
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, (c * PR + 4 + tid) * 4, 0, 16);
    }
    if (tid == 0) {
        const float lc = (ew[0] * wl[0] + ew[1] * wl[1]) + (ew[2] * wl[2] + ew[3] * wl[3]);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mc), rsrc, c * PR * 4, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lc), rsrc, (c * PR + 1) * 4, 0, 16);
    }
    // merge: chunk 0 polls (no ticket) or the ticket's last arriver merges
    const int nc = (len + DA3_CH - 1) / DA3_CH;
    const bool poll = a.err != nullptr && nc <= 24 && HD == 128;
    if (poll) {
        if (c != 0) return;
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            int* cnt = a.counters + (long)b * a.heads + h;
            const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == nc - 1;
            if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_s = last;
        }
        __syncthreads();
        if (!last_s) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    }
    auto ld1 = [&](int idx) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, idx * 4, 0, 16)); };
    float* ms = &wo[0][0];   // LDS reuse: [nc] maxima, [nc] sums (nc <= 24 here, else strided below)
    constexpr int KS = 256 / HD;
    const int dim = tid % HD, grp = tid / HD;
    float lsum = 0.f, acc = 0.f;
    if (poll) {
        constexpr int NJ = 12;  // 24 chunks / KS groups (HD 128)
        float ov[NJ];
        const int tc = min(tid, nc - 1);
        float mt, lt0;
        for (unsigned it = 0;; ++it) {
            asm volatile("" ::: "memory");  // the records change under us: re-load them every pass
#pragma unroll
            for (int j = 0; j < NJ; ++j) ov[j] = ld1(min(grp + KS * j, nc - 1) * PR + 4 + dim);
            mt = ld1(tc * PR);
            lt0 = ld1(tc * PR + 1);
            bool pend = __float_as_uint(mt) == DA3_SENT || __float_as_uint(lt0) == DA3_SENT;
#pragma unroll
            for (int j = 0; j < NJ; ++j) pend = pend || __float_as_uint(ov[j]) == DA3_SENT;
            if (!__syncthreads_or(pend)) break;
            if (it > (1u << 20)) {
                if (tid == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        // refill what was read (each word by exactly one thread) for the next launch
        const uint32_t sent = DA3_SENT;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (grp + KS * j < nc) __builtin_amdgcn_raw_buffer_store_b32(sent, rsrc, ((grp + KS * j) * PR + 4 + dim) * 4, 0, 16);
        if (tid < nc) {
            __builtin_amdgcn_raw_buffer_store_b32(sent, rsrc, (tid * PR) * 4, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b32(sent, rsrc, (tid * PR + 1) * 4, 0, 16);
        }
        __syncthreads();  // every wave is past its reads of wo / wm before ms overwrites them
        if (tid < nc) { ms[tid] = mt; ms[32 + tid] = lt0; }
        __syncthreads();
        float mm = -INFINITY;
        for (int cc = 0; cc < nc; ++cc) mm = fmaxf(mm, ms[cc]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int cc = grp + KS * j;
            if (cc < nc) {
                const float w = expf(ms[cc] - mm);
                lsum += ms[32 + cc] * w;
                acc += ov[j] * w;
            }
        }
    } else {
        // any length: running maximum over the chunks in order, each thread folding its strided subset
        float mm = -INFINITY;
        for (int cc = 0; cc < nc; ++cc) mm = fmaxf(mm, ld1(cc * PR));
#pragma unroll 4
        for (int cc = grp; cc < nc; cc += KS) {
            const float w = expf(ld1(cc * PR) - mm);
            lsum += ld1(cc * PR + 1) * w;
            acc += ld1(cc * PR + 4 + dim) * w;
        }
        __syncthreads();  // every wave is past its reads of wo before it is reused
    }
    mrg[0][tid] = acc;
    mrg[1][tid] = lsum;
    __syncthreads();
    if (tid < HD) {
        float at = 0.f, lt = 0.f;
#pragma unroll
        for (int g = 0; g < KS; ++g) { at += mrg[0][g * HD + tid]; lt += mrg[1][g * HD + tid]; }
        a.o[(long)b * a.o_ld + (long)h * HD + tid] = at / lt;
    }
}

void launch_dec_attn3(const DecAttn2Args& a, hipStream_t s) {
    if (!a.counters) throw std::runtime_error("EINTERNAL: dec_attn needs a zeroed counter array");
    if (a.hd != 128 && a.hd != 64 && a.hd != 32) throw std::runtime_error("EINVAL: decode attention supports head_dim 32 / 64 / 128");
    if (a.heads % a.kv_heads) throw std::runtime_error("EINVAL: num_attention_heads must be a multiple of num_key_value_heads");
    const bool early = a.kv_bound > 0 && a.kv_bound <= a.max_len;
    const int span = early ? a.kv_bound : a.max_len;
    dim3 g((span + DA3_CH - 1) / DA3_CH, a.heads, a.B);
    const bool pr = a.prerot != 0;
#define DSOCR_DA3(HDV)                                                                                              \
    do {                                                                                                            \
        if (pr && early) DSOCR_LAUNCH((dec_attn3_kernel<HDV, true, true>), g, dim3(256), 0, s, a);                 \
        else if (pr) DSOCR_LAUNCH((dec_attn3_kernel<HDV, true, false>), g, dim3(256), 0, s, a);                    \
        else if (early) DSOCR_LAUNCH((dec_attn3_kernel<HDV, false, true>), g, dim3(256), 0, s, a);                 \
        else DSOCR_LAUNCH((dec_attn3_kernel<HDV, false, false>), g, dim3(256), 0, s, a);                           \
    } while (0)
    if (a.hd == 128) DSOCR_DA3(128);
    else if (a.hd == 64) DSOCR_DA3(64);
    else DSOCR_DA3(32);
#undef DSOCR_DA3
}

}  // namespace dsocr
