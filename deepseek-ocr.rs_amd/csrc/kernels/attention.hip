// Attention kernels, f32 end to end (the reference keeps scores, softmax and PV
// in f32: sam.rs:837-872, clip.rs:449-453, block.rs:661-775).
//
// 1. attention_fwd: flash-style (online softmax) on the f32 matrix cores.  A wave
//    owns 32 queries; S^T = K.Q^T is computed with v_mfma_f32_32x32x2_f32 so that a
//    lane holds one query's scores, and P feeds the P.V MFMA straight from the
//    accumulator (the k-order of P is permuted and V rows are read in the same
//    permuted order: cdna_hip_programming.md §3 "An accumulator tile as the next
//    MFMA's operand").  K/V tiles of 32 keys are shared by the 4 waves via LDS.
//    Options: decomposed SAM rel-pos bias (sam.rs:1124-1192, never materialising
//    [S,S]), causal masking (block.rs:1504-1526), variable sequence lengths.
// 2. sam_relbias: per-query rel-pos dot products q.Rh / q.Rw.
// 3. rope_kv: rotate_half RoPE (block.rs:1403-1471) + KV-cache append (prefill rows;
//    the decode step fuses both into dec_attn_kernel, decode.hip).
#include <algorithm>
#include <cstdlib>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

constexpr int AT_Q = 32;   // queries per wave
constexpr int AT_KT = 32;  // keys per tile

template <int HD>
__global__ __launch_bounds__(256) void attention_fwd_kernel(AttnArgs a) {
    __shared__ float Ks[AT_KT][HD + 1];
    __shared__ float Vs[AT_KT][HD + 1];
    const int s = blockIdx.z, h = blockIdx.y;
    const int len = a.seq_len ? a.seq_len[s] : a.L;
    const int qb0 = blockIdx.x * (4 * AT_Q);
    if (qb0 >= len) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int half = lane >> 5, l32 = lane & 31;
    const int kvh = h / (a.heads / a.kv_heads);

    const long qoff = a.q.seq_off ? a.q.seq_off[s] : (long)s * a.L * a.q.row_stride;
    const long koff = a.k.seq_off ? a.k.seq_off[s] : (long)s * a.L * a.k.row_stride;
    const long voff = a.v.seq_off ? a.v.seq_off[s] : (long)s * a.L * a.v.row_stride;
    const long ooff = a.o_seq_off ? a.o_seq_off[s] : (long)s * a.L * a.o_row_stride;
    const float* Q = a.q.ptr + qoff + (long)h * a.q.head_stride;
    const float* K = a.k.ptr + koff + (long)kvh * a.k.head_stride;
    const float* V = a.v.ptr + voff + (long)kvh * a.v.head_stride;

    const int q_lane = qb0 + wave * AT_Q + l32;  // this lane's query (lanes l and l+32 share it)
    const bool q_valid = q_lane < len;
    float qreg[HD / 2];
    {
        const float* qr = Q + (long)(q_valid ? q_lane : 0) * a.q.row_stride;
#pragma unroll
        for (int i = 0; i < HD / 2; ++i) qreg[i] = qr[2 * i + half];
    }
    const float* rb = nullptr;
    int R = 0;
    if (a.relbias) {
        R = a.rel_h + a.rel_w;
        rb = a.relbias + (((long)s * a.heads + h) * a.L + (q_valid ? q_lane : 0)) * R;
    }

    f32x16 o[HD / 32];
#pragma unroll
    for (int t = 0; t < HD / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    int kend = len;
    if (a.causal) kend = min(len, qb0 + 4 * AT_Q);
    for (int k0 = 0; k0 < kend; k0 += AT_KT) {
        // stage K/V tile (32 x HD floats each)
        constexpr int F4 = AT_KT * HD / 4;
        for (int i = tid; i < F4; i += 256) {
            const int row = i / (HD / 4), c4 = (i % (HD / 4)) * 4;
            const int key = k0 + row;
            float4 kv4 = make_float4(0.f, 0.f, 0.f, 0.f), vv4 = kv4;
            if (key < len) {
                kv4 = *reinterpret_cast<const float4*>(K + (long)key * a.k.row_stride + c4);
                vv4 = *reinterpret_cast<const float4*>(V + (long)key * a.v.row_stride + c4);
            }
            Ks[row][c4] = kv4.x; Ks[row][c4 + 1] = kv4.y; Ks[row][c4 + 2] = kv4.z; Ks[row][c4 + 3] = kv4.w;
            Vs[row][c4] = vv4.x; Vs[row][c4 + 1] = vv4.y; Vs[row][c4 + 2] = vv4.z; Vs[row][c4 + 3] = vv4.w;
        }
        __syncthreads();

        f32x16 sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
        for (int i = 0; i < HD / 2; ++i)
            sc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ks[l32][2 * i + half], qreg[i], sc, 0, 0, 0);

        float tmax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            float v = sc[r] * a.scale;
            if (rb) v += rb[key / a.rel_w] + rb[a.rel_h + key % a.rel_w];
            if (key >= len || (a.causal && key > q_lane)) v = -INFINITY;
            sc[r] = v;
            tmax = fmaxf(tmax, v);
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = (m_new == -INFINITY) ? 1.f : __expf(m_run - m_new);
        float psum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float p = (m_new == -INFINITY) ? 0.f : __expf(sc[r] - m_new);
            sc[r] = p;
            psum += p;
        }
        psum += __shfl_xor(psum, 32, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
        // rescale O rows (query row of O acc register r lives on lane `row`)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float al = __shfl(alpha, (r & 3) + 8 * (r >> 2) + 4 * half, 64);
#pragma unroll
            for (int t = 0; t < HD / 32; ++t) o[t][r] *= al;
        }
        // O += P.V with the permuted key order kappa(s, half) = (s&3)+8*(s>>2)+4*half
#pragma unroll
        for (int st = 0; st < 16; ++st) {
            const int kr = (st & 3) + 8 * (st >> 2) + 4 * half;
#pragma unroll
            for (int t = 0; t < HD / 32; ++t)
                o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(sc[st], Vs[kr][t * 32 + l32], o[t], 0, 0, 0);
        }
        __syncthreads();
    }
    // normalise and store: O acc col = d (lane&31), row = query
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int qrow = (r & 3) + 8 * (r >> 2) + 4 * half;
        const float lr = __shfl(l_run, qrow, 64);
        const int q = qb0 + wave * AT_Q + qrow;
        if (q < len) {
            float* op = a.o + ooff + (long)q * a.o_row_stride + (long)h * a.o_head_stride;
#pragma unroll
            for (int t = 0; t < HD / 32; ++t) op[t * 32 + l32] = o[t][r] / lr;
        }
    }
}

// attention_fwd2: the same flash attention with the P.V product computed TRANSPOSED
// (O^T = V^T . P^T: the accumulator's column is the lane's own query, so the online-softmax
// rescale needs no cross-lane shuffles), the dot-product dims split as d = i + half * HD/2 so
// every K fragment is a 16-byte LDS read, V staged transposed in LDS (16-byte reads of 4 keys),
// K/V tile t+1 prefetched into registers while tile t is consumed (one barrier per tile), and the
// rel-pos bias column indices of a tile computed once per tile in LDS (no per-score division).
//
// SPLIT (the causal prefill, round 4): the keys of a 128-query block are split into pieces of AT_KSPLIT keys,
// one block per (query block, piece) — at one 706-token page 60 blocks with 1..6 pieces of work became 210
// blocks of one piece each — and every block writes its unnormalised partial (m, l, o) per query;
// attention_merge_kernel combines a query's pieces in piece order (flash-decoding combine).
constexpr int AT_KSPLIT = 128;

// (query block, key piece) of pair p, pairs enumerated query-block-major over the grid's length L
__device__ __forceinline__ void split_pair(int p, int L, int& qb, int& ks) {
    for (qb = 0;; ++qb) {
        const int n = (min(L, (qb + 1) * 4 * AT_Q) + AT_KSPLIT - 1) / AT_KSPLIT;
        if (p < n || n == 0) { ks = p; return; }
        p -= n;
    }
}
// first pair of query block qb
__device__ __host__ inline int split_first_pair(int qb, int L) {
    int off = 0;
    for (int j = 0; j < qb; ++j) off += (std::min(L, (j + 1) * 4 * AT_Q) + AT_KSPLIT - 1) / AT_KSPLIT;
    return off;
}

template <int HD, bool REL, bool SPLIT = false>
__global__ __launch_bounds__(256, 1) void attention_fwd2_kernel(AttnArgs a) {
    constexpr int KP = HD + 4, VP = AT_KT + 4;
    constexpr int F4 = AT_KT * HD / 4 / 256;  // float4 per thread per operand per tile
    static_assert(!(SPLIT && REL), "the split form serves the causal prefill (no rel-pos bias)");
    __shared__ __attribute__((aligned(16))) float Ks[2][AT_KT][KP];
    __shared__ __attribute__((aligned(16))) float Vt[2][HD][VP];
    __shared__ int rbh[2][AT_KT], rbw[2][AT_KT];
    const int s = blockIdx.z, h = blockIdx.y;
    const int len = a.seq_len ? a.seq_len[s] : a.L;
    int qblk = blockIdx.x, kpiece = 0;
    if (SPLIT) split_pair(blockIdx.x, a.L, qblk, kpiece);
    const int qb0 = qblk * (4 * AT_Q);
    if (qb0 >= len) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int half = lane >> 5, l32 = lane & 31;
    const int kvh = h / (a.heads / a.kv_heads);
    const long qoff = a.q.seq_off ? a.q.seq_off[s] : (long)s * a.L * a.q.row_stride;
    const long koff = a.k.seq_off ? a.k.seq_off[s] : (long)s * a.L * a.k.row_stride;
    const long voff = a.v.seq_off ? a.v.seq_off[s] : (long)s * a.L * a.v.row_stride;
    const long ooff = a.o_seq_off ? a.o_seq_off[s] : (long)s * a.L * a.o_row_stride;
    const float* Q = a.q.ptr + qoff + (long)h * a.q.head_stride;
    const float* K = a.k.ptr + koff + (long)kvh * a.k.head_stride;
    const float* V = a.v.ptr + voff + (long)kvh * a.v.head_stride;
    const int q_lane = qb0 + wave * AT_Q + l32;
    const bool q_valid = q_lane < len;
    float qreg[HD / 2];
    {
        const float* qr = Q + (long)(q_valid ? q_lane : 0) * a.q.row_stride + half * (HD / 2);
#pragma unroll
        for (int i = 0; i < HD / 2; i += 4) {
            const float4 v4 = *reinterpret_cast<const float4*>(qr + i);
            qreg[i] = v4.x; qreg[i + 1] = v4.y; qreg[i + 2] = v4.z; qreg[i + 3] = v4.w;
        }
    }
    // REL: the block's 128 query rows of the rel-pos table staged once into LDS (row pitch R + 1:
    // the lanes of a wave read 32 different rows at one column without bank conflicts)
    extern __shared__ __attribute__((aligned(16))) float rbs[];
    const int R = a.rel_h + a.rel_w, RP = R + 1;
    const float* rb = nullptr;
    if (REL) {
        const float* tab = a.relbias + (((long)s * a.heads + h) * a.L) * R;
        for (int i = tid; i < 4 * AT_Q * R; i += 256) {
            const int ql = i / R, j = i % R;
            rbs[ql * RP + j] = tab[(long)min(qb0 + ql, len - 1) * R + j];
        }
        rb = rbs + (wave * AT_Q + l32) * RP;
    }
    int kend = len;
    if (a.causal) kend = min(len, qb0 + 4 * AT_Q);
    int kbeg = 0;
    if (SPLIT) {
        kbeg = kpiece * AT_KSPLIT;
        if (kbeg >= kend) return;  // past this sequence's keys (a shorter sequence of the batch)
        kend = min(kend, kbeg + AT_KSPLIT);
    }
    // staging: thread covers float4 f = tid + 256 j of the tile: key f / (HD/4), cols (f % (HD/4)) * 4
    // (macros, not lambdas: a captured register array is demoted to scratch)
    float4 rk[F4], rv[F4];
#define AT2_GLOAD(K0)                                                                          \
    _Pragma("unroll") for (int j = 0; j < F4; ++j) {                                           \
        const int f = tid + 256 * j;                                                           \
        const int key = min((K0) + f / (HD / 4), len - 1);                                     \
        const int c4 = (f % (HD / 4)) * 4;                                                     \
        rk[j] = *reinterpret_cast<const float4*>(K + (long)key * a.k.row_stride + c4);         \
        rv[j] = *reinterpret_cast<const float4*>(V + (long)key * a.v.row_stride + c4);         \
    }
#define AT2_LSTORE(BUF, K0)                                                                    \
    _Pragma("unroll") for (int j = 0; j < F4; ++j) {                                           \
        const int f = tid + 256 * j;                                                           \
        const int kr = f / (HD / 4), c4 = (f % (HD / 4)) * 4;                                  \
        *reinterpret_cast<float4*>(&Ks[BUF][kr][c4]) = rk[j];                                  \
        Vt[BUF][c4 + 0][kr] = rv[j].x;                                                         \
        Vt[BUF][c4 + 1][kr] = rv[j].y;                                                         \
        Vt[BUF][c4 + 2][kr] = rv[j].z;                                                         \
        Vt[BUF][c4 + 3][kr] = rv[j].w;                                                         \
    }                                                                                          \
    if (REL && tid < AT_KT) {                                                                  \
        const int key = (K0) + tid;                                                            \
        rbh[BUF][tid] = key / a.rel_w;                                                         \
        rbw[BUF][tid] = a.rel_h + key % a.rel_w;                                               \
    }
    f32x16 o[HD / 32];
#pragma unroll
    for (int t = 0; t < HD / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    AT2_GLOAD(kbeg);
    AT2_LSTORE(0, kbeg);
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += AT_KT, buf ^= 1) {
        AT2_GLOAD(k0 + AT_KT);  // unconditional (clamped keys): a guarded prefetch demotes rk/rv to scratch
        // S^T = K . Q^T: lane (half, l32) feeds dims i + half*HD/2
        f32x16 sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
        for (int i = 0; i < HD / 2; i += 4) {
            const float4 k4 = *reinterpret_cast<const float4*>(&Ks[buf][l32][half * (HD / 2) + i]);
            sc = __builtin_amdgcn_mfma_f32_32x32x2f32(k4.x, qreg[i], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x2f32(k4.y, qreg[i + 1], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x2f32(k4.z, qreg[i + 2], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x2f32(k4.w, qreg[i + 3], sc, 0, 0, 0);
        }
        // rel-pos bias: every table load of the tile issued together (REL is a template flag:
        // a runtime `if (rb)` per score became 16 exec-masked branches with a vmcnt(0) each)
        float bias[16];
        if (REL) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int kl = (r & 3) + 8 * (r >> 2) + 4 * half;
                bias[r] = rb[rbh[buf][kl]] + rb[rbw[buf][kl]];
            }
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int kl = (r & 3) + 8 * (r >> 2) + 4 * half;
            const int key = k0 + kl;
            float v = sc[r] * a.scale;
            if (REL) v += bias[r];
            if (key >= len || (a.causal && key > q_lane)) v = -INFINITY;
            sc[r] = v;
            tmax = fmaxf(tmax, v);
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = (m_new == -INFINITY) ? 1.f : __expf(m_run - m_new);
        float psum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = (m_new == -INFINITY) ? 0.f : __expf(sc[r] - m_new);
            sc[r] = p;
            psum += p;
        }
        psum += __shfl_xor(psum, 32, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
#pragma unroll
        for (int t = 0; t < HD / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
        // O^T += V^T . P^T, keys in the accumulator's permuted order kappa(st, half)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int kb = 8 * g4 + 4 * half;
#pragma unroll
            for (int t = 0; t < HD / 32; ++t) {
                const float4 v4 = *reinterpret_cast<const float4*>(&Vt[buf][t * 32 + l32][kb]);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.x, sc[4 * g4 + 0], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.y, sc[4 * g4 + 1], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.z, sc[4 * g4 + 2], o[t], 0, 0, 0);
                o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.w, sc[4 * g4 + 3], o[t], 0, 0, 0);
            }
        }
        AT2_LSTORE(buf ^ 1, k0 + AT_KT);
        __syncthreads();
    }
    if (SPLIT) {  // unnormalised partial of this key piece: [m, l, o[HD]] per query of the block
        if (q_valid) {
            const int npairs = split_first_pair((a.L + 4 * AT_Q - 1) / (4 * AT_Q), a.L);
            float* rec = a.part + ((((long)s * a.heads + h) * npairs + blockIdx.x) * (4 * AT_Q) + (q_lane - qb0)) * (HD + 2);
            if (half == 0) { rec[0] = m_run; rec[1] = l_run; }
#pragma unroll
            for (int t = 0; t < HD / 32; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) rec[2 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * half] = o[t][r];
        }
        return;
    }
    // O^T accumulator: row = d (within t), column = this lane's query
    if (q_valid) {
        float* op = a.o + ooff + (long)q_lane * a.o_row_stride + (long)h * a.o_head_stride;
#pragma unroll
        for (int t = 0; t < HD / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) op[t * 32 + (r & 3) + 8 * (r >> 2) + 4 * half] = o[t][r] / l_run;
    }
#undef AT2_GLOAD
#undef AT2_LSTORE
}

// combine of the key pieces (SPLIT above): thread (query, d); m = max m_i, l = sum l_i e^(m_i - m),
// o = sum o_i e^(m_i - m), all in piece order; out = o / l
template <int HD>
__global__ __launch_bounds__(256) void attention_merge_kernel(AttnArgs a) {
    const int s = blockIdx.z, h = blockIdx.y;
    const int len = a.seq_len ? a.seq_len[s] : a.L;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    const int q = (int)(idx / HD), d = (int)(idx % HD);
    if (q >= len) return;
    const int qb = q / (4 * AT_Q), ql = q % (4 * AT_Q);
    const int kend = a.causal ? min(len, (qb + 1) * 4 * AT_Q) : len;
    const int n = (kend + AT_KSPLIT - 1) / AT_KSPLIT;
    const int npairs = split_first_pair((a.L + 4 * AT_Q - 1) / (4 * AT_Q), a.L);
    const float* rec0 = a.part + ((((long)s * a.heads + h) * npairs + split_first_pair(qb, a.L)) * (4 * AT_Q) + ql) * (HD + 2);
    const long pstride = (long)(4 * AT_Q) * (HD + 2);
    float m = -INFINITY;
    for (int i = 0; i < n; ++i) m = fmaxf(m, rec0[i * pstride]);
    float l = 0.f, acc = 0.f;
    for (int i = 0; i < n; ++i) {
        const float* r = rec0 + i * pstride;
        const float w = r[0] == -INFINITY ? 0.f : __expf(r[0] - m);
        l += r[1] * w;
        acc += r[2 + d] * w;
    }
    const long ooff = a.o_seq_off ? a.o_seq_off[s] : (long)s * a.L * a.o_row_stride;
    a.o[ooff + (long)q * a.o_row_stride + (long)h * a.o_head_stride + d] = acc / l;
}

size_t attention_causal_part_floats(int n_seq, int heads, int L, int hd) {
    const int nqb = (L + 4 * AT_Q - 1) / (4 * AT_Q);
    return (size_t)n_seq * heads * split_first_pair(nqb, L) * (4 * AT_Q) * (hd + 2);
}

// attention_split: the same exact-f32 attention (64-dim heads, uniform sequences, no causal mask: the
// SAM and CLIP towers) on the bf16 matrix cores.  Every f32 operand is split exactly into three bf16
// planes x = hi + mid + lo (RNE at each step, residuals exact) and each product takes the six plane
// pairs whose weight reaches the f32 rounding of the product (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi,
// mid.mid; the dropped mid.lo, lo.mid, lo.lo are below 2^-24 of |x||y|): QK^T and P.V as 6 bf16 MFMA
// passes each, 16x the f32-MFMA rate per pass, so 2.7x fewer MFMA cycles than attention_fwd2 for
// the same f32-accurate result (summation order aside).  Layout as attention_bf16_tr_kernel: S^T = K.Q^T
// (the lane's own query in the accumulator column), O^T = V^T.P^T with V stored row-major as planes and
// read as the V^T operand through ds_read_b64_tr_b16; K / V planes split once per tile at staging
// (the next tile's f32 loads in registers under the current tile's compute); SAM's decomposed rel-pos
// bias from the block's table rows in LDS as in attention_fwd2.
// Eight waves per block, two per SIMD: waves w and w + 4 own the same 32 queries and take the two 32-key
// halves of every 64-key tile, each with its own running (m, l, O); the pair combines through LDS at the
// end (flash-decoding combine of two pieces).  One wave's softmax and plane splits then run under the
// other wave's MFMAs on the same SIMD (the block's LDS — the rel-pos rows of its 128 queries, 66 KB for
// the 64x64 SAM grid — allows one block per CU, so a second wave per SIMD has to come from the block).
typedef __bf16 bf16x8s_t __attribute__((ext_vector_type(8)));
typedef short v4i16s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16s_t lds_v4i16s;

__device__ __forceinline__ void split3_bf16(float v, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)v;
    const float r1 = v - (float)h;
    m = (__bf16)r1;
    l = (__bf16)(r1 - (float)m);
}

constexpr int AS_NT = 512;

template <bool REL>
__global__ __launch_bounds__(AS_NT, 1) void attention_split_kernel(AttnArgs a) {
    constexpr int HD = 64, KT = 64;
    constexpr int KP = HD + 8, VP = HD + 32;   // plane row pitches (bf16): VP keeps 4 rows on distinct banks
    constexpr int QS = HD / 16, DC = HD / 32;
    constexpr int F4 = KT * HD / 4 / AS_NT;    // float4 per thread per operand per tile
    constexpr int OW = DC * 16 + 2;            // floats a key-half wave hands its partner: O, m, l
    __shared__ __attribute__((aligned(16))) uint16_t Kp[3][KT][KP];
    __shared__ __attribute__((aligned(16))) uint16_t Vp[3][KT][VP];
    static_assert(sizeof(Vp) >= 4 * OW * 64 * sizeof(float), "combine records reuse the V planes");
    __shared__ int rbh[KT], rbw[KT];
    extern __shared__ __attribute__((aligned(16))) float rbs[];
    const int s = blockIdx.z, h = blockIdx.y;
    const int len = a.L;
    const int qb0 = blockIdx.x * (4 * AT_Q);
    if (qb0 >= len) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qg = wave & 3, kh = wave >> 2;   // query group, key half of each tile
    const int half = lane >> 5, l32 = lane & 31;
    const int kvh = h / (a.heads / a.kv_heads);
    const float* Q = a.q.ptr + (long)s * a.L * a.q.row_stride + (long)h * a.q.head_stride;
    const float* K = a.k.ptr + (long)s * a.L * a.k.row_stride + (long)kvh * a.k.head_stride;
    const float* V = a.v.ptr + (long)s * a.L * a.v.row_stride + (long)kvh * a.v.head_stride;
    const int q_lane = qb0 + qg * AT_Q + l32;
    const bool q_valid = q_lane < len;
    // this lane's query as three planes: dims 16 st + 8 half + j
    bf16x8s_t qh[QS], qm[QS], ql[QS];
    {
        const float* qr = Q + (long)(q_valid ? q_lane : 0) * a.q.row_stride + 8 * half;
#pragma unroll
        for (int st = 0; st < QS; ++st) {
            const float4 x0 = *reinterpret_cast<const float4*>(qr + 16 * st);
            const float4 x1 = *reinterpret_cast<const float4*>(qr + 16 * st + 4);
            const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 hh, mm, ll;
                split3_bf16(xv[j], hh, mm, ll);
                qh[st][j] = hh; qm[st][j] = mm; ql[st][j] = ll;
            }
        }
    }
    const int R = a.rel_h + a.rel_w, RP = R + 1;
    const float* rb = nullptr;
    if (REL) {
        const float* tab = a.relbias + (((long)s * a.heads + h) * a.L) * R;
        for (int i = tid; i < 4 * AT_Q * R; i += AS_NT) {
            const int qq = i / R, j = i % R;
            rbs[qq * RP + j] = tab[(long)min(qb0 + qq, len - 1) * R + j];
        }
        rb = rbs + (qg * AT_Q + l32) * RP;
    }
    const int i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3, gd = 16 * ((lane >> 4) & 1);
    // next tile's K / V in registers: buffer loads bounded at the sequence's last key (keys past it read
    // as zeros: no clamps), one per-lane offset plus the tile's uniform row offset
    f32x4 rk[F4], rv[F4];
    const auto rsk = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(K), (short)0, len * a.k.row_stride * 4, 0x00020000);
    const auto rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(V), (short)0, len * a.v.row_stride * 4, 0x00020000);
    const int ko = ((tid / (HD / 4)) * a.k.row_stride + (tid % (HD / 4)) * 4) * 4;
    const int vo = ((tid / (HD / 4)) * a.v.row_stride + (tid % (HD / 4)) * 4) * 4;
#define AS_GLOAD(K0)                                                                           \
    _Pragma("unroll") for (int j = 0; j < F4; ++j) {                                           \
        const int kr_ = (K0) + j * (AS_NT / (HD / 4));                                         \
        rk[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsk, ko + kr_ * a.k.row_stride * 4, 0, 0)); \
        rv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsv, vo + kr_ * a.v.row_stride * 4, 0, 0)); \
    }
#define AS_PUT(P, KEY, C4, X)                                                                  \
    {                                                                                          \
        const float xv_[4] = {(X)[0], (X)[1], (X)[2], (X)[3]};                                 \
        uint16_t hb_[4], mb_[4], lb_[4];                                                       \
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                        \
            __bf16 hh, mm, ll;                                                                 \
            split3_bf16(xv_[e], hh, mm, ll);                                                   \
            __builtin_memcpy(&hb_[e], &hh, 2);                                                 \
            __builtin_memcpy(&mb_[e], &mm, 2);                                                 \
            __builtin_memcpy(&lb_[e], &ll, 2);                                                 \
        }                                                                                      \
        __builtin_memcpy(&P[0][KEY][C4], hb_, 8);                                              \
        __builtin_memcpy(&P[1][KEY][C4], mb_, 8);                                              \
        __builtin_memcpy(&P[2][KEY][C4], lb_, 8);                                              \
    }
#define AS_LSTORE(K0)                                                                          \
    _Pragma("unroll") for (int j = 0; j < F4; ++j) {                                           \
        const int f = tid + AS_NT * j;                                                         \
        const int kr = f / (HD / 4), c4 = (f % (HD / 4)) * 4;                                  \
        AS_PUT(Kp, kr, c4, rk[j]);                                                             \
        AS_PUT(Vp, kr, c4, rv[j]);                                                             \
    }                                                                                          \
    if (REL && tid < KT) {                                                                     \
        const int key = (K0) + tid;                                                            \
        rbh[tid] = key / a.rel_w;                                                              \
        rbw[tid] = a.rel_h + key % a.rel_w;                                                    \
    }
    f32x16 o[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[c][r] = 0.f;
    const float c2 = (REL ? 1.f : a.scale) * 1.4426950408889634f;  // score -> log2 units
    float m_run = -INFINITY, l_run = 0.f;
    const int u = kh;  // this wave's 32 keys of every tile: 32 u .. 32 u + 31
    AS_GLOAD(0);
    AS_LSTORE(0);
    __syncthreads();
    for (int k0 = 0; k0 < len; k0 += KT) {
        AS_GLOAD(k0 + KT);  // the next tile in flight under this one
        f32x16 sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
        for (int st = 0; st < QS; ++st) {
            const int kr = u * 32 + l32, kc = 16 * st + 8 * half;
            const bf16x8s_t kh8 = *reinterpret_cast<const bf16x8s_t*>(&Kp[0][kr][kc]);
            const bf16x8s_t km8 = *reinterpret_cast<const bf16x8s_t*>(&Kp[1][kr][kc]);
            const bf16x8s_t kl8 = *reinterpret_cast<const bf16x8s_t*>(&Kp[2][kr][kc]);
            sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl8, qh[st], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(km8, qm[st], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8, ql[st], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(km8, qh[st], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8, qm[st], sc, 0, 0, 0);
            sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8, qh[st], sc, 0, 0, 0);
        }
        // softmax in the log2 domain (p = 2^(v c - m), one FMA before the exponential); SAM adds its rel-pos
        // bias to the scaled score first, as the reference does.  A key half can be all past the sequence
        // (the last tile, or every tile when len <= 32): m stays -inf and exponentials are taken against 0.
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int kl = u * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            if (REL) sc[r] = fmaf(sc[r], a.scale, rb[rbh[kl]] + rb[rbw[kl]]);
        }
        if (k0 + KT > len) {  // the last, partial tile
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (k0 + u * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= len) sc[r] = -INFINITY;
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sc[r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float m_new = fmaxf(m_run, tmax * c2);
        const float m_ref = m_new == -INFINITY ? 0.f : m_new;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_ref);
        float psum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sc[r], c2, -m_ref));
            sc[r] = p;
            psum += p;
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
        // O^T += V^T . P^T: the lane's P registers 8t .. 8t+7 hold keys 32u + 16t + 4 half + {0..3, 8..11};
        // the transposed reads fetch exactly those rows of each V plane
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            // p = hi + mid + lo exactly by truncation (low 16 bits cleared, twice; the rest has <= 8
            // significant bits), two bf16 of a plane packed per register by one byte permute
            f32x4 phv, pmv, plv;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float p0 = sc[8 * t + 2 * q], p1 = sc[8 * t + 2 * q + 1];
                const uint32_t b0 = __float_as_uint(p0), b1 = __float_as_uint(p1);
                const float r0 = p0 - __uint_as_float(b0 & 0xffff0000u), r1 = p1 - __uint_as_float(b1 & 0xffff0000u);
                const uint32_t c0 = __float_as_uint(r0), c1 = __float_as_uint(r1);
                const float e0 = r0 - __uint_as_float(c0 & 0xffff0000u), e1 = r1 - __uint_as_float(c1 & 0xffff0000u);
                phv[q] = __uint_as_float(__builtin_amdgcn_perm(b1, b0, 0x07060302u));
                pmv[q] = __uint_as_float(__builtin_amdgcn_perm(c1, c0, 0x07060302u));
                plv[q] = __uint_as_float(__builtin_amdgcn_perm(__float_as_uint(e1), __float_as_uint(e0), 0x07060302u));
            }
            const bf16x8s_t ph = __builtin_bit_cast(bf16x8s_t, phv), pm = __builtin_bit_cast(bf16x8s_t, pmv),
                            pl = __builtin_bit_cast(bf16x8s_t, plv);
            const int kr0 = u * 32 + 16 * t + 4 * half + tq;
#pragma unroll
            for (int c = 0; c < DC; ++c) {
                const int d0 = c * 32 + gd + 4 * tp;
                bf16x8s_t vf[3];
#pragma unroll
                for (int pl_ = 0; pl_ < 3; ++pl_) {
                    const v4i16s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16s*)&Vp[pl_][kr0][d0]);
                    const v4i16s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16s*)&Vp[pl_][kr0 + 8][d0]);
                    __builtin_memcpy(&vf[pl_], &lo, 8);
                    __builtin_memcpy(reinterpret_cast<char*>(&vf[pl_]) + 8, &hi, 8);
                }
                o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2], ph, o[c], 0, 0, 0);
                o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[1], pm, o[c], 0, 0, 0);
                o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[0], pl, o[c], 0, 0, 0);
                o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[1], ph, o[c], 0, 0, 0);
                o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[0], pm, o[c], 0, 0, 0);
                o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[0], ph, o[c], 0, 0, 0);
            }
        }
        __syncthreads();  // every wave is done with the tile before it is refilled
        AS_LSTORE(k0 + KT);
        __syncthreads();
    }
    // combine the two key halves: the second half's waves hand (O, m, l) over through the V planes' LDS
    // (no wave reads a plane after the loop's last barrier), lane-contiguous records
    float* rec = reinterpret_cast<float*>(&Vp[0][0][0]) + qg * OW * 64 + lane;
    if (kh == 1) {
#pragma unroll
        for (int c = 0; c < DC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) rec[(c * 16 + r) * 64] = o[c][r];
        rec[(DC * 16) * 64] = m_run;
        rec[(DC * 16 + 1) * 64] = l_run;
    }
    __syncthreads();
    if (kh == 0 && q_valid) {
        const float m_b = rec[(DC * 16) * 64], l_b = rec[(DC * 16 + 1) * 64];
        const float m = fmaxf(m_run, m_b);
        const float a0 = __builtin_amdgcn_exp2f(m_run - m), a1 = __builtin_amdgcn_exp2f(m_b - m);
        const float inv = 1.f / (l_run * a0 + l_b * a1);
        float* op = a.o + (long)s * a.L * a.o_row_stride + (long)q_lane * a.o_row_stride + (long)h * a.o_head_stride;
#pragma unroll
        for (int c = 0; c < DC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                op[c * 32 + (r & 3) + 8 * (r >> 2) + 4 * half] = (o[c][r] * a0 + rec[(c * 16 + r) * 64] * a1) * inv;
    }
#undef AS_GLOAD
#undef AS_PUT
#undef AS_LSTORE
}

// DSOCR_ATTN_SPLIT=0 (A/B switch, read once): the SAM / CLIP attention on the f32 MFMA (attention_fwd2)
static bool attn_split_on() {
    static const bool v = !(getenv("DSOCR_ATTN_SPLIT") && atoi(getenv("DSOCR_ATTN_SPLIT")) == 0);
    return v;
}

// DSOCR_ATTN_KSPLIT=0 (A/B switch, read at every launch): the causal prefill without key pieces
static bool attn_ksplit_on() {
    const char* e = getenv("DSOCR_ATTN_KSPLIT");
    return !(e && atoi(e) == 0);
}

void launch_attention(const AttnArgs& a, hipStream_t s) {
    int maxlen = a.L;
    dim3 grid((maxlen + 4 * AT_Q - 1) / (4 * AT_Q), a.heads, a.n_seq);
    if (grid.x == 0 || a.n_seq == 0) return;
    AttnArgs b = a;
    if (b.kv_heads == 0) b.kv_heads = b.heads;
    if (a.hd == 64 && !a.causal && !a.seq_len && !a.q.seq_off && !a.k.seq_off && !a.v.seq_off && !a.o_seq_off &&
        (long)(a.L + 64) * std::max(a.k.row_stride, a.v.row_stride) * 4 < (1L << 31) && attn_split_on()) {
        // the vision towers: exact-f32 products on the bf16 matrix cores (6 plane pairs)
        const bool rel = b.relbias != nullptr;
        const size_t lds = rel ? (size_t)4 * AT_Q * (b.rel_h + b.rel_w + 1) * 4 : 0;
        static bool attr_s = false;
        if (!attr_s) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_split_kernel<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 90 * 1024);
            attr_s = true;
        }
        if (lds <= 90 * 1024) {
            if (rel) hipLaunchKernelGGL((attention_split_kernel<true>), grid, dim3(AS_NT), lds, s, b);
            else hipLaunchKernelGGL((attention_split_kernel<false>), grid, dim3(AS_NT), 0, s, b);
            return;
        }
    }
    if ((a.hd == 64 || a.hd == 128) && a.causal && !a.relbias && a.part &&
        a.part_floats >= attention_causal_part_floats(a.n_seq, a.heads, a.L, a.hd) && attn_ksplit_on()) {
        // the causal prefill: one block per (query block, key piece), then the piece combine
        const int nqb = (a.L + 4 * AT_Q - 1) / (4 * AT_Q);
        const dim3 g1(split_first_pair(nqb, a.L), a.heads, a.n_seq);
        const dim3 g2((unsigned)(((long)a.L * a.hd + 255) / 256), a.heads, a.n_seq);
        if (a.hd == 64) {
            hipLaunchKernelGGL((attention_fwd2_kernel<64, false, true>), g1, dim3(256), 0, s, b);
            hipLaunchKernelGGL(attention_merge_kernel<64>, g2, dim3(256), 0, s, b);
        } else {
            hipLaunchKernelGGL((attention_fwd2_kernel<128, false, true>), g1, dim3(256), 0, s, b);
            hipLaunchKernelGGL(attention_merge_kernel<128>, g2, dim3(256), 0, s, b);
        }
        return;
    }
    if (a.hd == 64 || a.hd == 128) {  // exact-f32 MFMA flash attention; other head dims: attention_fwd_kernel
        const bool rel = b.relbias != nullptr;
        const size_t lds = rel ? (size_t)4 * AT_Q * (b.rel_h + b.rel_w + 1) * 4 : 0;
        static bool attr = false;
        if (!attr) {  // dynamic LDS beyond 64 KB (the global SAM table: 128 rows x 129 floats)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_fwd2_kernel<64, true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_fwd2_kernel<128, true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
            attr = true;
        }
        if (a.hd == 64) {
            if (rel) hipLaunchKernelGGL((attention_fwd2_kernel<64, true>), grid, dim3(256), lds, s, b);
            else hipLaunchKernelGGL((attention_fwd2_kernel<64, false>), grid, dim3(256), 0, s, b);
        } else {
            if (rel) hipLaunchKernelGGL((attention_fwd2_kernel<128, true>), grid, dim3(256), lds, s, b);
            else hipLaunchKernelGGL((attention_fwd2_kernel<128, false>), grid, dim3(256), 0, s, b);
        }
        return;
    }
    if (a.hd == 64) hipLaunchKernelGGL(attention_fwd_kernel<64>, grid, dim3(256), 0, s, b);
    else if (a.hd == 128) hipLaunchKernelGGL(attention_fwd_kernel<128>, grid, dim3(256), 0, s, b);
    else if (a.hd == 32) hipLaunchKernelGGL(attention_fwd_kernel<32>, grid, dim3(256), 0, s, b);
}

// ------------------------------------------------------------------ SAM rel-pos bias
__global__ __launch_bounds__(256) void sam_relbias_kernel(const float* q, long q_rs, int n_seq, int gh, int gw,
                                                          int heads, int hd, const float* Rh, const float* Rw,
                                                          float* out) {
    const int R = gh + gw;
    const int L = gh * gw;
    const long total = (long)n_seq * heads * L * R;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
        const int j = (int)(idx % R);
        long t = idx / R;
        const int qi = (int)(t % L);
        t /= L;
        const int h = (int)(t % heads);
        const int s = (int)(t / heads);
        const float* qr = q + ((long)s * L + qi) * q_rs + (long)h * hd;
        const float* rr;
        if (j < gh) {
            const int qh = qi / gw;
            rr = Rh + (long)(qh - j + gh - 1) * hd;
        } else {
            const int qw = qi % gw, kw = j - gh;
            rr = Rw + (long)(qw - kw + gw - 1) * hd;
        }
        float acc = 0.f;
        for (int d = 0; d < hd; d += 4) {
            float4 a4 = *reinterpret_cast<const float4*>(qr + d);
            float4 b4 = *reinterpret_cast<const float4*>(rr + d);
            acc = fmaf(a4.x, b4.x, acc);
            acc = fmaf(a4.y, b4.y, acc);
            acc = fmaf(a4.z, b4.z, acc);
            acc = fmaf(a4.w, b4.w, acc);
        }
        out[idx] = acc;
    }
}

// Thread per query (one head per block row): the query row lives in registers, the two rel-pos
// tables of the head dim in LDS (row pitch hd + 1: lanes reading different rows of one column do
// not collide on a bank), the R outputs of the query written contiguously.  Same dot-product order
// as sam_relbias_kernel (d ascending, one fmaf chain).
template <int HD>
__global__ __launch_bounds__(256) void sam_relbias2_kernel(const float* q, long q_rs, int n_seq, int gh, int gw,
                                                           int heads, const float* Rh, const float* Rw, float* out) {
    extern __shared__ __attribute__((aligned(16))) float tabs[];
    constexpr int P = HD + 1;
    const int nh = 2 * gh - 1, nw = 2 * gw - 1;
    float* th = tabs;
    float* tw = tabs + nh * P;
    for (int i = threadIdx.x; i < nh * HD; i += 256) th[(i / HD) * P + i % HD] = Rh[i];
    for (int i = threadIdx.x; i < nw * HD; i += 256) tw[(i / HD) * P + i % HD] = Rw[i];
    __syncthreads();
    const int L = gh * gw, R = gh + gw;
    const int sh = blockIdx.y, h = sh % heads, s = sh / heads;
    const int qi = blockIdx.x * 256 + threadIdx.x;
    if (qi >= L) return;
    float qr[HD];
    const float* qp = q + ((long)s * L + qi) * q_rs + (long)h * HD;
#pragma unroll
    for (int d = 0; d < HD; d += 4) {
        const float4 v = *reinterpret_cast<const float4*>(qp + d);
        qr[d] = v.x; qr[d + 1] = v.y; qr[d + 2] = v.z; qr[d + 3] = v.w;
    }
    const int qh = qi / gw, qw = qi % gw;
    float* o = out + (((long)s * heads + h) * L + qi) * R;
    for (int j = 0; j < R; ++j) {
        const float* rr = j < gh ? th + (qh - j + gh - 1) * P : tw + (qw - (j - gh) + gw - 1) * P;
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) acc = fmaf(qr[d], rr[d], acc);
        o[j] = acc;
    }
}

void launch_sam_relbias(const float* q, long q_row_stride, int n_seq, int gh, int gw, int heads, int hd,
                        const float* Rh, const float* Rw, float* out, hipStream_t s) {
    long total = (long)n_seq * heads * gh * gw * (gh + gw);
    if (total == 0) return;
    const size_t lds = (size_t)((2 * gh - 1) + (2 * gw - 1)) * (hd + 1) * 4;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sam_relbias2_kernel<64>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        attr = true;
    }
    if (hd == 64 && lds <= 96 * 1024) {  // tables staged in LDS; otherwise the direct kernel below
        dim3 grid((gh * gw + 255) / 256, n_seq * heads);
        hipLaunchKernelGGL(sam_relbias2_kernel<64>, grid, dim3(256), lds, s, q, q_row_stride, n_seq, gh, gw, heads, Rh,
                           Rw, out);
        return;
    }
    long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(sam_relbias_kernel, dim3((unsigned)blocks), dim3(256), 0, s, q, q_row_stride, n_seq, gh, gw,
                       heads, hd, Rh, Rw, out);
}

// ------------------------------------------------------------------ RoPE + KV append
__global__ __launch_bounds__(256) void rope_kv_kernel(RopeKvArgs a) {
    const int r = blockIdx.x;
    const int page = a.row_page[r], pos = a.row_pos[r];
    float* row = a.qkv + (long)r * a.ld;
    const int H = a.heads * a.hd, KVH = a.kv_heads * a.hd;
    const float* cs = a.cos + (long)pos * a.rope_dim;
    const float* sn = a.sin + (long)pos * a.rope_dim;
    const int half = a.rope_dim / 2;
    const int nq = a.heads, nk = a.kv_heads;
    const int total = (nq + nk) * a.hd;
    constexpr int MAXPER = 32;  // supports (heads + kv_heads) * hd <= 8192
    float outv[MAXPER];
    const int iters = (total + 255) / 256;
    // phase 1: read + rotate (q rotated in place, so every read precedes every write)
    for (int it = 0; it < iters && it < MAXPER; ++it) {
        const int idx = threadIdx.x + it * 256;
        if (idx >= total) break;
        const int hh = idx / a.hd, d = idx % a.hd;
        const float* base = (hh < nq) ? (row + hh * a.hd) : (row + H + (hh - nq) * a.hd);
        float out;
        if (d < a.rope_dim) {
            // x' = optional MLA even/odd regroup of x (block.rs:1405-1424)
            auto xr = [&](int i) -> float {
                if (!a.use_mla) return base[i];
                return i < half ? base[2 * i] : base[2 * (i - half) + 1];
            };
            const float x = xr(d);
            const float rot = d < half ? -xr(d + half) : xr(d - half);
            out = x * cs[d] + rot * sn[d];
        } else {
            out = base[d];
        }
        outv[it] = out;
    }
    __syncthreads();
    for (int it = 0; it < iters && it < MAXPER; ++it) {
        const int idx = threadIdx.x + it * 256;
        if (idx >= total) break;
        const int hh = idx / a.hd, d = idx % a.hd;
        if (hh < nq) {
            row[hh * a.hd + d] = outv[it];
        } else {
            const int kh = hh - nq;
            a.kc[(long)page * a.page_stride + (long)kh * a.head_stride + (long)pos * a.hd + d] = outv[it];
        }
    }
    for (int idx = threadIdx.x; idx < nk * a.hd; idx += blockDim.x) {
        const int kh = idx / a.hd, d = idx % a.hd;
        float* vc = a.vc + (long)page * a.page_stride + (long)kh * a.head_stride + (long)pos * a.hd;
        vc[d] = row[H + KVH + kh * a.hd + d];
    }
}

void launch_rope_kv(const RopeKvArgs& a, hipStream_t s) {
    if (a.rows == 0) return;
    hipLaunchKernelGGL(rope_kv_kernel, dim3(a.rows), dim3(256), 0, s, a);
}

}  // namespace dsocr
