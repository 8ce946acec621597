// Screened greedy selection for the decode step (B <= 2 pages): the full-precision lm_head
// (129280 x 1280 bf16, 331 MB, transformer/model.rs:243-270) is replaced on the critical path by
// an int8 copy (per-row scale, 165 MB) that gives every row an approximate logit A_v and a
// RIGOROUS bound eps_v with |L_v - A_v| <= eps_v, where L_v is the logit the exact kernel
// (dec_gemv_stream over the bf16 rows) would produce bit for bit.  Selection then keeps every
// row whose interval [A - eps, A + eps] can still reach the best lower bound T, rescores exactly
// those candidates with the exact kernel's arithmetic, and takes the first-index argmax
// (sampling.rs:104-118) over them: the same token as the exact path, from half the bytes.
//
// Bound (per row v, K = hidden, x = the RMS-normalised row, u = 2^-24):
//   L_v - A_v = [fl(x.W) - x.W] + [x.(W - s Q)] + [s x.Q - fl(s fl(x.Q))]
//   |.| <= ||x|| (E_v + g (||W_v|| + s_v ||Q_v||)) + |A_v| 2u          (g = 2 K u, generous)
// with E_v = ||W_v - s_v Q_v||, all row constants computed in f64 at load and rounded up.
#include <cstdint>
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

// ---------------------------------------------------------------- load time: quantise one row per block
// (WT: the lm_head's 16-bit storage — bf16 checkpoints, f16 where a DSQ snapshot's Q8_0 lm_head was dequantised)
template <typename WT>
__global__ __launch_bounds__(256) void lmhead_quantize_kernel(const uint16_t* __restrict__ w, int K, int8_t* q,
                                                              float* scale, float* bound, float* qnorm, int8_t* qf) {
    __shared__ double red[256];
    const int v = blockIdx.x;
    const uint16_t* row = w + (long)v * K;
    float mx = 0.f;
    for (int k = threadIdx.x; k < K; k += 256) mx = fmaxf(mx, fabsf(wbits_to_f32<WT>(row[k])));
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    const float s = red[0] > 0.0 ? (float)(red[0] / 127.0) : 1.f;
    __syncthreads();
    double e2 = 0.0, w2 = 0.0, q2 = 0.0;
    int8_t* const qf_out = qf;
    for (int k = threadIdx.x; k < K; k += 256) {
        const float x = wbits_to_f32<WT>(row[k]);
        float qf = rintf(x / s);
        qf = fminf(127.f, fmaxf(-127.f, qf));
        q[(long)v * K + k] = (int8_t)qf;
        if (qf_out) {  // fragment order of the multi-token kernel: [v/16][k/64][lane = v%16 + 16 (k%64)/16][k%16]
            const int kk = k & 63;
            qf_out[(((long)(v >> 4) * (K >> 6) + (k >> 6)) * 64 + (v & 15) + 16 * (kk >> 4)) * 16 + (kk & 15)] = (int8_t)qf;
        }
        const double e = (double)x - (double)s * (double)qf;
        e2 += e * e;
        w2 += (double)x * x;
        q2 += (double)qf * qf;
    }
    double* sums = red;
    for (int part = 0; part < 3; ++part) {
        __syncthreads();
        sums[threadIdx.x] = part == 0 ? e2 : (part == 1 ? w2 : q2);
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (threadIdx.x < o) sums[threadIdx.x] += sums[threadIdx.x + o];
            __syncthreads();
        }
        if (part == 0) e2 = sums[0];
        else if (part == 1) w2 = sums[0];
        else q2 = sums[0];
    }
    if (threadIdx.x == 0) {
        const double g = 2.0 * K * 5.9604644775390625e-8;  // 2 K u
        const double b = (sqrt(e2) + g * (sqrt(w2) + (double)s * sqrt(q2))) * (1.0 + 1e-6) + 1e-30;
        scale[v] = s;
        bound[v] = __double2float_ru(b);
        if (qnorm) qnorm[v] = __double2float_ru((double)s * sqrt(q2) * (1.0 + 1e-6));  // s ||Q||, rounded up
    }
}

void launch_lmhead_quantize(const void* w, int V, int K, void* q, float* scale, float* bound, hipStream_t s,
                            float* qnorm, void* qfrag, int wdtype) {
    if (qfrag && K % 64) throw std::runtime_error("EINVAL: fragment-ordered int8 lm_head needs K % 64 == 0");
    if (qfrag && V % 16 && hipMemsetAsync(qfrag, 0, lmhead_qfrag_bytes(V, K), s) != hipSuccess)
        throw std::runtime_error("EINTERNAL: hipMemsetAsync (int8 lm_head tail tile)");
    if (wdtype == WDT_F16)
        DSOCR_LAUNCH(lmhead_quantize_kernel<f16_t>, dim3(V), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(w), K,
                     reinterpret_cast<int8_t*>(q), scale, bound, qnorm, reinterpret_cast<int8_t*>(qfrag));
    else
        DSOCR_LAUNCH(lmhead_quantize_kernel<bf16_t>, dim3(V), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(w), K,
                     reinterpret_cast<int8_t*>(q), scale, bound, qnorm, reinterpret_cast<int8_t*>(qfrag));
}

size_t lmhead_qfrag_bytes(int V, int K) { return (size_t)((V + 15) / 16) * 16 * K; }

// ---------------------------------------------------------------- per step: screened lm_head
// x staged once per block exactly as dec_gemv_stream stages it (RMSNorm fused); block 0 also
// writes the staged row (the exact rescoring reads it).  A wave walks groups of RB rows with a
// two-deep register pipeline of 16-byte int8 loads (K / 16 chunks per row); per row it forms the
// interval [lo, hi] (row r's in lane r: one pass, one ballot) and keeps the row when hi reaches
// the wave's running threshold Tw (the best lo of the unbanned rows seen by this wave or,
// refreshed once per group, by its block: an LDS atomicMax key).  Kept rows go to an LDS list;
// at the end the block writes its list, count and best lo to its own slot, and the final kernel
// reduces the blocks (no cross-block atomics: a device-wide threshold / counter was 2-10x
// slower, every wave hitting one address).
constexpr int LQ_RB = 8;   // rows per group
constexpr int LQ_XS = 128;
constexpr int LQ_LIST = 1024;  // rows one block may keep (the grid keeps rows per block <= this)
// Load layout of one group (K/16 16-byte chunks per row): load r (r < RB) is row r's chunks
// 0..63, one per lane; the rows' remaining chunks (TSEG = 16 or 32 of them at most) are packed
// TSEG lanes per row into RB*TSEG/64 shared tail loads — every lane's bytes are useful.
template <int TSEG>
struct LqGroup {
    static constexpr int NTL = TSEG ? LQ_RB * TSEG / 64 : 0;
    uint4 m[LQ_RB];
    uint4 t[NTL > 0 ? NTL : 1];
    float sc, bd;  // lane r: row r's scale / bound
};

template <int TSEG>
__device__ __forceinline__ void lq_issue(LqGroup<TSEG>& q, const LmHeadQ8Args& a, const int8_t* W, int n0, int lane) {
    const int chunks = a.K >> 4, N = a.N, K = a.K;
    const int nr = min(n0 + (lane & (LQ_RB - 1)), N - 1);
    q.sc = a.scale[nr];
    q.bd = a.bound[nr];
#pragma unroll
    for (int r = 0; r < LQ_RB; ++r) {
        const int n = min(n0 + r, N - 1);
        q.m[r] = ldg_nt16(W + (long)n * K + (min(lane, chunks - 1) << 4));
    }
    if (TSEG) {
        constexpr int RPT = TSEG ? 64 / TSEG : 1;
#pragma unroll
        for (int t = 0; t < LqGroup<TSEG>::NTL; ++t) {
            const int n = min(n0 + t * RPT + lane / TSEG, N - 1);
            q.t[t] = ldg_nt16(W + (long)n * K + (min(64 + lane % TSEG, chunks - 1) << 4));
        }
    }
}

__device__ __forceinline__ float i8f(uint32_t w, int byte) {
    // signed byte: shift it to the top, arithmetic shift back (one sdwa sext convert).
    // (__builtin_amdgcn_sbfe on this compiler folds into an UNSIGNED sdwa convert: wrong.)
    return (float)((int32_t)(w << (24 - 8 * byte)) >> 24);
}

// the page's banned rows: staged in LDS (a global read here would drain the prefetch: vmcnt is
// in order); longer lists are read from global memory
constexpr int LQ_BANS = 256;
__device__ __forceinline__ float lq_dot16(const float* xv, uint4 q, float acc) {
    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = fmaf(xv[4 * i + j], i8f(wd[i], j), acc);
    return acc;
}

__device__ __forceinline__ void ld_x16(const float* p, float* xv) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 t = *reinterpret_cast<const float4*>(p + 4 * i);
        xv[4 * i] = t.x; xv[4 * i + 1] = t.y; xv[4 * i + 2] = t.z; xv[4 * i + 3] = t.w;
    }
}

__device__ __forceinline__ bool lq_banned(int n, int nban, const int* ban_s, const int* ban_g) {
    if (nban <= LQ_BANS) {
        for (int j = 0; j < nban; ++j)
            if (ban_s[j] == n) return true;
        return false;
    }
    for (int j = 0; j < nban; ++j)
        if (ban_g[j] == n) return true;
    return false;
}

template <int TSEG>
__global__ __launch_bounds__(256) void lmhead_q8_kernel(LmHeadQ8Args a) {
    __shared__ __attribute__((aligned(16))) float xs[LQ_XS + 1536];
    __shared__ float nrm_s;
    __shared__ unsigned tkey_s;
    __shared__ int ban_s[LQ_BANS];
    __shared__ int lst_n;
    __shared__ int lst_idx[LQ_LIST];
    __shared__ float lst_hi[LQ_LIST];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int K = a.K, chunks = K >> 4;
    const int b = blockIdx.y;
    const float* xrow = a.x + (long)b * a.ldx;
    const int8_t* W = reinterpret_cast<const int8_t*>(a.q);
    const int ngroups = (a.N + LQ_RB - 1) / LQ_RB;
    const int stride = gridDim.x * 4;
    LqGroup<TSEG> qa;
    int g = blockIdx.x * 4 + wave;
    // loads in order of use: x / norm weight, the ban list, then the first row group (its
    // latency overlaps the norm prologue)
    float4 v[2], w[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int k = min((tid + i * 256) * 4, K - 4);
        v[i] = *reinterpret_cast<const float4*>(xrow + k);
        w[i] = *reinterpret_cast<const float4*>(a.norm_w + k);
    }
    int nban = 0, bent = 0;
    const int* ban_g = nullptr;
    if (a.ban) {
        ban_g = a.ban + (long)b * a.ban_ld + 1;
        nban = a.ban[(long)b * a.ban_ld];
        bent = ban_g[min(tid, (int)a.ban_ld - 2)];
    }
    lq_issue<TSEG>(qa, a, W, min(g, ngroups - 1) * LQ_RB, lane);
    // stage x = rmsnorm(x) (the dec_gemv staging arithmetic: 256 threads, float4 each, XR = 2)
    {
        float qs = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if ((tid + i * 256) * 4 < K) qs += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
        qs = wave_sum(qs);
        if (lane == 0) xs[wave] = qs;
        if (tid == 0) { tkey_s = 0u; lst_n = 0; }
        if (tid < LQ_BANS) ban_s[tid] = bent;
        __syncthreads();
        float q = 0.f;
        for (int ww = 0; ww < 4; ++ww) q += xs[ww];
        const float den = sqrtf(q / (float)K + a.eps);
        __syncthreads();
        float n2 = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int k = (tid + i * 256) * 4;
            if (k < K) {
                float4 o;
                o.x = (v[i].x / den) * w[i].x;
                o.y = (v[i].y / den) * w[i].y;
                o.z = (v[i].z / den) * w[i].z;
                o.w = (v[i].w / den) * w[i].w;
                *reinterpret_cast<float4*>(xs + LQ_XS + k) = o;
                n2 += (o.x * o.x + o.y * o.y) + (o.z * o.z + o.w * o.w);
            }
        }
        n2 = wave_sum(n2);
        if (lane == 0) xs[4 + wave] = n2;
        __syncthreads();
        if (tid == 0) {
            // ||x||, rounded up (the partial-sum rounding is < 1e-4 relative at K <= 1536)
            nrm_s = sqrtf((xs[4] + xs[5] + xs[6] + xs[7]) * (1.f + 1e-4f)) * (1.f + 1e-6f);
        }
        __syncthreads();
    }
    const float nrm = nrm_s;
    const float* x = xs + LQ_XS;
    float Tw = -INFINITY;
    for (; g < ngroups; g += stride) {
        LqGroup<TSEG> qn;
        const int g2 = g + stride;
        lq_issue<TSEG>(qn, a, W, min(g2, ngroups - 1) * LQ_RB, lane);  // clamped: no predicated loads
        float acc[LQ_RB];
        {
            // every lane computes (clamped chunks past K hold valid bytes), masked after
            float xv[16];
            ld_x16(x + (min(lane, chunks - 1) << 4), xv);
            const bool ok = lane < chunks;
#pragma unroll
            for (int r = 0; r < LQ_RB; ++r) {
                const float d = lq_dot16(xv, qa.m[r], 0.f);
                acc[r] = ok ? d : 0.f;
            }
            if (TSEG) {
                constexpr int RPT = TSEG ? 64 / TSEG : 1;
                const int tc = 64 + lane % TSEG;
                ld_x16(x + (min(tc, chunks - 1) << 4), xv);
                const bool tok = tc < chunks;
                const int seg = lane / TSEG;
#pragma unroll
                for (int t = 0; t < LqGroup<TSEG>::NTL; ++t) {
                    float tv = lq_dot16(xv, qa.t[t], 0.f);
                    tv = tok ? tv : 0.f;
#pragma unroll
                    for (int rr = 0; rr < RPT; ++rr) acc[t * RPT + rr] += seg == rr ? tv : 0.f;
                }
            }
        }
        // row r's dot product to lane r (which holds its scale / bound): the intervals of the
        // group in one pass, one ballot; only rows that can matter take the serial path
        float my = 0.f;
#pragma unroll
        for (int r = 0; r < LQ_RB; ++r) {
            const float sd = wave_sum(acc[r]);
            my = (lane & (LQ_RB - 1)) == r ? sd : my;
        }
        const float A = qa.sc * my;
        // |L - A| <= nrm * bound + |A| 2u; the extra factors cover the rounding of e and of A -/+ e
        const float e = (nrm * qa.bd) * (1.f + 4.8e-7f) + fabsf(A) * 3.6e-7f;
        const float lo = A - e, hi = A + e;
        const int nrow = g * LQ_RB + lane;
        const bool trig = lane < LQ_RB && nrow < a.N && (lo > Tw || hi >= Tw);
        unsigned long long m = __ballot(trig);
        while (m) {
            const int r = __ffsll((long long)m) - 1;
            m &= m - 1;
            const float lo_r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lo), r));
            const float hi_r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hi), r));
            const int n = g * LQ_RB + r;
            if (!(lo_r > Tw) && !(hi_r >= Tw)) continue;
            if (lq_banned(n, nban, ban_s, ban_g)) continue;
            if (lo_r > Tw) {
                Tw = lo_r;
                if (lane == 0) atomicMax(&tkey_s, fkey(lo_r));
            }
            if (lane == 0) {
                const int p = atomicAdd(&lst_n, 1);
                lst_idx[p] = n;
                lst_hi[p] = hi_r;
            }
        }
        Tw = fmaxf(Tw, __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(fkey_dec(tkey_s)))));
        qa = qn;
    }
    __syncthreads();
    // the block's list against its final threshold (most rows kept early fall out here)
    const int cnt = lst_n;
    const float Tb = fkey_dec(tkey_s);
    // entry p of this block at [b][p][block] (the final kernel reads a row of blocks per load); wave 0
    // compacts the list by ballots and writes the count itself: no barrier after the global stores (a barrier
    // waits for the acknowledgement of every store before it)
    const long sb = (long)b * a.nblk * a.slot + blockIdx.x;
    if (wave == 0) {
        int kept = 0;
        for (int i0 = 0; i0 < cnt; i0 += 64) {
            const int i = i0 + lane;
            const bool keep = i < cnt && lst_hi[i] >= Tb;
            const unsigned long long bm = __ballot(keep);
            if (keep) {
                const int p = kept + __popcll(bm & ((1ull << lane) - 1ull));
                a.cand[sb + (long)p * a.nblk] = lst_idx[i];
                a.cand_hi[sb + (long)p * a.nblk] = lst_hi[i];
            }
            kept += __popcll(bm);
        }
        if (lane == 0) {
            a.blk_cnt[(long)b * a.nblk + blockIdx.x] = kept;
            a.blk_t[(long)b * a.nblk + blockIdx.x] = Tb;
        }
    }
    // block 0 hands the staged row to the final selection (exact rescoring) here, after its last barrier:
    // stored during the staging, the staging's barriers waited for the stores and block 0 started ~1 us late
    if (blockIdx.x == 0 && a.xn_out)
        for (int k = tid * 4; k < K; k += 256 * 4)
            *reinterpret_cast<float4*>(a.xn_out + (long)b * K + k) = *reinterpret_cast<const float4*>(x + k);
}

static int lq_tseg(int K) {
    const int chunks = K >> 4;
    return chunks <= 64 ? 0 : (chunks <= 80 ? 16 : 32);
}

void lmhead_q8_grid(int N, int K, int B, int* nblk, long* slot) {
    static int resident[3] = {0, 0, 0};
    const int ti = lq_tseg(K) / 16;
    if (!resident[ti]) {
        int per_cu = 0, dev = 0, cus = 0;
        if (ti == 0) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lmhead_q8_kernel<0>, 256, 0);
        else if (ti == 1) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lmhead_q8_kernel<16>, 256, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lmhead_q8_kernel<32>, 256, 0);
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        resident[ti] = std::max(1, per_cu) * std::max(1, cus);
    }
    const int groups = (N + LQ_RB - 1) / LQ_RB;
    int blocks = std::min((groups + 3) / 4, std::max(1, resident[ti] / std::max(1, B)));
    // rows one block walks (its kept list is bounded by them) must fit the LDS list
    constexpr int max_per_wave = LQ_LIST / (4 * LQ_RB);
    blocks = std::max(blocks, (groups + 4 * max_per_wave - 1) / (4 * max_per_wave));
    const int per_wave = (groups + 4 * blocks - 1) / (4 * blocks);
    *nblk = blocks;
    *slot = (long)per_wave * 4 * LQ_RB;
}



// ---------------------------------------------------------------- 3..8 tokens: one int8 stream for all
// The same intervals for B = 3..8 decode rows, with the int8 rows read ONCE for every token on the
// int8 matrix cores (v_mfma_i32_16x16x64_i8: 16 vocabulary rows x 64 k as the A operand, straight from
// the fragment-ordered copy, one 1 KiB block per wave load; the B operand = the token rows).  Each
// token's normalised row x (staged as dec_gemv / the single-token kernel stage it, block 0 writes it for
// the exact rescoring) is represented in two int8 planes, x~ = t1 Xh + t2 Xl (t1 = max|x| / 127,
// Xh = rint(x / t1), t2 = t1 / 254, Xl = rint((x - t1 Xh) / t2)), so Ih = Xh.Q_v and Il = Xl.Q_v are exact
// int32 dot products and A_v = s_v (t1 Ih + t2 Il) is formed in f64.  Bound (per row v, token t):
//   L_v - A_v = [fl(x.W) - x.W] + [x.(W - s Q)] + [s (x - x~).Q] + [s x~.Q - A_v]
//   |.| <= ||x|| bound_v + (s_v ||Q_v||) ||x - x~|| + (f64 rounding of A_v, covered by the margin)
// with ||x||, ||x - x~|| summed in f64 and rounded up, s ||Q|| stored at load (lmhead_quantize).  The
// kept-row lists, per-block thresholds and the final kernel (dec_screen_final) are the single-token
// kernel's, one list per token (page).
constexpr int LM_T = 8, LM_WV = 8, LM_LIST = 256, LM_KMAX = 1536, LM_BANS = 128, LM_TPB = LM_LIST / 16;
typedef int v4i32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int KS>  // k-steps of 64 held in registers: KS == K / 64
__global__ __launch_bounds__(512, 4) void lmhead_q8mm_kernel(LmHeadQ8Args a, int tpb) {
    __shared__ __attribute__((aligned(16))) int8_t xq[2][LM_T][LM_KMAX + 16];
    __shared__ float t1_s[LM_T], t2_s[LM_T], nrm_s[LM_T], errn_s[LM_T];
    __shared__ unsigned tkey_s[LM_T];
    __shared__ float den_s[LM_T];
    __shared__ int lst_n[LM_T], nban_s[LM_T];
    __shared__ int lst_idx[LM_T][LM_LIST];
    __shared__ float lst_hi[LM_T][LM_LIST];
    __shared__ int ban_s[LM_T][LM_BANS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int ks = KS;
    const int K = KS * 64, B = a.B, N = a.N;
    const int ntiles = (N + 15) >> 4;
    const int t_beg = blockIdx.x * tpb, t_end = min(ntiles, t_beg + tpb);
    const v4i32* QF = reinterpret_cast<const v4i32*>(a.qfrag);
    // weight fragments stream through a ring of PF k-steps per wave: step t + PF (of this tile, or of the
    // wave's next tile) is issued as step t is consumed, so PF KiB stay in flight per wave across tile
    // boundaries; the first tile's first PF steps go out before the staging (their latency overlaps it)
    constexpr int PF = KS / 2;
    v4i32 wa[PF];
    auto ld = [&](int T_, int t) {
        return __builtin_nontemporal_load(QF + ((long)min(T_, ntiles - 1) * ks + t) * 64 + lane);
    };
    int T = t_beg + wave;
#pragma unroll
    for (int t = 0; t < PF; ++t) wa[t] = ld(T, t);
    // nban_s[t] has ONE writer: the staging wave t < B below, lane t of wave 0 for the unused t >= B (a
    // zeroing by wave 0 of every entry could land after a staging wave's count: no barrier between them)
    if (tid < LM_T) { tkey_s[tid] = 0u; lst_n[tid] = 0; if (tid >= B) nban_s[tid] = 0; }
    // ---- stage: wave w normalises token row w (K <= 1536: float4 chunks lane + 64 j), quantises it
    // into the two planes and sums ||x||^2 and ||x - x~||^2 in f64
    if (wave < B) {
        // three passes over the row (L1-resident after the first): sum of squares; max |x|; quantise
        const float* xr = a.x + (long)wave * a.ldx;
        constexpr int J = LM_KMAX / 256;
        int nb = 0;
        if (a.ban) {
            const int* bg = a.ban + (long)wave * a.ban_ld;
            nb = bg[0];
            for (int i = lane; i < min(nb, LM_BANS); i += 64) ban_s[wave][i] = bg[1 + i];
        }
        if (lane == 0) nban_s[wave] = nb;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int k = (lane + 64 * j) * 4;
            if (k < K) {
                const float4 v = *reinterpret_cast<const float4*>(xr + k);
                q += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
            }
        }
        q = wave_sum(q);
        const float den = sqrtf(q / (float)K + a.eps);
        if (lane == 0) den_s[wave] = den;
        auto xhat = [&](int k) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k), w = *reinterpret_cast<const float4*>(a.norm_w + k);
            return make_float4((v.x / den) * w.x, (v.y / den) * w.y, (v.z / den) * w.z, (v.w / den) * w.w);
        };
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int k = (lane + 64 * j) * 4;
            if (k < K) {
                const float4 o = xhat(k);
                mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            }
        }
        mx = wave_max(mx);
        const float t1 = mx > 0.f ? mx / 127.f : 1.f, t2 = t1 / 254.f;
        double n2 = 0.0, e2 = 0.0;
        for (int j = 0; j < J; ++j) {
            const int k = (lane + 64 * j) * 4;
            if (k < K) {
                const float4 o = xhat(k);
                const float xv[4] = {o.x, o.y, o.z, o.w};
                uint32_t hw = 0, lw = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float h = fminf(127.f, fmaxf(-127.f, rintf(xv[e] / t1)));
                    const float l = fminf(127.f, fmaxf(-127.f, rintf(fmaf(-t1, h, xv[e]) / t2)));
                    hw |= (uint32_t)(uint8_t)(int8_t)h << (8 * e);
                    lw |= (uint32_t)(uint8_t)(int8_t)l << (8 * e);
                    const double d = (double)xv[e] - ((double)t1 * (double)h + (double)t2 * (double)l);
                    e2 += d * d;
                    n2 += (double)xv[e] * (double)xv[e];
                }
                *reinterpret_cast<uint32_t*>(&xq[0][wave][k]) = hw;
                *reinterpret_cast<uint32_t*>(&xq[1][wave][k]) = lw;
            }
        }
        n2 = wave_sum_d(n2);
        e2 = wave_sum_d(e2);
        if (lane == 0) {
            t1_s[wave] = t1;
            t2_s[wave] = t2;
            nrm_s[wave] = __double2float_ru(sqrt(n2) * (1.0 + 1e-9));
            errn_s[wave] = __double2float_ru(sqrt(e2) * (1.0 + 1e-9) + 1e-30);
        }
    }
    __syncthreads();
    // ---- per lane: token column c (lanes of columns >= B compute on a clamped row and are dropped),
    // rows 16 T + 4 g + i (the int32 accumulator layout of the 16x16 MFMA)
    const int c = lane & 15, g = lane >> 4, cr = min(c, B - 1);
    const bool col_ok = c < B;
    const float t1 = t1_s[cr], t2 = t2_s[cr], nrm = nrm_s[cr], errn = errn_s[cr];
    const int8_t* xh = &xq[0][cr][16 * g];
    const int8_t* xl = &xq[1][cr][16 * g];
    // ---- phase 1: every tile of the wave (at most TPW) -> the lane's row intervals, kept in registers, and
    // the lane's best unbanned lower bound; the block threshold per token from those (LDS atomicMax)
    // ---- phase 2: the lane's rows whose upper bound reaches the threshold (and not banned) join the list.
    // No per-row serial path: a row is tested against the BLOCK's final threshold, not a running one.
    constexpr int TPW = (LM_TPB + LM_WV - 1) / LM_WV;
    float lo_a[TPW][4], hi_a[TPW][4];
    auto banned = [&](int n) {
        const int nb = nban_s[cr];
        bool hit = false;
        if (nb <= LM_BANS) {
            for (int j = 0; j < nb; ++j) hit = hit || ban_s[cr][j] == n;
        } else {
            const int* bg = a.ban + (long)cr * a.ban_ld + 1;
            for (int j = 0; j < nb; ++j) hit = hit || bg[j] == n;
        }
        return hit;
    };
    float best = -INFINITY;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int Tu = T + u * LM_WV;
        if (Tu >= t_end) break;  // wave-uniform
        const int Tn = Tu + LM_WV;
        // scale / bound / s||Q|| of this lane's 4 rows (the arrays are padded to whole tiles)
        const int r0 = 16 * Tu + 4 * g;
        const float4 sc4 = *reinterpret_cast<const float4*>(a.scale + r0);
        const float4 bd4 = *reinterpret_cast<const float4*>(a.bound + r0);
        const float4 qn4 = *reinterpret_cast<const float4*>(a.qnorm + r0);
        v4i32 ch = {0, 0, 0, 0}, cl = {0, 0, 0, 0};
        // the token planes are re-read from LDS per tile (kept live across tiles they would take 8 KS VGPRs)
        const int8_t* ph = xh;
        const int8_t* pl = xl;
        asm volatile("" : "+v"(ph), "+v"(pl));
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const v4i32 bh = *reinterpret_cast<const v4i32*>(ph + 64 * t);
            const v4i32 bl = *reinterpret_cast<const v4i32*>(pl + 64 * t);
            const v4i32 w = wa[t % PF];
            ch = __builtin_amdgcn_mfma_i32_16x16x64_i8(w, bh, ch, 0, 0, 0);
            cl = __builtin_amdgcn_mfma_i32_16x16x64_i8(w, bl, cl, 0, 0, 0);
            // refill the slot: step t + PF of this tile, else step t + PF - KS of the next (clamped: a wave
            // without a next tile re-reads its last tile's rows, never used)
            wa[t % PF] = t + PF < KS ? ld(Tu, t + PF) : ld(Tn < t_end ? Tn : Tu, t + PF - KS);
            __builtin_amdgcn_sched_barrier(0);  // keep each step's two LDS reads next to its MFMAs
        }
        const float scv[4] = {sc4.x, sc4.y, sc4.z, sc4.w}, bdv[4] = {bd4.x, bd4.y, bd4.z, bd4.w},
                    qnv[4] = {qn4.x, qn4.y, qn4.z, qn4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double A = (double)scv[i] * ((double)t1 * (double)ch[i] + (double)t2 * (double)cl[i]);
            const double e = ((double)nrm * (double)bdv[i] + (double)qnv[i] * (double)errn) * (1.0 + 1e-6) +
                             fabs(A) * 1e-12 + 1e-30;
            const int row = r0 + i;
            const bool ok = col_ok && row < N;
            lo_a[u][i] = ok ? __double2float_rd(A - e) : -INFINITY;
            hi_a[u][i] = ok ? __double2float_ru(A + e) : -INFINITY;
            if (lo_a[u][i] > best && !banned(row)) best = lo_a[u][i];
        }
    }
    // the token's best over the wave's 4 lanes of that column (lanes c, c + 16, c + 32, c + 48), then the block
    best = fmaxf(best, __shfl_xor(best, 16));
    best = fmaxf(best, __shfl_xor(best, 32));
    if (col_ok && g == 0 && best > -INFINITY) atomicMax(&tkey_s[c], fkey(best));
    __syncthreads();
    const float Tb = fkey_dec(tkey_s[cr]);
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int Tu = T + u * LM_WV;
        if (Tu >= t_end) break;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 16 * Tu + 4 * g + i;
            if (col_ok && row < N && hi_a[u][i] >= Tb && !banned(row)) {
                const int p = atomicAdd(&lst_n[c], 1);
                lst_idx[c][p] = row;
                lst_hi[c][p] = hi_a[u][i];
            }
        }
    }
    __syncthreads();
    // ---- every token's list against its block threshold -> cand[b][p][block] (the single-token layout)
    for (int tk = wave; tk < B; tk += LM_WV) {
        const int cnt = lst_n[tk];
        const float Tb = fkey_dec(tkey_s[tk]);
        const long sb = (long)tk * a.nblk * a.slot + blockIdx.x;
        int kept = 0;
        for (int i0 = 0; i0 < cnt; i0 += 64) {
            const int i = i0 + lane;
            const bool keep = i < cnt && lst_hi[tk][i] >= Tb;
            const unsigned long long bm = __ballot(keep);
            if (keep) {
                const int p = kept + __popcll(bm & ((1ull << lane) - 1ull));
                a.cand[sb + (long)p * a.nblk] = lst_idx[tk][i];
                a.cand_hi[sb + (long)p * a.nblk] = lst_hi[tk][i];
            }
            kept += __popcll(bm);
        }
        if (lane == 0) {
            a.blk_cnt[(long)tk * a.nblk + blockIdx.x] = kept;
            a.blk_t[(long)tk * a.nblk + blockIdx.x] = Tb;
        }
    }
    // block 0 hands the normalised rows to the final selection here, after its last barrier (recomputed with the
    // staging's arithmetic: the same values), not during the staging, whose barriers would wait for the stores
    if (blockIdx.x == 0 && a.xn_out && wave < B) {
        const float* xr = a.x + (long)wave * a.ldx;
        const float den = den_s[wave];
        for (int k = lane * 4; k < K; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k), w = *reinterpret_cast<const float4*>(a.norm_w + k);
            *reinterpret_cast<float4*>(a.xn_out + (long)wave * K + k) =
                make_float4((v.x / den) * w.x, (v.y / den) * w.y, (v.z / den) * w.z, (v.w / den) * w.w);
        }
    }
}

bool lmhead_q8mm_ok(int B, int N, int K) {
    return B >= 1 && B <= LM_T && (K == 768 || K == 1024 || K == 1280 || K == 1536) && N >= 16;
}

void lmhead_q8mm_grid(int N, int K, int B, int* nblk, long* slot) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    (void)K;
    (void)B;
    const int tiles = (N + 15) / 16;
    // two blocks of 8 waves per CU; a block's tiles (its rows) never exceed its LDS lists
    int blocks = std::max(2 * cus, (tiles + LM_TPB - 1) / LM_TPB);
    const int tpb = (tiles + blocks - 1) / blocks;
    blocks = (tiles + tpb - 1) / tpb;
    *nblk = blocks;
    *slot = (long)tpb * 16;
}

void launch_lmhead_q8(const LmHeadQ8Args& a, hipStream_t s) {
    if (a.K % 16 || a.K > 1536 || a.K < 16) throw std::runtime_error("EINVAL: lmhead_q8 needs K % 16 == 0, K <= 1536");
    int nblk = 0;
    long slot = 0;
    if (a.B >= 3 && a.qfrag) {  // one int8 stream for all B tokens on the matrix cores
        if (!lmhead_q8mm_ok(a.B, a.N, a.K) || !a.qnorm) throw std::runtime_error("EINVAL: lmhead_q8mm outside its range");
        lmhead_q8mm_grid(a.N, a.K, a.B, &nblk, &slot);
        if (!a.blk_cnt || !a.blk_t || !a.cand || !a.cand_hi || a.nblk != nblk || a.slot != slot)
            throw std::runtime_error("EINVAL: lmhead_q8mm block lists missing or not sized by lmhead_q8_grid");
        if (a.ban && a.ban_ld < 2) throw std::runtime_error("EINVAL: lmhead_q8 ban list stride < 2");
        const int tpb = (int)(slot / 16);
        if (a.K == 1280) DSOCR_LAUNCH(lmhead_q8mm_kernel<20>, dim3(nblk), dim3(512), 0, s, a, tpb);
        else if (a.K == 1536) DSOCR_LAUNCH(lmhead_q8mm_kernel<24>, dim3(nblk), dim3(512), 0, s, a, tpb);
        else if (a.K == 1024) DSOCR_LAUNCH(lmhead_q8mm_kernel<16>, dim3(nblk), dim3(512), 0, s, a, tpb);
        else DSOCR_LAUNCH(lmhead_q8mm_kernel<12>, dim3(nblk), dim3(512), 0, s, a, tpb);
        return;
    }
    lmhead_q8_grid(a.N, a.K, a.B, &nblk, &slot);
    if (!a.blk_cnt || !a.blk_t || !a.cand || !a.cand_hi || a.nblk != nblk || a.slot != slot)
        throw std::runtime_error("EINVAL: lmhead_q8 block lists missing or not sized by lmhead_q8_grid");
    if (a.ban && a.ban_ld < 2) throw std::runtime_error("EINVAL: lmhead_q8 ban list stride < 2");
    const int tseg = lq_tseg(a.K);
    const dim3 grid(nblk, a.B);
    if (tseg == 0) DSOCR_LAUNCH(lmhead_q8_kernel<0>, grid, dim3(256), 0, s, a);
    else if (tseg == 16) DSOCR_LAUNCH(lmhead_q8_kernel<16>, grid, dim3(256), 0, s, a);
    else DSOCR_LAUNCH(lmhead_q8_kernel<32>, grid, dim3(256), 0, s, a);
}

}  // namespace dsocr
