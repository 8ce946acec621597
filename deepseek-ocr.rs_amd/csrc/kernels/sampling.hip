// Stochastic token selection on the GPU: the `do_sample && temperature > 0` branch of
// select_token_id (core/src/sampling.rs:67-86) with apply_top_k (:160-175), apply_top_p
// (:177-223), sample_from_logits (:225-256) and the reference's RNG, rand 0.8.5 StdRng
// (ChaCha12, rand_chacha 0.3.1) seeded by rand_core 0.6.4 seed_from_u64 (host side,
// engine.cpp) and drawn through WeightedIndex<f64> / UniformFloat<f64>.
//
// One block of 1024 threads per page, after the lm_head + repetition penalty:
//   1. n-gram ban bitmap of the whole vocabulary in LDS; ban ignored if it leaves nothing
//   2. candidates = finite logit/T, compacted in index order (contiguous per-thread ranges)
//   3. top-k / top-p: stable LSD radix sort (8 x 4-bit digits) of the candidates by descending
//      logit — ties keep the lower index first, as Rust's stable sort_by does; top-p's f64 sums
//      run in sorted order on one thread (the reference's sequential fold, bit for bit)
//   4. kept candidates back in index order, weights exp(q - qmax) (f64), WeightedIndex's
//      cumulative left fold on one thread, one u64 from the page's ChaCha12 state, the
//      partition point of the chosen weight
//   5. the chosen id goes to the selection slots dec_sample_final_kernel reduces (it keeps the
//      EOS / output / context / embedding / KV bookkeeping of the greedy path)
// The f64 multiply-adds of rand's float sampling use __dmul_rn / __dadd_rn (no contraction).
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

constexpr int ST_NT = 1024;
constexpr int ST_DIG = 16;  // 4-bit digits

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define ST_QR(a, b, c, d)                                  \
    s[a] += s[b]; s[d] = rotl32(s[d] ^ s[a], 16);          \
    s[c] += s[d]; s[b] = rotl32(s[b] ^ s[c], 12);          \
    s[a] += s[b]; s[d] = rotl32(s[d] ^ s[a], 8);           \
    s[c] += s[d]; s[b] = rotl32(s[b] ^ s[c], 7);

// ChaCha block (djb layout: 64-bit counter in words 12-13, 64-bit stream 0 in 14-15)
__device__ void chacha_block(const uint32_t* key, uint64_t ctr, int rounds, uint32_t* out) {
    uint32_t init[16] = {0x61707865u, 0x3320646Eu, 0x79622D32u, 0x6B206574u, key[0], key[1], key[2], key[3],
                         key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    uint32_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = init[i];
    for (int r = 0; r < rounds; r += 2) {
        ST_QR(0, 4, 8, 12) ST_QR(1, 5, 9, 13) ST_QR(2, 6, 10, 14) ST_QR(3, 7, 11, 15)
        ST_QR(0, 5, 10, 15) ST_QR(1, 6, 11, 12) ST_QR(2, 7, 8, 13) ST_QR(3, 4, 9, 14)
    }
    for (int i = 0; i < 16; ++i) out[i] = s[i] + init[i];
}
#undef ST_QR

// BlockRng<ChaCha12Core> refill: four consecutive blocks into the 64-word buffer
__device__ void rng_refill(uint32_t* st) {
    uint64_t ctr = (uint64_t)st[RNG_CTR] | ((uint64_t)st[RNG_CTR + 1] << 32);
    for (int j = 0; j < 4; ++j) chacha_block(st + RNG_KEY, ctr + j, 12, st + RNG_BUF + 16 * j);
    ctr += 4;
    st[RNG_CTR] = (uint32_t)ctr;
    st[RNG_CTR + 1] = (uint32_t)(ctr >> 32);
}

// rand_core 0.6 BlockRng::next_u64 (low word first; the odd-index case straddles a refill)
__device__ uint64_t rng_next_u64(uint32_t* st) {
    uint32_t* buf = st + RNG_BUF;
    const uint32_t idx = st[RNG_IDX];
    if (idx < 63) {
        st[RNG_IDX] = idx + 2;
        return (uint64_t)buf[idx] | ((uint64_t)buf[idx + 1] << 32);
    }
    if (idx >= 64) {
        rng_refill(st);
        st[RNG_IDX] = 2;
        return (uint64_t)buf[0] | ((uint64_t)buf[1] << 32);
    }
    const uint64_t x = buf[63];
    rng_refill(st);
    st[RNG_IDX] = 1;
    return x | ((uint64_t)buf[0] << 32);
}

// ascending key order == descending logit order (-0.0 and +0.0 compare equal, as partial_cmp)
__device__ __forceinline__ uint32_t desc_key(float x) {
    uint32_t u = x == 0.f ? 0u : __float_as_uint(x);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ~u;
}

// exclusive block scan of one int per thread (ST_NT threads); returns the prefix, *total the sum
__device__ int block_excl_scan(int v, int* lds16, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) lds16[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < ST_NT / 64; ++w) {
        const int s = lds16[w];
        if (w < wave) base += s;
        tot += s;
    }
    *total = tot;
    return base + incl - v;
}

__device__ __forceinline__ bool is_banned(const uint32_t* ban, int v) { return (ban[v >> 5] >> (v & 31)) & 1u; }

// In-order f64 scan over n values produced by load(g) (the reference's sequential loops, bit for
// bit).  The block stages ST_TILE values at a time in LDS (waves 1.. fetch tile t+1 while lane 0 of
// wave 0 folds tile t out of LDS), so the serial chain pays LDS, not HBM/L2, latency.
// stop(S) is a predicate on the running sum that can only turn true as S grows; the fold ends at
// the first g with stop(S_g) and calls on_stop(g) on thread 0.  If cum_out is set, cum_out[g]
// receives the running total S_g (WeightedIndex's cumulative weights are S_0..S_{n-2}).  The
// total is returned on thread 0.  Terms must be non-negative (weights, shares).
constexpr int ST_TILE = 4096;
template <class Load, class Stop, class OnStop>
__device__ double block_serial_fold(int n, double* tiles, int* stop_s, double* cum_out, Load load, Stop stop,
                                    OnStop on_stop) {
    const int tid = threadIdx.x;
    double total = 0.0;
    const int ntile = (n + ST_TILE - 1) / ST_TILE;
    for (int i = tid; i < min(n, ST_TILE); i += ST_NT) tiles[i] = load(i);
    if (tid == 0) *stop_s = 0;
    __syncthreads();
    for (int t = 0; t < ntile; ++t) {
        double* cur = tiles + (t & 1) * ST_TILE;
        double* nxt = tiles + ((t + 1) & 1) * ST_TILE;
        const int g0 = t * ST_TILE, len = min(ST_TILE, n - g0);
        if (tid >= 64 && t + 1 < ntile) {
            const int g1 = g0 + ST_TILE, len1 = min(ST_TILE, n - g1);
            for (int i = tid - 64; i < len1; i += ST_NT - 64) nxt[i] = load(g1 + i);
        }
        if (tid == 0 && !*stop_s) {
            // 16-value register batches, the next batch's LDS reads in flight while this one folds;
            // the chain is one f64 add per value (0 + v is exact for the non-negative terms, so the
            // first value needs no special case) and the stop test runs once per batch: the running
            // sums never decrease, so `stop` can only turn true and its first index is searched in
            // the batch that crossed
            constexpr int RB = 16;
            double nb[RB];
#pragma unroll
            for (int j = 0; j < RB; ++j) nb[j] = cur[min(j, len - 1)];
            int stop_at = -1;
            for (int i0 = 0; i0 < len; i0 += RB) {
                double v[RB];
#pragma unroll
                for (int j = 0; j < RB; ++j) v[j] = nb[j];
#pragma unroll
                for (int j = 0; j < RB; ++j) nb[j] = cur[min(i0 + RB + j, len - 1)];
                const int cnt = min(RB, len - i0);
                if (cnt == RB) {
#pragma unroll
                    for (int j = 0; j < RB; ++j) { total = total + v[j]; v[j] = total; }
                } else {
                    for (int j = 0; j < cnt; ++j) { total = total + v[j]; v[j] = total; }
                }
                if (cum_out) {
#pragma unroll
                    for (int j = 0; j < RB; ++j)
                        if (j < cnt) cur[i0 + j] = v[j];
                }
                if (stop(total)) {
                    for (int j = 0; j < cnt; ++j)
                        if (stop(v[j])) { stop_at = g0 + i0 + j; break; }
                    break;
                }
            }
            if (stop_at >= 0) { *stop_s = 1; on_stop(stop_at); }
        }
        __syncthreads();
        if (cum_out)
            for (int i = tid; i < len; i += ST_NT) cum_out[g0 + i] = cur[i];
        const bool stop = *stop_s != 0;
        __syncthreads();
        if (stop) break;
    }
    return total;
}

__global__ __launch_bounds__(ST_NT) void dec_stoch_select_kernel(DecSampleArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ban[];  // (V + 31) / 32 words: n-gram ban, later the kept set
    __shared__ double lds_big[ST_DIG * ST_NT / 2];  // radix histograms, later two fold tiles
    int* hist = reinterpret_cast<int*>(lds_big);
    __shared__ int stop_s;
    __shared__ int lds16[ST_NT / 64];
    __shared__ float fmax_s[ST_NT / 64];
    __shared__ int keep_s, tok_s;
    __shared__ double total_s, chosen_s;
    const int b = blockIdx.x, tid = threadIdx.x, V = a.V;
    const int nwords = (V + 31) >> 5;
    const float* lg = a.logits + (long)b * a.ld;
    uint32_t* sk0 = a.st_key + (long)b * 2 * a.st_ld;
    uint32_t* sk1 = sk0 + a.st_ld;
    int* si0 = a.st_idx + (long)b * 2 * a.st_ld;
    int* si1 = si0 + a.st_ld;
    double* sw = a.st_w + (long)b * a.st_ld;
    const double T = a.temperature;
#define ST_STAMP(i) \
    if (a.st_stamps && b == 0 && tid == 0) a.st_stamps[i] = __builtin_amdgcn_s_memtime();
    ST_STAMP(0)

    // ---- 1. n-gram ban (sampling.rs:141-158) over the whole vocabulary
    for (int i = tid; i < nwords; i += ST_NT) ban[i] = 0u;
    __syncthreads();
    {
        const int n = a.ctx_len[b], g = a.ngram;
        const int* cx = a.ctx + (long)b * a.ctx_cap;
        if (g > 1 && n >= g - 1)
            for (int i = tid; i <= n - g; i += ST_NT) {
                const int t = cx[i + g - 1];
                if (t < 0 || t >= V) continue;
                bool match = true;
                for (int jj = 0; jj < g - 1; ++jj)
                    if (cx[i + jj] != cx[n - g + 1 + jj]) { match = false; break; }
                if (match) atomicOr(&ban[t >> 5], 1u << (t & 31));
            }
    }
    __syncthreads();
    // has_valid_logits(filtered) (sampling.rs:62-64): else the ban is dropped
    int nv = 0;
    for (int v = tid; v < V; v += ST_NT) {
        const float x = lg[v];
        nv += (x > -INFINITY && x < INFINITY && !is_banned(ban, v)) ? 1 : 0;
    }
    int nvalid;
    (void)block_excl_scan(nv, lds16, &nvalid);
    const bool use_ban = nvalid > 0;
    ST_STAMP(1)

    // ---- 2. candidates in index order: finite logit / T (f64), contiguous range per thread
    const int chunk = (V + ST_NT - 1) / ST_NT;
    const int v0 = min(V, tid * chunk), v1 = min(V, v0 + chunk);
    int c = 0;
    float lmax = -INFINITY;
    for (int v = v0; v < v1; ++v) {
        const float x = lg[v];
        const double q = (double)x / T;
        if (q > -INFINITY && q < INFINITY && !(use_ban && is_banned(ban, v))) {
            ++c;
            lmax = fmaxf(lmax, x);
        }
    }
    int nc;
    int off = block_excl_scan(c, lds16, &nc);
    for (int u0 = v0; u0 < v1; u0 += 8) {  // loads batched ahead of the stores
        float xx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xx[j] = u0 + j < v1 ? lg[u0 + j] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int v = u0 + j;
            const double q = (double)xx[j] / T;
            if (v < v1 && q > -INFINITY && q < INFINITY && !(use_ban && is_banned(ban, v))) {
                sk0[off] = desc_key(xx[j]);
                si0[off] = v;
                ++off;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o, 64));
    if ((tid & 63) == 0) fmax_s[tid >> 6] = lmax;
    __syncthreads();
    lmax = fmax_s[0];
    for (int w = 1; w < ST_NT / 64; ++w) lmax = fmaxf(lmax, fmax_s[w]);
    // max of the kept logits64 (top-k / top-p keep the largest): the division is monotonic
    const double qmax = (double)lmax / T;
    ST_STAMP(2)

    if (nc == 0) {  // sample_from_logits -> None: the argmax chain of the final kernel decides
        for (int j = tid; j < a.red_blocks; j += ST_NT) a.red_idx[(long)b * a.red_blocks + j] = 0x7fffffff;
        return;
    }

    const bool topk = a.top_k > 0 && a.top_k < V && nc > a.top_k;
    const bool topp = a.top_p >= 0.0 && a.top_p < 1.0;
    const int* kept = si0;
    int nk = nc;
    if (topk || topp) {
      if (topp) {
        // ---- 3. stable LSD radix sort of (key, index) by key ascending = logit descending
        uint32_t *ks = sk0, *kd = sk1;
        int *is = si0, *id = si1;
        const int sc = (nc + ST_NT - 1) / ST_NT;
        const int s0 = min(nc, tid * sc), s1 = min(nc, s0 + sc);
        for (int pass = 0; pass < 8; ++pass) {
            const int sh = pass * 4;
            for (int d = 0; d < ST_DIG; ++d) hist[d * ST_NT + tid] = 0;
            for (int i0 = s0; i0 < s1; i0 += 8) {  // 8 loads in flight per round
                uint32_t kk[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) kk[j] = i0 + j < s1 ? ks[i0 + j] : 0u;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (i0 + j < s1) hist[((kk[j] >> sh) & 15) * ST_NT + tid] += 1;
            }
            __syncthreads();
            // exclusive scan over (digit, thread): thread t owns flattened entries [16t, 16t+16)
            int loc[ST_DIG], sum = 0;
            for (int j = 0; j < ST_DIG; ++j) { loc[j] = hist[tid * ST_DIG + j]; sum += loc[j]; }
            int tot;
            int base = block_excl_scan(sum, lds16, &tot);
            for (int j = 0; j < ST_DIG; ++j) { hist[tid * ST_DIG + j] = base; base += loc[j]; }
            __syncthreads();
            for (int i0 = s0; i0 < s1; i0 += 8) {  // loads batched ahead of the scattered stores
                uint32_t kk[8];
                int ii[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    kk[j] = i0 + j < s1 ? ks[i0 + j] : 0u;
                    ii[j] = i0 + j < s1 ? is[i0 + j] : 0;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (i0 + j < s1) {
                        const int p = hist[((kk[j] >> sh) & 15) * ST_NT + tid]++;
                        kd[p] = kk[j];
                        id[p] = ii[j];
                    }
            }
            __syncthreads();
            uint32_t* tk = ks; ks = kd; kd = tk;
            int* ti = is; is = id; id = ti;
        }
        // 8 passes: sorted data is back in (sk0, si0)
        ST_STAMP(3)
        int m = topk ? (int)a.top_k : nc;
        if (topp) {
            // apply_top_p: weights exp(q - qmax) in sorted order; the total, then the cumulative share
            // until it exceeds top_p, both as in-order folds (sampling.rs:195-211)
            auto wsorted = [&](int j) { return exp((double)lg[si0[j]] / T - qmax); };
            auto never = [](double) { return false; };
            auto none = [](int) {};
            const double total = block_serial_fold(m, lds_big, &stop_s, nullptr, wsorted, never, none);
            if (tid == 0) { total_s = total; keep_s = m; }
            __syncthreads();
            const double tot = total_s;
            if (tot > 0.0) {
                const double tp = a.top_p;
                (void)block_serial_fold(m, lds_big, &stop_s, nullptr, [&](int j) { return wsorted(j) / tot; },
                                        [&](double cumv) { return cumv > tp; }, [&](int j) { keep_s = j + 1; });
            }
            __syncthreads();
            if (keep_s < 1) keep_s = 1;
            __syncthreads();
            m = keep_s;
        }
        ST_STAMP(4)
        // kept set back in index order (bitmap, then per-thread word ranges)
        for (int i = tid; i < nwords; i += ST_NT) ban[i] = 0u;
        __syncthreads();
        for (int j = tid; j < m; j += ST_NT) atomicOr(&ban[si0[j] >> 5], 1u << (si0[j] & 31));
        __syncthreads();
      } else {
        // top-k alone needs the kept SET, not its order: radix-select the k-th smallest key (8-bit
        // digits from the top), keep every key below it and, of the keys equal to it, the first ones
        // in index order — exactly the first k of the stable sort
        for (int i = tid; i < nwords; i += ST_NT) ban[i] = 0u;
        uint32_t prefix = 0u, pmask = 0u;
        int need = (int)a.top_k;
        for (int sh = 24; sh >= 0; sh -= 8) {
            for (int d = tid; d < 256; d += ST_NT) hist[d] = 0;
            __syncthreads();
            for (int i = tid; i < nc; i += ST_NT) {
                const uint32_t k = sk0[i];
                if ((k & pmask) == prefix) atomicAdd(&hist[(k >> sh) & 255], 1);
            }
            __syncthreads();
            if (tid == 0) {
                int cum = 0, d = 0;
                for (; d < 255; ++d) {
                    if (cum + hist[d] >= need) break;
                    cum += hist[d];
                }
                keep_s = d;
                tok_s = need - cum;
            }
            __syncthreads();
            prefix |= (uint32_t)keep_s << sh;
            pmask |= 255u << sh;
            need = tok_s;
            __syncthreads();
        }
        // mark: keys < threshold, then the first `need` keys == threshold in index order
        const int sc = (nc + ST_NT - 1) / ST_NT;
        const int s0 = min(nc, tid * sc), s1 = min(nc, s0 + sc);
        int eq = 0;
        for (int i = s0; i < s1; ++i) eq += sk0[i] == prefix ? 1 : 0;
        int eq_tot;
        int rank = block_excl_scan(eq, lds16, &eq_tot);
        for (int i = s0; i < s1; ++i) {
            const uint32_t k = sk0[i];
            bool keep = k < prefix;
            if (k == prefix) keep = rank++ < need;
            if (keep) atomicOr(&ban[si0[i] >> 5], 1u << (si0[i] & 31));
        }
        __syncthreads();
        ST_STAMP(3)
      }
        const int wc = (nwords + ST_NT - 1) / ST_NT;
        const int w0 = min(nwords, tid * wc), w1 = min(nwords, w0 + wc);
        int cnt = 0;
        for (int w = w0; w < w1; ++w) cnt += __popc(ban[w]);
        int tot;
        int o2 = block_excl_scan(cnt, lds16, &tot);
        for (int w = w0; w < w1; ++w) {
            uint32_t bits = ban[w];
            while (bits) {
                const int bpos = __ffs(bits) - 1;
                bits &= bits - 1;
                si1[o2++] = (w << 5) + bpos;
            }
        }
        kept = si1;
        nk = tot;
        __syncthreads();
        ST_STAMP(5)
    }

    // ---- 4. sample_from_logits over the kept candidates in index order: weights, WeightedIndex's
    // cumulative left fold (sw[0..nk-1) = cumulative_weights) and the total
    // weights first, by the whole block (coalesced), then the in-order fold reads them back
    for (int i = tid; i < nk; i += ST_NT) {
        const double w = exp((double)lg[kept[i]] / T - qmax);
        sw[i] = (w < INFINITY && w > 0.0) ? w : 0.0;
    }
    __syncthreads();
    ST_STAMP(5)
    // the total (one fold), the draw, then a second fold of the same terms that stops at the first
    // running sum above the chosen weight: that index is WeightedIndex's partition point over
    // cumulative_weights = S_0..S_{n-2} (n - 1 when none exceeds it), without storing the sums
    auto wload = [&](int i) { return sw[i]; };
    const double total = block_serial_fold(nk, lds_big, &stop_s, nullptr, wload, [](double) { return false; },
                                           [](int) {});
    if (tid == 0) {
        total_s = total;
        if (!(total > 0.0)) {
            // every weight zero: Iterator::max_by over the logits (the LAST maximum)
            int best = kept[0];
            for (int i = 1; i < nk; ++i)
                if (!(lg[kept[i]] < lg[best])) best = kept[i];
            tok_s = best;
        } else {
            // UniformFloat::<f64>::new(0, total): shrink scale until scale * max_rand < total
            const double max_rand = 1.0 - 0x1p-52;
            double scale = total;
            while (!(__dadd_rn(__dmul_rn(scale, max_rand), 0.0) < total))
                scale = __longlong_as_double(__double_as_longlong(scale) - 1);
            uint32_t* st = a.rng + (long)b * RNG_WORDS;
            const uint64_t u = rng_next_u64(st);
            const double v12 = __longlong_as_double((long long)((u >> 12) | 0x3FF0000000000000ull));
            chosen_s = __dadd_rn(__dmul_rn(v12 - 1.0, scale), 0.0);
        }
        keep_s = nk - 1;
    }
    __syncthreads();
    ST_STAMP(6)
    if (total_s > 0.0) {
        const double chosen = chosen_s;
        (void)block_serial_fold(nk, lds_big, &stop_s, nullptr, wload, [&](double S) { return S > chosen; },
                                [&](int g) { keep_s = min(g, nk - 1); });
        __syncthreads();
        if (tid == 0) tok_s = kept[keep_s];
    }
    __syncthreads();
    ST_STAMP(7)
#undef ST_STAMP
    // ---- 5. hand the id to the final selection kernel
    for (int j = tid; j < a.red_blocks; j += ST_NT) {
        a.red_idx[(long)b * a.red_blocks + j] = j == 0 ? tok_s : 0x7fffffff;
        if (j == 0) a.red_val[(long)b * a.red_blocks] = 0.f;
    }
}

void launch_dec_stoch_select(const DecSampleArgs& a, hipStream_t s) {
    if (!(a.temperature > 0.0)) throw std::runtime_error("EINVAL: sampling needs temperature > 0");
    if (!a.rng || !a.st_key || !a.st_idx || !a.st_w || a.st_ld < a.V)
        throw std::runtime_error("EINTERNAL: sampling workspaces missing");
    const size_t lds = sizeof(uint32_t) * (size_t)((a.V + 31) / 32);
    if (lds + sizeof(int) * (ST_DIG * ST_NT + 64) > 160 * 1024)
        throw std::runtime_error("EINVAL: vocabulary too large for the sampling kernel");
    hipLaunchKernelGGL(dec_stoch_select_kernel, dim3(a.B), dim3(ST_NT), lds, s, a);
}

}  // namespace dsocr
