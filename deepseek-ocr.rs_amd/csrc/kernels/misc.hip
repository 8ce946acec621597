// Data-movement kernels of the page path (HBM-bound byte work: no MFMA) and the
// on-device greedy token selection.
#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

static inline unsigned grid_for(long total, int block = 256, long cap = 16384) {
    long b = (total + block - 1) / block;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (unsigned)b;
}

// SAM PatchEmbed conv k=s=ps (sam.rs:427-456) as im2col: img NCHW [n][3][H][W] ->
// cols [n*gh*gw][3*ps*ps], K order (c, ky, kx) == the [O][C][kh][kw] weight layout.
__global__ void patch_im2col_kernel(const float* img, int n, int H, int W, int ps, float* cols) {
    const int gh = H / ps, gw = W / ps, K = 3 * ps * ps;
    const long total = (long)n * gh * gw * K;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int k = (int)(i % K);
        const long row = i / K;
        const int gx = (int)(row % gw);
        const int gy = (int)((row / gw) % gh);
        const int b = (int)(row / ((long)gw * gh));
        const int c = k / (ps * ps), ky = (k / ps) % ps, kx = k % ps;
        cols[i] = img[(((long)b * 3 + c) * H + gy * ps + ky) * W + gx * ps + kx];
    }
}
void launch_patch_im2col(const float* img, int n, int H, int W, int ps, float* cols, hipStream_t s) {
    long total = (long)n * (H / ps) * (W / ps) * 3 * ps * ps;
    hipLaunchKernelGGL(patch_im2col_kernel, dim3(grid_for(total)), dim3(256), 0, s, img, n, H, W, ps, cols);
}

// Conv2d on NHWC activations (SAM neck + downsample, sam.rs:475-576): cols
// [n*oh*ow][kh*kw*C] with K order (ky, kx, c); the weight is re-laid out on load.
__global__ void conv_im2col_nhwc_kernel(const float* x, int n, int H, int W, int C, int kh, int kw, int stride, int pad,
                                        float* cols) {
    const int oh = (H + 2 * pad - kh) / stride + 1, ow = (W + 2 * pad - kw) / stride + 1;
    const int K = kh * kw * C;
    const int C4 = C / 4;
    const long total = (long)n * oh * ow * kh * kw * C4;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        long t = i / C4;
        const int kx = (int)(t % kw); t /= kw;
        const int ky = (int)(t % kh); t /= kh;
        const int ox = (int)(t % ow); t /= ow;
        const int oy = (int)(t % oh);
        const int b = (int)(t / oh);
        const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (iy >= 0 && iy < H && ix >= 0 && ix < W)
            v = *reinterpret_cast<const float4*>(x + (((long)b * H + iy) * W + ix) * C + c4 * 4);
        const long row = ((long)b * oh + oy) * ow + ox;
        *reinterpret_cast<float4*>(cols + row * K + (ky * kw + kx) * C + c4 * 4) = v;
    }
}
void launch_conv_im2col_nhwc(const float* x, int n, int H, int W, int C, int kh, int kw, int stride, int pad,
                             float* cols, hipStream_t s) {
    const int oh = (H + 2 * pad - kh) / stride + 1, ow = (W + 2 * pad - kw) / stride + 1;
    long total = (long)n * oh * ow * kh * kw * (C / 4);
    hipLaunchKernelGGL(conv_im2col_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, n, H, W, C, kh, kw, stride,
                       pad, cols);
}

// x[rep][r][c] += t[r][c]  (absolute position embedding add, sam.rs:249-267)
__global__ void add_broadcast_kernel(float* x, const float* t, long per, int reps) {
    const long total = per * reps;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
        x[i] += t[i % per];
}
void launch_add_broadcast(float* x, const float* t, long rows_per_rep, int cols, int reps, hipStream_t s) {
    long per = rows_per_rep * cols;
    hipLaunchKernelGGL(add_broadcast_kernel, dim3(grid_for(per * reps)), dim3(256), 0, s, x, t, per, reps);
}

// CLIP embeddings (clip.rs:165-236): out[b][0] = cls + pos[0]; out[b][1+i] = sam[b][i] + pos[1+i]
__global__ void clip_embed_kernel(const float* sam, const float* cls, const float* pos, int n, int S, int C,
                                  float* out) {
    const long total = (long)n * (S + 1) * C;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long r = i / C;
        const int tok = (int)(r % (S + 1));
        const int b = (int)(r / (S + 1));
        const float base = tok == 0 ? cls[c] : sam[((long)b * S + tok - 1) * C + c];
        out[i] = base + pos[(long)tok * C + c];
    }
}
void launch_clip_embed(const float* sam, const float* cls, const float* pos, int n, int S, int C, float* out,
                       hipStream_t s) {
    long total = (long)n * (S + 1) * C;
    hipLaunchKernelGGL(clip_embed_kernel, dim3(grid_for(total)), dim3(256), 0, s, sam, cls, pos, n, S, C, out);
}

// build_clip_sam_tokens (model/mod.rs:604-650): [clip[b][1+i] || sam[b][i]]
__global__ void concat_clip_sam_kernel(const float* clip, const float* sam, int n, int S, int C1, int C2, float* out) {
    const int C = C1 + C2;
    const long total = (long)n * S * C;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long r = i / C;
        const int tok = (int)(r % S);
        const int b = (int)(r / S);
        out[i] = c < C1 ? clip[((long)b * (S + 1) + tok + 1) * C1 + c] : sam[((long)b * S + tok) * C2 + (c - C1)];
    }
}
void launch_concat_clip_sam(const float* clip, const float* sam, int n, int S, int C1, int C2, float* out,
                            hipStream_t s) {
    long total = (long)n * S * (C1 + C2);
    hipLaunchKernelGGL(concat_clip_sam_kernel, dim3(grid_for(total)), dim3(256), 0, s, clip, sam, n, S, C1, C2, out);
}

__device__ __forceinline__ float table_val(const void* table, int dt, long idx) {
    const uint16_t* t = reinterpret_cast<const uint16_t*>(table);
    return dt == WDT_BF16 ? bf16_bits_to_f32(t[idx]) : f16_bits_to_f32(t[idx]);
}

// Prefill input rows: token embeddings with image rows injected at mask slots
// (inject_image_tokens, model/mod.rs:1760-1857) and the formatted image tokens
// (newline / view_separator rows, model/mod.rs:590-709, 879-923).
__global__ void assemble_rows_kernel(const int* kind, const int* index, int rows, int H, const void* table, int dt,
                                     const float* srcA, const float* srcB, const float* vecA, const float* vecB,
                                     float* dst, long ld) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const int k = kind[r];
    const long ix = index[r];
    for (int c = threadIdx.x; c < H; c += blockDim.x) {
        float v;
        switch (k) {
            case 0: v = table_val(table, dt, ix * H + c); break;
            case 1: v = srcA[ix * H + c]; break;
            case 2: v = srcB[ix * H + c]; break;
            case 3: v = vecA[c]; break;
            default: v = vecB[c]; break;
        }
        dst[(long)r * ld + c] = v;
    }
}
void launch_assemble_rows(const int* kind, const int* index, int rows, int H, const void* table, int table_dt,
                          const float* srcA, const float* srcB, const float* vecA, const float* vecB, float* dst,
                          long ld_dst, hipStream_t s) {
    if (rows == 0) return;
    hipLaunchKernelGGL(assemble_rows_kernel, dim3(rows), dim3(256), 0, s, kind, index, rows, H, table, table_dt, srcA,
                       srcB, vecA, vecB, dst, ld_dst);
}

__global__ void embed_tokens_kernel(const void* table, int dt, const int* ids, int n, int H, float* out, long ld) {
    const int r = blockIdx.x;
    if (r >= n) return;
    const long id = ids[r];
    for (int c = threadIdx.x; c < H; c += blockDim.x) out[(long)r * ld + c] = table_val(table, dt, id * H + c);
}
void launch_embed_tokens(const void* table, int table_dt, const int* ids, int n, int H, float* out, long ld,
                         hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(embed_tokens_kernel, dim3(n), dim3(256), 0, s, table, table_dt, ids, n, H, out, ld);
}

// ------------------------------------------------------------------ parity trace
// grid (chunks, B): page b's raw logits row -> trace[b][out_len[b]] while the page is running
__global__ void trace_logits_kernel(const float* lg, int V, long ld, const int* out_len, const int* done, float* trace,
                                    long steps) {
    const int b = blockIdx.y;
    const int n = out_len[b];
    if (done[b] || n >= steps) return;
    float* dst = trace + ((long)b * steps + n) * V;
    const float* src = lg + (long)b * ld;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V; i += gridDim.x * blockDim.x) dst[i] = src[i];
}
void launch_trace_logits(const float* logits, int B, int V, long ld, const int* out_len, const int* done, float* trace,
                         long steps, hipStream_t s) {
    if (B == 0 || V == 0) return;
    hipLaunchKernelGGL(trace_logits_kernel, dim3(64, B), dim3(256), 0, s, logits, V, ld, out_len, done, trace, steps);
}

// ------------------------------------------------------------------ repetition penalty
// sampling.rs:34-96: every distinct context token's logit is divided (>0) or multiplied
// (<=0) by the penalty once.  Selection itself is dec_argmax_partial / dec_sample_final (decode.hip).
__global__ void rep_penalty_kernel(SampleArgs a) {
    // apply once per distinct context token: the first occurrence applies it
    const int b = blockIdx.y;
    const int n = a.ctx_len[b];
    const int* ctx = a.ctx + (long)b * a.ctx_cap;
    float* lg = a.logits + (long)b * a.ld;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int t = ctx[i];
        if (t < 0 || t >= a.V) continue;
        bool first = true;
        for (int j = 0; j < i; ++j)
            if (ctx[j] == t) { first = false; break; }
        if (!first) continue;
        float v = lg[t];
        lg[t] = v > 0.f ? v / a.rep_penalty : v * a.rep_penalty;
    }
}

void launch_rep_penalty(const SampleArgs& a, hipStream_t s) {
    if (a.rep_penalty > 0.f && fabsf(a.rep_penalty - 1.0f) > 1.1920929e-07f)
        hipLaunchKernelGGL(rep_penalty_kernel, dim3(8, a.B), dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ launch spans (diagnostics)
// One block folds the per-wave (entry, exit) slots of the launch just made (dev_common.hpp WaveSpan):
// first entry, last exit, slots seen; clears them; counts the distinct ids of the launch (e.g. the
// experts its routing picked) and stores the record at the step the device is on (out_len of page 0).
__global__ __launch_bounds__(1024) void span_reduce_kernel(unsigned long long* slots, unsigned long long* rec,
                                                            const int* step, int cap, const int* ids, int n_ids) {
    __shared__ unsigned long long lo_s[16], hi_s[16];
    __shared__ int cnt_s[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long lo = ~0ull, hi = 0;
    int cnt = 0;
    for (long i = tid; i < SPAN_SLOTS; i += 1024) {
        const unsigned long long a = slots[2 * i], b = slots[2 * i + 1];
        if (a != 0) {
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
            ++cnt;
            slots[2 * i] = 0;
            slots[2 * i + 1] = 0;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
        cnt += __shfl_xor(cnt, o);
    }
    if (lane == 0) { lo_s[wave] = lo; hi_s[wave] = hi; cnt_s[wave] = cnt; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 16; ++w) {
            lo = lo_s[w] < lo ? lo_s[w] : lo;
            hi = hi_s[w] > hi ? hi_s[w] : hi;
            cnt += cnt_s[w];
        }
        int distinct = 0;
        for (int i = 0; i < n_ids; ++i) {
            bool seen = false;
            for (int j = 0; j < i; ++j) seen = seen || ids[j] == ids[i];
            distinct += (!seen && ids[i] >= 0) ? 1 : 0;
        }
        int k = step ? *step : 0;
        k = k < 0 ? 0 : (k >= cap ? cap - 1 : k);
        unsigned long long* r = rec + 4L * k;
        r[0] = cnt ? lo : 0;
        r[1] = hi;
        r[2] = (unsigned long long)distinct;
        r[3] = (unsigned long long)cnt;
    }
}

void launch_span_reduce(unsigned long long* slots, unsigned long long* rec, const int* step, int cap, const int* ids,
                        int n_ids, hipStream_t s) {
    hipLaunchKernelGGL(span_reduce_kernel, dim3(1), dim3(1024), 0, s, slots, rec, step, cap, ids, n_ids);
}

// Chain spans: block r folds region r's slots stamped since the previous fold (entry > tmark[step & 1]); block 0
// then stamps tmark[(step + 1) & 1] (read by the next step's fold, never by this one).
__global__ __launch_bounds__(1024) void span_chain_fold_kernel(const unsigned long long* slots, unsigned long long* rec,
                                                               const int* step, int cap, unsigned long long* tmark) {
    __shared__ unsigned long long lo_s[16], hi_s[16];
    __shared__ int cnt_s[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = blockIdx.x;
    int k = step ? *step : 0;
    k = k < 0 ? 0 : (k >= cap ? cap - 1 : k);
    const unsigned long long since = tmark[k & 1];
    const unsigned long long* sl = slots + (size_t)r * SPAN_SLOTS * 2;
    unsigned long long lo = ~0ull, hi = 0;
    int cnt = 0;
    for (long i = tid; i < SPAN_SLOTS; i += 1024) {
        const unsigned long long a = sl[2 * i], b = sl[2 * i + 1];
        if (a > since) {
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
            ++cnt;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
        cnt += __shfl_xor(cnt, o);
    }
    if (lane == 0) { lo_s[wave] = lo; hi_s[wave] = hi; cnt_s[wave] = cnt; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 16; ++w) {
            lo = lo_s[w] < lo ? lo_s[w] : lo;
            hi = hi_s[w] > hi ? hi_s[w] : hi;
            cnt += cnt_s[w];
        }
        unsigned long long* o = rec + ((size_t)k * gridDim.x + r) * 4;
        o[0] = cnt ? lo : 0;
        o[1] = cnt ? hi : 0;
        o[2] = (unsigned long long)cnt;
        o[3] = 0;
        if (r == 0) tmark[(k + 1) & 1] = __builtin_amdgcn_s_memrealtime();
    }
}

void launch_span_chain_fold(const unsigned long long* slots, int nreg, unsigned long long* rec, const int* step, int cap,
                            unsigned long long* tmark, hipStream_t s) {
    hipLaunchKernelGGL(span_chain_fold_kernel, dim3(nreg), dim3(1024), 0, s, slots, rec, step, cap, tmark);
}

}  // namespace dsocr
