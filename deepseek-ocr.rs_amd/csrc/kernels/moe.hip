// MoE routing on device (no host sync, unlike the reference's to_vec1 at
// block.rs:1304): router softmax + greedy top-k, grouping of assignments by
// expert, weighted combine with the shared experts, and SwiGLU for the
// grouped-GEMM prefill path.
#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

// One wave per token.  block.rs:1263-1301: softmax (or sigmoid) over E logits,
// sort descending (stable: ties keep the lower expert id), take top-k,
// optional renormalisation (+1e-20) and routed scaling.
__global__ __launch_bounds__(256) void router_topk_kernel(const float* logits, int T, int E, int topk, int softmax_scoring,
                                                          int norm_topk, float scaling, int* ids, float* w) {
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= T) return;
    const float* lg = logits + (long)t * E;
    constexpr int MAXE = 4;  // E <= 256
    float sc[MAXE];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
        int e = lane + 64 * j;
        sc[j] = e < E ? lg[e] : -INFINITY;
        mx = fmaxf(mx, sc[j]);
    }
    if (softmax_scoring) {
        mx = wave_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < MAXE; ++j) {
            int e = lane + 64 * j;
            sc[j] = e < E ? expf(sc[j] - mx) : 0.f;
            sum += sc[j];
        }
        sum = wave_sum(sum);
#pragma unroll
        for (int j = 0; j < MAXE; ++j) sc[j] = (lane + 64 * j) < E ? sc[j] / sum : -INFINITY;
    } else {
#pragma unroll
        for (int j = 0; j < MAXE; ++j) sc[j] = (lane + 64 * j) < E ? 1.0f / (1.0f + expf(-sc[j])) : -INFINITY;
    }
    float wsum = 0.f;
    float picked[8];
    for (int k = 0; k < topk; ++k) {
        // wave argmax: larger value wins, ties -> lower expert id
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < MAXE; ++j) {
            int e = lane + 64 * j;
            if (e < E && (sc[j] > bv || (sc[j] == bv && e < bi))) { bv = sc[j]; bi = e; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            float ov = __shfl_xor(bv, o, 64);
            int oi = __shfl_xor(bi, o, 64);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
#pragma unroll
        for (int j = 0; j < MAXE; ++j)
            if (lane + 64 * j == bi) sc[j] = -INFINITY;
        picked[k < 8 ? k : 7] = bv;
        if (lane == 0) ids[(long)t * topk + k] = bi;
        wsum += bv;
    }
    if (lane == 0) {
        for (int k = 0; k < topk; ++k) {
            float v = picked[k < 8 ? k : 7];
            if (topk > 1 && norm_topk) v = v / (wsum + 1e-20f);
            if (scaling != 1.0f) v = v * scaling;
            w[(long)t * topk + k] = v;
        }
    }
}

void launch_router_topk(const float* logits, int T, int E, int topk, int softmax_scoring, int norm_topk, float scaling,
                        int* topk_ids, float* topk_w, hipStream_t s) {
    if (T == 0) return;
    hipLaunchKernelGGL(router_topk_kernel, dim3((T + 3) / 4), dim3(256), 0, s, logits, T, E, topk, softmax_scoring,
                       norm_topk, scaling, topk_ids, topk_w);
}

// Single workgroup: histogram, exclusive scan, placement (order inside an expert
// is irrelevant: every assignment row is computed independently and the
// combine reads it back by position, so results are placement-independent).
__global__ __launch_bounds__(1024) void moe_group_kernel(const int* ids, int n, int E, int* eoff, int* arow, int* apos,
                                                         int topk) {
    __shared__ int cnt[257];
    __shared__ int cur[257];
    for (int e = threadIdx.x; e <= E; e += blockDim.x) { cnt[e] = 0; cur[e] = 0; }
    __syncthreads();
    for (int a = threadIdx.x; a < n; a += blockDim.x) atomicAdd(&cnt[ids[a]], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int e = 0; e < E; ++e) { int c = cnt[e]; cnt[e] = acc; acc += c; }
        cnt[E] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e <= E; e += blockDim.x) eoff[e] = cnt[e];
    for (int a = threadIdx.x; a < n; a += blockDim.x) {
        int e = ids[a];
        int p = cnt[e] + atomicAdd(&cur[e], 1);
        arow[p] = a / topk;
        apos[a] = p;
    }
}

void launch_moe_group(const int* topk_ids, int T, int topk, int E, int* eoff, int* arow, int* apos, int* scratch,
                      hipStream_t s) {
    (void)scratch;
    hipLaunchKernelGGL(moe_group_kernel, dim3(1), dim3(1024), 0, s, topk_ids, T * topk, E, eoff, arow, apos, topk);
}

// combine: v = sum_k w_k * y_k (top-k order, f32), v += shared, out (+)= v
// (block.rs:1374-1389 then the block's residual add, block.rs:184).
__global__ __launch_bounds__(256) void moe_combine_kernel(const float* y, const int* apos, const float* w,
                                                          const float* shared, int T, int topk, int H, float* out,
                                                          int accumulate) {
    const int t = blockIdx.x;
    for (int j = threadIdx.x; j < H; j += blockDim.x) {
        float v = 0.f;
        for (int k = 0; k < topk; ++k) v += y[(long)apos[t * topk + k] * H + j] * w[t * topk + k];
        if (shared) v = v + shared[(long)t * H + j];
        float* op = out + (long)t * H + j;
        *op = accumulate ? (*op + v) : v;
    }
}

void launch_moe_combine(const float* y, const int* apos, const float* topk_w, const float* shared, int T, int topk,
                        int H, float* out, int accumulate, hipStream_t s) {
    if (T == 0) return;
    hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, s, y, apos, topk_w, shared, T, topk, H, out,
                       accumulate);
}

__global__ void silu_mul_kernel(const float* g, int ldg, int I, int rows, float* h, int ldh) {
    long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    long total = (long)rows * I;
    for (; idx < total; idx += (long)gridDim.x * blockDim.x) {
        long r = idx / I;
        int i = (int)(idx % I);
        float gv = g[r * ldg + i];
        float uv = g[r * ldg + I + i];
        h[r * ldh + i] = (gv / (1.0f + expf(-gv))) * uv;
    }
}

void launch_silu_mul(const float* g, int ldg, int I, int rows, float* h, int ldh, hipStream_t s) {
    long total = (long)rows * I;
    if (total == 0) return;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(silu_mul_kernel, dim3(blocks), dim3(256), 0, s, g, ldg, I, rows, h, ldh);
}

}  // namespace dsocr
