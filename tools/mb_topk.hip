// Microbenchmark: latency of the fused gate/up routing tail in isolation — topk_wave64 on waves 0..7 (one token
// each), the expert grouping on wave 0, and bare __syncthreads — one 512-thread block per CU slot (grid 1 or 512),
// no memory traffic beyond LDS.  Per launch: median over blocks of each phase, in s_memrealtime ticks (10 ns).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ideepseek-ocr.rs_amd/csrc/kernels tools/mb_topk.hip -o tools/mb_topk
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "dev_common.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

using namespace dsocr;

constexpr int NST = 6;

__global__ __launch_bounds__(512) void k(const float* logits, unsigned long long* out, int* sink, int T, int E, int K) {
    __shared__ float lg_s[8 * 64];
    __shared__ __attribute__((aligned(16))) float rank_s[8 * 128];
    __shared__ __attribute__((aligned(16))) int ids_s[64];
    __shared__ float w_s[64];
    __shared__ int grp_s[65 * MOE_GRP_REC];
    __shared__ unsigned long long st[NST];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    lg_s[tid] = logits[tid];
    __syncthreads();
#define ST(i) if (tid == 0) st[i] = __builtin_amdgcn_s_memrealtime();
    ST(0);
    __syncthreads();
    __syncthreads();
    __syncthreads();
    __syncthreads();
    ST(1);  // four bare barriers
    if (wave < T) topk_wave64(lg_s[wave * 64 + lane], E, K, 1, 1, 1.f, rank_s + wave * 128, ids_s + wave * 8, w_s + wave * 8);
    __syncthreads();
    ST(2);  // top-k + barrier
    if (wave == 0) group_picks_wave64<8>(ids_s, w_s, T, K, E, grp_s, reinterpret_cast<int*>(rank_s));
    __syncthreads();
    ST(3);  // grouping + barrier
    if (wave < T) topk_wave64(lg_s[wave * 64 + lane], E, K, 1, 1, 1.f, rank_s + wave * 128, ids_s + wave * 8, w_s + wave * 8);
    ST(4);  // top-k alone (wave 0's view, no barrier)
    __syncthreads();
    ST(5);
    if (tid < 64 * 18 / 18) sink[blockIdx.x * 64 + tid] = grp_s[tid] + ids_s[tid];
    if (tid < NST) out[blockIdx.x * NST + tid] = st[tid];
}

int main() {
    const int T = 8, E = 64, K = 6;
    float* lg;
    unsigned long long* out;
    int* sink;
    CK(hipMalloc(&lg, 512 * 4));
    CK(hipMalloc(&out, 512 * NST * 8));
    CK(hipMalloc(&sink, 512 * 64 * 4));
    std::vector<float> h(512);
    for (int i = 0; i < 512; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.01f;
    CK(hipMemcpy(lg, h.data(), 512 * 4, hipMemcpyHostToDevice));
    const char* names[NST - 1] = {"4 bare barriers", "topk + barrier", "grouping + barrier", "topk alone (wave 0)",
                                  "barrier"};
    for (int grid : {1, 512}) {
        for (int rep = 0; rep < 4; ++rep) {
            hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, 0, lg, out, sink, T, E, K);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> o(grid * NST);
            CK(hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost));
            if (rep == 0) continue;
            printf("grid %3d rep %d:", grid, rep);
            for (int p = 0; p < NST - 1; ++p) {
                std::vector<double> d(grid);
                for (int b = 0; b < grid; ++b) d[b] = (double)(o[b * NST + p + 1] - o[b * NST + p]) * 0.01;
                std::sort(d.begin(), d.end());
                printf("  %s %.2f us", names[p], d[grid / 2]);
            }
            printf("\n");
        }
    }
    printf("mb_topk done\n");
    return 0;
}
