// Microbenchmark: every block of a one-block-per-CU grid reading the same small matrix (the fused 8-page gate/up
// prologue's router rows: 64 x 1280 f16 = 160 KB, wave w: rows 16 (w & 3) .., k half w >> 2, 20 k-steps of 16-byte
// lane loads), all issued before one wait.  Per launch: median over blocks of (all loads back - entry), in
// s_memrealtime ticks (10 ns).  Variants: 0 same order in every block; 1 the wave -> (tile, half) map rotated by
// block; 2 the k-step issue order rotated by block; 3 a single block (no sharing); 4 every block its own copy
// (no sharing, same bytes); 5 a fragment-ordered copy (each wave's 20 fragments contiguous: 1 KB per load
// instruction); 6 the same, a single block.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_bcast.hip -o tools/mb_bcast
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int K = 1280, E = 64, STEPS = K / 32, HALF = STEPS / 2;

__global__ __launch_bounds__(512) void k(const uint16_t* R, long copy_stride, int mode, unsigned long long* out,
                                         float* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, b = blockIdx.x;
    const int col = lane & 15, g = lane >> 4;
    int tile = wave & 3, kh = wave >> 2;
    if (mode == 1) { tile = (wave + b) & 3; kh = ((wave >> 2) + (b >> 2)) & 1; }
    const uint16_t* base = R + (mode == 4 ? (long)b * copy_stride : 0) + (long)(16 * tile + col) * K + 8 * g +
                           32L * kh * HALF;
    // fragment-ordered copy: wave w's 20 fragments are 20 KB contiguous, lane l's 16 bytes at 1 KB step + 16 l
    if (mode >= 5) base = R + (long)wave * (HALF * 512) + 8 * lane - 32L * 0;
    uint4 q[HALF];
    const int rot = mode == 2 ? (b % HALF) : 0;
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
        int s = i + rot;
        s = s >= HALF ? s - HALF : s;
        q[i] = *reinterpret_cast<const uint4*>(base + (mode >= 5 ? 512L : 32L) * s);
    }
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < HALF; ++i) acc += q[i].x ^ q[i].y ^ q[i].z ^ q[i].w;
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) out[b] = t2 - t0;
    if (acc == 0x12345u) sink[b] = (float)(t1 - t0);
}

int main() {
    const int grid = 256;
    const long copy = (long)E * K + 4096;  // elements per private copy (mode 4), padded
    uint16_t* R;
    unsigned long long* out;
    float* sink;
    CK(hipMalloc(&R, copy * grid * 2));
    CK(hipMemset(R, 1, copy * grid * 2));
    CK(hipMalloc(&out, grid * 8));
    CK(hipMalloc(&sink, grid * 4));
    const char* names[7] = {"same order", "tile/half rotated", "k-steps rotated", "one block", "private copies",
                            "fragment order", "fragment, 1 block"};
    for (int mode = 0; mode < 7; ++mode) {
        const int gr = (mode == 3 || mode == 6) ? 1 : grid;
        for (int rep = 0; rep < 6; ++rep) {
            // a fresh buffer touch pattern per launch is not needed: the matrix is L2/MALL-resident after the first
            hipLaunchKernelGGL(k, dim3(gr), dim3(512), 0, 0, R, copy, mode, out, sink);
            CK(hipDeviceSynchronize());
            if (rep < 2) continue;
            std::vector<unsigned long long> o(gr);
            CK(hipMemcpy(o.data(), out, gr * 8, hipMemcpyDeviceToHost));
            std::sort(o.begin(), o.end());
            printf("%-18s rep %d: med %.2f us  max %.2f us\n", names[mode], rep, o[gr / 2] * 0.01, o[gr - 1] * 0.01);
        }
    }
    printf("mb_bcast done\n");
    return 0;
}
