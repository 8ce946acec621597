// Microbenchmark: cost of executing straight-line (once-fetched) code vs the same instruction count from a short
// loop body, one wave per CU, every CU at once (the decode kernels' prologues are straight-line code executed
// once per block).  Per launch: median over waves of (exit - entry) in s_memrealtime ticks (10 ns).
//   hipcc --offload-arch=gfx950 -O3 tools/mb_icache.hip -o tools/mb_icache && tools/mb_icache
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R64(x) R4(R16(x))
#define R256(x) R4(R64(x))
#define R1024(x) R4(R256(x))

template <int MODE>
__global__ __launch_bounds__(64) void k(unsigned long long* out, float* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float v = (float)threadIdx.x;
    if (MODE == 0) {  // 4096 instructions straight-line (16 KB of VOP1 code)
        asm volatile(R1024(R4("v_add_f32 %0, 1.0, %0\n")) : "+v"(v));
    } else if (MODE == 1) {  // the same 4096 from a 64-instruction loop body
        for (int i = 0; i < 64; ++i) asm volatile(R64("v_add_f32 %0, 1.0, %0\n") : "+v"(v));
    } else if (MODE == 2) {  // 1024 straight-line (4 KB)
        asm volatile(R1024("v_add_f32 %0, 1.0, %0\n") : "+v"(v));
    } else {  // 1024 from a loop
        for (int i = 0; i < 16; ++i) asm volatile(R64("v_add_f32 %0, 1.0, %0\n") : "+v"(v));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (v == -1.f) sink[0] = v;
}

int main() {
    unsigned long long* d;
    float* sink;
    CK(hipMalloc(&d, 4096 * 8));
    CK(hipMalloc(&sink, 64));
    const char* names[4] = {"4096 straight (16 KB)", "4096 loop (256 B body)", "1024 straight (4 KB)", "1024 loop"};
    for (int rep = 0; rep < 3; ++rep)
        for (int m = 0; m < 4; ++m) {
            for (int it = 0; it < 2; ++it) {
                if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(64), 0, 0, d, sink);
                if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(64), 0, 0, d, sink);
                if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(64), 0, 0, d, sink);
                if (m == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(64), 0, 0, d, sink);
                CK(hipDeviceSynchronize());
                std::vector<unsigned long long> h(256);
                CK(hipMemcpy(h.data(), d, 256 * 8, hipMemcpyDeviceToHost));
                std::sort(h.begin(), h.end());
                printf("%-26s launch %d: wave time us min %.2f med %.2f max %.2f\n", names[m], it, h[0] / 100.0, h[128] / 100.0,
                       h[255] / 100.0);
            }
        }
    return 0;
}
