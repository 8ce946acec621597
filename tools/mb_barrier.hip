// What a device-wide barrier inside one persistent launch costs on MI355X, next to the kernel
// boundary it would replace (the persistent per-layer decode kernel question):
//   boundary: N dependent launches of a tiny kernel (G blocks of 256 threads) replayed from one hipGraph;
//   barrier:  one launch of G blocks crossing N grid barriers (arrival counter: one relaxed agent-scope
//             add per block, release / acquire fences, bounded spin on a monotonic target);
//   xcd:      the same launch with the XCD-hierarchical barrier (MI355X_MICROARCH.md barrier-xcd): each block
//             adds to its XCC's counter (XCC from HW_REG_XCC_ID); the XCC's last arriver adds to the top
//             counter, waits for all eight, publishes the XCC's generation; the others poll only their
//             XCC's generation word (one line per XCC), then an agent acquire;
// all per step, G in {64, 128, 256, 512} (every block resident: at most 2 per CU).
// build: hipcc --offload-arch=gfx950 -O3 tools/mb_barrier.hip -o tools/mb_barrier
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(256) void k_step(float* buf, int step) {
    // a dependent step: block b reads what block b - 1 wrote last step (the boundary orders them)
    if (threadIdx.x == 0) {
        const int b = blockIdx.x, g = gridDim.x;
        buf[b] = buf[(b + g - 1) % g] * 0.5f + (float)step;
    }
}

__global__ __launch_bounds__(256) void k_barrier(float* buf, int* cnt, int* err, int steps) {
    __shared__ int bail;
    const int b = blockIdx.x, g = gridDim.x;
    for (int s = 0; s < steps; ++s) {
        if (threadIdx.x == 0) {
            buf[b] = buf[(b + g - 1) % g] * 0.5f + (float)s;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int target = (s + 1) * g;
            int ok = 0;
            for (unsigned it = 0; it < (1u << 22); ++it) {
                if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) { ok = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            bail = !ok;
        }
        __syncthreads();
        if (bail) return;  // every wave of the block leaves together; the grid drains
    }
}

// XCC id of the executing CU (s_getreg HW_REG_XCC_ID = 20, bits [3:0]: size 4 -> (3 << 11) | 20)
__device__ __forceinline__ int xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7; }

// xc: [8 XCC counters][8 XCC generations][top], each on its own 128-B line (32 ints); per_xcc[x] = blocks on
// XCC x (counted by a census launch before)
__global__ __launch_bounds__(256) void k_census(int* per_xcc) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(per_xcc + xcc_id(), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_barrier_xcd(float* buf, int* xc, const int* per_xcc, int* err, int steps) {
    __shared__ int bail;
    const int b = blockIdx.x, g = gridDim.x;
    const int x = xcc_id();
    int* cnt_x = xc + 32 * x;
    int* gen_x = xc + 32 * (8 + x);
    int* top = xc + 32 * 16;
    const int mine = per_xcc[x];
    int nx = 0;
    for (int i = 0; i < 8; ++i) nx += per_xcc[i] > 0 ? 1 : 0;
    for (int s = 0; s < steps; ++s) {
        if (threadIdx.x == 0) {
            buf[b] = buf[(b + g - 1) % g] * 0.5f + (float)s;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const int old = __hip_atomic_fetch_add(cnt_x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int ok = 0;
            if (old == (s + 1) * mine - 1) {  // the XCC's last arriver: top counter, then publish
                __hip_atomic_fetch_add(top, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (unsigned it = 0; it < (1u << 22); ++it) {
                    if (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (s + 1) * nx) { ok = 1; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                __hip_atomic_store(gen_x, s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                for (unsigned it = 0; it < (1u << 22); ++it) {
                    if (__hip_atomic_load(gen_x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= s + 1) { ok = 1; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (!ok) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            bail = !ok;
        }
        __syncthreads();
        if (bail) return;
    }
}

int main() {
    const int N = 2000;
    float* buf;
    int *cnt, *err;
    CK(hipMalloc(&buf, 4096 * 4));
    CK(hipMalloc(&cnt, 4));
    CK(hipMalloc(&err, 4));
    int *xc, *per_xcc;
    CK(hipMalloc(&xc, 32 * 17 * 4));
    CK(hipMalloc(&per_xcc, 8 * 4));
    CK(hipMemset(buf, 0, 4096 * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int G : {64, 128, 256, 512}) {
        // boundary
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_step, dim3(G), dim3(256), 0, s, buf, i);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms_b = 0;
        CK(hipEventElapsedTime(&ms_b, e0, e1));
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(gr);
        // barrier (warm launch first)
        float ms_p = 0;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemsetAsync(cnt, 0, 4, s));
            CK(hipMemsetAsync(err, 0, 4, s));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_barrier, dim3(G), dim3(256), 0, s, buf, cnt, err, N);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms_p, e0, e1));
        }
        int herr = 0;
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        // XCD-hierarchical barrier
        float ms_x = 0;
        int herr_x = 0;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemsetAsync(xc, 0, 32 * 17 * 4, s));
            CK(hipMemsetAsync(per_xcc, 0, 8 * 4, s));
            CK(hipMemsetAsync(err, 0, 4, s));
            hipLaunchKernelGGL(k_census, dim3(G), dim3(256), 0, s, per_xcc);
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_barrier_xcd, dim3(G), dim3(256), 0, s, buf, xc, per_xcc, err, N);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms_x, e0, e1));
        }
        CK(hipMemcpy(&herr_x, err, 4, hipMemcpyDeviceToHost));
        int px[8];
        CK(hipMemcpy(px, per_xcc, 32, hipMemcpyDeviceToHost));
        printf("G=%4d  kernel boundary (graph replay) %6.2f us/step   grid barrier (one launch) %6.2f us/step%s"
               "   XCD-hierarchical barrier %6.2f us/step%s  (blocks per XCC %d %d %d %d %d %d %d %d)\n", G,
               1e3 * ms_b / N, 1e3 * ms_p / N, herr ? "  [barrier gave up]" : "", 1e3 * ms_x / N,
               herr_x ? " [gave up]" : "", px[0], px[1], px[2], px[3], px[4], px[5], px[6], px[7]);
        fflush(stdout);
    }
    printf("mb_barrier done\n");
    return 0;
}
