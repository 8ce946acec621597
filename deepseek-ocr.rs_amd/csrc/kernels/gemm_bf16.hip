// bf16 x bf16 -> f32 GEMM on the gfx950 matrix cores for the f32-exact split formulation of the
// vision linears (sam.rs:656-701 linear_forward, clip.rs:418-447 apply_linear, model/mod.rs:392-444
// projector): every f32 activation row is split exactly into three bf16 planes
// a = lo + mid + hi (split3_rows_kernel; RNE at each step, residuals exact by Sterbenz) laid out
// [lo | mid | hi] along K, and the bf16 weight is tripled [W | W | W] at load, so
//     A . W^T = A3 . W3^T   with K3 = 3 K,
// a plain NT GEMM whose bf16 x bf16 products are exact in the f32 accumulator (the small planes
// accumulate first).  Same result as f32 matmul up to summation order.
//
// Kernel: 128 x 128 x 64 tiles, 256 threads = 4 waves as 2 x 2 of 64 x 64 (2 x 2 MFMA 32x32x16),
// two LDS stages filled by 16-byte global_load_lds (lane-linear LDS image, XOR-swizzled 16-byte
// chunks via the SOURCE address so the fragment ds_read_b128s are conflict-free), counted vmcnt +
// raw s_barrier (cdna_hip_programming.md §5, "Pipelining across barriers"), XCD-aware tile order.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dsocr {

typedef __bf16 bf16x8_v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int TB_M = 128, TB_N = 128, TB_K = 64;
constexpr int TB_STAGE = (TB_M + TB_N) * TB_K;  // bf16 elements per stage

// 128 rows x 64 bf16 (128-byte rows): wave w, instruction i fills rows (4w + i) * 8 .. + 7; lane L
// writes LDS row R + L / 8, slot L % 8, which holds global chunk (L % 8) ^ ((row >> 1) & 7).  Two rows
// share a 256-B bank row, so row r's 16-B chunk c sits in slot (r & 1) * 8 + (c ^ ((r >> 1) & 7)): the 16
// rows of each ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, + 32) land on 16
// distinct slots (MI355X_MICROARCH.md §LDS; the former c ^ (r & 7) put rows 12 and 20 on one slot).
__device__ __forceinline__ void stage_tile(const uint16_t* g, long ld, int r0, int rmax, int k0, uint16_t* lds,
                                           int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int R = (wave * 4 + i) * 8;
        const int r = R + (lane >> 3);
        const int j = (lane & 7) ^ ((r >> 1) & 7);
        const long row = min(r0 + r, rmax);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g + row * ld + k0 + j * 8),
                                         (lds_void*)(lds + R * TB_K), 16, 0, 0);
    }
}

// fragment of rows r .. r + 31 (lane & 31), k chunk kc + (lane >> 5), from a swizzled tile
__device__ __forceinline__ bf16x8_v frag(const uint16_t* lds, int r, int kc) {
    const int c = kc ^ ((r >> 1) & 7);
    return *reinterpret_cast<const bf16x8_v*>(lds + r * TB_K + c * 8);
}

__device__ __forceinline__ float rnd_bf16(float v) { return (float)(__bf16)v; }

// tile -> (M band, N column) in grouped order: gm bands per group, consecutive tiles walk down the
// group's bands of one column, then the next column (gm = 1: one band across every column)
__device__ __forceinline__ void tile_coords(int tile, int ntm, int ntn, int gm, int& bm, int& bn) {
    if (gm <= 1) {
        bm = tile / ntn;
        bn = tile % ntn;
        return;
    }
    const int per_group = gm * ntn;
    const int first = (tile / per_group) * gm;
    const int gsz = min(ntm - first, gm);
    const int t = tile % per_group;
    bm = first + t % gsz;
    bn = t / gsz;
}

static int gemm_group_m(int requested) {
    if (requested >= 0) return requested;
    static const int v = getenv("DSOCR_GEMM_GROUP_M") ? atoi(getenv("DSOCR_GEMM_GROUP_M")) : 8;
    return v;
}

// bf16-output epilogue: each reference op rounds to bf16 on its own (matmul, + bias, activation,
// + residual), so the rounding chain is rnd(rnd(rnd(acc) + b) ...)
__device__ __forceinline__ void bf16_store_epilogue(const GemmBf16Args& g, long orow, int col, float acc, float bv) {
    float v = rnd_bf16(acc);
    if (g.bias) v = rnd_bf16(v + bv);
    if (g.act) v = rnd_bf16(apply_act(v, g.act));
    __bf16* cp = reinterpret_cast<__bf16*>(g.C) + orow * (long)g.ldc + col;
    if (g.accumulate) v = rnd_bf16((float)*cp + v);
    *cp = (__bf16)v;
}

template <int NST>
__global__ __launch_bounds__(256, 2) void gemm_bf16_nt_kernel(GemmBf16Args g) {
    __shared__ __attribute__((aligned(16))) uint16_t smem[NST * TB_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware tile order (bijective; blocks b and b + 8 share an XCD): consecutive tiles of one
    // XCD walk the N tiles of one M row band, so the A band stays in that XCD's L2
    const int ntn = (g.N + TB_N - 1) / TB_N;
    const int nwg = gridDim.x;
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    // split-K: wgid = tile * splits + split (a tile's K slices on one XCD, adjacent in time)
    const int split = wgid % g.splits, tile = wgid / g.splits;
    int bm, bn;
    tile_coords(tile, (g.M + TB_M - 1) / TB_M, ntn, g.group_m, bm, bn);
    const int m0 = bm * TB_M, n0 = bn * TB_N;
    const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A);
    const uint16_t* W = reinterpret_cast<const uint16_t*>(g.W);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nk_all = g.K / TB_K;
    const int kbeg = (int)((long)nk_all * split / g.splits), kend = (int)((long)nk_all * (split + 1) / g.splits);
    const int nk = kend - kbeg;
    auto issue = [&](int kt) {
        uint16_t* st = smem + (NST == 1 ? 0 : (kt & 1) * TB_STAGE);
        stage_tile(A, g.lda, m0, g.M - 1, (kbeg + kt) * TB_K, st, wave, lane);
        stage_tile(W, g.ldw, n0, g.N - 1, (kbeg + kt) * TB_K, st + TB_M * TB_K, wave, lane);
    };
    if (NST == 2 && nk > 0) issue(0);
    for (int kt = 0; kt < nk; ++kt) {
        if (NST == 1) {  // one stage: the other blocks of the CU hide this block's stage loads
            issue(kt);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (kt + 1 < nk) {
            issue(kt + 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage kt landed (8 DMAs of kt+1 in flight)
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const uint16_t* As = smem + (NST == 1 ? 0 : (kt & 1) * TB_STAGE);
        const uint16_t* Bs = As + TB_M * TB_K;
#pragma unroll
        for (int ks = 0; ks < TB_K / 16; ++ks) {
            const int kc = ks * 2 + (lane >> 5);
            bf16x8_v af[2], bfv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = frag(As, wm * 64 + i * 32 + (lane & 31), kc);
#pragma unroll
            for (int j = 0; j < 2; ++j) bfv[j] = frag(Bs, wn * 64 + j * 32 + (lane & 31), kc);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave is done with this stage before it is refilled
        asm volatile("" ::: "memory");
    }
    // epilogue: D layout col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int half = lane >> 5, l32 = lane & 31;
    if (g.splits > 1) {  // raw partial sums of this K slice: [split][M][N], reduced in split order
        float* P = g.part + (long)split * g.M * g.N;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int col = n0 + wn * 64 + j * 32 + l32;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    if (row < g.M && col < g.N) P[(long)row * g.N + col] = acc[i][j][r];
                }
            }
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + l32;
            if (col >= g.N) continue;
            const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (row >= g.M) continue;
                const long orow = g.c_rows ? (long)g.c_rows[row] : (long)row;
                if (orow < 0) continue;
                if (g.out_bf16) {
                    bf16_store_epilogue(g, orow, col, acc[i][j][r], bv);
                    continue;
                }
                float v = apply_act(acc[i][j][r] + bv, g.act);
                float* cp = g.C + orow * (long)g.ldc + col;
                if (g.accumulate) v += *cp;
                *cp = v;
            }
        }
    }
}

// split-K reduction: C = act(sum_s P[s] + bias) (+ C), rows scattered through c_rows
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmBf16Args g) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)g.M * g.N) return;
    const int row = (int)(i / g.N), col = (int)(i % g.N);
    float v = 0.f;
    for (int sp = 0; sp < g.splits; ++sp) v += g.part[(long)sp * g.M * g.N + i];
    const long orow = g.c_rows ? (long)g.c_rows[row] : (long)row;
    if (orow < 0) return;
    if (g.out_bf16) {
        bf16_store_epilogue(g, orow, col, v, g.bias ? g.bias[col] : 0.f);
        return;
    }
    v = apply_act(v + (g.bias ? g.bias[col] : 0.f), g.act);
    float* cp = g.C + orow * g.ldc + col;
    if (g.accumulate) v += *cp;
    *cp = v;
}

// the same, four columns per thread (N % 4 == 0): 16-byte partial loads, one row per grid.y, no
// index division, all slices in flight at once (the scalar kernel ran ~11 us per call on the CLIP /
// projector shapes, 125 calls per vision pass)
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(GemmBf16Args g) {
    const int col = (blockIdx.x * 256 + threadIdx.x) * 4;
    const int row = blockIdx.y;
    if (col >= g.N) return;
    const long i = (long)row * g.N + col;
    const long mn = (long)g.M * g.N;
    const long orow = g.c_rows ? (long)g.c_rows[row] : (long)row;  // issued with the slice loads
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (g.bias)
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = g.bias[col + e];
    // every slice's load issued before the first add (a runtime-bounded loop waited for each in turn:
    // one HBM round trip per slice), then summed in slice order as before
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int sp0 = 0; sp0 < g.splits; sp0 += 8) {
        float4 p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sp0 + j < g.splits) p[j] = *reinterpret_cast<const float4*>(g.part + (sp0 + j) * mn + i);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sp0 + j < g.splits) { v.x += p[j].x; v.y += p[j].y; v.z += p[j].z; v.w += p[j].w; }
    }
    if (orow < 0) return;
    const float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (g.out_bf16) {
            bf16_store_epilogue(g, orow, col + e, r[e], bv[e]);
            continue;
        }
        float x = apply_act(r[e] + bv[e], g.act);
        float* cp = g.C + orow * g.ldc + col + e;
        if (g.accumulate) x += *cp;
        *cp = x;
    }
}

static void launch_splitk_reduce(const GemmBf16Args& g, hipStream_t s) {
    if (g.N % 4 == 0 && g.M <= 65535 && (reinterpret_cast<uintptr_t>(g.part) & 15) == 0) {
        hipLaunchKernelGGL(splitk_reduce4_kernel, dim3((unsigned)((g.N / 4 + 255) / 256), (unsigned)g.M), dim3(256), 0, s, g);
        return;
    }
    const long n = (long)g.M * g.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
}

// ---------------------------------------------------------------------------------------
// Ping-pong form for the large bf16-output linears (the dots.ocr tower: 21316 rows x 1536 / 4608 / 8448
// columns).  256 x 256 tiles, 32 k per LDS stage, four stages (128 KiB, one block per CU), 8 waves as
// 2 (M) x 4 (N) of 128 x 64 (4 x 2 tiles of v_mfma_f32_32x32x16_bf16).  The two wave rows run one
// barrier apart: in every interval between two workgroup barriers one row issues its LDS DMAs and reads
// its fragments (12 ds_read_b128) while the other runs its 16 MFMAs, and the two waves sharing a SIMD
// (w and w + 4) belong to different rows, so the matrix core always has a wave to run.  Stage use, with
// interval I_j ending at barrier b_j, row g loading k-tile t in I_{2t+g} and multiplying in I_{2t+g+1}:
//  - at the start of its load interval for k-tile t a row issues the DMAs of k-tile t + 3 (its share:
//    its own 128 A rows, 128 of the 256 W rows) into stage (t + 3) & 3 = (t - 1) & 3, whose last
//    reads (k-tile t - 1) both rows finished (lgkmcnt(0)) before b_{2t-1};
//  - k-tile u + 1 is waited for (counted vmcnt: the DMAs of the k-tiles after it stay in flight) by row
//    1 at the end of its load interval for u and by row 0 at the end of its multiply interval for u, both
//    before b_{2u+1}; it is read in I_{2u+2} and I_{2u+3}, after that barrier.
// Row 1 takes one extra barrier before its first k-tile, row 0 one after its last, so both rows pass the
// same number.  The DMA images are lane-linear per instruction (16 rows of 64 B) with the 16-byte chunk
// XOR-swizzled by the SOURCE address (chunk ^ ((row >> 2) & 3)), which puts every ds_read_b128 lane group
// on 16 distinct slots of the 256-byte bank row.  Every output element sees the same MFMA sequence as
// gemm_bf16_nt_kernel (k ascending, 16 per instruction), so the results are bitwise equal to it
// (tools/kbench dgemm compares them).
constexpr int PP_M = 256, PP_N = 256, PP_K = 32, PP_NST = 4;
constexpr int PP_STAGE = (PP_M + PP_N) * PP_K;  // bf16 elements per stage (32 KiB)
constexpr int PP_LDS = PP_NST * PP_STAGE * 2;    // bytes

__device__ __forceinline__ bf16x8_v pp_frag(const uint16_t* lds, int r, int kc) {
    return *reinterpret_cast<const bf16x8_v*>(lds + r * PP_K + ((kc ^ ((r >> 2) & 3)) * 8));
}

// row g's share of k-tile kt: 128 A rows (g * 128 + ...) and 128 W rows, 2 + 2 DMAs of 16 rows per wave;
// piece p: rows (wg * 2 + (p >> 1)) * 16 of A (p even) or W (p odd)
__device__ __forceinline__ void pp_issue(int p, const uint16_t* A, long lda, int m0, int mmax, const uint16_t* W,
                                         long ldw, int n0, int nmax, int k0, uint16_t* st, int grp, int wg, int lane) {
    const int R = grp * 128 + (wg * 2 + (p >> 1)) * 16;
    const int r = R + (lane >> 2);
    const int j = (lane & 3) ^ ((r >> 2) & 3);
    if ((p & 1) == 0) {
        const long ra = min(m0 + r, mmax);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(A + ra * lda + k0 + j * 8),
                                         (lds_void*)(st + R * PP_K), 16, 0, 0);
    } else {
        const long rw = min(n0 + r, nmax);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(W + rw * ldw + k0 + j * 8),
                                         (lds_void*)(st + PP_M * PP_K + R * PP_K), 16, 0, 0);
    }
}

// a k-tile landed: the n DMAs issued after its last one stay in flight (n is 0..8, even)
__device__ __forceinline__ void pp_wait_n(int n) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void pp_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// diagnostic stamp (separate instantiation; read shares, not the run time): s_memtime with its own wait
#define PP_STAMP(var)                                                                           \
    if (STAMPS) {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                      \
    }

// rotary element as dots_rope8_kernel: x cos + rot sin, no contraction (rot = -partner on the low half)
__device__ __forceinline__ float pp_rope(float x, float pt, float cs, float sn, bool lo) {
#pragma clang fp contract(off)
    const float rot = lo ? -pt : pt;
    const float a = x * cs;
    const float b = rot * sn;
    return a + b;
}

template <bool STAMPS>
__global__ __launch_bounds__(512, 1) void gemm_bf16_pp_kernel(GemmBf16Args g) {
    extern __shared__ __attribute__((aligned(16))) uint16_t pp_smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 2, wc = wave & 3;  // wave row = staggered group, wave column
    const int ntn = (g.N + PP_N - 1) / PP_N;
    const int nwg = gridDim.x;
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    int bm, bn;
    tile_coords(tile, (g.M + PP_M - 1) / PP_M, ntn, g.group_m, bm, bn);
    const int m0 = bm * PP_M, n0 = bn * PP_N;
    const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A);
    const uint16_t* W = reinterpret_cast<const uint16_t*>(g.W);
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nk = g.K / PP_K;
    auto issue = [&](int p, int kt) {
        pp_issue(p, A, g.lda, m0, g.M - 1, W, g.ldw, n0, g.N - 1, kt * PP_K, pp_smem + (kt & 3) * PP_STAGE, wr, wc, lane);
    };
    // prologue: k-tiles 0..2 in flight, k-tile 0 landed everywhere before the first barrier
    unsigned long long p0 = 0, rt0 = 0;
    if (STAMPS) {
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(p0)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt0)::"memory");
    }
    for (int kt = 0; kt < 3 && kt < nk; ++kt)
#pragma unroll
        for (int p = 0; p < 4; ++p) issue(p, kt);
    pp_wait_n(4 * min(2, nk - 1));
    pp_barrier();
    if (wr == 1) pp_barrier();
    unsigned long long seg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sa = 0, sb = 0, sc = 0, sd = 0, se = 0, sf = 0, sh = 0, si = 0, s0 = 0;
    PP_STAMP(s0);
    for (int t = 0; t < nk; ++t) {
        // load interval: this wave's fragments of k-tile t (every DMA of k-tile t + 3 goes out in the multiply
        // interval: issued beside the ds_reads here a DMA cost ~180 cycles vs ~25-65 between MFMAs, qkv 406 vs
        // 313 us, profiles/r05_dots/gemm_pp/kb_dgemm_lp{0,2}.log)
        const bool more = t + 3 < nk;
        PP_STAMP(sa);
        PP_STAMP(sb);
        const uint16_t* As = pp_smem + (t & 3) * PP_STAGE;
        const uint16_t* Bs = As + PP_M * PP_K;
        bf16x8_v af[2][4], bfv[2][2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kc = ks * 2 + (lane >> 5);
#pragma unroll
            for (int j = 0; j < 2; ++j) bfv[ks][j] = pp_frag(Bs, wc * 64 + j * 32 + (lane & 31), kc);
#pragma unroll
            for (int i = 0; i < 4; ++i) af[ks][i] = pp_frag(As, wr * 128 + i * 32 + (lane & 31), kc);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PP_STAMP(sc);
        // DMAs issued after k-tile t + 1's: k-tile t + 2's four
        if (wr == 1 && t + 1 < nk) pp_wait_n(t + 2 < nk ? 4 : 0);
        PP_STAMP(sd);
        pp_barrier();
        PP_STAMP(se);
        // multiply interval, the DMAs of k-tile t + 3 one after every 4 MFMAs (their issue cost, ~100 cycles
        // each, runs in the MFMA shadow instead of lengthening the load interval); raised wave priority over the
        // interval (measured neutral against none, profiles/r05_dots/gemm_pp, kept as built)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks][i], bfv[ks][j], acc[i][j], 0, 0, 0);
                // MFMA group m = ks * 4 + i (2 MFMAs each): the 4 pieces after groups 1, 3, 5, 7
                const int m = ks * 4 + i;
                if (m % 2 == 1) {
                    if (more) issue(m / 2, t + 3);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        __builtin_amdgcn_s_setprio(0);
        PP_STAMP(sf);
        if (wr == 0 && t + 1 < nk) pp_wait_n((t + 2 < nk ? 4 : 0) + (more ? 4 : 0));
        PP_STAMP(sh);
        pp_barrier();
        PP_STAMP(si);
        if (STAMPS) {
            seg[0] += sb - sa; seg[1] += sc - sb; seg[2] += sd - sc; seg[3] += se - sd;
            seg[4] += sf - se; seg[5] += sh - sf; seg[6] += si - sh;
        }
    }
    if (wr == 0) pp_barrier();
    // epilogue (bf16 out, no activation, no row scatter, 16-byte aligned C rows: the launch checks).  The
    // wave's 128 x 64 result goes through its own 16 KiB of the (now idle) staging LDS: the D layout
    // (col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) is written as bf16 rnd(rnd(acc) + b)
    // with ds_write_b16 (16-byte chunk ^ 4 on rows with bit 2 set: the two half-waves on distinct banks),
    // read back as 16-byte row chunks and stored with one global_store_dwordx4 per lane (128-byte rows per
    // 8 lanes) -- the 2-byte scattered stores took ~55k cycles per block, a third of the kernel
    const int half = lane >> 5, l32 = lane & 31;
    uint16_t* ep = pp_smem + wave * (128 * 64);
    if (g.swiglu) {
        // SwiGLU pair: this wave's 64 columns are fc1 (j = 0) and fc3 (j = 1) of the same 32 h columns, lane
        // for lane; h = rnd(rnd(g / rnd(1 + rnd(exp(-g)))) * u) as dots_swiglu8_kernel, g and u each
        // rnd(rnd(acc) + b) as the separate GEMM stored them.  Staged as [128][32] bf16 (64-byte rows), stored
        // as 16-byte row chunks (4 lanes per row)
        if (n0 + wc * 64 >= g.N) return;
        const int gc = n0 + wc * 64 + l32, uc = gc + 32;
        const float bg = g.bias ? g.bias[gc] : 0.f, bu = g.bias ? g.bias[uc] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                float gv = rnd_bf16(acc[i][0][r]), uv = rnd_bf16(acc[i][1][r]);
                if (g.bias) {
                    gv = rnd_bf16(gv + bg);
                    uv = rnd_bf16(uv + bu);
                }
                const float ex = rnd_bf16(expf(-gv));
                const float sv = rnd_bf16(gv / rnd_bf16(1.0f + ex));
                const __bf16 hv = (__bf16)(sv * uv);
                ep[row * 32 + l32] = *reinterpret_cast<const uint16_t*>(&hv);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        __bf16* H = reinterpret_cast<__bf16*>(g.C);
        const int hc = (n0 + wc * 64) / 2;
#pragma unroll 4
        for (int it = 0; it < 8; ++it) {
            const int row = it * 16 + (lane >> 2), ch = lane & 3;
            const int grow = m0 + wr * 128 + row;
            const u32x4 q = *reinterpret_cast<const u32x4*>(ep + row * 32 + ch * 8);
            if (grow < g.M) *reinterpret_cast<u32x4*>(H + (long)grow * g.ldc + hc + ch * 8) = q;
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = n0 + wc * 64 + j * 32 + l32;
        const float bv = (g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                float v = rnd_bf16(acc[i][j][r]);
                if (g.bias) v = rnd_bf16(v + bv);
                const int c = j * 32 + l32;
                const int cs = (((c >> 3) ^ (((row >> 2) & 1) << 2)) << 3) | (c & 7);
                const __bf16 hv = (__bf16)v;
                ep[row * 64 + cs] = *reinterpret_cast<const uint16_t*>(&hv);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    __bf16* C = reinterpret_cast<__bf16*>(g.C);
    if (g.rope_cos && n0 < g.rope_cols) {
        // q / k tile (two heads of 128): the partner half-head (dims d +- 64) is wave wc ^ 1's LDS region, same
        // rows and chunk; every wave wrote its region before this barrier
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const uint16_t* pe = pp_smem + (wr * 4 + (wc ^ 1)) * (128 * 64);
        const int d0 = (wc & 1) * 64;
#pragma unroll 2
        for (int it = 0; it < 16; ++it) {
            const int row = it * 8 + (lane >> 3), ch = lane & 7;
            const int off = row * 64 + ((ch ^ (((row >> 2) & 1) << 2)) << 3);
            const u32x4 q = *reinterpret_cast<const u32x4*>(ep + off);
            const u32x4 pq = *reinterpret_cast<const u32x4*>(pe + off);
            const int grow = m0 + wr * 128 + row;
            if (grow >= g.M) continue;
            const float* ct = g.rope_cos + (long)grow * 128 + d0 + ch * 8;
            const float* st = g.rope_sin + (long)grow * 128 + d0 + ch * 8;
            const float4 c0 = *reinterpret_cast<const float4*>(ct), c1 = *reinterpret_cast<const float4*>(ct + 4);
            const float4 s0 = *reinterpret_cast<const float4*>(st), s1 = *reinterpret_cast<const float4*>(st + 4);
            const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
            const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
            const uint16_t* xv = reinterpret_cast<const uint16_t*>(&q);
            const uint16_t* pv = reinterpret_cast<const uint16_t*>(&pq);
            u32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a0 = pp_rope(__uint_as_float((uint32_t)xv[2 * e] << 16), __uint_as_float((uint32_t)pv[2 * e] << 16),
                                         cs[2 * e], sn[2 * e], d0 == 0);
                const float a1 = pp_rope(__uint_as_float((uint32_t)xv[2 * e + 1] << 16),
                                         __uint_as_float((uint32_t)pv[2 * e + 1] << 16), cs[2 * e + 1], sn[2 * e + 1], d0 == 0);
                const __bf16 h0 = (__bf16)a0, h1 = (__bf16)a1;
                o[e] = (uint32_t)*reinterpret_cast<const uint16_t*>(&h0) | ((uint32_t)*reinterpret_cast<const uint16_t*>(&h1) << 16);
            }
            *reinterpret_cast<u32x4*>(C + (long)grow * g.ldc + n0 + wc * 64 + ch * 8) = o;
        }
        return;
    }
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3), ch = lane & 7;
        const u32x4 q = *reinterpret_cast<const u32x4*>(ep + row * 64 + ((ch ^ (((row >> 2) & 1) << 2)) << 3));
        const int grow = m0 + wr * 128 + row, gcol = n0 + wc * 64 + ch * 8;
        if (grow >= g.M || gcol >= g.N) continue;
        __bf16* cp = C + (long)grow * g.ldc + gcol;
        const uint16_t* qv = reinterpret_cast<const uint16_t*>(&q);
        if (gcol + 8 <= g.N && !g.accumulate) {
            *reinterpret_cast<u32x4*>(cp) = q;
            continue;
        }
        u32x4 cv = gcol + 8 <= g.N ? *reinterpret_cast<const u32x4*>(cp) : u32x4{0, 0, 0, 0};
        uint16_t* cw = reinterpret_cast<uint16_t*>(&cv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (gcol + e >= g.N) break;
            float v = __uint_as_float((uint32_t)qv[e] << 16);
            if (g.accumulate) {
                const float cold = gcol + 8 <= g.N ? __uint_as_float((uint32_t)cw[e] << 16) : (float)cp[e];
                v = rnd_bf16(cold + v);
            }
            const __bf16 hv = (__bf16)v;
            cw[e] = *reinterpret_cast<const uint16_t*>(&hv);
        }
        if (gcol + 8 <= g.N) *reinterpret_cast<u32x4*>(cp) = cv;
        else
            for (int e = 0; e < 8 && gcol + e < g.N; ++e) reinterpret_cast<uint16_t*>(cp)[e] = cw[e];
    }
    if (STAMPS) {
        unsigned long long e1 = 0, rt1 = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(e1)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt1)::"memory");
        if (lane == 0 && blockIdx.x < 64) {
            seg[7] = si - s0;
            unsigned long long* o = g.stamps + ((long)blockIdx.x * 8 + wave) * 12;
            for (int k = 0; k < 8; ++k) o[k] = seg[k];
            o[8] = s0 - p0; o[9] = e1 - si; o[10] = e1 - p0; o[11] = rt1 - rt0;
        }
    }
}

// DSOCR_GEMM_PP=0 keeps the 128 x 128 one-stage kernel for the large linears (A/B)
static bool gemm_pp_on() {
    static const int v = getenv("DSOCR_GEMM_PP") ? atoi(getenv("DSOCR_GEMM_PP")) : 1;
    return v != 0;
}

int gemm_bf16_splits(int M, int N, int K) {
    const int tiles = ((M + TB_M - 1) / TB_M) * ((N + TB_N - 1) / TB_N);
    const int nk = K / TB_K;
    int sp = 1;
    // fill the chip (>= 256 blocks) while every slice keeps >= 8 K steps of 64
    while (tiles * sp < 256 && nk / (sp * 2) >= 8) sp *= 2;
    return sp;
}

void launch_gemm_bf16(const GemmBf16Args& g0, hipStream_t s) {
    GemmBf16Args g = g0;
    if (g.M <= 0 || g.N <= 0) return;
    if (g.K % TB_K || g.lda % 8 || g.ldw % 8 || (reinterpret_cast<uintptr_t>(g.A) & 15) ||
        (reinterpret_cast<uintptr_t>(g.W) & 15))
        throw std::runtime_error("EINVAL: gemm_bf16 needs K % 64 == 0 and 16-byte aligned rows");
    if (g.splits < 1 || !g.part) g.splits = 1;
    g.group_m = gemm_group_m(g.group_m);
    // ping-pong 256 x 256 kernel: variant 3, or by default for one-slice problems of >= 256 such tiles
    const long pp_tiles = (long)((g.M + PP_M - 1) / PP_M) * ((g.N + PP_N - 1) / PP_N);
    if (g.swiglu && (g.splits != 1 || g.K % PP_K || !g.out_bf16 || g.act || g.c_rows || g.accumulate || g.N % 64 ||
                     g.ldc % 8 || (reinterpret_cast<uintptr_t>(g.C) & 15)))
        throw std::runtime_error("EINVAL: the SwiGLU-pair GEMM needs one K slice, K % 32, N % 64, bf16 out, 16-byte rows");
    if (g.rope_cos && (g.swiglu || g.splits != 1 || g.K % PP_K || !g.out_bf16 || g.act || g.c_rows || g.accumulate ||
                       g.rope_cols % PP_N || g.rope_cols > g.N || g.ldc % 8 || (reinterpret_cast<uintptr_t>(g.C) & 15) ||
                       !g.rope_sin))
        throw std::runtime_error("EINVAL: the rotary GEMM epilogue needs one K slice, K % 32, bf16 out, q|k columns "
                                 "in whole 256-column tiles, 16-byte rows");
    if (g.swiglu || g.rope_cos || (g.splits == 1 && g.K % PP_K == 0 && g.out_bf16 && !g.act && !g.c_rows && g.ldc % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(g.C) & 15) == 0 &&
                     (g.variant == 3 || (g.variant == 0 && gemm_pp_on() && pp_tiles >= 256)))) {
        static bool attr = false;
        if (!attr) {
            const void* fns[2] = {reinterpret_cast<const void*>(gemm_bf16_pp_kernel<false>),
                                  reinterpret_cast<const void*>(gemm_bf16_pp_kernel<true>)};
            for (const void* f : fns)
                if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS) != hipSuccess)
                    throw std::runtime_error("gemm_bf16_pp: cannot reserve 128 KiB of LDS");
            attr = true;
        }
        const dim3 grid((unsigned)pp_tiles), blk(512);
        if (g.stamps) hipLaunchKernelGGL((gemm_bf16_pp_kernel<true>), grid, blk, PP_LDS, s, g);
        else hipLaunchKernelGGL((gemm_bf16_pp_kernel<false>), grid, blk, PP_LDS, s, g);
        return;
    }
    const int tiles = ((g.M + TB_M - 1) / TB_M) * ((g.N + TB_N - 1) / TB_N);
    // one LDS stage unless variant 2 (tools/kbench dgemm A/B: 1.2-1.4x on the dots.ocr linears,
    // profiles/r03_kbench_dgemm.log; bitwise equal results)
    if (g.variant == 2) hipLaunchKernelGGL(gemm_bf16_nt_kernel<2>, dim3(tiles * g.splits), dim3(256), 0, s, g);
    else hipLaunchKernelGGL(gemm_bf16_nt_kernel<1>, dim3(tiles * g.splits), dim3(256), 0, s, g);
    if (g.splits > 1) launch_splitk_reduce(g, s);
}

// ---------------------------------------------------------------------------------------
// The same exact-f32 linear with the plane split fused into the fragment loads: A stays f32 in HBM
// and LDS, W is the plain bf16 [N][K] weight (not tripled).  Per 16-k step a wave reads its two f32 A
// fragments (8 values per lane), splits each value exactly into hi + mid + lo bf16 (split3_rows'
// RNE steps) in registers, and issues lo.W, mid.W, hi.W on v_mfma_f32_32x32x16_bf16 against the
// same B fragment: the weight bytes per product fall to 1/3, the separate split pass (6 bytes per
// activation written and re-read) disappears, and every product stays exact in the f32 accumulator.
// Tiles 128 x 128 x 32, 4 waves as 2 x 2 of 64 x 64, two LDS stages of A 16 KB f32 + W 8 KB (three
// blocks per CU) filled by 16-byte global_load_lds, one raw s_barrier per k-step (stage k + 1 is issued
// after it, into the buffer every wave finished reading before it), counted vmcnt.  XOR-swizzled
// 16-byte chunks (A rows 128 B: chunk ^ ((r >> 1) & 7); W rows 64 B: chunk ^ ((r >> 2) & 3)) put every
// ds_read_b128 lane group on 16 distinct slots of the 256-B bank row (SQ_LDS_BANK_CONFLICT 0).  The
// bijective XCD-aware tile order and deterministic split-K of gemm_bf16_nt_kernel.  Measured and not
// kept: a third / fourth stage (fewer blocks per CU, slower or equal), register-staged loads with
// ds_write_b128 (1.7x slower).
constexpr int FX_M = 128, FX_N = 128, FX_K = 32;
constexpr int FX_AS = FX_M * FX_K;      // f32 elements of an A stage
constexpr int FX_WS = FX_N * FX_K;      // bf16 elements of a W stage

__device__ __forceinline__ bf16x8_v fx_pack(const float* v) {
    bf16x8_v r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
    return r;
}

// F16W: f16 weights (the decoder's prefill linears): each weight splits exactly into w_hi + w_lo bf16
// in registers (f16 has 11 significant bits) and the products lo.hi, mid.lo, mid.hi, hi.lo, hi.hi are
// issued (lo.lo is below f32 rounding: the W5 formulation's set) — 5 MFMAs per fragment pair, A and W
// read once instead of as 5 bf16 planes each.
// Wave layout: bf16 weights use 4 x 1 waves of 32 x 128 (each A row is split by exactly one wave; a
// 2 x 2 layout splits every A fragment in two waves and the split VALU work, not the MFMAs, bounds
// the k-step); f16 weights keep 2 x 2 of 64 x 64 (their W split would double instead).
// NST = 1: one LDS stage (24 KB: four blocks per CU at <= 128 VGPRs), the latency of a block's stage
// loads hidden by the other blocks of its CU instead of by a second stage
template <bool F16W, bool W22 = F16W, int NST = 2, int BN = FX_N>  // (BN 256 measured slower on every vision shape)
__global__ __launch_bounds__(256, 2) void gemm_f32a_nt_kernel(GemmBf16Args g) {
    constexpr int WN = W22 ? 2 : 1, WM = 4 / WN;     // waves along N / M
    constexpr int TI = FX_M / WM / 32, TJ = BN / WN / 32;
    constexpr int WS = BN * FX_K;  // bf16 elements of a W stage
    __shared__ __attribute__((aligned(16))) float a_lds[NST * FX_AS];
    __shared__ __attribute__((aligned(16))) uint16_t w_lds[NST * WS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int ntn = (g.N + BN - 1) / BN;
    const int nwg = gridDim.x;
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int split = wgid % g.splits, tile = wgid / g.splits;
    int bm, bn;
    tile_coords(tile, (g.M + FX_M - 1) / FX_M, ntn, g.group_m, bm, bn);
    const int m0 = bm * FX_M, n0 = bn * BN;
    const float* A = reinterpret_cast<const float*>(g.A);
    const uint16_t* W = reinterpret_cast<const uint16_t*>(g.W);
    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nk_all = g.K / FX_K;
    const int kbeg = (int)((long)nk_all * split / g.splits), kend = (int)((long)nk_all * (split + 1) / g.splits);
    const int nk = kend - kbeg;
    // A: 128 rows x 32 f32 (8 chunks of 16 B per row); instruction i of wave w fills rows (4w + i) * 8 .. + 7
    // W: 128 rows x 32 bf16 (4 chunks per row);     instruction i of wave w fills rows (2w + i) * 16 .. + 15
    // (LDS-DMA writes lane-linearly: lane L's 16 B land in row R + L / 8 (W: L / 4), slot L % 8 (L % 4),
    // so the lane fetches the global chunk that the swizzle puts in that slot)
    auto issue = [&](int kt) {
        const int k0 = (kbeg + kt) * FX_K;
        float* as = a_lds + (NST == 1 ? 0 : (kt & 1) * FX_AS);
        uint16_t* ws_ = w_lds + (NST == 1 ? 0 : (kt & 1) * WS);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int R = (wave * 4 + i) * 8;
            const int r = R + (lane >> 3);
            const int j = (lane & 7) ^ ((r >> 1) & 7);
            const long row = min(m0 + r, g.M - 1);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(A + row * g.lda + k0 + j * 4),
                                             (lds_void*)(as + R * FX_K), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < BN / 64; ++i) {
            const int R = (wave * (BN / 64) + i) * 16;
            const int r = R + (lane >> 2);
            const int j = (lane & 3) ^ ((r >> 2) & 3);
            const long row = min(n0 + r, g.N - 1);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(W + row * g.ldw + k0 + j * 8),
                                             (lds_void*)(ws_ + R * FX_K), 16, 0, 0);
        }
    };
    if (NST == 2 && nk > 0) issue(0);
    for (int kt = 0; kt < nk; ++kt) {
        if (NST == 1) issue(kt);  // the stage is free: every wave passed the barrier after its last read
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stage kt landed
        __builtin_amdgcn_s_barrier();  // every wave's stage kt landed; every wave is done with stage kt - 1
        asm volatile("" ::: "memory");
        if (NST == 2 && kt + 1 < nk) issue(kt + 1);  // into stage (kt - 1) & 1
        const float* As = a_lds + (NST == 1 ? 0 : (kt & 1) * FX_AS);
        const uint16_t* Ws = w_lds + (NST == 1 ? 0 : (kt & 1) * WS);
#pragma unroll
        for (int ks = 0; ks < FX_K / 16; ++ks) {
            const int kc = ks * 2 + (lane >> 5);  // this lane's 8-value k chunk (of 4)
            bf16x8_v bfv[TJ], blo[TJ];
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int r = wn * (BN / WN) + j * 32 + (lane & 31);
                if constexpr (F16W) {
                    const uint4 raw = *reinterpret_cast<const uint4*>(Ws + r * FX_K + ((kc ^ ((r >> 2) & 3)) * 8));
                    float wv[8], wh[8], wl[8];
                    unpack8<f16_t>(raw, wv);
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        wh[e] = (float)(__bf16)wv[e];
                        wl[e] = wv[e] - wh[e];
                    }
                    bfv[j] = fx_pack(wh);
                    blo[j] = fx_pack(wl);
                } else {
                    bfv[j] = *reinterpret_cast<const bf16x8_v*>(Ws + r * FX_K + ((kc ^ ((r >> 2) & 3)) * 8));
                }
            }
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const int r = wm * (FX_M / WM) + i * 32 + (lane & 31);
                const int sw = (r >> 1) & 7;
                const float4 lo4 = *reinterpret_cast<const float4*>(As + r * FX_K + (((2 * kc) ^ sw) * 4));
                const float4 hi4 = *reinterpret_cast<const float4*>(As + r * FX_K + (((2 * kc + 1) ^ sw) * 4));
                const float av[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
                float h[8], m[8], l[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    h[e] = (float)(__bf16)av[e];
                    const float r1 = av[e] - h[e];
                    m[e] = (float)(__bf16)r1;
                    l[e] = r1 - m[e];
                }
                const bf16x8_v ph = fx_pack(h), pm = fx_pack(m), pl = fx_pack(l);
#pragma unroll
                for (int j = 0; j < TJ; ++j) {
                    if constexpr (F16W) {  // small terms first
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pl, bfv[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm, blo[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm, bfv[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph, blo[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph, bfv[j], acc[i][j], 0, 0, 0);
                    } else {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pl, bfv[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm, bfv[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph, bfv[j], acc[i][j], 0, 0, 0);
                    }
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's reads done before the next barrier
        if (NST == 1) {
            __builtin_amdgcn_s_barrier();  // every wave's reads of the stage done before it is refilled
            asm volatile("" ::: "memory");
        }
    }
    const int half = lane >> 5, l32 = lane & 31;
    if (g.splits > 1) {
        float* P = g.part + (long)split * g.M * g.N;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int col = n0 + wn * (BN / WN) + j * 32 + l32;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * (FX_M / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    if (row < g.M && col < g.N) P[(long)row * g.N + col] = acc[i][j][r];
                }
            }
        return;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int col = n0 + wn * (BN / WN) + j * 32 + l32;
            if (col >= g.N) continue;
            const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * (FX_M / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (row >= g.M) continue;
                const long orow = g.c_rows ? (long)g.c_rows[row] : (long)row;
                if (orow < 0) continue;
                float v = apply_act(acc[i][j][r] + bv, g.act);
                float* cp = g.C + orow * (long)g.ldc + col;
                if (g.accumulate) v += *cp;
                *cp = v;
            }
        }
    }
}

// K slices: up to ~2 blocks per CU while every slice keeps >= 2 k-steps of 32 (tools/kbench vgemm: the CLIP
// 257 / 404-row linears, the neck convolutions and the projector ran 1.2-1.3x faster at 4-8x the slices
// of the former >= 16-step rule, the 6400-row K 3072 fc2 1.35x at 2 slices)
int gemm_f32a_splits(int M, int N, int K) {
    const int tiles = ((M + FX_M - 1) / FX_M) * ((N + FX_N - 1) / FX_N);
    const int nk = K / FX_K;
    int sp = 1;
    while (tiles * sp < 512 && nk / (sp * 2) >= 2) sp *= 2;
    return sp;
}

bool gemm_f32a_ok(const GemmBf16Args& g) {
    return g.K % FX_K == 0 && g.lda % 4 == 0 && g.ldw % 8 == 0 && (reinterpret_cast<uintptr_t>(g.A) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(g.W) & 15) == 0 && !g.out_bf16;
}

// DSOCR_GEMM_NST=2 (A/B switch, read once): the bf16-weight linears on the two-stage kernel
static int gemm_nst_env() {
    static const int v = getenv("DSOCR_GEMM_NST") ? atoi(getenv("DSOCR_GEMM_NST")) : 1;
    return v;
}

void launch_gemm_f32a(const GemmBf16Args& g0, hipStream_t s) {
    GemmBf16Args g = g0;
    if (!g.variant) g.variant = gemm_nst_env();
    if (g.M <= 0 || g.N <= 0) return;
    if (!gemm_f32a_ok(g)) throw std::runtime_error("EINVAL: gemm_f32a needs K % 32 == 0 and 16-byte aligned rows");
    if (g.splits < 1 || !g.part) g.splits = 1;
    g.group_m = gemm_group_m(g.group_m);
    const int tiles = ((g.M + FX_M - 1) / FX_M) * ((g.N + FX_N - 1) / FX_N);
    // bf16 weights: 4 x 1 waves of 32 x 128 (each A row split once), ONE LDS stage (24 KB, four blocks per
    // CU: kbench vgemm 1.00-1.18x the two-stage kernel on the SAM linears, within 3 % elsewhere); f16
    // weights: 2 x 2 (their W split would double under 4 x 1), two stages
    if (g.w_f16) hipLaunchKernelGGL((gemm_f32a_nt_kernel<true>), dim3(tiles * g.splits), dim3(256), 0, s, g);
    else if (g.variant == 2) hipLaunchKernelGGL((gemm_f32a_nt_kernel<false, false, 2>), dim3(tiles * g.splits), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_f32a_nt_kernel<false, false, 1>), dim3(tiles * g.splits), dim3(256), 0, s, g);
    if (g.splits > 1) launch_splitk_reduce(g, s);
}

// ---------------------------------------------------------------------------------------
// Grouped (MoE prefill) exact-f32 GEMM: the routed experts' gate/up and down over the token rows
// sorted by expert (block.rs:1215-1395 applies each expert to the tokens that picked it).  A prompt
// of T tokens gives each of the 64 experts ~T·topk/64 rows (28 at one 1024 px page), so the 128-row
// tiles of gemm_x3 issued >= 4x the needed MFMAs and staged every plane through register stores.
// Here tiles are 32 rows x 128 columns x 32 k: a block's tile index is mapped to (expert, row tile)
// by a 64-lane prefix sum over the per-expert tile counts (the launch covers the bound
// sum ceil(rows_e / 32) <= M / 32 + groups; surplus blocks leave), 4 waves own 32 columns each,
// the A rows are gathered by the LDS DMA itself (per-lane addresses), W rows of the expert's slab,
// and the planes are split in registers as in gemm_f32a_nt_kernel (same products, same order).
constexpr int GX_N = 128, GX_K = 32;

// GM = 32: 4 x 1 waves of 32 x 32; GM = 128 (many rows per expert): 2 x 2 waves of 64 x 64
template <bool F16W, int GM>
__global__ __launch_bounds__(256) void gemm_f32a_grp_kernel(GemmArgs g) {
    constexpr int GX_M = GM, WM = GM == 32 ? 1 : 2, WN = 4 / WM, TI = GM / WM / 32, TJ = GX_N / WN / 32;
    constexpr int AI = GM / 32;  // A DMA instructions per thread
    __shared__ __attribute__((aligned(16))) float a_lds[2 * GX_M * GX_K];
    __shared__ __attribute__((aligned(16))) uint16_t w_lds[2 * GX_N * GX_K];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // tile -> (group, row tile): inclusive prefix of ceil(rows / 32) over the groups (lane = group)
    const int t = blockIdx.y;
    int cnt = 0;
    if (lane < g.groups) cnt = g.group_off[lane + 1] - g.group_off[lane];
    const int nt = (cnt + GX_M - 1) / GX_M;
    int pre = nt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(pre, d);
        if (lane >= d) pre += o;
    }
    const unsigned long long hit = __ballot(lane < g.groups && pre > t);
    if (!hit) return;  // whole block: surplus tile
    const int grp = __builtin_ctzll(hit);
    const int m_begin = __shfl(g.group_off[min(lane, g.groups - 1)], grp);
    const int rows = __shfl(cnt, grp);
    const int mt = t - (__shfl(pre, grp) - __shfl(nt, grp));
    const int m0 = mt * GX_M, n0 = blockIdx.x * GX_N;
    const uint16_t* W = reinterpret_cast<const uint16_t*>(g.W) + (long)grp * g.w_group_stride;
    const float* bias = g.bias ? g.bias + (long)grp * g.bias_group_stride : nullptr;
    // DMA sources: A rows (wave * AI + i) * 8 + lane / 8 of the tile, W rows (2 * wave + i) * 16 + lane / 4
    const float* a_src[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
        const int ar = (wave * AI + i) * 8 + (lane >> 3);
        const int aj = (lane & 7) ^ ((ar >> 1) & 7);
        const int arr = m_begin + min(m0 + ar, rows - 1);
        a_src[i] = g.A + (long)(g.a_rows ? g.a_rows[arr] : arr) * g.lda + aj * 4;
    }
    const uint16_t* w_src[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (wave * 2 + i) * 16 + (lane >> 2);
        const int j = (lane & 3) ^ ((r >> 2) & 3);
        w_src[i] = W + (long)min(n0 + r, g.N - 1) * g.ldw + j * 8;
    }
    auto issue = [&](int kt) {
        const int k0 = kt * GX_K;
        float* as = a_lds + (kt & 1) * GX_M * GX_K;
        uint16_t* ws_ = w_lds + (kt & 1) * GX_N * GX_K;
#pragma unroll
        for (int i = 0; i < AI; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(a_src[i] + k0),
                                             (lds_void*)(as + (wave * AI + i) * 8 * GX_K), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(w_src[i] + k0),
                                             (lds_void*)(ws_ + (wave * 2 + i) * 16 * GX_K), 16, 0, 0);
    };
    const int wm = wave / WN, wn = wave % WN;
    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nk = g.K / GX_K;
    issue(0);
    for (int kt = 0; kt < nk; ++kt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 1 < nk) issue(kt + 1);
        const float* As = a_lds + (kt & 1) * GX_M * GX_K;
        const uint16_t* Ws = w_lds + (kt & 1) * GX_N * GX_K;
#pragma unroll
        for (int ks = 0; ks < GX_K / 16; ++ks) {
            const int kc = ks * 2 + (lane >> 5);
            bf16x8_v bfv[TJ], blo[TJ];
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int r = wn * (GX_N / WN) + j * 32 + (lane & 31);
                if constexpr (F16W) {
                    const uint4 raw = *reinterpret_cast<const uint4*>(Ws + r * GX_K + ((kc ^ ((r >> 2) & 3)) * 8));
                    float wv[8], wh[8], wl[8];
                    unpack8<f16_t>(raw, wv);
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        wh[e] = (float)(__bf16)wv[e];
                        wl[e] = wv[e] - wh[e];
                    }
                    bfv[j] = fx_pack(wh);
                    blo[j] = fx_pack(wl);
                } else {
                    bfv[j] = *reinterpret_cast<const bf16x8_v*>(Ws + r * GX_K + ((kc ^ ((r >> 2) & 3)) * 8));
                }
            }
#pragma unroll
            for (int i = 0; i < TI; ++i) {
            const int r = wm * (GX_M / WM) + i * 32 + (lane & 31);
            const int sw = (r >> 1) & 7;
            const float4 lo4 = *reinterpret_cast<const float4*>(As + r * GX_K + (((2 * kc) ^ sw) * 4));
            const float4 hi4 = *reinterpret_cast<const float4*>(As + r * GX_K + (((2 * kc + 1) ^ sw) * 4));
            const float av[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
            float h[8], m[8], l[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                h[e] = (float)(__bf16)av[e];
                const float r1 = av[e] - h[e];
                m[e] = (float)(__bf16)r1;
                l[e] = r1 - m[e];
            }
            const bf16x8_v ph = fx_pack(h), pm = fx_pack(m), pl = fx_pack(l);
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                if constexpr (F16W) {  // small terms first
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pl, bfv[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm, blo[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm, bfv[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph, blo[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph, bfv[j], acc[i][j], 0, 0, 0);
                } else {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pl, bfv[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm, bfv[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph, bfv[j], acc[i][j], 0, 0, 0);
                }
            }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const int half = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int col = n0 + wn * (GX_N / WN) + j * 32 + l32;
        if (col >= g.N) continue;
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * (GX_M / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (row >= rows) continue;
                const long orow = g.c_rows ? (long)g.c_rows[m_begin + row] : (long)(m_begin + row);
                if (orow < 0) continue;
                float v = apply_act(acc[i][j][r] + bv, g.act);
                float* cp = g.C + orow * (long)g.ldc + col;
                if (g.accumulate) v += *cp;
                *cp = v;
            }
        }
    }
}

bool gemm_f32a_grouped_ok(const GemmArgs& g) {
    return g.group_off && g.groups >= 1 && g.groups <= 64 && g.K % GX_K == 0 && g.lda % 4 == 0 && g.ldw % 8 == 0 &&
           g.w_group_stride % 8 == 0 && (reinterpret_cast<uintptr_t>(g.A) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(g.W) & 15) == 0;
}

void launch_gemm_f32a_grouped(const GemmArgs& g, hipStream_t s, int tile_rows) {
    if (!gemm_f32a_grouped_ok(g)) throw std::runtime_error("EINVAL: grouped gemm_f32a outside its range");
    if (g.M <= 0 || g.N <= 0) return;
    // 32-row tiles up to 256 mean rows per group, 128-row tiles above (each expert's weights re-read
    // once per row tile); tiles: sum over groups of ceil(rows / GM) <= M / GM + groups
    const int gm = (tile_rows == 32 || tile_rows == 128) ? tile_rows : ((long)g.M <= 256L * g.groups ? 32 : 128);
    const long bound = std::min<long>((long)(g.M + gm - 1) / gm + g.groups,
                                      (long)g.groups * ((std::max(g.max_group_rows, 1) + gm - 1) / gm));
    dim3 grid((g.N + GX_N - 1) / GX_N, (unsigned)bound);
    if (gm == 32) {
        if (g.wdtype == WDT_F16) hipLaunchKernelGGL((gemm_f32a_grp_kernel<true, 32>), grid, dim3(256), 0, s, g);
        else hipLaunchKernelGGL((gemm_f32a_grp_kernel<false, 32>), grid, dim3(256), 0, s, g);
    } else {
        if (g.wdtype == WDT_F16) hipLaunchKernelGGL((gemm_f32a_grp_kernel<true, 128>), grid, dim3(256), 0, s, g);
        else hipLaunchKernelGGL((gemm_f32a_grp_kernel<false, 128>), grid, dim3(256), 0, s, g);
    }
}

}  // namespace dsocr
