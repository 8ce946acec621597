// Dev microbenchmark of the decode kernels in isolation (full DeepSeek-OCR decoder shapes, random
// weights), timed per launch from the dispatch-packet timestamps (prof_events / DSOCR_LAUNCH, the
// figures rocprofv3's kernel trace reports) and as back-to-back hipGraph replays.  Weight buffers
// rotate over more than the 256 MiB Infinity Cache so every launch streams from HBM.
//   tools/build_kbench.sh && tools/kbench [case ...]
//   cases: router8 moe1 moe8 gemv1 gemv8 attn1 attn8 lm8 (default: all)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "../deepseek-ocr.rs_amd/csrc/kernels/kernels.hpp"

using namespace dsocr;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

__global__ void fill_f16(uint16_t* p, size_t n, uint32_t seed, float amp) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        const float u = ((h & 0xffffff) / 16777216.0f - 0.5f) * 2.f * amp;
        _Float16 f = (_Float16)u;
        uint16_t b;
        __builtin_memcpy(&b, &f, 2);
        p[i] = b;
    }
}
__global__ void fill_f32(float* p, size_t n, uint32_t seed, float amp, float off) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        p[i] = off + ((h & 0xffffff) / 16777216.0f - 0.5f) * 2.f * amp;
    }
}

static uint32_t g_seed = 1;
static void* dalloc(size_t bytes) {
    void* p = nullptr;
    CK(hipMalloc(&p, bytes ? bytes : 16));
    CK(hipMemset(p, 0, bytes ? bytes : 16));
    return p;
}
static uint16_t* rand_f16(size_t n, float amp = 0.05f) {
    auto* p = (uint16_t*)dalloc(n * 2);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, p, n, g_seed++ * 7919u, amp);
    return p;
}
static float* rand_f32(size_t n, float amp = 1.f, float off = 0.f) {
    auto* p = (float*)dalloc(n * 4);
    hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, 0, p, n, g_seed++ * 104729u, amp, off);
    return p;
}

struct Timing {
    double avg_us = 0, replay_us = 0;
};

static double ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

// per-launch dispatch timestamps (the body's first DSOCR_LAUNCH) + graph replay of n bodies
static Timing timeit(int n, const std::function<void(int)>& body, hipStream_t s) {
    Timing t;
    body(0);
    CK(hipStreamSynchronize(s));
    std::vector<hipEvent_t> ev(2 * n);
    for (auto& e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < n; ++i) {
        prof_events() = ProfEvents{ev[2 * i], ev[2 * i + 1]};
        body(i);
        if (prof_events().start) { fprintf(stderr, "body made no instrumented launch\n"); exit(3); }
    }
    CK(hipEventSynchronize(ev[2 * n - 1]));
    double sum = 0;
    for (int i = 0; i < n; ++i) sum += ms_between(ev[2 * i], ev[2 * i + 1]);
    t.avg_us = 1000.0 * sum / n;
    for (auto& e : ev) (void)hipEventDestroy(e);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) body(i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    t.replay_us = 1000.0 * ms_between(e0, e1) / n;
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return t;
}

static void report(const char* name, const Timing& t, double bytes) {
    printf("%-34s avg %8.2f us  (%6.3f TB/s)   replay %8.2f us  (%6.3f TB/s)   bytes %.2f MB\n", name, t.avg_us,
           bytes / t.avg_us / 1e6, t.replay_us, bytes / t.replay_us / 1e6, bytes / 1e6);
    fflush(stdout);
}

// DeepSeek-OCR decoder (deepseek-ocr.json language config)
constexpr int H = 1280, E = 64, TOPK = 6, I = 896, IS = 1792, HEADS = 10, HD = 128, V = 129280;
constexpr int NL = 11;  // MoE layers

struct MoeLayerW {
    uint16_t *router, *gu, *d, *sgu, *sd;
    uint16_t *gu_s = nullptr, *sgu_s = nullptr, *d_s = nullptr, *sd_s = nullptr;  // fragment-ordered copies
    uint16_t* router_s = nullptr;
    float* norm;
};
static bool g_swz = getenv("KB_SWZ") && atoi(getenv("KB_SWZ")) != 0;

static std::vector<MoeLayerW> g_moe;
static void moe_weights() {
    if (!g_moe.empty()) return;
    for (int l = 0; l < NL; ++l) {
        MoeLayerW w;
        w.router = rand_f16((size_t)E * H, 0.05f);
        w.gu = rand_f16((size_t)E * 2 * I * H);
        w.d = rand_f16((size_t)E * H * I);
        w.sgu = rand_f16((size_t)2 * IS * H);
        w.sd = rand_f16((size_t)H * IS);
        w.norm = rand_f32(H, 0.2f, 1.0f);
        if (g_swz) {
            w.gu_s = (uint16_t*)dalloc(mm_swizzle_elems(E * 2 * I, H) * 2);
            launch_mm_swizzle(w.gu, E * 2 * I, H, w.gu_s, nullptr);
            w.sgu_s = (uint16_t*)dalloc(mm_swizzle_elems(2 * IS, H) * 2);
            launch_mm_swizzle(w.sgu, 2 * IS, H, w.sgu_s, nullptr);
            w.d_s = (uint16_t*)dalloc(mm_swizzle_elems(E * H, I) * 2);
            launch_mm_swizzle(w.d, E * H, I, w.d_s, nullptr);
            w.sd_s = (uint16_t*)dalloc(mm_swizzle_elems(H, IS) * 2);
            launch_mm_swizzle(w.sd, H, IS, w.sd_s, nullptr);
            w.router_s = (uint16_t*)dalloc(mm_swizzle_elems(E, H) * 2);
            launch_mm_swizzle(w.router, E, H, w.router_s, nullptr);
        }
        g_moe.push_back(w);
    }
}

static void case_moe(int T, hipStream_t s, bool route_only) {
    moe_weights();
    float* x = rand_f32((size_t)T * H);
    MoeDecodeArgs a;
    a.T = T; a.H = H; a.E = E; a.topk = TOPK; a.I = I; a.Is = IS;
    a.x = x; a.eps = 1e-6f; a.out = x;
    a.router_wdt = WDT_F16; a.wdtype = WDT_F16;
    a.softmax_scoring = 1; a.norm_topk = 0; a.scaling = 1.f;
    a.xn = (float*)dalloc((size_t)T * H * 4);
    a.xn_router = (float*)dalloc((size_t)T * H * 4);
    a.logits = (float*)dalloc((size_t)T * E * 4);
    a.ids = (int*)dalloc((size_t)T * TOPK * 4);
    a.wts = (float*)dalloc((size_t)T * TOPK * 4);
    a.h = (float*)dalloc((size_t)T * TOPK * I * 4);
    a.hs = (float*)dalloc((size_t)T * IS * 4);
    a.grp = (int*)dalloc(moe_grp_ints(E, T, TOPK) * 4);
    a.route_cnt = (int*)dalloc(64);
    if (T >= 3 && T <= 8) {
        a.dn_part = (float*)dalloc(moe_down_mm_part_floats(E, T, TOPK, I, IS, H) * 4);
        a.dn_tick = (int*)dalloc(256);
    }
    auto set = [&](int l) {
        const MoeLayerW& w = g_moe[l % NL];
        a.norm_w = w.norm; a.router = w.router; a.Wgu = w.gu; a.Wd = w.d; a.sWgu = w.sgu; a.sWd = w.sd;
        a.Wgu_swz = w.gu_s; a.sWgu_swz = w.sgu_s; a.Wd_swz = w.d_s; a.sWd_swz = w.sd_s; a.router_swz = w.router_s;
    };
    const int n = 4 * NL;
    CK(hipDeviceSynchronize());  // the fills ran on the null stream; s does not wait for it
    set(0);
    launch_moe_decode(a, s, MOE_ALL);
    CK(hipStreamSynchronize(s));
    {
        std::vector<float> lg((size_t)T * E);
        CK(hipMemcpy(lg.data(), a.logits, lg.size() * 4, hipMemcpyDeviceToHost));
        printf("logits[0][0..7]:");
        for (int e = 0; e < 8; ++e) printf(" %.4f", lg[e]);
        printf("\n");
    }
    std::vector<int> ids(T * TOPK);
    CK(hipMemcpy(ids.data(), a.ids, ids.size() * 4, hipMemcpyDeviceToHost));
    std::vector<char> seen(E, 0);
    int touched = 0;
    for (int v : ids) if (v >= 0 && v < E && !seen[v]) { seen[v] = 1; ++touched; }
    const char *gun, *dnn;
    moe_decode_kernel_names(a, &gun, &dnn);
    printf("moe T=%d: %d distinct experts, kernels %s / %s; ids", T, touched, gun, dnn);
    for (int v : ids) printf(" %d", v);
    printf("\n");
    char nm[96];
    const bool fused = T >= 3 && !(getenv("DSOCR_ROUTE_FUSED") && atoi(getenv("DSOCR_ROUTE_FUSED")) == 0);
    snprintf(nm, sizeof nm, "moe%d route", T);
    if (!fused) report(nm, timeit(n, [&](int i) { set(i); launch_moe_decode(a, s, MOE_ROUTE); }, s), (double)E * H * 2);
    if (route_only && !fused) {
        // phase clocks of the one-block router (wall clock, 100 MHz)
        auto* st = (unsigned long long*)dalloc(128);
        for (int it = 0; it < 3; ++it) {
            CK(hipMemset(st, 0, 128));
            set(it);
            DecGemvArgs g;
            g.M = T; g.N = E; g.K = H; g.x = x; g.ldx = H; g.W = a.router; g.ldw = H; g.wdtype = WDT_F16;
            g.y = a.logits; g.ldy = E; g.norm_w = a.norm_w; g.eps = a.eps; g.xn_out = a.xn;
            DecRouteEpi re;
            re.topk = TOPK; re.ids = a.ids; re.w = a.wts; re.grp = a.grp; re.stamps = st; re.counter = a.route_cnt;
            launch_dec_route_grp(g, re, s);
            CK(hipStreamSynchronize(s));
            unsigned long long h[16];
            CK(hipMemcpy(h, st, sizeof h, hipMemcpyDeviceToHost));
            printf("route stamps (us from block 0 entry):");
            for (int i = 1; i < 8; ++i) printf(" %d:%.2f", i, ((long long)h[i] - (long long)h[0]) / 100.0);
            printf("\n");
        }
        return;
    }
    // gate/up / down rotate layers but keep layer 0's routing state (same expert set per layer)
    set(0);
    launch_moe_decode(a, s, MOE_ROUTE);
    const double gub = ((double)touched * 2 * I + 2.0 * IS) * H * 2;
    const double dnb = ((double)touched * I + IS) * H * 2;
    snprintf(nm, sizeof nm, "moe%d gateup", T);
    report(nm, timeit(n, [&](int i) { set(i); launch_moe_decode(a, s, MOE_GATEUP); }, s), gub);
    snprintf(nm, sizeof nm, "moe%d down", T);
    report(nm, timeit(n, [&](int i) { set(i); launch_moe_decode(a, s, MOE_DOWN); }, s), dnb);
    if (T >= 3) {
        // phase clocks of the grouped gate/up (per block: entry, staged, router MFMAs, top-k, records, unit loop,
        // first unit batch computed, exit), us from the first block's entry: min / median / max over blocks
        auto* st = (unsigned long long*)dalloc(1024 * 8 * 8);
        for (int it = 0; it < 3; ++it) {
            CK(hipMemset(st, 0, 1024 * 64));
            set(it + 1);
            launch_moe_decode(a, s, MOE_ROUTE);
            a.stamps = st;
            launch_moe_decode(a, s, MOE_GATEUP);
            a.stamps = nullptr;
            CK(hipStreamSynchronize(s));
            std::vector<unsigned long long> h(1024 * 8);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int b = 0; b < 1024; ++b) if (h[b * 8] && h[b * 8] < t0) t0 = h[b * 8];
            printf("gateup%d stamps (us; min/med/max):", T);
            for (int i = 0; i < 8; ++i) {
                std::vector<double> v;
                for (int b = 0; b < 1024; ++b) if (h[b * 8 + i]) v.push_back(((long long)h[b * 8 + i] - (long long)t0) / 100.0);
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                printf(" %d:%.2f/%.2f/%.2f", i, v.front(), v[v.size() / 2], v.back());
            }
            printf("\n");
        }
    }
    if (T >= 3) {
        // phase clocks of the grouped down (per block: entry, staged, streamed, ticket taken, last arriver done)
        auto* st = (unsigned long long*)dalloc(2048 * 8 * 8);
        for (int it = 0; it < 3; ++it) {
            CK(hipMemset(st, 0, 2048 * 64));
            set(it + 1);
            launch_moe_decode(a, s, MOE_ROUTE);
            launch_moe_decode(a, s, MOE_GATEUP);
            a.stamps = st;
            launch_moe_decode(a, s, MOE_DOWN);
            a.stamps = nullptr;
            CK(hipStreamSynchronize(s));
            std::vector<unsigned long long> h(2048 * 8);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            int nb = 0;
            for (int b = 0; b < 2048; ++b) if (h[b * 8]) { ++nb; if (h[b * 8] < t0) t0 = h[b * 8]; }
            printf("down%d stamps, %d blocks (us; min/med/max):", T, nb);
            for (int i = 0; i < 5; ++i) {
                std::vector<double> v;
                for (int b = 0; b < 2048; ++b) if (h[b * 8 + i]) v.push_back(((long long)h[b * 8 + i] - (long long)t0) / 100.0);
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                printf(" %d:%.2f/%.2f/%.2f(n%zu)", i, v.front(), v[v.size() / 2], v.back(), v.size());
            }
            printf("\n");
        }
    }
    if (T != 1 || !getenv("KB_WAVES")) return;
    // per-wave entry / exit clocks (WaveSpan slots) of single gate/up and down launches after a fresh route,
    // by role: the gate/up's shared-expert and routed waves, the down's routed and shared waves
    auto* slots = (unsigned long long*)dalloc((size_t)SPAN_SLOTS * 16);
    const int order = getenv("DSOCR_GU_ORDER") ? atoi(getenv("DSOCR_GU_ORDER")) : 0;
    const int n_rt = TOPK * I, nbr = (n_rt + 3) / 4;
    for (int it = 0; it < 3; ++it) {
        for (int part : {MOE_GATEUP, MOE_DOWN}) {
            set(it + 1);
            launch_moe_decode(a, s, MOE_ROUTE);
            CK(hipMemsetAsync(slots, 0, (size_t)SPAN_SLOTS * 16, s));
            a.span = slots;
            launch_moe_decode(a, s, part);
            a.span = nullptr;
            CK(hipStreamSynchronize(s));
            std::vector<unsigned long long> h((size_t)SPAN_SLOTS * 2);
            CK(hipMemcpy(h.data(), slots, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (size_t w = 0; w < (size_t)SPAN_SLOTS; ++w) if (h[2 * w] && h[2 * w] < t0) t0 = h[2 * w];
            std::vector<double> ent[2], ext[2];
            for (size_t w = 0; w < (size_t)SPAN_SLOTS; ++w) {
                if (!h[2 * w]) continue;
                int role;
                if (part == MOE_GATEUP) role = order ? ((int)(w / 4) >= nbr ? 0 : 1) : (w % 4 == 0 ? 0 : 1);
                else role = (w % 8) >= 6 ? 0 : 1;  // down: waves 6, 7 of a block hold the shared chunks
                ent[role].push_back(((long long)h[2 * w] - (long long)t0) / 100.0);
                ext[role].push_back(((long long)h[2 * w + 1] - (long long)t0) / 100.0);
            }
            printf("%s waves (us from first entry; min/p10/p50/p90/max):", part == MOE_GATEUP ? "gateup" : "down  ");
            for (int r = 0; r < 2; ++r) {
                for (auto* v : {&ent[r], &ext[r]}) {
                    if (v->empty()) continue;
                    std::sort(v->begin(), v->end());
                    auto q = [&](double f) { return (*v)[(size_t)(f * (v->size() - 1))]; };
                    printf(" %s %s %.2f/%.2f/%.2f/%.2f/%.2f |", r ? "routed" : "shared", v == &ent[r] ? "entry" : "exit",
                           q(0), q(0.1), q(0.5), q(0.9), q(1));
                }
            }
            printf(" n %zu/%zu\n", ent[0].size(), ent[1].size());
        }
    }
}

static void case_gemv(int M, hipStream_t s) {
    // q/k/v (3840 x 1280) and o_proj (1280 x 1280), 40 layers' worth (> the Infinity Cache)
    constexpr int NB = 40;
    std::vector<uint16_t*> wq(NB), wo(NB);
    for (int i = 0; i < NB; ++i) { wq[i] = rand_f16((size_t)3 * H * H); wo[i] = rand_f16((size_t)H * H); }
    float* x = rand_f32((size_t)M * H);
    float* nw = rand_f32(H, 0.2f, 1.f);
    float* y = (float*)dalloc((size_t)M * 3 * H * 4);
    for (int norm = 0; norm < 2; ++norm) {
        DecGemvArgs g;
        g.M = M; g.K = H; g.x = x; g.ldx = H; g.wdtype = WDT_F16; g.y = y; g.ldw = H;
        if (norm) { g.norm_w = nw; g.eps = 1e-6f; }
        char nm[96];
        g.N = 3 * H; g.ldy = 3 * H;
        snprintf(nm, sizeof nm, "gemv M=%d N=3840%s", M, norm ? " +norm" : "");
        report(nm, timeit(NB, [&](int i) { g.W = wq[i]; launch_dec_gemv(g, s); }, s), 3.0 * H * H * 2);
        g.N = H; g.ldy = H;
        snprintf(nm, sizeof nm, "gemv M=%d N=1280%s", M, norm ? " +norm" : "");
        report(nm, timeit(NB, [&](int i) { g.W = wo[i]; launch_dec_gemv(g, s); }, s), 1.0 * H * H * 2);
    }
    for (int i = 0; i < NB; ++i) { (void)hipFree(wq[i]); (void)hipFree(wo[i]); }
}

// per-block phase records (DecAttn2Args::stamps): block range [p0, p1) = projection blocks, [a0, a1) = attention
// blocks; times in us from the first block entry: entry (first / last), and per phase the time by which every
// block that reached it had (max) and the median
static void print_stamps(const char* what, const std::vector<unsigned long long>& h, int p0, int p1, int a0, int a1) {
    unsigned long long t0 = ~0ull;
    for (size_t b = 0; b * 8 < h.size(); ++b) if (h[b * 8] && h[b * 8] < t0) t0 = h[b * 8];
    auto us = [&](unsigned long long t) { return ((long long)t - (long long)t0) / 100.0; };
    auto stat = [&](int lo, int hi, int slot, const char* nm) {
        std::vector<double> v;
        for (int b = lo; b < hi; ++b) if (h[(size_t)b * 8 + slot]) v.push_back(us(h[(size_t)b * 8 + slot]));
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        printf(" %s %.2f/%.2f/%.2f |", nm, v.front(), v[v.size() / 2], v.back());
    };
    printf("%s stamps us (min/median/max):", what);
    if (p1 > p0) { stat(p0, p1, 0, "proj entry"); stat(p0, p1, 1, "proj stored"); }
    stat(a0, a1, 0, "attn entry");
    stat(a0, a1, 2, p1 > p0 ? "q polled" : "softmax");
    stat(a0, a1, 3, "record");
    stat(a0, a1, 4, "merge polled");
    stat(a0, a1, 5, "exit");
    printf("\n");
}

static void case_attn(int B, int pos, hipStream_t s) {
    const int max_len = 1218;
    constexpr int NLA = 12;
    const long head_stride = (long)max_len * HD, page_stride = (long)HEADS * head_stride;
    std::vector<float*> kc(NLA), vc(NLA);
    for (int l = 0; l < NLA; ++l) { kc[l] = rand_f32((size_t)B * page_stride); vc[l] = rand_f32((size_t)B * page_stride); }
    float* qkv = rand_f32((size_t)B * 3 * HEADS * HD);
    std::vector<int> hpos(B, pos);
    int* kv_pos = (int*)dalloc(B * 4);
    CK(hipMemcpy(kv_pos, hpos.data(), B * 4, hipMemcpyHostToDevice));
    float* cs = rand_f32((size_t)max_len * HD, 1.f);
    float* sn = rand_f32((size_t)max_len * HD, 1.f);
    float* part = (float*)dalloc(dec_attn_workspace(B, HEADS, HD, max_len) + 64);
    dec_attn_part_init(part, dec_attn_workspace(B, HEADS, HD, max_len), nullptr);
    int* cnt = (int*)dalloc((size_t)B * HEADS * 4 + 16);
    float* o = (float*)dalloc((size_t)B * HEADS * HD * 4);
    DecAttn2Args a;
    a.qkv = qkv; a.ld = 3 * HEADS * HD; a.kv_pos = kv_pos; a.B = B; a.heads = HEADS; a.kv_heads = HEADS; a.hd = HD;
    a.rope_dim = HD; a.max_len = max_len; a.cos = cs; a.sin = sn; a.page_stride = page_stride; a.head_stride = head_stride;
    a.scale = 1.f / sqrtf((float)HD); a.part = part; a.counters = cnt; a.o = o; a.o_ld = HEADS * HD; a.prerot = B == 1;
    a.err = cnt + B * HEADS;
    char nm[96];
    snprintf(nm, sizeof nm, "attn B=%d L=%d", B, pos + 1);
    const double bytes = 2.0 * B * (pos + 1) * HEADS * HD * 4;
    report(nm, timeit(4 * NLA, [&](int i) { a.kc = kc[i % NLA]; a.vc = vc[i % NLA]; launch_dec_attn(a, s); }, s), bytes);
    const int chunks = (max_len + 63) / 64, nb = chunks * HEADS * B;
    auto* st = (unsigned long long*)dalloc((size_t)nb * 64);
    for (int it = 0; it < 2; ++it) {
        CK(hipMemset(st, 0, (size_t)nb * 64));
        a.kc = kc[it + 1]; a.vc = vc[it + 1]; a.stamps = st;
        launch_dec_attn(a, s);
        a.stamps = nullptr;
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h((size_t)nb * 8);
        CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        print_stamps("attn", h, 0, 0, 0, nb);
    }
    for (int l = 0; l < NLA; ++l) { (void)hipFree(kc[l]); (void)hipFree(vc[l]); }
}

// one page's fused q/k/v projection + decode attention (dec_qkv_attn) at L = pos + 1, 12 layers' weights and
// caches rotating, timed; then the phase clocks of three single launches (DecAttn2Args::stamps)
static void case_qkvattn1(int pos, hipStream_t s) {
    const int max_len = 1218;
    constexpr int NLA = 12;
    const long head_stride = (long)max_len * HD, page_stride = (long)HEADS * head_stride;
    std::vector<float*> kc(NLA), vc(NLA);
    std::vector<uint16_t*> wq(NLA);
    for (int l = 0; l < NLA; ++l) {
        kc[l] = rand_f32((size_t)page_stride); vc[l] = rand_f32((size_t)page_stride);
        wq[l] = rand_f16((size_t)3 * H * H);
    }
    float* x = rand_f32(H);
    float* nw = rand_f32(H, 0.2f, 1.f);
    float* row = (float*)dalloc((size_t)3 * H * 4);
    dec_qkv_sentinel_init(row, 3 * H, nullptr);
    int* kv_pos = (int*)dalloc(16);
    CK(hipMemcpy(kv_pos, &pos, 4, hipMemcpyHostToDevice));
    float* cs = rand_f32((size_t)max_len * HD, 1.f);
    float* sn = rand_f32((size_t)max_len * HD, 1.f);
    const size_t pb = dec_attn_workspace(1, HEADS, HD, max_len);
    float* part = (float*)dalloc(pb + 64);
    dec_attn_part_init(part, pb, nullptr);
    int* cnt = (int*)dalloc(HEADS * 4 + 16);
    float* o = (float*)dalloc((size_t)HEADS * HD * 4);
    DecGemvArgs g;
    g.M = 1; g.N = 3 * H; g.K = H; g.ldw = H; g.wdtype = WDT_F16; g.y = row; g.ldy = 3 * H; g.x = x; g.ldx = H;
    g.norm_w = nw; g.eps = 1e-6f;
    DecRopeEpi re;
    re.kv_pos = kv_pos; re.cos = cs; re.sin = sn; re.hd = HD; re.rot_rows = 2 * H;
    DecAttn2Args a;
    a.qkv = row; a.ld = 3 * H; a.kv_pos = kv_pos; a.B = 1; a.heads = HEADS; a.kv_heads = HEADS; a.hd = HD;
    a.rope_dim = HD; a.max_len = max_len; a.cos = cs; a.sin = sn; a.page_stride = page_stride; a.head_stride = head_stride;
    a.scale = 1.f / sqrtf((float)HD); a.part = part; a.counters = cnt; a.o = o; a.o_ld = HEADS * HD; a.prerot = 1;
    a.err = cnt + HEADS;
    auto set = [&](int i) { g.W = wq[i % NLA]; a.kc = kc[i % NLA]; a.vc = vc[i % NLA]; };
    if (!dec_qkv_attn_ok(g, re, a)) { printf("qkvattn1: fused launch refused\n"); return; }
    char nm[96];
    snprintf(nm, sizeof nm, "qkv+attn B=1 L=%d", pos + 1);
    const double bytes = 3.0 * H * H * 2 + 2.0 * (pos + 1) * HEADS * HD * 4;
    report(nm, timeit(4 * NLA, [&](int i) { set(i); launch_dec_qkv_attn(g, re, a, s); }, s), bytes);
    for (int dl : {50, 100, 150, 200, 300}) {  // K / V loads held back behind the projection (10 ns ticks)
        a.kv_delay = dl;
        snprintf(nm, sizeof nm, "qkv+attn B=1 L=%d kv_delay %d", pos + 1, dl);
        report(nm, timeit(4 * NLA, [&](int i) { set(i); launch_dec_qkv_attn(g, re, a, s); }, s), bytes);
    }
    a.kv_delay = getenv("KB_KV_DELAY") ? atoi(getenv("KB_KV_DELAY")) : 0;
    const int nq = (3 * H / 2 + 3) / 4, nb = nq + ((max_len + 63) / 64) * HEADS;
    auto* st = (unsigned long long*)dalloc((size_t)nb * 64);
    for (int it = 0; it < 3; ++it) {
        CK(hipMemset(st, 0, (size_t)nb * 64));
        set(it + 1);
        a.stamps = st;
        launch_dec_qkv_attn(g, re, a, s);
        a.stamps = nullptr;
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h((size_t)nb * 8);
        CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        print_stamps("qkv+attn", h, 0, nq, nq, nb);
    }
    for (int l = 0; l < NLA; ++l) { (void)hipFree(kc[l]); (void)hipFree(vc[l]); (void)hipFree(wq[l]); }
}

static void case_lm(int M, hipStream_t s) {
    constexpr int NB = 2;  // 2 x 331 MB > the Infinity Cache
    std::vector<uint16_t*> w(NB);
    for (int i = 0; i < NB; ++i) w[i] = rand_f16((size_t)V * H);
    float* x = rand_f32((size_t)M * H);
    float* y = (float*)dalloc((size_t)M * V * 4);
    DecGemvArgs g;
    g.M = M; g.N = V; g.K = H; g.x = x; g.ldx = H; g.wdtype = WDT_BF16; g.y = y; g.ldy = V; g.ldw = H;
    char nm[96];
    snprintf(nm, sizeof nm, "lm_head exact M=%d", M);
    report(nm, timeit(8, [&](int i) { g.W = w[i % NB]; launch_dec_gemv(g, s); }, s), (double)V * H * 2);
    // fragment-ordered copies
    std::vector<uint16_t*> ws(NB);
    for (int i = 0; i < NB; ++i) {
        ws[i] = (uint16_t*)dalloc(mm_swizzle_elems(V, H) * 2);
        launch_mm_swizzle(w[i], V, H, ws[i], s);
    }
    snprintf(nm, sizeof nm, "lm_head exact M=%d swizzled", M);
    report(nm, timeit(8, [&](int i) { g.W = w[i % NB]; g.w_swz = ws[i % NB]; launch_dec_gemv(g, s); }, s), (double)V * H * 2);
    g.w_swz = nullptr;
    for (int i = 0; i < NB; ++i) { (void)hipFree(w[i]); (void)hipFree(ws[i]); }
}

// mean stream time of n back-to-back launches of an uninstrumented body (after one warm-up)
static double time_plain(int n, const std::function<void()>& body, hipStream_t s) {
    body();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < n; ++i) body();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    const double us = 1000.0 * ms_between(e0, e1) / n;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return us;
}

// vision linears (exact-f32 3-plane GEMM, bf16 weights) at the shapes one 1024 px page runs: every
// pipeline variant (GemmBf16Args::variant) timed in interleaved rounds, outputs compared bitwise to
// variant 1 (the k order per output element is the same in all of them)
static void case_vgemm(hipStream_t s) {
    struct Shape { int M, N, K; const char* what; };
    const Shape shapes[] = {
        {4900, 2304, 768, "sam1 qkv (windows)"}, {4096, 3072, 768, "sam1 fc1"}, {4096, 768, 3072, "sam1 fc2"},
        {4900, 768, 768, "sam1 proj"}, {7056, 2304, 768, "sam4 qkv (windows)"}, {6400, 3072, 768, "sam4 fc1"},
        {6400, 768, 3072, "sam4 fc2"}, {257, 3072, 1024, "clip1 qkv"}, {404, 4096, 1024, "clip4 fc1"},
        {404, 1024, 4096, "clip4 fc2"}, {257, 1024, 1024, "clip1 out"}, {1024, 512, 2304, "net2"},
        {256, 1024, 4608, "net3"}, {400, 1280, 2048, "projector"}};
    // KB_VARIANTS: comma list of <variant>[x<split multiplier>] (e.g. 1,7,1x4,7x4)
    const char* env = getenv("KB_VARIANTS");
    std::vector<int> vars, smul;
    for (const char* p = env ? env : "2,1,2x4,1x4"; *p;) {
        vars.push_back(atoi(p));
        while (*p && *p != ',' && *p != 'x') ++p;
        smul.push_back(*p == 'x' ? atoi(p + 1) : 1);
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
    }
    for (const Shape& sh : shapes) {
        float* A = rand_f32((size_t)sh.M * sh.K);
        uint16_t* W = rand_f16((size_t)sh.N * sh.K, 0.05f);  // bit patterns as bf16: any finite values do
        float* bias = rand_f32(sh.N, 0.1f);
        const int splits = gemm_f32a_splits(sh.M, sh.N, sh.K);
        int max_mul = 1;
        for (int m : smul) max_mul = std::max(max_mul, m);
        float* part = (float*)dalloc((size_t)splits * max_mul * sh.M * sh.N * 4);
        std::vector<float*> C(vars.size());
        for (auto& c : C) c = (float*)dalloc((size_t)sh.M * sh.N * 4);
        std::vector<std::vector<double>> us(vars.size());
        const double flop = 2.0 * sh.M * sh.N * sh.K;
        for (int round = 0; round < 3; ++round)
            for (size_t v = 0; v < vars.size(); ++v) {
                GemmBf16Args g;
                g.M = sh.M; g.N = sh.N; g.K = sh.K; g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.bias = bias;
                g.C = C[v]; g.ldc = sh.N; g.part = part; g.variant = vars[v];
                g.splits = std::max(1, std::min(splits * smul[v], sh.K / 32 / 2));
                us[v].push_back(time_plain(8, [&] { launch_gemm_f32a(g, s); }, s));
            }
        std::vector<float> ref((size_t)sh.M * sh.N), got(ref.size());
        CK(hipMemcpy(ref.data(), C[0], ref.size() * 4, hipMemcpyDeviceToHost));
        printf("vgemm %-20s M %5d N %5d K %5d splits %d:", sh.what, sh.M, sh.N, sh.K, splits);
        for (size_t v = 0; v < vars.size(); ++v) {
            CK(hipMemcpy(got.data(), C[v], got.size() * 4, hipMemcpyDeviceToHost));
            const bool same = memcmp(ref.data(), got.data(), ref.size() * 4) == 0;
            std::sort(us[v].begin(), us[v].end());
            printf("  v%dx%d %7.1f us %5.0f TF%s", vars[v], smul[v], us[v][1], flop / us[v][1] / 1e6, same ? "" : " DIFF");
        }
        printf("\n");
        fflush(stdout);
        for (auto& c : C) (void)hipFree(c);
        (void)hipFree(A); (void)hipFree(W); (void)hipFree(bias);
        (void)hipFree(part);
    }
}

// dots.ocr tower linears (bf16 x bf16 -> bf16 epilogue, gemm_bf16_nt) at the 2044 px page's 21316 rows:
// variant 1 (one LDS stage, the default) vs 2 (two stages), interleaved rounds, outputs compared bitwise
// (a 256 x 256 eight-wave tile measured 0.7x of variant 1 here and was dropped: profiles/r03_kbench_dgemm.log)
static void case_dgemm(hipStream_t s) {
    struct Shape { int M, N, K; const char* what; };
    const Shape shapes[] = {{21316, 4608, 1536, "qkv"}, {21316, 1536, 1536, "proj"}, {21316, 8448, 1536, "fc1|fc3"},
                            {21316, 1536, 4224, "fc2"}};
    const int vars[2] = {1, getenv("KB_DGEMM_V") ? atoi(getenv("KB_DGEMM_V")) : 3};
    for (const Shape& sh : shapes) {
        uint16_t* A = rand_f16((size_t)sh.M * sh.K, 0.5f);
        uint16_t* W = rand_f16((size_t)sh.N * sh.K, 0.05f);
        float* bias = rand_f32(sh.N, 0.1f);
        uint16_t* C[2] = {(uint16_t*)dalloc((size_t)sh.M * sh.N * 2), (uint16_t*)dalloc((size_t)sh.M * sh.N * 2)};
        const int acc_mode = getenv("KB_DGEMM_ACC") ? 1 : 0;  // C += A W^T + b (the residual linears), same start
        if (acc_mode) {
            uint16_t* c0 = rand_f16((size_t)sh.M * sh.N, 1.0f);
            for (auto* c : C) CK(hipMemcpy(c, c0, (size_t)sh.M * sh.N * 2, hipMemcpyDeviceToDevice));
            (void)hipFree(c0);
        }
        std::vector<double> us[2];
        const double flop = 2.0 * sh.M * sh.N * sh.K;
        for (int round = 0; round < 3; ++round)
            for (int v = 0; v < 2; ++v) {
                GemmBf16Args g;
                g.M = sh.M; g.N = sh.N; g.K = sh.K; g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.bias = bias;
                g.C = reinterpret_cast<float*>(C[v]); g.ldc = sh.N; g.out_bf16 = 1; g.variant = vars[v]; g.accumulate = acc_mode;
                us[v].push_back(time_plain(4, [&] { launch_gemm_bf16(g, s); }, s));
            }
        std::vector<uint16_t> r1((size_t)sh.M * sh.N), r2(r1.size());
        CK(hipMemcpy(r1.data(), C[0], r1.size() * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r2.data(), C[1], r2.size() * 2, hipMemcpyDeviceToHost));
        printf("dgemm %-8s M %5d N %5d K %5d:", sh.what, sh.M, sh.N, sh.K);
        for (int v = 0; v < 2; ++v) {
            std::sort(us[v].begin(), us[v].end());
            printf("  v%d %8.1f us %5.0f TF", vars[v], us[v][1], flop / us[v][1] / 1e6);
        }
        printf("  v%d==v%d %s\n", vars[0], vars[1], memcmp(r1.data(), r2.data(), r1.size() * 2) ? "NO" : "yes");
        fflush(stdout);
        if (getenv("KB_STAMPS")) {  // ping-pong diagnostic build: per-wave segment shares (row 0 = waves 0-3, row 1 = 4-7)
            unsigned long long* st = (unsigned long long*)dalloc(64 * 8 * 12 * 8);
            CK(hipMemset(st, 0, 64 * 8 * 12 * 8));
            GemmBf16Args g;
            g.M = sh.M; g.N = sh.N; g.K = sh.K; g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.bias = bias;
            g.C = reinterpret_cast<float*>(C[1]); g.ldc = sh.N; g.out_bf16 = 1; g.variant = 3; g.stamps = st;
            launch_gemm_bf16(g, s);
            CK(hipStreamSynchronize(s));
            std::vector<unsigned long long> h(64 * 8 * 12);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            const char* nm[8] = {"issue", "reads", "vm_r1", "bar1", "mfma", "vm_r0", "bar2", "total"};
            for (int row = 0; row < 2; ++row) {
                double sum[12] = {0};
                for (int b = 0; b < 64; ++b)
                    for (int w = row * 4; w < row * 4 + 4; ++w)
                        for (int k = 0; k < 12; ++k) sum[k] += (double)h[((size_t)b * 8 + w) * 12 + k];
                printf("  stamps row %d (cycles per k-tile):", row);
                const double nk = (double)(sh.K / 32) * 64 * 4;
                for (int k = 0; k < 8; ++k) printf(" %s %.0f", nm[k], sum[k] / nk);
                printf(" | per block: prologue %.0f epilogue %.0f kernel %.0f cycles, %.2f us (%.2f GHz)\n", sum[8] / 256,
                       sum[9] / 256, sum[10] / 256, sum[11] / 256 / 100.0, sum[10] / sum[11] / 10.0);
            }
            (void)hipFree(st);
        }
        for (auto* c : C) (void)hipFree(c);
        (void)hipFree(A); (void)hipFree(W); (void)hipFree(bias);
    }
}

int main(int argc, char** argv) {
    std::vector<std::string> cases;
    for (int i = 1; i < argc; ++i) cases.push_back(argv[i]);
    if (cases.empty()) cases = {"router8", "moe1", "moe8", "gemv1", "gemv8", "attn1", "attn8", "lm8"};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (const auto& c : cases) {
        if (c == "router8") case_moe(8, s, true);
        else if (c == "moe1") case_moe(1, s, false);
        else if (c == "moe8") case_moe(8, s, false);
        else if (c == "gemv1") case_gemv(1, s);
        else if (c == "gemv8") case_gemv(8, s);
        else if (c == "attn1") { case_attn(1, 706, s); case_attn(1, 1216, s); }
        else if (c == "attn8") { case_attn(8, 706, s); case_attn(8, 1216, s); }
        else if (c == "qkvattn1") { case_qkvattn1(706, s); case_qkvattn1(1216, s); }
        else if (c == "lm8") case_lm(8, s);
        else if (c == "vgemm") case_vgemm(s);
        else if (c == "dgemm") case_dgemm(s);
        else fprintf(stderr, "unknown case %s\n", c.c_str());
        CK(hipStreamSynchronize(s));
    }
    printf("kbench done\n");
    return 0;
}
