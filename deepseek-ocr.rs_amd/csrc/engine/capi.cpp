// C ABI (include/dsocr.h).  Exceptions never cross this boundary: messages are
// prefixed with a status tag ("EINVAL: ...") and mapped to dsocr_status.
#include "../../../include/dsocr.h"

#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>

#include "../common/host_util.hpp"
#include "dots.hpp"
#include "engine.hpp"
#include "host_ops.hpp"

struct dsocr_engine {
    std::unique_ptr<dsocr::Engine> impl;
};
struct dsocr_page_pixels {
    dsocr::PagePixels px;
};
struct dsocr_dots {
    std::unique_ptr<dsocr::DotsVision> impl;
};

namespace {
thread_local std::string g_last_error;

dsocr_status status_from(const std::string& msg) {
    g_last_error = msg;
    auto starts = [&](const char* p) { return msg.rfind(p, 0) == 0; };
    if (starts("EINVAL")) return DSOCR_EINVAL;
    if (starts("ENOENT")) return DSOCR_ENOENT;
    if (starts("EDEVICE")) return DSOCR_EDEVICE;
    if (starts("ENOMEM")) return DSOCR_ENOMEM;
    return DSOCR_EINTERNAL;
}

template <typename F>
dsocr_status guarded(F&& f) {
    try {
        f();
        g_last_error.clear();
        return DSOCR_OK;
    } catch (const std::exception& e) {
        return status_from(e.what());
    } catch (...) {
        return status_from("EINTERNAL: unknown error");
    }
}

// Diagnostics (DSOCR_SEGV_MAPS=1): on SIGSEGV write the fault address and /proc/self/maps to stderr
// (async-signal-safe: open/read/write only), then hand the signal back to the handler that was there
// before (a profiler's or the default), so unsymbolised PCs in its stack dump resolve to library + offset.
struct sigaction g_prev_segv;
// "0x" + 16 hex digits of v into out (no libc formatting: snprintf is not async-signal-safe)
size_t hex_u64(uint64_t v, char* out) {
    static const char dig[] = "0123456789abcdef";
    out[0] = '0';
    out[1] = 'x';
    for (int i = 0; i < 16; ++i) out[2 + i] = dig[(v >> (60 - 4 * i)) & 15];
    return 18;
}
void segv_maps_handler(int sig, siginfo_t* si, void* uc) {
    char buf[4096];
    static const char head[] = "\n[dsocr] SIGSEGV at ", tail[] = "; /proc/self/maps follows\n";
    size_t n = 0;
    memcpy(buf, head, sizeof(head) - 1);
    n += sizeof(head) - 1;
    n += hex_u64(si ? (uint64_t)(uintptr_t)si->si_addr : 0, buf + n);
    memcpy(buf + n, tail, sizeof(tail) - 1);
    n += sizeof(tail) - 1;
    (void)!write(2, buf, n);
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        ssize_t r;
        while ((r = read(fd, buf, sizeof(buf))) > 0) (void)!write(2, buf, (size_t)r);
        close(fd);
    }
    (void)!write(2, "[dsocr] end of maps\n", 20);
    sigaction(SIGSEGV, &g_prev_segv, nullptr);  // the faulting instruction re-runs under the previous handler
    (void)sig;
    (void)uc;
}
void install_segv_maps_once() {
    static bool done = false;
    if (done || !getenv("DSOCR_SEGV_MAPS")) return;
    done = true;
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = segv_maps_handler;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
}

void check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("EDEVICE: ") + what + ": " + hipGetErrorString(e));
}

dsocr::GenParams to_params(const dsocr_decode_params* p) {
    if (!p) throw std::runtime_error("EINVAL: decode params are NULL");
    dsocr::GenParams g;
    g.use_cache = p->use_cache != 0;  // false: generate_without_cache (model/mod.rs:2051-2283)
    g.max_new = p->max_new_tokens;
    g.rep_penalty = p->repetition_penalty;
    g.ngram = p->no_repeat_ngram_size > 1 ? (int)p->no_repeat_ngram_size : 0;
    g.eos = p->eos_token_id;
    g.ignore_eos = p->ignore_eos != 0;
    // select_token_id samples only when do_sample && temperature > 0 (sampling.rs:67); otherwise
    // it is the greedy path
    g.do_sample = p->do_sample != 0 && p->temperature > 0.0;
    g.temperature = p->temperature;
    g.top_p = p->top_p;
    g.top_k = (long)p->top_k;
    g.seed_set = p->has_seed != 0;
    g.seed = p->seed;
    return g;
}

dsocr::GenRequest to_request(const dsocr_request& r) {
    dsocr::GenRequest g;
    if (!r.input_ids || r.prompt_len == 0) throw std::runtime_error("EINVAL: empty prompt");
    g.ids.resize(r.prompt_len);
    for (size_t i = 0; i < r.prompt_len; ++i) {
        if (r.input_ids[i] < 0 || r.input_ids[i] > INT32_MAX) throw std::runtime_error("EINVAL: token id out of range");
        g.ids[i] = (int)r.input_ids[i];
    }
    if (r.image_mask) g.mask.assign(r.image_mask, r.image_mask + r.prompt_len);
    g.page = r.page ? &r.page->px : nullptr;
    g.image_rows = r.image_rows;
    g.n_image_rows = r.n_image_rows;
    return g;
}
}  // namespace

extern "C" {

const char* dsocr_last_error(void) { return g_last_error.c_str(); }

dsocr_status dsocr_engine_load(const dsocr_load_args* args, dsocr_engine** out) {
    return guarded([&] {
        if (!args || !out) throw std::runtime_error("EINVAL: NULL argument");
        if (!args->config_path) throw std::runtime_error("EINVAL: config_path is required");
        if (args->dtype < DSOCR_F32 || args->dtype > DSOCR_BF16) throw std::runtime_error("EINVAL: bad dtype");
        install_segv_maps_once();
        auto* e = new dsocr_engine;
        try {
            e->impl.reset(new dsocr::Engine(args->config_path, args->weights_path ? args->weights_path : "",
                                            args->device_ordinal, (int)args->dtype, args->synthetic_seed,
                                            args->snapshot_path ? args->snapshot_path : ""));
        } catch (...) {
            delete e;
            throw;
        }
        *out = e;
    });
}

void dsocr_engine_free(dsocr_engine* e) { delete e; }

dsocr_status dsocr_engine_info(const dsocr_engine* e, size_t* hidden, size_t* vocab, int64_t* eos, size_t* layers) {
    return guarded([&] {
        if (!e) throw std::runtime_error("EINVAL: NULL engine");
        const auto& c = e->impl->cfg();
        if (hidden) *hidden = c.lang.hidden;
        if (vocab) *vocab = c.lang.vocab;
        if (eos) *eos = c.lang.eos;
        if (layers) *layers = c.lang.layers;
    });
}

dsocr_status dsocr_prepare_page(const uint8_t* rgb, uint32_t w, uint32_t h, const dsocr_vision_settings* vs,
                                dsocr_page_pixels** out) {
    return guarded([&] {
        if (!rgb || !vs || !out) throw std::runtime_error("EINVAL: NULL argument");
        std::unique_ptr<dsocr_page_pixels> p(new dsocr_page_pixels);  // released only on success
        dsocr::PagePixels& px = p->px;
        px.base = (int)vs->base_size;
        px.tile = (int)vs->image_size;
        px.crop = vs->crop_mode != 0;
        const int gsize = px.crop ? px.base : px.tile;  // model/mod.rs:1714
        std::vector<uint8_t> gview = dsocr::build_global_view(rgb, (int)w, (int)h, gsize);
        px.gsize = gsize;
        px.global_chw.resize((size_t)3 * gsize * gsize);
        dsocr::image_to_chw(gview.data(), gsize, gsize, px.global_chw.data());
        if (px.crop) {
            int gw = 1, gh = 1;
            auto tiles = dsocr::dynamic_preprocess(rgb, (int)w, (int)h, px.tile, 2, 9, &gw, &gh);
            px.crop_w = gw;
            px.crop_h = gh;
            px.n_tiles = (int)tiles.size();
            px.tiles_chw.resize((size_t)px.n_tiles * 3 * px.tile * px.tile);
            for (int i = 0; i < px.n_tiles; ++i)
                dsocr::image_to_chw(tiles[i].data(), px.tile, px.tile, px.tiles_chw.data() + (size_t)i * 3 * px.tile * px.tile);
        }
        px.n_image_tokens = dsocr::image_placeholder_count(px.base, px.tile, px.crop, px.crop_w, px.crop_h);
        *out = p.release();
    });
}

dsocr_status dsocr_prepare_page_device(dsocr_engine* e, const uint8_t* rgb, uint32_t w, uint32_t h,
                                       const dsocr_vision_settings* vs, dsocr_page_pixels** out) {
    return guarded([&] {
        if (!e || !rgb || !vs || !out) throw std::runtime_error("EINVAL: NULL argument");
        auto* p = new dsocr_page_pixels;
        p->px.base = (int)vs->base_size;
        p->px.tile = (int)vs->image_size;
        p->px.crop = vs->crop_mode != 0;
        try {
            e->impl->prepare_page_device(rgb, (int)w, (int)h, p->px);
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
    });
}

dsocr_status dsocr_page_read_device(const dsocr_page_pixels* p, float* global_out, float* tiles_out) {
    return guarded([&] {
        if (!p) throw std::runtime_error("EINVAL: NULL page");
        if (!p->px.global_dev) throw std::runtime_error("EINVAL: page has no device pixels");
        const size_t G = (size_t)p->px.gsize, T = (size_t)p->px.tile;
        check_hip(hipSetDevice(p->px.dev_ordinal), "hipSetDevice");
        if (global_out) check_hip(hipMemcpy(global_out, p->px.global_dev, 3 * G * G * 4, hipMemcpyDeviceToHost), "d2h");
        if (tiles_out && p->px.tiles_dev)
            check_hip(hipMemcpy(tiles_out, p->px.tiles_dev, (size_t)p->px.n_tiles * 3 * T * T * 4, hipMemcpyDeviceToHost), "d2h");
    });
}

void dsocr_page_free(dsocr_page_pixels* p) { delete p; }

dsocr_status dsocr_page_to_device(dsocr_engine* e, dsocr_page_pixels* p) {
    return guarded([&] {
        if (!e || !p) throw std::runtime_error("EINVAL: NULL argument");
        e->impl->upload_page(p->px);
    });
}

dsocr_status dsocr_page_info(const dsocr_page_pixels* p, uint32_t* cw, uint32_t* ch, uint32_t* nt, size_t* ntok) {
    return guarded([&] {
        if (!p) throw std::runtime_error("EINVAL: NULL page");
        if (cw) *cw = p->px.crop_w;
        if (ch) *ch = p->px.crop_h;
        if (nt) *nt = p->px.n_tiles;
        if (ntok) *ntok = p->px.n_image_tokens;
    });
}

dsocr_status dsocr_page_pixels_view(const dsocr_page_pixels* p, const float** g, uint32_t* gs, const float** t,
                                    uint32_t* ts) {
    return guarded([&] {
        if (!p) throw std::runtime_error("EINVAL: NULL page");
        if (g) *g = p->px.global_chw.empty() ? nullptr : p->px.global_chw.data();
        if (gs) *gs = p->px.gsize;
        if (t) *t = p->px.tiles_chw.empty() ? nullptr : p->px.tiles_chw.data();
        if (ts) *ts = p->px.tile;
    });
}

dsocr_status dsocr_image_embeddings(dsocr_engine* e, const dsocr_page_pixels* const* pages, size_t n, float* out,
                                    size_t cap_rows, size_t* rows_per_page) {
    return guarded([&] {
        if (!e || (!pages && n)) throw std::runtime_error("EINVAL: NULL argument");
        std::vector<const dsocr::PagePixels*> ps;
        for (size_t i = 0; i < n; ++i) {
            if (!pages[i]) throw std::runtime_error("EINVAL: page " + std::to_string(i) + " is NULL");
            ps.push_back(&pages[i]->px);
        }
        auto rows = e->impl->image_embeddings(ps);
        const size_t H = e->impl->cfg().lang.hidden;
        size_t off = 0;
        for (size_t i = 0; i < n; ++i) {
            const size_t r = rows[i].size() / H;
            if (rows_per_page) rows_per_page[i] = r;
            if (off + r > cap_rows) throw std::runtime_error("EINVAL: output capacity too small");
            if (out) std::memcpy(out + off * H, rows[i].data(), rows[i].size() * 4);
            off += r;
        }
    });
}

dsocr_status dsocr_generate(dsocr_engine* e, const dsocr_request* req, const dsocr_decode_params* params,
                            dsocr_stream_cb cb, void* user, int64_t* out_ids, size_t cap, size_t* n_out) {
    return guarded([&] {
        if (!e || !req || !out_ids || !n_out) throw std::runtime_error("EINVAL: NULL argument");
        std::vector<dsocr::GenRequest> reqs{to_request(*req)};
        auto r = e->impl->generate(reqs, to_params(params), cb, user);
        if (r[0].size() > cap) throw std::runtime_error("EINVAL: output capacity too small");
        std::memcpy(out_ids, r[0].data(), r[0].size() * sizeof(int64_t));
        *n_out = r[0].size();
    });
}

dsocr_status dsocr_generate_batch(dsocr_engine* e, size_t n, const dsocr_request* reqs,
                                  const dsocr_decode_params* params, dsocr_result* results) {
    return guarded([&] {
        if (!e || (!reqs && n) || (!results && n)) throw std::runtime_error("EINVAL: NULL argument");
        std::vector<dsocr::GenRequest> rq;
        for (size_t i = 0; i < n; ++i) rq.push_back(to_request(reqs[i]));
        auto r = e->impl->generate(rq, to_params(params), nullptr, nullptr);
        for (size_t i = 0; i < n; ++i) {
            results[i].status = DSOCR_OK;
            size_t m = std::min(r[i].size(), results[i].cap);
            if (results[i].out_ids) std::memcpy(results[i].out_ids, r[i].data(), m * sizeof(int64_t));
            results[i].n_out = m;
            if (m < r[i].size()) results[i].status = DSOCR_EINVAL;
        }
    });
}

dsocr_status dsocr_generate_trace(dsocr_engine* e, size_t n, const dsocr_request* reqs,
                                  const dsocr_decode_params* params, dsocr_result* results, float* logits_out,
                                  size_t logits_cap) {
    return guarded([&] {
        if (!e || (!reqs && n) || (!results && n) || !logits_out || !params) throw std::runtime_error("EINVAL: NULL argument");
        const size_t need = n * (size_t)params->max_new_tokens * e->impl->cfg().lang.vocab;
        if (need > logits_cap)
            throw std::runtime_error("EINVAL: logits_out holds " + std::to_string(logits_cap) + " floats, the trace needs " +
                                     std::to_string(need) + " (n * max_new_tokens * vocab)");
        std::vector<dsocr::GenRequest> rq;
        for (size_t i = 0; i < n; ++i) rq.push_back(to_request(reqs[i]));
        dsocr::GenParams g = to_params(params);
        g.trace = logits_out;
        auto r = e->impl->generate(rq, g, nullptr, nullptr);
        for (size_t i = 0; i < n; ++i) {
            results[i].status = DSOCR_OK;
            size_t m = std::min(r[i].size(), results[i].cap);
            if (results[i].out_ids) std::memcpy(results[i].out_ids, r[i].data(), m * sizeof(int64_t));
            results[i].n_out = m;
            if (m < r[i].size()) results[i].status = DSOCR_EINVAL;
        }
    });
}

dsocr_status dsocr_last_timings(const dsocr_engine* e, dsocr_timings* t) {
    return guarded([&] {
        if (!e || !t) throw std::runtime_error("EINVAL: NULL argument");
        dsocr::Timings x = e->impl->last_timings();
        t->vision_prepare_ms = x.vision_prepare_ms;
        t->vision_compute_ms = x.vision_compute_ms;
        t->decode_prefill_ms = x.prefill_ms;
        t->decode_iterative_ms = x.iterative_ms;
        t->decode_generate_ms = x.generate_ms;
        t->decode_steps = x.steps;
        t->pages = x.pages;
        t->vision_flops = x.vision_flops;
        t->prefill_flops = x.prefill_flops;
    });
}

dsocr_status dsocr_profile_decode(dsocr_engine* e, int iters, dsocr_decode_profile* out) {
    return guarded([&] {
        if (!e || iters <= 0 || !out) throw std::runtime_error("EINVAL: bad arguments");
        auto p = e->impl->profile_decode(iters);
        auto cp = [](const dsocr::Engine::KernelProfile& k) {
            dsocr_kernel_profile r;
            r.avg_us = k.avg_us; r.bytes = k.bytes; r.flops = k.flops; r.launches = k.launches; r.replay_us = k.replay_us;
            r.ctx_us = k.ctx_us;
            return r;
        };
        out->moe_gateup = cp(p.moe_gateup);
        out->moe_down = cp(p.moe_down);
        out->attention = cp(p.attention);
        out->lm_head = cp(p.lm_head);
        out->experts_touched = p.experts_touched;
        out->tokens = p.tokens;
        out->kv_len = p.kv_len;
        out->qkv = cp(p.qkv);
        out->o_proj = cp(p.o_proj);
        out->router = cp(p.router);
        out->layers_step = cp(p.layers_step);
        out->lm_head_screened = cp(p.lm_head_screened);
        out->moe_gateup_kernel = p.gateup_kernel;
        out->moe_down_kernel = p.down_kernel;
    });
}

// ---------------------------------------------------------------- device helpers
dsocr_status dsocr_engine_set_spans(dsocr_engine* e, int enable) {
    return guarded([&] {
        if (!e) throw std::runtime_error("EINVAL: NULL engine");
        e->impl->set_spans(enable);
    });
}

dsocr_status dsocr_engine_spans(const dsocr_engine* e, uint64_t* out, size_t cap, size_t* kinds, size_t* layers,
                                size_t* steps) {
    return guarded([&] {
        if (!e) throw std::runtime_error("EINVAL: NULL engine");
        const auto& v = e->impl->spans();
        const size_t nl = e->impl->cfg().lang.layers;
        const size_t ns = v.empty() ? 0 : (size_t)e->impl->span_steps();
        if (kinds) *kinds = (size_t)e->impl->span_kinds();
        if (layers) *layers = nl;
        if (steps) *steps = ns;
        if (!out) return;  // size query
        if (v.size() > cap)
            throw std::runtime_error("EINVAL: span buffer holds " + std::to_string(cap) + " values, " +
                                     std::to_string(v.size()) + " needed");
        if (!v.empty()) std::memcpy(out, v.data(), v.size() * 8);
    });
}
static_assert(dsocr::Engine::SPAN_FIELDS == 5, "dsocr.h documents 5 fields per span record");

dsocr_status dsocr_engine_set_persist_stamps(dsocr_engine* e, int mode) {
    return guarded([&] {
        if (!e) throw std::runtime_error("EINVAL: NULL engine");
        e->impl->set_persist_stamps(mode);
    });
}

dsocr_status dsocr_engine_persist_info(const dsocr_engine* e, int* used, double* durations, size_t cap_d,
                                       size_t* n_launches, uint64_t* stamps, size_t cap_s, size_t* n_stamps) {
    return guarded([&] {
        if (!e) throw std::runtime_error("EINVAL: NULL engine");
        const auto& d = e->impl->persist_launch_us();
        const auto& st = e->impl->persist_stamps();
        if (used) *used = e->impl->persist_used() ? 1 : 0;
        if (n_launches) *n_launches = d.size();
        if (n_stamps) *n_stamps = st.size();
        if (durations) {
            if (d.size() > cap_d) throw std::runtime_error("EINVAL: duration buffer too small");
            if (!d.empty()) std::memcpy(durations, d.data(), d.size() * sizeof(double));
        }
        if (stamps) {
            if (st.size() > cap_s) throw std::runtime_error("EINVAL: stamp buffer too small");
            if (!st.empty()) std::memcpy(stamps, st.data(), st.size() * 8);
        }
    });
}

dsocr_status dsocr_device_count(int* n) {
    return guarded([&] { check_hip(hipGetDeviceCount(n), "hipGetDeviceCount"); });
}
dsocr_status dsocr_dev_alloc(size_t bytes, void** ptr) {
    return guarded([&] {
        if (hipMalloc(ptr, bytes ? bytes : 16) != hipSuccess) throw std::runtime_error("ENOMEM: hipMalloc failed");
    });
}
dsocr_status dsocr_dev_free(void* ptr) {
    return guarded([&] { check_hip(hipFree(ptr), "hipFree"); });
}
dsocr_status dsocr_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    return guarded([&] { check_hip(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D"); });
}
dsocr_status dsocr_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    return guarded([&] { check_hip(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "hipMemcpy D2H"); });
}
dsocr_status dsocr_dev_sync(void) {
    return guarded([&] { check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize"); });
}
dsocr_status dsocr_synth_bf16(const char* name, uint64_t seed, uint64_t n, uint16_t* out) {
    return guarded([&] {
        if (!name || (!out && n)) throw std::runtime_error("EINVAL: NULL argument");
        dsocr::synth_bf16(name, seed, n, out);
    });
}
dsocr_status dsocr_resize_bicubic(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw, uint32_t dh) {
    return guarded([&] {
        if (!src || !dst) throw std::runtime_error("EINVAL: NULL argument");
        dsocr::resize_bicubic(src, (int)sw, (int)sh, dst, (int)dw, (int)dh);
    });
}

dsocr_status dsocr_resize_catmull_rom(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw,
                                      uint32_t dh) {
    return guarded([&] {
        if (!src || !dst || !sw || !sh || !dw || !dh) throw std::runtime_error("EINVAL: NULL argument or empty image");
        dsocr::resize_catmull_rom_fir(src, (int)sw, (int)sh, dst, (int)dw, (int)dh);
    });
}

// ---------------------------------------------------------------- kernel-level entry points
dsocr_status dsocr_k_gemm(int M, int N, int K, const float* A, const void* W, int wdtype, const float* bias, float* C,
                          int act, int accumulate) {
    return guarded([&] {
        if (K % 8) throw std::runtime_error("EINVAL: K must be a multiple of 8");
        dsocr::GemmArgs g;
        g.M = M; g.N = N; g.K = K; g.A = A; g.lda = K; g.W = W; g.ldw = K; g.wdtype = wdtype; g.bias = bias;
        g.C = C; g.ldc = N; g.act = act; g.accumulate = accumulate;
        dsocr::launch_gemm(g, nullptr);
        check_hip(hipGetLastError(), "gemm launch");
        check_hip(hipDeviceSynchronize(), "gemm");
    });
}
dsocr_status dsocr_k_gemm_grouped(int M, int N, int K, const float* A, int lda, const int* a_rows, const void* W,
                                  int wdtype, long long w_group_stride, const float* bias, long long bias_group_stride,
                                  float* C, int ldc, const int* c_rows, int act, int accumulate, const int* group_off,
                                  int groups, int max_group_rows, int kernel) {
    return guarded([&] {
        if (!A || !W || !C || !group_off || groups < 1 || M < 0 || N < 1 || K < 1)
            throw std::runtime_error("EINVAL: grouped gemm arguments");
        dsocr::GemmArgs g;
        g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.a_rows = a_rows; g.W = W; g.ldw = K; g.wdtype = wdtype;
        g.w_group_stride = (long)w_group_stride; g.bias = bias; g.bias_group_stride = (long)bias_group_stride;
        g.C = C; g.ldc = ldc; g.c_rows = c_rows; g.act = act; g.accumulate = accumulate;
        g.group_off = group_off; g.groups = groups; g.max_group_rows = max_group_rows;
        if (kernel == 1 || kernel == 2) dsocr::launch_gemm_f32a_grouped(g, nullptr, kernel == 2 ? 128 : 32);
        else dsocr::launch_gemm(g, nullptr);
        check_hip(hipGetLastError(), "grouped gemm launch");
        check_hip(hipDeviceSynchronize(), "grouped gemm");
    });
}
dsocr_status dsocr_k_gemm_f32a(int M, int N, int K, const float* A, const void* W, int wdtype, const float* bias,
                               float* C, int act, int accumulate, int splits) {
    return guarded([&] {
        if (wdtype != dsocr::WDT_BF16 && wdtype != dsocr::WDT_F16) throw std::runtime_error("EINVAL: weights must be bf16 or f16");
        dsocr::GemmBf16Args g;
        g.M = M; g.N = N; g.K = K; g.A = A; g.lda = K; g.W = W; g.ldw = K; g.bias = bias;
        g.w_f16 = wdtype == dsocr::WDT_F16;
        g.C = C; g.ldc = N; g.act = act; g.accumulate = accumulate;
        if (!dsocr::gemm_f32a_ok(g)) throw std::runtime_error("EINVAL: gemm_f32a needs K % 32 == 0 and 16-byte aligned rows");
        g.splits = splits > 0 ? splits : dsocr::gemm_f32a_splits(M, N, K);
        float* part = nullptr;
        if (g.splits > 1) {
            check_hip(hipMalloc(&part, sizeof(float) * (size_t)g.splits * M * N), "hipMalloc");
            g.part = part;
        }
        dsocr::launch_gemm_f32a(g, nullptr);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (part) (void)hipFree(part);
        check_hip(e, "gemm_f32a");
    });
}
dsocr_status dsocr_k_gemv(int M, int N, int K, const float* x, const float* norm_w, float eps, const void* W,
                          int wdtype, const float* bias, float* y, int act, int accumulate) {
    return guarded([&] {
        if (K % 8) throw std::runtime_error("EINVAL: K must be a multiple of 8");
        dsocr::DecGemvArgs a;
        a.M = M; a.N = N; a.K = K; a.x = x; a.ldx = K; a.W = W; a.ldw = K; a.wdtype = wdtype; a.bias = bias;
        a.y = y; a.ldy = N; a.act = act; a.accumulate = accumulate; a.norm_w = norm_w; a.eps = eps;
        dsocr::launch_dec_gemv(a, nullptr);
        check_hip(hipGetLastError(), "gemv launch");
        check_hip(hipDeviceSynchronize(), "gemv");
    });
}
dsocr_status dsocr_k_gemv_splitk(int M, int N, int K, const float* x, const void* W, int wdtype, const float* bias,
                                 float* y, int accumulate) {
    return guarded([&] {
        dsocr::DecGemvArgs a;
        a.M = M; a.N = N; a.K = K; a.x = x; a.ldx = K; a.W = W; a.ldw = K; a.wdtype = wdtype; a.bias = bias;
        a.y = y; a.ldy = N; a.accumulate = accumulate;
        if (!dsocr::dec_mm_splitk_ok(a)) throw std::runtime_error("EINVAL: gemv_splitk needs M <= 8, K % 64 == 0");
        float* part = nullptr;
        int* tick = nullptr;
        check_hip(hipMalloc(&part, sizeof(float) * dsocr::dec_mm_splitk_part_floats(N, K)), "hipMalloc");
        check_hip(hipMalloc(&tick, sizeof(int) * dsocr::dec_mm_splitk_ticks(N)), "hipMalloc");
        check_hip(hipMemset(tick, 0, sizeof(int) * dsocr::dec_mm_splitk_ticks(N)), "hipMemset");
        dsocr::launch_dec_mm_splitk(a, part, tick, nullptr);
        hipError_t e = hipDeviceSynchronize();
        (void)hipFree(part);
        (void)hipFree(tick);
        check_hip(e, "gemv_splitk");
    });
}
dsocr_status dsocr_k_layernorm(int rows, int cols, const float* x, const float* w, const float* b, float eps, float* y) {
    return guarded([&] {
        if (cols % 4) throw std::runtime_error("EINVAL: cols must be a multiple of 4");
        dsocr::launch_layernorm(x, cols, y, cols, nullptr, rows, cols, w, b, eps, nullptr);
        check_hip(hipDeviceSynchronize(), "layernorm");
    });
}
dsocr_status dsocr_k_dsq_dequant(int qtype, const void* src, size_t src_bytes, size_t out_dim, size_t in_dim,
                                 void* out_f16) {
    return guarded([&] {
        const size_t need = dsocr::dsq_payload_bytes(qtype, (long)out_dim, (long)in_dim);
        if (need == 0) throw std::runtime_error("EINVAL: unsupported snapshot tensor dtype code " + std::to_string(qtype));
        if (src_bytes != need)
            throw std::runtime_error("EINVAL: payload is " + std::to_string(src_bytes) + " bytes, expected " + std::to_string(need));
        dsocr::launch_dsq_dequant(qtype, src, (long)out_dim, (long)in_dim, out_f16, nullptr);
        check_hip(hipGetLastError(), "dsq_dequant launch");
        check_hip(hipDeviceSynchronize(), "dsq_dequant");
    });
}
dsocr_status dsocr_k_rmsnorm(int rows, int cols, const float* x, const float* w, float eps, float* y) {
    return guarded([&] {
        if (cols % 4) throw std::runtime_error("EINVAL: cols must be a multiple of 4");
        dsocr::launch_rmsnorm(x, cols, y, cols, rows, cols, w, eps, nullptr);
        check_hip(hipDeviceSynchronize(), "rmsnorm");
    });
}
dsocr_status dsocr_k_attention(int n_seq, int L, int heads, int hd, float scale, int causal, const float* q,
                               const float* k, const float* v, float* o, const float* relh, const float* relw, int gh,
                               int gw) {
    return guarded([&] {
        if (hd != 32 && hd != 64 && hd != 128) throw std::runtime_error("EINVAL: head_dim must be 32, 64 or 128");
        const long C = (long)heads * hd;
        dsocr::AttnArgs a;
        a.q = {q, C, hd, nullptr};
        a.k = {k, C, hd, nullptr};
        a.v = {v, C, hd, nullptr};
        a.o = o; a.o_row_stride = C; a.o_head_stride = hd; a.n_seq = n_seq; a.L = L; a.heads = heads;
        a.kv_heads = heads; a.hd = hd; a.scale = scale; a.causal = causal;
        float* rb = nullptr;
        float* part = nullptr;
        if (causal) {  // the engine's prefill form: key pieces + combine
            a.part_floats = dsocr::attention_causal_part_floats(n_seq, heads, L, hd);
            check_hip(hipMalloc(&part, sizeof(float) * a.part_floats), "hipMalloc attention pieces");
            a.part = part;
        }
        if (relh && relw) {
            if (gh * gw != L) throw std::runtime_error("EINVAL: rel-pos grid does not match L");
            check_hip(hipMalloc(&rb, sizeof(float) * (size_t)n_seq * heads * L * (gh + gw)), "hipMalloc relbias");
            dsocr::launch_sam_relbias(q, C, n_seq, gh, gw, heads, hd, relh, relw, rb, nullptr);
            a.relbias = rb; a.rel_h = gh; a.rel_w = gw;
        }
        dsocr::launch_attention(a, nullptr);
        hipError_t e = hipDeviceSynchronize();
        if (rb) (void)hipFree(rb);
        if (part) (void)hipFree(part);
        check_hip(e, "attention");
    });
}
dsocr_status dsocr_k_attention_bf16(int n_seq, int L, int heads, int hd, float scale, const void* qkv, long ld,
                                    void* o, long o_ld, int o_bf16) {
    return guarded([&] {
        if (!qkv || !o || n_seq <= 0 || L <= 0 || heads <= 0) throw std::runtime_error("EINVAL: bad attention arguments");
        const long D = (long)heads * hd;
        if (ld < 3 * D || o_ld < D) throw std::runtime_error("EINVAL: row strides too small");
        dsocr::AttnBf16Args a;
        a.q = (const uint16_t*)qkv; a.k = (const uint16_t*)qkv + D; a.v = (const uint16_t*)qkv + 2 * D;
        a.q_rs = a.k_rs = a.v_rs = ld; a.q_hs = a.k_hs = a.v_hs = hd;
        a.o = o; a.o_rs = o_ld; a.o_hs = hd; a.o_bf16 = o_bf16;
        a.n_seq = n_seq; a.L = L; a.heads = heads; a.kv_heads = heads; a.hd = hd; a.scale = scale;
        const char* pv = getenv("DSOCR_DOTS_PV_PLANES");  // the tower's P.V plane count (3 unless set to 2)
        a.pv_planes = (pv && atoi(pv) == 2) ? 2 : 3;
        dsocr::launch_attention_bf16(a, nullptr);
        check_hip(hipGetLastError(), "attention_bf16 launch");
        check_hip(hipDeviceSynchronize(), "attention_bf16");
    });
}
dsocr_status dsocr_k_decode_attention(int B, int heads, int kv_heads, int hd, int rope_dim, int max_len, float scale,
                                      const float* qkv, const float* cos, const float* sin, float* kc, float* vc,
                                      const int* kv_pos, float* o, int prerot) {
    return guarded([&] {
        if (hd != 32 && hd != 64 && hd != 128) throw std::runtime_error("EINVAL: head_dim must be 32, 64 or 128");
        if (prerot && rope_dim != hd) throw std::runtime_error("EINVAL: pre-rotated rows need rope_dim == head_dim");
        if (kv_heads <= 0 || heads % kv_heads || rope_dim > hd || rope_dim % 2)
            throw std::runtime_error("EINVAL: bad head / rope configuration");
        float* part = nullptr;
        int* cnt = nullptr;
        const size_t pb = dsocr::dec_attn_workspace(B, heads, hd, max_len);
        check_hip(hipMalloc(&part, pb), "hipMalloc");
        check_hip(hipMalloc(&cnt, sizeof(int) * (B * heads + 1)), "hipMalloc");
        check_hip(hipMemset(cnt, 0, sizeof(int) * (B * heads + 1)), "hipMemset");
        dsocr::dec_attn_part_init(part, pb, nullptr);
        dsocr::DecAttn2Args a;
        a.qkv = qkv; a.ld = (long)(heads + 2 * kv_heads) * hd; a.kv_pos = kv_pos; a.B = B; a.heads = heads;
        a.kv_heads = kv_heads; a.hd = hd; a.rope_dim = rope_dim; a.use_mla = 0; a.max_len = max_len;
        a.cos = cos; a.sin = sin; a.kc = kc; a.vc = vc; a.head_stride = (long)max_len * hd;
        a.page_stride = (long)kv_heads * max_len * hd; a.scale = scale; a.part = part; a.o = o;
        a.o_ld = (long)heads * hd; a.counters = cnt; a.err = cnt + B * heads;
        a.prerot = prerot != 0;
        dsocr::launch_dec_attn(a, nullptr);
        hipError_t e = hipDeviceSynchronize();
        int herr = 0;
        if (e == hipSuccess) e = hipMemcpy(&herr, a.err, sizeof(int), hipMemcpyDeviceToHost);
        (void)hipFree(part);
        (void)hipFree(cnt);
        check_hip(e, "decode attention");
        if (herr) throw std::runtime_error("EINTERNAL: decode attention merge timed out");
    });
}
dsocr_status dsocr_k_qkv_attention(int fused, int steps, int H, int heads, int hd, int max_len, float scale,
                                   float eps, const float* x, const float* norm_w, const void* Wqkv, int wdtype,
                                   const float* cos, const float* sin, float* kc, float* vc, const int* kv_pos,
                                   float* qkv_row, float* o, int* used_fused) {
    return guarded([&] {
        if (steps <= 0 || H <= 0 || heads <= 0 || hd != 128 || heads * hd != H)
            throw std::runtime_error("EINVAL: qkv_attention needs 128-dim MHA heads with heads * hd == H");
        if (wdtype != dsocr::WDT_F16 && wdtype != dsocr::WDT_BF16) throw std::runtime_error("EINVAL: 16-bit weights only");
        const int QKVN = 3 * H;
        {  // range check once, before anything is allocated (it does not depend on the step)
            dsocr::DecGemvArgs g;
            g.M = 1; g.N = QKVN; g.K = H; g.W = Wqkv; g.ldw = H; g.wdtype = wdtype; g.y = qkv_row; g.ldy = QKVN;
            g.x = x; g.ldx = H; g.norm_w = norm_w; g.eps = eps;
            dsocr::DecRopeEpi re;
            re.kv_pos = kv_pos; re.cos = cos; re.sin = sin; re.hd = hd; re.rot_rows = 2 * H;
            if (!dsocr::dec_qkv_rope_ok(g, re)) throw std::runtime_error("EINVAL: q/k/v projection outside dec_qkv_rope's range");
        }
        float* part = nullptr;
        int* cnt = nullptr;
        const size_t pb = dsocr::dec_attn_workspace(1, heads, hd, max_len);
        check_hip(hipMalloc(&part, pb), "hipMalloc");
        check_hip(hipMalloc(&cnt, sizeof(int) * (heads + 1)), "hipMalloc");
        check_hip(hipMemset(cnt, 0, sizeof(int) * (heads + 1)), "hipMemset");
        dsocr::dec_attn_part_init(part, pb, nullptr);
        bool took = false;
        for (int s = 0; s < steps; ++s) {
            dsocr::DecGemvArgs g;
            g.M = 1; g.N = QKVN; g.K = H; g.W = Wqkv; g.ldw = H; g.wdtype = wdtype; g.y = qkv_row; g.ldy = QKVN;
            g.x = x + (size_t)s * H; g.ldx = H; g.norm_w = norm_w; g.eps = eps;
            dsocr::DecRopeEpi re;
            re.kv_pos = kv_pos + s; re.cos = cos; re.sin = sin; re.hd = hd; re.rot_rows = 2 * H;
            dsocr::DecAttn2Args a;
            a.qkv = qkv_row; a.ld = QKVN; a.kv_pos = kv_pos + s; a.B = 1; a.heads = heads; a.kv_heads = heads;
            a.hd = hd; a.rope_dim = hd; a.use_mla = 0; a.max_len = max_len; a.cos = cos; a.sin = sin;
            a.kc = kc; a.vc = vc; a.head_stride = (long)max_len * hd; a.page_stride = (long)heads * max_len * hd;
            a.scale = scale; a.part = part; a.o = o + (size_t)s * H; a.o_ld = H; a.counters = cnt; a.err = cnt + heads;
            a.prerot = 1;
            if (fused && dsocr::dec_qkv_attn_ok(g, re, a)) {
                dsocr::launch_dec_qkv_attn(g, re, a, nullptr);
                took = true;
            } else {
                dsocr::launch_dec_qkv_rope(g, re, nullptr);
                dsocr::launch_dec_attn(a, nullptr);
            }
        }
        hipError_t e = hipDeviceSynchronize();
        int herr = 0;
        if (e == hipSuccess) e = hipMemcpy(&herr, cnt + heads, sizeof(int), hipMemcpyDeviceToHost);
        (void)hipFree(part);
        (void)hipFree(cnt);
        check_hip(e, "qkv_attention");
        if (herr) throw std::runtime_error("EINTERNAL: q/k/v hand-off or attention merge timed out");
        if (used_fused) *used_fused = took ? 1 : 0;
    });
}
int dsocr_k_poll_wait_fits(long waiting_blocks, int api_blocks_per_cu, int cus) {
    return dsocr::poll_wait_fits(waiting_blocks, api_blocks_per_cu, cus) ? 1 : 0;
}
dsocr_status dsocr_k_moe(int T, int H, int E, int topk, int I, int Is, const float* x, const float* norm_w,
                         float eps, const void* router, const void* Wgu, const void* Wd, const void* sWgu,
                         const void* sWd, int wdtype, int norm_topk, float scaling, float* out, int* ids_out,
                         float* w_out) {
    return guarded([&] {
        if (T <= 0 || H <= 0 || E <= 0 || topk <= 0 || I <= 0) throw std::runtime_error("EINVAL: bad MoE shape");
        std::vector<void*> bufs;
        auto alloc = [&](size_t b) {
            void* p = nullptr;
            check_hip(hipMalloc(&p, b ? b : 16), "hipMalloc");
            bufs.push_back(p);
            return p;
        };
        try {
            const int TK = T * topk;
            // the engine's own dispatch (Engine::decode_step -> launch_moe_decode): mix kernels at one
            // token, slot kernels at two, the grouped (expert-deduplicated) kernels at 3..8, sorted groups above
            dsocr::MoeDecodeArgs a;
            a.T = T; a.H = H; a.E = E; a.topk = topk; a.I = I;
            a.x = x; a.norm_w = norm_w; a.eps = eps; a.out = out;
            a.router = router; a.router_wdt = wdtype; a.Wgu = Wgu; a.Wd = Wd; a.wdtype = wdtype;
            if (sWgu && sWd && Is > 0) {
                a.Is = Is; a.sWgu = sWgu; a.sWd = sWd; a.hs = (float*)alloc(sizeof(float) * (size_t)T * Is);
            }
            a.softmax_scoring = 1; a.norm_topk = norm_topk; a.scaling = scaling;
            a.xn = (float*)alloc(sizeof(float) * (size_t)T * H);
            a.xn_router = (float*)alloc(sizeof(float) * (size_t)T * H);
            a.logits = (float*)alloc(sizeof(float) * (size_t)T * E);
            a.ids = (int*)alloc(sizeof(int) * TK);
            a.wts = (float*)alloc(sizeof(float) * TK);
            a.h = (float*)alloc(sizeof(float) * (size_t)TK * I);
            a.grp = (int*)alloc(sizeof(int) * dsocr::moe_grp_ints(E, T, topk));
            a.route_cnt = (int*)alloc(sizeof(int) * 16);
            check_hip(hipMemset(a.route_cnt, 0, sizeof(int) * 16), "hipMemset");
            if (wdtype == 1 && H % 32 == 0 && I % 32 == 0 && T <= 8) {
                // fragment-ordered expert copies, as Engine::ensure_mm_weights keeps them
                a.Wgu_swz = alloc(sizeof(uint16_t) * dsocr::mm_swizzle_elems(E * 2 * I, H));
                dsocr::launch_mm_swizzle(Wgu, E * 2 * I, H, const_cast<void*>(a.Wgu_swz), nullptr);
                a.Wd_swz = alloc(sizeof(uint16_t) * dsocr::mm_swizzle_elems(E * H, I));
                dsocr::launch_mm_swizzle(Wd, E * H, I, const_cast<void*>(a.Wd_swz), nullptr);
                if (a.Is > 0 && a.Is % 32 == 0) {
                    a.sWgu_swz = alloc(sizeof(uint16_t) * dsocr::mm_swizzle_elems(2 * a.Is, H));
                    dsocr::launch_mm_swizzle(sWgu, 2 * a.Is, H, const_cast<void*>(a.sWgu_swz), nullptr);
                    a.sWd_swz = alloc(sizeof(uint16_t) * dsocr::mm_swizzle_elems(H, a.Is));
                    dsocr::launch_mm_swizzle(sWd, H, a.Is, const_cast<void*>(a.sWd_swz), nullptr);
                }
            }
            if (T >= 3 && T <= 8) {
                a.dn_part = (float*)alloc(sizeof(float) * dsocr::moe_down_mm_part_floats(E, T, topk, I, a.Is, H));
                a.dn_tick = (int*)alloc(sizeof(int) * (H / 64 + 1));
                check_hip(hipMemset(a.dn_tick, 0, sizeof(int) * (H / 64 + 1)), "hipMemset");
            }
            if (T > 8) {
                a.eoff = (int*)alloc(sizeof(int) * (E + 1)); a.arow = (int*)alloc(sizeof(int) * TK);
                a.apos = (int*)alloc(sizeof(int) * TK); a.active = (int*)alloc(sizeof(int) * E);
                a.aw = (float*)alloc(sizeof(float) * TK); a.n_active = (int*)alloc(sizeof(int));
            }
            dsocr::launch_moe_decode(a, nullptr);
            check_hip(hipGetLastError(), "moe launch");
            check_hip(hipDeviceSynchronize(), "moe");
            if (ids_out) check_hip(hipMemcpy(ids_out, a.ids, sizeof(int) * TK, hipMemcpyDeviceToHost), "d2h");
            if (w_out) check_hip(hipMemcpy(w_out, a.wts, sizeof(float) * TK, hipMemcpyDeviceToHost), "d2h");
        } catch (...) {
            for (void* p : bufs) (void)hipFree(p);
            throw;
        }
        for (void* p : bufs) (void)hipFree(p);
    });
}
dsocr_status dsocr_k_moe_kernels(int T, int H, int E, int topk, int I, int Is, int has_norm, const char** gateup,
                                 const char** down) {
    return guarded([&] {
        dsocr::MoeDecodeArgs a;
        a.T = T; a.H = H; a.E = E; a.topk = topk; a.I = I; a.Is = Is;
        int dummy = 0;
        float fd = 0.f;
        a.x = &fd; a.out = &fd; a.norm_w = has_norm ? &fd : nullptr;
        if (Is > 0) { a.sWgu = &dummy; a.sWd = &dummy; a.hs = &fd; }
        a.xn = a.xn_router = a.logits = a.wts = a.h = &fd;
        a.ids = a.grp = a.route_cnt = &dummy;
        if (T >= 3 && T <= 8) { a.dn_part = &fd; a.dn_tick = &dummy; }
        // the engine keeps fragment-ordered expert copies (Engine::ensure_mm_weights)
        a.Wgu_swz = a.Wd_swz = &dummy;
        if (Is > 0) a.sWgu_swz = a.sWd_swz = &dummy;
        if (T > 8) { a.eoff = a.arow = a.apos = a.active = a.n_active = &dummy; a.aw = &fd; }
        dsocr::moe_decode_kernel_names(a, gateup, down);
    });
}
dsocr_status dsocr_k_lmhead_screened(int B, int V, int K, const float* x, const float* norm_w, float eps,
                                     const void* W, const int* ban, int ban_ld, int* out_tok) {
    return guarded([&] {
        if (B <= 0 || V <= 0 || K % 16 || K > 1536 || !x || !norm_w || !W || !out_tok)
            throw std::runtime_error("EINVAL: screened lm_head needs B, V > 0, K % 16 == 0, K <= 1536, x / norm / W / out");
        if (ban && ban_ld < 2) throw std::runtime_error("EINVAL: ban list stride < 2");
        std::vector<void*> bufs;
        auto alloc = [&](size_t b) {
            void* p = nullptr;
            check_hip(hipMalloc(&p, b ? b : 16), "hipMalloc");
            bufs.push_back(p);
            return p;
        };
        try {
            // the engine's load-time quantisation and its per-step launches (Engine::decode_head)
            // (B = 3..8: the one-stream matrix-core form, as the engine runs it at 3..8 pages)
            const bool mm = B >= 3 && dsocr::lmhead_q8mm_ok(B, V, K);
            if (B > 2 && !mm) throw std::runtime_error("EINVAL: screened lm_head for 3..8 rows needs K in {768, 1024, 1280, 1536}");
            const size_t vp = (size_t)(V + 15) / 16 * 16;
            void* q = alloc((size_t)V * K);
            float* scale = (float*)alloc(sizeof(float) * vp);
            float* bound = (float*)alloc(sizeof(float) * vp);
            float* qnorm = mm ? (float*)alloc(sizeof(float) * vp) : nullptr;
            void* qfrag = mm ? alloc(dsocr::lmhead_qfrag_bytes(V, K)) : nullptr;
            check_hip(hipMemset(scale, 0, sizeof(float) * vp), "hipMemset");
            check_hip(hipMemset(bound, 0, sizeof(float) * vp), "hipMemset");
            if (qnorm) check_hip(hipMemset(qnorm, 0, sizeof(float) * vp), "hipMemset");
            dsocr::launch_lmhead_quantize(W, V, K, q, scale, bound, nullptr, qnorm, qfrag);
            dsocr::LmHeadQ8Args a;
            a.x = x; a.ldx = K; a.norm_w = norm_w; a.eps = eps; a.q = q; a.scale = scale; a.bound = bound;
            a.B = B; a.N = V; a.K = K; a.ban = ban; a.ban_ld = ban ? ban_ld : 0;
            a.qfrag = qfrag; a.qnorm = qnorm;
            if (mm) dsocr::lmhead_q8mm_grid(V, K, B, &a.nblk, &a.slot);
            else dsocr::lmhead_q8_grid(V, K, B, &a.nblk, &a.slot);
            a.blk_cnt = (int*)alloc(sizeof(int) * B * a.nblk);
            a.blk_t = (float*)alloc(sizeof(float) * B * a.nblk);
            a.cand = (int*)alloc(sizeof(int) * B * a.nblk * a.slot);
            a.cand_hi = (float*)alloc(sizeof(float) * B * a.nblk * a.slot);
            a.xn_out = (float*)alloc(sizeof(float) * B * K);
            dsocr::launch_lmhead_q8(a, nullptr);
            dsocr::DecSampleArgs ss;  // selection only: empty contexts, no bookkeeping
            ss.B = B; ss.V = V; ss.ld = V; ss.ctx = (int*)alloc(sizeof(int) * 64); ss.ctx_cap = 64;
            ss.ctx_len = (int*)alloc(sizeof(int) * B); ss.ngram = 0; ss.out_tok = out_tok;
            check_hip(hipMemset(ss.ctx_len, 0, sizeof(int) * B), "hipMemset");
            ss.blk_cnt = a.blk_cnt; ss.blk_t = a.blk_t; ss.cand = a.cand; ss.cand_hi = a.cand_hi; ss.nblk = a.nblk;
            ss.slot = a.slot; ss.w_exact = W; ss.xn = a.xn_out; ss.K = K;
            dsocr::launch_dec_sample(ss, nullptr);
            check_hip(hipGetLastError(), "screened lm_head launch");
            check_hip(hipDeviceSynchronize(), "screened lm_head");
        } catch (...) {
            for (void* p : bufs) (void)hipFree(p);
            throw;
        }
        for (void* p : bufs) (void)hipFree(p);
    });
}
dsocr_status dsocr_k_sample_greedy(int B, int V, float* logits, const int* ctx, int ctx_cap, const int* ctx_len,
                                   int ngram, float rep_penalty, int* out_tok) {
    return guarded([&] {
        const int rb = (int)dsocr::dec_sample_blocks(V);
        int *ridx, *done;
        float* rval;
        check_hip(hipMalloc(&ridx, sizeof(int) * B * rb), "hipMalloc");
        check_hip(hipMalloc(&rval, sizeof(float) * B * rb), "hipMalloc");
        check_hip(hipMalloc(&done, sizeof(int) * B), "hipMalloc");
        check_hip(hipMemset(done, 0, sizeof(int) * B), "hipMemset");
        dsocr::SampleArgs p;
        p.logits = logits; p.B = B; p.V = V; p.ld = V; p.ctx = ctx; p.ctx_cap = ctx_cap; p.ctx_len = ctx_len;
        p.rep_penalty = rep_penalty;
        dsocr::launch_rep_penalty(p, nullptr);
        dsocr::DecSampleArgs a;  // selection only: no bookkeeping buffers
        a.logits = logits; a.B = B; a.V = V; a.ld = V; a.ctx = const_cast<int*>(ctx); a.ctx_cap = ctx_cap;
        a.ctx_len = const_cast<int*>(ctx_len); a.ngram = ngram; a.red_val = rval; a.red_idx = ridx;
        a.out_tok = out_tok; a.done = done;
        dsocr::launch_dec_sample(a, nullptr);
        hipError_t e = hipDeviceSynchronize();
        (void)hipFree(ridx); (void)hipFree(rval); (void)hipFree(done);
        check_hip(e, "sample");
    });
}

dsocr_status dsocr_k_sample_stoch(int B, int V, float* logits, const int* ctx, int ctx_cap, const int* ctx_len,
                                  int ngram, float rep_penalty, double temperature, size_t top_k, double top_p,
                                  uint64_t seed, int draws, int* out_tok) {
    return guarded([&] {
        if (B <= 0 || V <= 0 || draws <= 0 || !(temperature > 0.0)) throw std::runtime_error("EINVAL: bad sampling arguments");
        const int rb = (int)dsocr::dec_sample_blocks(V);
        std::vector<void*> bufs;
        auto dalloc = [&](size_t bytes) {
            void* p = nullptr;
            check_hip(hipMalloc(&p, bytes), "hipMalloc");
            bufs.push_back(p);
            return p;
        };
        try {
            int* ridx = (int*)dalloc(sizeof(int) * B * rb);
            float* rval = (float*)dalloc(sizeof(float) * B * rb);
            int* done = (int*)dalloc(sizeof(int) * B);
            check_hip(hipMemset(done, 0, sizeof(int) * B), "hipMemset");
            dsocr::SampleArgs p;
            p.logits = logits; p.B = B; p.V = V; p.ld = V; p.ctx = ctx; p.ctx_cap = ctx_cap; p.ctx_len = ctx_len;
            p.rep_penalty = rep_penalty;
            dsocr::launch_rep_penalty(p, nullptr);
            dsocr::DecSampleArgs a;
            a.logits = logits; a.B = B; a.V = V; a.ld = V; a.ctx = const_cast<int*>(ctx); a.ctx_cap = ctx_cap;
            a.ctx_len = const_cast<int*>(ctx_len); a.ngram = ngram; a.red_val = rval; a.red_idx = ridx; a.done = done;
            a.do_sample = 1; a.temperature = temperature; a.top_k = (long)top_k; a.top_p = top_p; a.st_ld = V;
            a.st_key = (uint32_t*)dalloc(sizeof(uint32_t) * 2 * (size_t)B * V);
            a.st_idx = (int*)dalloc(sizeof(int) * 2 * (size_t)B * V);
            a.st_w = (double*)dalloc(sizeof(double) * (size_t)B * V);
            const std::vector<uint32_t> st = dsocr::rng_state_from_u64(seed);
            a.rng = (uint32_t*)dalloc(sizeof(uint32_t) * dsocr::RNG_WORDS * B);
            for (int b = 0; b < B; ++b)
                check_hip(hipMemcpy(a.rng + (size_t)b * dsocr::RNG_WORDS, st.data(), sizeof(uint32_t) * dsocr::RNG_WORDS,
                                    hipMemcpyHostToDevice), "hipMemcpy");
            const bool stamps = getenv("DSOCR_SAMPLE_STAMPS") != nullptr;  // diagnostics: phase clocks to stderr
            if (stamps) {
                a.st_stamps = (unsigned long long*)dalloc(sizeof(unsigned long long) * 8);
                check_hip(hipMemset(a.st_stamps, 0, sizeof(unsigned long long) * 8), "hipMemset");
            }
            for (int d = 0; d < draws; ++d) {
                a.out_tok = out_tok + (size_t)d * B;
                dsocr::launch_dec_sample(a, nullptr);
            }
            check_hip(hipDeviceSynchronize(), "sample");
            if (stamps) {
                unsigned long long h[8];
                check_hip(hipMemcpy(h, a.st_stamps, sizeof(h), hipMemcpyDeviceToHost), "hipMemcpy");
                fprintf(stderr, "[sample stamps] phase clocks (shader cycles) from start:");
                for (int i = 1; i < 8; ++i) fprintf(stderr, " %lld", h[i] ? (long long)(h[i] - h[0]) : -1LL);
                fprintf(stderr, "\n");
            }
        } catch (...) {
            for (void* q : bufs) (void)hipFree(q);
            throw;
        }
        for (void* q : bufs) (void)hipFree(q);
    });
}

// ---------------------------------------------------------------- dots.ocr vision tower
dsocr_status dsocr_dots_load(const char* config_path, const char* weights_path, uint64_t seed, int device,
                             dsocr_dots** out) {
    return guarded([&] {
        if (!config_path || !out) throw std::runtime_error("EINVAL: NULL argument");
        std::unique_ptr<dsocr_dots> d(new dsocr_dots);
        d->impl.reset(new dsocr::DotsVision(config_path, weights_path ? weights_path : "", seed, device));
        *out = d.release();
    });
}
void dsocr_dots_free(dsocr_dots* d) { delete d; }
dsocr_status dsocr_dots_info(const dsocr_dots* d, size_t* hidden, size_t* embed, size_t* layers, size_t* patch_dim) {
    return guarded([&] {
        if (!d) throw std::runtime_error("EINVAL: NULL handle");
        const dsocr::DotsConfig& c = d->impl->cfg();
        if (hidden) *hidden = c.hidden;
        if (embed) *embed = c.embed;
        if (layers) *layers = c.layers;
        if (patch_dim) *patch_dim = (size_t)c.channels * c.patch * c.patch;
    });
}
dsocr_status dsocr_dots_preprocess(const char* config_path, const uint8_t* rgb, uint32_t w, uint32_t h, float* patches,
                                   size_t cap, size_t* n_patches, uint32_t* grid) {
    return guarded([&] {
        if (!config_path || !rgb || !n_patches) throw std::runtime_error("EINVAL: NULL argument");
        std::ifstream f(config_path);
        if (!f) throw std::runtime_error(std::string("ENOENT: cannot read config ") + config_path);
        std::stringstream ss;
        ss << f.rdbuf();
        const dsocr::DotsConfig c = dsocr::parse_dots_config(dsocr::Json::parse(ss.str()));
        const dsocr::DotsPatches p = dsocr::dots_preprocess(c, rgb, (int)w, (int)h);
        const size_t n = (size_t)p.grid_t * p.grid_h * p.grid_w;
        *n_patches = n;
        if (grid) { grid[0] = p.grid_t; grid[1] = p.grid_h; grid[2] = p.grid_w; }
        if (patches) {
            if (n > cap) throw std::runtime_error("EINVAL: patch capacity too small");
            std::memcpy(patches, p.data.data(), p.data.size() * 4);
        }
    });
}
dsocr_status dsocr_dots_embed(dsocr_dots* d, const uint8_t* rgb, uint32_t w, uint32_t h, float* out, size_t cap_rows,
                              size_t* n_rows, uint32_t* grid) {
    return guarded([&] {
        if (!d || !rgb || !n_rows) throw std::runtime_error("EINVAL: NULL argument");
        const dsocr::DotsConfig& c = d->impl->cfg();
        const dsocr::DotsPatches p = dsocr::dots_preprocess(c, rgb, (int)w, (int)h);
        const size_t groups = (size_t)p.grid_t * p.grid_h * p.grid_w / (c.merge * c.merge);
        *n_rows = groups;
        if (grid) { grid[0] = p.grid_t; grid[1] = p.grid_h; grid[2] = p.grid_w; }
        if (groups > cap_rows) throw std::runtime_error("EINVAL: output capacity too small");
        std::vector<float> r = d->impl->embed(p);
        if (out) std::memcpy(out, r.data(), r.size() * 4);
    });
}
dsocr_status dsocr_dots_embed_device(dsocr_dots* d, const float* patches, uint32_t gt, uint32_t gh, uint32_t gw,
                                     float* out, int time_attention_layers) {
    return guarded([&] {
        if (!d || !patches || !out || !gt || !gh || !gw) throw std::runtime_error("EINVAL: bad arguments");
        d->impl->time_layers = std::max(0, time_attention_layers);
        d->impl->embed_device(patches, (int)gt, (int)gh, (int)gw, out);
        d->impl->time_layers = 0;
    });
}
dsocr_status dsocr_dots_last_timings(const dsocr_dots* d, dsocr_dots_timings* t) {
    return guarded([&] {
        if (!d || !t) throw std::runtime_error("EINVAL: NULL argument");
        const dsocr::DotsTimings x = d->impl->last_timings();
        t->total_ms = x.total_ms; t->patch_ms = x.patch_ms; t->blocks_ms = x.blocks_ms;
        t->attention_ms = x.attention_ms; t->merger_ms = x.merger_ms; t->tokens = x.tokens; t->groups = x.groups;
    });
}

}  // extern "C"
