// DeepSeek-OCR page engine (host orchestration of the gfx950 kernels).
// Reference call stacks followed here: SURVEY §3.2-3.4; per-stage citations inline.
#include "engine.hpp"

#include <algorithm>
#include <chrono>
#include <random>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>

#include "../common/host_util.hpp"
#include "dsq.hpp"
#include "host_ops.hpp"

namespace dsocr {

// ============================================================================ weight source
namespace {

struct HostMat {
    std::vector<uint16_t> data;
    int dt = WDT_BF16;
};

struct Source {
    std::unique_ptr<SafeTensors> st;
    uint64_t seed = 0;
    bool synth = false;
    int mode = 1;  // dsocr_dtype: 0 f32, 1 f16, 2 bf16
    // .dsq snapshot (crates/dsq-runtime): its records replace the checkpoint's linears, decoded to
    // fp16 on the GPU (dequant); a snapshot linear's bias comes from its record only, as
    // SnapshotLinear::{Quantized, Float} carries it (dsq-runtime/src/lib.rs:336-366)
    const DsqFile* snap = nullptr;
    std::function<void(const DsqRecord&, uint16_t*)> dequant;

    const DsqRecord* snap_weight_of_bias(const std::string& n) const {
        if (!snap || n.size() < 5 || n.compare(n.size() - 5, 5, ".bias") != 0) return nullptr;
        return snap->find(n.substr(0, n.size() - 5) + ".weight");
    }
    bool has(const std::string& n) const {
        if (snap) {
            if (snap->find(n)) return true;
            if (const DsqRecord* r = snap_weight_of_bias(n)) return r->has_bias;
        }
        return synth ? synth_has(n) : st->has(n);
    }

    static bool is_language(const std::string& n) {
        return n.rfind("model.layers.", 0) == 0 || n.rfind("model.embed_tokens.", 0) == 0;
    }
    bool round16(const std::string& n) const { return mode == 1 && is_language(n); }

    // exact f32 values (with the f16 rounding rule applied)
    std::vector<float> f32(const std::string& n, size_t numel) const {
        if (const DsqRecord* r = snap_weight_of_bias(n)) {
            std::vector<float> b = snap->bias(*r);
            if (b.size() != numel)
                throw std::runtime_error("EINVAL: snapshot bias for `" + r->name + "` has " + std::to_string(b.size()) +
                                         " values, expected " + std::to_string(numel));
            return b;
        }
        std::vector<float> out(numel);
        if (synth) {
            std::vector<uint16_t> b(numel);
            synth_bf16(n, seed, numel, b.data());
            for (size_t i = 0; i < numel; ++i) out[i] = bf16_to_f32(b[i]);
        } else {
            const StTensor& t = st->get(n);
            if ((size_t)t.numel() != numel)
                throw std::runtime_error("EINVAL: shape mismatch for `" + n + "`: " + std::to_string(t.numel()) +
                                         " vs expected " + std::to_string(numel));
            if (t.dtype == "BF16") {
                const uint16_t* p = (const uint16_t*)t.data;
                for (size_t i = 0; i < numel; ++i) out[i] = bf16_to_f32(p[i]);
            } else if (t.dtype == "F16") {
                const uint16_t* p = (const uint16_t*)t.data;
                for (size_t i = 0; i < numel; ++i) out[i] = f16_to_f32(p[i]);
            } else if (t.dtype == "F32") {
                std::memcpy(out.data(), t.data, numel * 4);
            } else {
                throw std::runtime_error("EINVAL: unsupported dtype " + t.dtype + " for `" + n + "`");
            }
        }
        if (round16(n))
            for (auto& v : out) v = f16_to_f32(f32_to_f16_rne(v));
        return out;
    }

    // 16-bit storage: f16 for language tensors in f16 mode (bf16 -> f16 RNE, the
    // reference's VarBuilder F16 load), otherwise the checkpoint's own 16-bit type.
    // out_dim / in_dim (when known) are checked against a snapshot record (dsq-runtime/src/lib.rs:326-334)
    HostMat h16(const std::string& n, size_t numel, long out_dim = -1, long in_dim = -1) const {
        HostMat m;
        m.data.resize(numel);
        if (const DsqRecord* r = snap ? snap->find(n) : nullptr) {
            if ((size_t)r->out_dim * r->in_dim != numel || (out_dim >= 0 && (long)r->out_dim != out_dim) ||
                (in_dim >= 0 && (long)r->in_dim != in_dim))
                throw std::runtime_error("EINVAL: snapshot tensor `" + n + "` dims mismatch (" + std::to_string(r->out_dim) +
                                         "x" + std::to_string(r->in_dim) + " for " + std::to_string(numel) + " values)");
            dequant(*r, m.data.data());
            m.dt = WDT_F16;
            return m;
        }
        const bool to_f16 = round16(n);
        if (synth) {
            synth_bf16(n, seed, numel, m.data.data());
            if (to_f16) {
#pragma omp parallel for schedule(static)
                for (long i = 0; i < (long)numel; ++i) m.data[i] = f32_to_f16_rne(bf16_to_f32(m.data[i]));
                m.dt = WDT_F16;
            } else {
                m.dt = WDT_BF16;
            }
            return m;
        }
        const StTensor& t = st->get(n);
        if ((size_t)t.numel() != numel)
            throw std::runtime_error("EINVAL: shape mismatch for `" + n + "`: " + std::to_string(t.numel()) +
                                     " vs expected " + std::to_string(numel));
        const uint16_t* p = (const uint16_t*)t.data;
        if (t.dtype == "BF16") {
            if (to_f16) {
#pragma omp parallel for schedule(static)
                for (long i = 0; i < (long)numel; ++i) m.data[i] = f32_to_f16_rne(bf16_to_f32(p[i]));
                m.dt = WDT_F16;
            } else {
                std::memcpy(m.data.data(), p, numel * 2);
                m.dt = WDT_BF16;
            }
        } else if (t.dtype == "F16") {
            std::memcpy(m.data.data(), p, numel * 2);
            m.dt = WDT_F16;
        } else if (t.dtype == "F32" && to_f16) {
            const float* f = (const float*)t.data;
            for (size_t i = 0; i < numel; ++i) m.data[i] = f32_to_f16_rne(f[i]);
            m.dt = WDT_F16;
        } else {
            throw std::runtime_error("EINVAL: matrix `" + n + "` has dtype " + t.dtype +
                                     "; only BF16/F16 checkpoints are supported for large tensors");
        }
        return m;
    }
};

std::string read_file(const std::string& p) {
    std::ifstream f(p);
    if (!f) throw std::runtime_error("ENOENT: cannot read config " + p);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

double ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

}  // namespace

// ============================================================================ lifecycle
void* Engine::dev_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) throw std::runtime_error("ENOMEM: hipMalloc(" + std::to_string(bytes) + ") failed");
    allocations_.push_back(p);
    return p;
}

void* Engine::ws(const std::string& name0, size_t bytes) {
    const std::string name = ws_prefix_.empty() ? name0 : ws_prefix_ + name0;
    auto it = ws_.find(name);
    if (it != ws_.end() && it->second.second >= bytes) return it->second.first;
    if (capturing_) throw std::runtime_error("EINTERNAL: workspace growth during graph capture: " + name);
    if (it != ws_.end()) {
        HIP_CHECK(hipDeviceSynchronize());  // both vision streams may still read it
        HIP_CHECK(hipFree(it->second.first));
    }
    void* p = nullptr;
    size_t cap = bytes + bytes / 8 + 256;
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) throw std::runtime_error("ENOMEM: workspace " + name + " (" + std::to_string(cap) + " bytes)");
    ws_[name] = {p, cap};
    return p;
}

Engine::Engine(const std::string& config_path, const std::string& weights_path, int device, int dtype, uint64_t seed,
               const std::string& snapshot_path)
    : device_(device), dtype_(dtype) {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) throw std::runtime_error("EDEVICE: no HIP device with ordinal " + std::to_string(device));
    HIP_CHECK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        throw std::runtime_error(std::string("EDEVICE: device is ") + prop.gcnArchName + ", engine is built for gfx950");
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    cfg_ = resolve_config(Json::parse(read_file(config_path)));
    const LangConfig& L = cfg_.lang;
    if (L.has_lora) throw std::runtime_error("EINVAL: LoRA attention path not yet implemented");  // block.rs:452-454
    if (L.topk_method != "greedy") throw std::runtime_error("EINVAL: MoE topk_method `" + L.topk_method + "` not yet supported (greedy only)");
    if (L.scoring != "softmax" && L.scoring != "sigmoid") throw std::runtime_error("EINVAL: MoE scoring `" + L.scoring + "` not yet supported");
    if (L.hidden_act != "silu" && L.hidden_act != "swish") throw std::runtime_error("EINVAL: activation `" + L.hidden_act + "` not implemented on this engine");
    if (L.n_routed > 256) throw std::runtime_error("EINVAL: at most 256 routed experts supported");
    if (L.topk > 8) throw std::runtime_error("EINVAL: at most 8 experts per token supported");
    if (!snapshot_path.empty() && dtype != 1)
        throw std::runtime_error("EINVAL: .dsq snapshots load as fp16 (dequant-on-load): use dtype f16");
    load_weights(weights_path, seed, snapshot_path);
    ensure_rope(4096);
    ensure_small(64);
    HIP_CHECK(hipStreamSynchronize(stream_));
}

PagePixels::~PagePixels() {
    if (global_dev) (void)hipFree(global_dev);
    if (tiles_dev) (void)hipFree(tiles_dev);
}

void* Engine::pinned(const std::string& name, size_t bytes) {
    auto it = pinned_.find(name);
    if (it != pinned_.end() && it->second.second >= bytes) return it->second.first;
    if (it != pinned_.end()) {
        HIP_CHECK(hipStreamSynchronize(stream_));  // an in-flight copy may still read the old buffer
        (void)hipHostFree(it->second.first);
    }
    void* h = nullptr;
    const size_t cap = bytes + bytes / 8 + 256;
    if (hipHostMalloc(&h, cap) != hipSuccess) throw std::runtime_error("ENOMEM: pinned staging " + name);
    pinned_[name] = {h, cap};
    return h;
}

// Stage a page's preprocessed pixels in HBM once (outside any timed region): generate() then
// gathers them device-to-device.
void Engine::upload_page(PagePixels& pg) {
    if (pg.global_dev && pg.dev_ordinal == device_) return;
    if (pg.global_chw.empty()) throw std::runtime_error("EINVAL: page pixels live on another device");
    if (pg.global_dev) { (void)hipFree(pg.global_dev); pg.global_dev = nullptr; }
    if (pg.tiles_dev) { (void)hipFree(pg.tiles_dev); pg.tiles_dev = nullptr; }
    HIP_CHECK(hipMalloc(&pg.global_dev, pg.global_chw.size() * 4));
    HIP_CHECK(hipMemcpy(pg.global_dev, pg.global_chw.data(), pg.global_chw.size() * 4, hipMemcpyHostToDevice));
    if (!pg.tiles_chw.empty()) {
        HIP_CHECK(hipMalloc(&pg.tiles_dev, pg.tiles_chw.size() * 4));
        HIP_CHECK(hipMemcpy(pg.tiles_dev, pg.tiles_chw.data(), pg.tiles_chw.size() * 4, hipMemcpyHostToDevice));
    }
    pg.dev_ordinal = device_;
}

// a1-a3 on the GPU (preprocess.hip): the page's RGB8 bytes go up once; the tap tables and the
// geometry come from the host functions the host path uses; the f32 CHW tensors are produced in
// HBM (px.global_dev / px.tiles_dev), bit-identical to dsocr_prepare_page's arrays
void Engine::prepare_page_device(const uint8_t* rgb, int w, int h, PagePixels& px) {
    hipStream_t st = stream_;
    const int G = px.crop ? px.base : px.tile;  // model/mod.rs:1714
    px.gsize = G;
    if (px.global_dev) { (void)hipFree(px.global_dev); px.global_dev = nullptr; }
    if (px.tiles_dev) { (void)hipFree(px.tiles_dev); px.tiles_dev = nullptr; }
    HIP_CHECK(hipMalloc(&px.global_dev, (size_t)3 * G * G * 4));
    const size_t nbytes = (size_t)w * h * 3;
    uint8_t* d_rgb = nbytes ? (uint8_t*)ws("pp_rgb", nbytes) : nullptr;
    if (nbytes) HIP_CHECK(hipMemcpyAsync(d_rgb, rgb, nbytes, hipMemcpyHostToDevice, st));
    auto upload_taps = [&](const ResampleCoeffs& rc, const char* name) -> std::pair<int*, int*> {
        std::vector<int> b(rc.bounds.size() * 2);
        for (size_t i = 0; i < rc.bounds.size(); ++i) { b[2 * i] = rc.bounds[i].first; b[2 * i + 1] = rc.bounds[i].second; }
        int* db = (int*)ws(std::string(name) + "_b", b.size() * 4);
        int* dc = (int*)ws(std::string(name) + "_c", rc.coeffs.size() * 4);
        HIP_CHECK(hipMemcpyAsync(db, b.data(), b.size() * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(dc, rc.coeffs.data(), rc.coeffs.size() * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));  // the host tables die with this lambda
        return {db, dc};
    };
    // ---- global view
    PpOut g;
    g.mode = 0; g.size = G; g.n_out = 1; g.out = px.global_dev;
    if (w > 0 && h > 0) {
        int nw, nh, xo, yo;
        global_view_geometry(w, h, G, &nw, &nh, &xo, &yo);
        const ResampleCoeffs cx = compute_resample_coeffs(w, nw), cy = compute_resample_coeffs(h, nh);
        auto tx = upload_taps(cx, "pp_gx");
        auto ty = upload_taps(cy, "pp_gy");
        uint8_t* hz = (uint8_t*)ws("pp_hz", (size_t)h * nw * 3);
        launch_pp_resize_h(d_rgb, w, h, tx.first, tx.second, cx.ksize, nw, hz, st);
        g.hz = hz; g.dw = nw; g.bounds = ty.first; g.coeffs = ty.second; g.ksize = cy.ksize;
        g.ox = xo; g.oy = yo; g.nw = nw; g.nh = nh;
    }
    launch_pp_resize_v_chw(g, st);
    // ---- tiles (vision/preprocess.rs:67-138, PreprocessParams::ocr1: 2..9 tiles)
    px.n_tiles = 0;
    px.crop_w = px.crop_h = 1;
    int gw = 1, gh = 1;
    if (px.crop && w > 0 && h > 0 && choose_tile_grid(w, h, px.tile, 2, 9, &gw, &gh)) {
        const int T = px.tile, tw = T * gw, th = T * gh;
        px.crop_w = gw;
        px.crop_h = gh;
        px.n_tiles = gw * gh;
        HIP_CHECK(hipMalloc(&px.tiles_dev, (size_t)px.n_tiles * 3 * T * T * 4));
        const ResampleCoeffs cx = compute_resample_coeffs(w, tw), cy = compute_resample_coeffs(h, th);
        auto tx = upload_taps(cx, "pp_tx");
        auto ty = upload_taps(cy, "pp_ty");
        uint8_t* hz = (uint8_t*)ws("pp_thz", (size_t)h * tw * 3);
        launch_pp_resize_h(d_rgb, w, h, tx.first, tx.second, cx.ksize, tw, hz, st);
        PpOut t;
        t.mode = 1; t.size = T; t.n_out = px.n_tiles; t.grid_w = gw; t.out = px.tiles_dev;
        t.hz = hz; t.dw = tw; t.bounds = ty.first; t.coeffs = ty.second; t.ksize = cy.ksize;
        launch_pp_resize_v_chw(t, st);
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(st));
    px.global_chw.clear();
    px.tiles_chw.clear();
    px.dev_ordinal = device_;
    px.n_image_tokens = image_placeholder_count(px.base, px.tile, px.crop, px.crop_w, px.crop_h);
}

Engine::~Engine() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (vstream_) (void)hipStreamSynchronize(vstream_);
    for (auto& e : span_ev_) (void)hipEventDestroy(e);
    for (auto& e : vis_ev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& kv : pinned_) (void)hipHostFree(kv.second.first);
    for (auto& kv : winmaps_) { (void)hipFree(kv.second.first); (void)hipFree(kv.second.second); }
    for (auto& kv : ws_) (void)hipFree(kv.second.first);
    for (void* p : allocations_) (void)hipFree(p);
    if (stream_) (void)hipStreamDestroy(stream_);
    if (vstream_) (void)hipStreamDestroy(vstream_);
}

void Engine::ensure_small(int n) {
    if (n <= small_cap_) return;
    std::vector<float> ones(n, 1.f);
    std::vector<int> iota(n);
    for (int i = 0; i < n; ++i) iota[i] = i;
    ones_ = (float*)dev_alloc(n * sizeof(float));
    iota_ = (int*)dev_alloc(n * sizeof(int));
    HIP_CHECK(hipMemcpy(ones_, ones.data(), n * sizeof(float), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(iota_, iota.data(), n * sizeof(int), hipMemcpyHostToDevice));
    small_cap_ = n;
}

// RoPE tables exactly as rope.rs:172-207 (f32 inv_freq, angle = pos * inv_freq, [half | half]).
void Engine::ensure_rope(int len) {
    if (len <= rope_cap_) return;
    int cap = rope_cap_ > 0 ? rope_cap_ : 1;
    while (cap < len) cap *= 2;
    const int rd = cfg_.lang.rope_dim, half = rd / 2;
    std::vector<float> inv(half), c((size_t)cap * rd), s((size_t)cap * rd);
    for (int i = 0; i < half; ++i) inv[i] = 1.0f / powf(cfg_.lang.rope_theta, ((float)i * 2.0f) / (float)rd);
    for (int p = 0; p < cap; ++p)
        for (int i = 0; i < half; ++i) {
            float a = (float)p * inv[i];
            c[(size_t)p * rd + i] = c[(size_t)p * rd + half + i] = cosf(a);
            s[(size_t)p * rd + i] = s[(size_t)p * rd + half + i] = sinf(a);
        }
    rope_cos_ = (float*)dev_alloc(c.size() * 4);
    rope_sin_ = (float*)dev_alloc(s.size() * 4);
    HIP_CHECK(hipMemcpy(rope_cos_, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(rope_sin_, s.data(), s.size() * 4, hipMemcpyHostToDevice));
    rope_cap_ = cap;
}

// ============================================================================ loading
void Engine::load_weights(const std::string& path, uint64_t seed, const std::string& snapshot_path) {
    Source src;
    src.mode = dtype_;
    if (path.empty()) {
        src.synth = true;
        src.seed = seed;
    } else {
        src.st.reset(new SafeTensors(path));
    }
    std::unique_ptr<DsqFile> snap;
    if (!snapshot_path.empty()) {
        snap.reset(new DsqFile(snapshot_path));
        src.snap = snap.get();
        src.dequant = [&](const DsqRecord& r, uint16_t* host_out) {
            const size_t need = dsq_payload_bytes(r.q_dtype, r.out_dim, r.in_dim);
            if (r.q_len != need)
                throw std::runtime_error("EINVAL: snapshot tensor `" + r.name + "` payload is " + std::to_string(r.q_len) +
                                         " bytes, expected " + std::to_string(need));
            const size_t n = (size_t)r.out_dim * r.in_dim;
            void* d_src = ws("load_dsq_src", need);
            void* d_dst = ws("load_dsq_dst", n * 2);
            HIP_CHECK(hipMemcpyAsync(d_src, snap->payload(r), need, hipMemcpyHostToDevice, stream_));
            launch_dsq_dequant(r.q_dtype, d_src, r.out_dim, r.in_dim, d_dst, stream_);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyAsync(host_out, d_dst, n * 2, hipMemcpyDeviceToHost, stream_));
            HIP_CHECK(hipStreamSynchronize(stream_));
        };
    }
    auto up16 = [&](const HostMat& m) -> void* {
        void* p = dev_alloc(m.data.size() * 2);
        HIP_CHECK(hipMemcpy(p, m.data.data(), m.data.size() * 2, hipMemcpyHostToDevice));
        return p;
    };
    auto upf = [&](const std::vector<float>& v) -> float* {
        float* p = (float*)dev_alloc(v.size() * 4);
        HIP_CHECK(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        return p;
    };
    auto vecf = [&](const std::string& n, size_t numel) -> float* { return upf(src.f32(n, numel)); };
    auto optvec = [&](const std::string& n, size_t numel) -> float* { return src.has(n) ? vecf(n, numel) : nullptr; };
    auto lin = [&](const std::string& pre, int N, int K, bool allow_bias) -> Lin {
        Lin l;
        HostMat m = src.h16(pre + ".weight", (size_t)N * K, N, K);
        l.W = up16(m);
        l.wdt = m.dt;
        l.N = N;
        l.K = K;
        if (allow_bias && src.has(pre + ".bias")) l.b = vecf(pre + ".bias", N);
        return l;
    };
    // concatenation of several [Ni][K] matrices (+ optional biases) into one [sum Ni][K]
    auto lin_cat = [&](const std::vector<std::string>& pres, const std::vector<int>& Ns, int K) -> Lin {
        Lin l;
        HostMat all;
        std::vector<float> bias;
        bool any_bias = false;
        int N = 0;
        for (size_t i = 0; i < pres.size(); ++i) {
            HostMat m = src.h16(pres[i] + ".weight", (size_t)Ns[i] * K, Ns[i], K);
            if (i == 0) all.dt = m.dt;
            else if (m.dt != all.dt) throw std::runtime_error("EINVAL: mixed dtypes in fused linear " + pres[i]);
            all.data.insert(all.data.end(), m.data.begin(), m.data.end());
            std::vector<float> b(Ns[i], 0.f);
            if (src.has(pres[i] + ".bias")) { b = src.f32(pres[i] + ".bias", Ns[i]); any_bias = true; }
            bias.insert(bias.end(), b.begin(), b.end());
            N += Ns[i];
        }
        l.W = up16(all);
        l.wdt = all.dt;
        l.N = N;
        l.K = K;
        if (any_bias) l.b = upf(bias);
        return l;
    };
    // conv [O][C][kh][kw] -> [O][kh][kw][C] (NHWC im2col order)
    auto conv = [&](const std::string& n, int O, int C, int kh, int kw) -> Lin {
        HostMat m = src.h16(n, (size_t)O * C * kh * kw);
        HostMat r;
        r.dt = m.dt;
        r.data.resize(m.data.size());
        for (int o = 0; o < O; ++o)
            for (int c = 0; c < C; ++c)
                for (int y = 0; y < kh; ++y)
                    for (int x = 0; x < kw; ++x)
                        r.data[(((size_t)o * kh + y) * kw + x) * C + c] = m.data[(((size_t)o * C + c) * kh + y) * kw + x];
        Lin l;
        l.W = up16(r);
        l.wdt = r.dt;
        l.N = O;
        l.K = C * kh * kw;
        return l;
    };

    // ---------------- SAM (vision/sam.rs:143-184)
    const SamConfig& S = cfg_.sam;
    const std::string sp = "model.sam_model.";
    sam_.patch = lin(sp + "patch_embed.proj", S.dim, 3 * S.patch * S.patch, true);
    const int tps = S.image_size / S.patch;
    if (src.has(sp + "pos_embed")) {
        sam_.has_pos = true;
        sam_.pos_grid = tps;
        std::vector<float> pos = src.f32(sp + "pos_embed", (size_t)tps * tps * S.dim);  // [1][g][g][C]
        sam_.pos_host.resize(pos.size());
        for (int y = 0; y < tps; ++y)
            for (int x = 0; x < tps; ++x)
                for (int c = 0; c < S.dim; ++c)
                    sam_.pos_host[((size_t)c * tps + y) * tps + x] = pos[((size_t)y * tps + x) * S.dim + c];
    }
    const int hd = S.dim / S.heads;
    for (int b = 0; b < S.depth; ++b) {
        SamBlock blk;
        const std::string bp = sp + "blocks." + std::to_string(b) + ".";
        blk.global = S.is_global(b);
        blk.n1 = {vecf(bp + "norm1.weight", S.dim), vecf(bp + "norm1.bias", S.dim)};
        blk.n2 = {vecf(bp + "norm2.weight", S.dim), vecf(bp + "norm2.bias", S.dim)};
        blk.qkv = lin(bp + "attn.qkv", 3 * S.dim, S.dim, true);
        blk.proj = lin(bp + "attn.proj", S.dim, S.dim, true);
        const int hid = (int)(S.dim * S.mlp_ratio);
        std::string f1 = src.has(bp + "mlp.fc1.weight") ? "mlp.fc1" : "mlp.lin1";
        std::string f2 = src.has(bp + "mlp.fc2.weight") ? "mlp.fc2" : "mlp.lin2";
        blk.fc1 = lin(bp + f1, hid, S.dim, true);
        blk.fc2 = lin(bp + f2, S.dim, hid, true);
        blk.use_rel = src.has(bp + "attn.rel_pos_h");
        if (blk.use_rel) {
            const int tokens = blk.global ? tps : S.window;
            blk.rel_len = 2 * tokens - 1;
            blk.relh = src.f32(bp + "attn.rel_pos_h", (size_t)blk.rel_len * hd);
            blk.relw = src.f32(bp + "attn.rel_pos_w", (size_t)blk.rel_len * hd);
        }
        sam_.blocks.push_back(std::move(blk));
    }
    sam_.neck0 = conv(sp + "neck.0.weight", S.neck, S.dim, 1, 1);
    sam_.neck1 = {vecf(sp + "neck.1.weight", S.neck), vecf(sp + "neck.1.bias", S.neck)};
    sam_.neck2 = conv(sp + "neck.2.weight", S.neck, S.neck, 3, 3);
    sam_.neck3 = {vecf(sp + "neck.3.weight", S.neck), vecf(sp + "neck.3.bias", S.neck)};
    sam_.net2 = conv(sp + "net_2.weight", S.out_ch[0], S.neck, 3, 3);
    sam_.net3 = conv(sp + "net_3.weight", S.out_ch[1], S.out_ch[0], 3, 3);

    // ---------------- CLIP (vision/clip.rs:73-88)
    const ClipConfig& C = cfg_.clip;
    const std::string cp = "model.vision_model.";
    clip_.cls = vecf(cp + "embeddings.class_embedding", C.hidden);
    clip_.pos_host = src.f32(cp + "embeddings.position_embedding.weight", (size_t)(C.seq + 1) * C.hidden);
    clip_.pre = {vecf(cp + "pre_layrnorm.weight", C.hidden), vecf(cp + "pre_layrnorm.bias", C.hidden)};
    for (int l = 0; l < C.layers; ++l) {
        ClipLayer cl;
        const std::string lp = cp + "transformer.layers." + std::to_string(l) + ".";
        cl.ln1 = {vecf(lp + "layer_norm1.weight", C.hidden), vecf(lp + "layer_norm1.bias", C.hidden)};
        cl.ln2 = {vecf(lp + "layer_norm2.weight", C.hidden), vecf(lp + "layer_norm2.bias", C.hidden)};
        cl.qkv = lin(lp + "self_attn.qkv_proj", 3 * C.hidden, C.hidden, true);
        cl.out = lin(lp + "self_attn.out_proj", C.hidden, C.hidden, true);
        cl.fc1 = lin(lp + "mlp.fc1", C.ffn, C.hidden, true);
        cl.fc2 = lin(lp + "mlp.fc2", C.hidden, C.ffn, true);
        clip_.layers.push_back(cl);
    }
    if (C.hidden != S.out_ch[1]) throw std::runtime_error("EINVAL: CLIP width must equal SAM output channels");
    if (C.hidden + S.out_ch[1] != cfg_.proj_in) throw std::runtime_error("EINVAL: combined hidden dims do not match projector input");

    // ---------------- projector (model/mod.rs:258-390)
    proj_ = lin("model.projector.layers", cfg_.proj_out, cfg_.proj_in, true);
    newline_ = src.has("model.image_newline") ? vecf("model.image_newline", cfg_.proj_out)
                                               : upf(std::vector<float>(cfg_.proj_out, 0.f));
    separator_ = vecf("model.view_seperator", cfg_.proj_out);

    // ---------------- language model (transformer/weights.rs:444-606)
    const LangConfig& L = cfg_.lang;
    {
        HostMat m = src.h16("model.embed_tokens.weight", (size_t)L.vocab * L.hidden);
        embed_ = up16(m);
        embed_dt_ = m.dt;
    }
    const int H = L.hidden, KVH = L.kv_heads * L.head_dim;
    for (int l = 0; l < L.layers; ++l) {
        DecLayer d;
        const std::string lp = "model.layers." + std::to_string(l) + ".";
        d.in_norm = {vecf(lp + "input_layernorm.weight", H), nullptr};
        d.post_norm = {vecf(lp + "post_attention_layernorm.weight", H), nullptr};
        d.qkv = lin_cat({lp + "self_attn.q_proj", lp + "self_attn.k_proj", lp + "self_attn.v_proj"},
                        {L.heads * L.head_dim, KVH, L.kv_heads * L.v_head_dim}, H);
        d.o = lin(lp + "self_attn.o_proj", H, L.heads * L.v_head_dim, true);
        d.moe = L.moe_layer(l);
        if (!d.moe) {
            d.gu = lin_cat({lp + "mlp.gate_proj", lp + "mlp.up_proj"}, {L.inter, L.inter}, H);
            d.down = lin(lp + "mlp.down_proj", H, L.inter, true);
            if (d.gu.b || d.down.b) throw std::runtime_error("EINVAL: biased dense MLP not supported");
        } else {
            const int E = L.n_routed, I = L.moe_inter;
            HostMat r = src.h16(lp + "mlp.gate.weight", (size_t)E * H);
            d.router.W = up16(r);
            d.router.wdt = r.dt;
            d.router.N = E;
            d.router.K = H;
            d.router.b = optvec(lp + "mlp.gate.e_score_correction_bias", E);
            HostMat gu, dn;
            gu.data.resize((size_t)E * 2 * I * H);
            dn.data.resize((size_t)E * H * I);
            for (int e = 0; e < E; ++e) {
                const std::string ep = lp + "mlp.experts." + std::to_string(e) + ".";
                HostMat g = src.h16(ep + "gate_proj.weight", (size_t)I * H, I, H);
                HostMat u = src.h16(ep + "up_proj.weight", (size_t)I * H, I, H);
                HostMat w = src.h16(ep + "down_proj.weight", (size_t)H * I, H, I);
                if (src.has(ep + "gate_proj.bias") || src.has(ep + "down_proj.bias"))
                    throw std::runtime_error("EINVAL: biased experts not supported");
                std::copy(g.data.begin(), g.data.end(), gu.data.begin() + (size_t)e * 2 * I * H);
                std::copy(u.data.begin(), u.data.end(), gu.data.begin() + (size_t)e * 2 * I * H + (size_t)I * H);
                std::copy(w.data.begin(), w.data.end(), dn.data.begin() + (size_t)e * H * I);
                gu.dt = dn.dt = g.dt;
            }
            d.e_gu = up16(gu);
            d.e_d = up16(dn);
            d.e_wdt = gu.dt;
            if (L.n_shared > 0) {
                const int Is = I * L.n_shared;
                d.has_shared = true;
                d.s_gu = lin_cat({lp + "mlp.shared_experts.gate_proj", lp + "mlp.shared_experts.up_proj"}, {Is, Is}, H);
                d.s_d = lin(lp + "mlp.shared_experts.down_proj", H, Is, true);
            }
        }
        layers_.push_back(d);
    }
    HIP_CHECK(hipDeviceSynchronize());
    final_norm_ = vecf("model.norm.weight", H);  // f32 copy (model/mod.rs:1008-1014)
    lm_head_ = lin("lm_head", L.vocab, H, false);
    if ((lm_head_.wdt == WDT_BF16 || lm_head_.wdt == WDT_F16) && H % 16 == 0 && H <= 1536) {
        // int8 screening copy of the lm_head (per-row scale + rigorous error bound), lmhead.hip
        // (+ for 3..8 pages: s ||Q|| per row and the fragment-ordered copy the int8 matrix cores read; the
        // per-row arrays padded to whole 16-row tiles)
        const size_t vp = (size_t)(L.vocab + 15) / 16 * 16;
        lmq_ = dev_alloc((size_t)L.vocab * H);
        lmq_scale_ = (float*)dev_alloc(vp * 4);
        lmq_bound_ = (float*)dev_alloc(vp * 4);
        HIP_CHECK(hipMemset(lmq_scale_, 0, vp * 4));
        HIP_CHECK(hipMemset(lmq_bound_, 0, vp * 4));
        if (lmhead_q8mm_ok(8, L.vocab, H)) {
            lmq_qnorm_ = (float*)dev_alloc(vp * 4);
            HIP_CHECK(hipMemset(lmq_qnorm_, 0, vp * 4));
            lmq_frag_ = dev_alloc(lmhead_qfrag_bytes(L.vocab, H));
        }
        launch_lmhead_quantize(lm_head_.W, L.vocab, H, lmq_, lmq_scale_, lmq_bound_, nullptr, lmq_qnorm_, lmq_frag_,
                               lm_head_.wdt);
        HIP_CHECK(hipDeviceSynchronize());
    }
}

// ============================================================================ compute helpers
void Engine::linear(const float* x, int M, int ldx, const Lin& l, float* y, int ldy, int act, int accumulate,
                    const int* c_rows) {
    flops_acc_ += 2.0 * M * (double)l.N * l.K;
    if (M <= 16 && !c_rows) {
        DecGemvArgs a;
        a.M = M; a.N = l.N; a.K = l.K; a.x = x; a.ldx = ldx; a.W = l.W; a.ldw = l.K; a.wdtype = l.wdt;
        a.bias = l.b; a.y = y; a.ldy = ldy; a.act = act; a.accumulate = accumulate;
        launch_dec_gemv(a, stream_);
    } else if ((l.wdt == WDT_F16 || l.wdt == WDT_BF16) && l.K % 32 == 0 && ldx % 4 == 0 &&
               (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        // the exact-f32 linear on the bf16 matrix cores: the f32 rows split into 3 bf16 planes (and f16
        // weights into hi / lo bf16) inside the GEMM's fragment loads (gemm_bf16.hip, gemm_f32a)
        GemmBf16Args g;
        g.M = M; g.N = l.N; g.K = l.K; g.A = x; g.lda = ldx; g.W = l.W; g.ldw = l.K; g.w_f16 = l.wdt == WDT_F16;
        g.bias = l.b; g.C = y; g.ldc = ldy; g.c_rows = c_rows; g.act = act; g.accumulate = accumulate;
        g.splits = gemm_f32a_splits(M, l.N, l.K);
        if (g.splits > 1) g.part = wsf("g_splitk", (size_t)g.splits * M * l.N);
        launch_gemm_f32a(g, stream_);
    } else {
        GemmArgs g;
        g.M = M; g.N = l.N; g.K = l.K; g.A = x; g.lda = ldx; g.W = l.W; g.ldw = l.K; g.wdtype = l.wdt;
        g.bias = l.b; g.C = y; g.ldc = ldy; g.c_rows = c_rows; g.act = act; g.accumulate = accumulate;
        launch_gemm(g, stream_);
    }
}

float* Engine::sam_pos(int g) {
    auto it = sam_.pos_dev.find(g);
    if (it != sam_.pos_dev.end()) return it->second;
    const int C = cfg_.sam.dim, src = sam_.pos_grid;
    std::vector<float> r = bicubic_resize_aa(sam_.pos_host, C, src, src, g, g);  // sam.rs:982-998
    std::vector<float> nhwc((size_t)g * g * C);
    for (int c = 0; c < C; ++c)
        for (int p = 0; p < g * g; ++p) nhwc[(size_t)p * C + c] = r[(size_t)c * g * g + p];
    float* d = (float*)dev_alloc(nhwc.size() * 4);
    HIP_CHECK(hipMemcpy(d, nhwc.data(), nhwc.size() * 4, hipMemcpyHostToDevice));
    sam_.pos_dev[g] = d;
    return d;
}

std::pair<float*, float*> Engine::sam_rel(SamBlock& b, int g) {
    auto it = b.rel_dev.find(g);
    if (it != b.rel_dev.end()) return it->second;
    const int hd = cfg_.sam.dim / cfg_.sam.heads;
    std::vector<float> rh = rel_pos_resize(b.relh, b.rel_len, hd, g);
    std::vector<float> rw = rel_pos_resize(b.relw, b.rel_len, hd, g);
    float* dh = (float*)dev_alloc(rh.size() * 4);
    float* dw = (float*)dev_alloc(rw.size() * 4);
    HIP_CHECK(hipMemcpy(dh, rh.data(), rh.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dw, rw.data(), rw.size() * 4, hipMemcpyHostToDevice));
    b.rel_dev[g] = {dh, dw};
    return {dh, dw};
}

float* Engine::clip_pos(int tokens) {
    auto it = clip_.pos_dev.find(tokens);
    if (it != clip_.pos_dev.end()) return it->second;
    const ClipConfig& C = cfg_.clip;
    std::vector<float> out;
    if (tokens == C.seq + 1) {
        out = clip_.pos_host;
    } else {  // clip.rs:486-544
        const int s = (int)std::lround(std::sqrt((double)C.seq)), t = (int)std::lround(std::sqrt((double)(tokens - 1)));
        if (t * t != tokens - 1) throw std::runtime_error("EINVAL: clip positional table tgt tokens not square");
        std::vector<float> grid((size_t)C.hidden * s * s);
        for (int p = 0; p < s * s; ++p)
            for (int c = 0; c < C.hidden; ++c) grid[(size_t)c * s * s + p] = clip_.pos_host[(size_t)(1 + p) * C.hidden + c];
        std::vector<float> r = bicubic_resize_aa(grid, C.hidden, s, s, t, t);
        out.resize((size_t)tokens * C.hidden);
        std::copy(clip_.pos_host.begin(), clip_.pos_host.begin() + C.hidden, out.begin());
        for (int p = 0; p < t * t; ++p)
            for (int c = 0; c < C.hidden; ++c) out[(size_t)(1 + p) * C.hidden + c] = r[(size_t)c * t * t + p];
    }
    float* d = (float*)dev_alloc(out.size() * 4);
    HIP_CHECK(hipMemcpy(d, out.data(), out.size() * 4, hipMemcpyHostToDevice));
    clip_.pos_dev[tokens] = d;
    return d;
}

// ============================================================================ vision
// DSOCR_VIS_STREAMS=0 (A/B switch, read once): every vision pass of a batch on the engine stream
static bool vis_streams_on() {
    static const bool v = !(getenv("DSOCR_VIS_STREAMS") && atoi(getenv("DSOCR_VIS_STREAMS")) == 0);
    return v;
}

// SamBackbone::forward (sam.rs:210-289) + ClipVisionModel::forward (clip.rs:98-102) +
// build_clip_sam_tokens + ImageProjector::project (model/mod.rs:604-650, 392-444).
float* Engine::vision_pass(const float* imgs, int n, int Spx, const std::string& out) {
    const SamConfig& S = cfg_.sam;
    const ClipConfig& CC = cfg_.clip;
    const int C = S.dim, heads = S.heads, hd = C / heads;
    if (Spx % S.patch) throw std::runtime_error("EINVAL: image dimensions must be divisible by patch size");
    const int g = Spx / S.patch;
    if (g % 2 || (g / 2) % 2) throw std::runtime_error("EINVAL: spatial dims cannot be evenly downsampled by stride 2");
    const long rows = (long)n * g * g;
    hipStream_t st = stream_;

    // patch embed
    float* cols = wsf("v_cols", (size_t)rows * 3 * S.patch * S.patch);
    launch_patch_im2col(imgs, n, Spx, Spx, S.patch, cols, st);
    float* x = wsf("v_x", (size_t)rows * C);
    linear(cols, (int)rows, 3 * S.patch * S.patch, sam_.patch, x, C);
    if (sam_.has_pos) launch_add_broadcast(x, sam_pos(g), (long)g * g, C, n, st);

    // window partition maps (sam.rs:926-980)
    const int W = S.window;
    const int gp = g + (W - g % W) % W, nw = gp / W;
    const long wrows = (long)n * nw * nw * W * W;
    auto wm = winmaps_.find({n, g});
    if (wm == winmaps_.end()) {  // built once per (images, grid): tok -> window slot and back
        std::vector<int> tok2win(rows), win2tok(wrows, -1);
        for (int b = 0; b < n; ++b)
            for (int y = 0; y < g; ++y)
                for (int xx = 0; xx < g; ++xx) {
                    long t = ((long)b * g + y) * g + xx;
                    long w = (((long)b * nw + y / W) * nw + xx / W) * W * W + (y % W) * W + (xx % W);
                    tok2win[t] = (int)w;
                    win2tok[w] = (int)t;
                }
        int *a = nullptr, *b2 = nullptr;
        HIP_CHECK(hipMalloc(&a, tok2win.size() * 4));
        HIP_CHECK(hipMalloc(&b2, win2tok.size() * 4));
        HIP_CHECK(hipMemcpy(a, tok2win.data(), tok2win.size() * 4, hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(b2, win2tok.data(), win2tok.size() * 4, hipMemcpyHostToDevice));
        wm = winmaps_.emplace(std::make_pair(n, g), std::make_pair(a, b2)).first;
    }
    int* d_tok2win = wm->second.first;
    int* d_win2tok = wm->second.second;
    const long maxrows = std::max(rows, wrows);
    float* xn = wsf("v_xn", (size_t)maxrows * C);
    float* qkv = wsf("v_qkv", (size_t)maxrows * 3 * C);
    float* ctx = wsf("v_ctx", (size_t)maxrows * C);
    const int hid = (int)(C * S.mlp_ratio);
    float* hbuf = wsf("v_h", (size_t)rows * hid);

    for (int bi = 0; bi < S.depth; ++bi) {
        SamBlock& blk = sam_.blocks[bi];
        const bool win = !blk.global;
        const int L = win ? W * W : g * g;
        const int nseq = win ? n * nw * nw : n;
        const long arows = (long)nseq * L;
        if (win) {
            HIP_CHECK(hipMemsetAsync(xn, 0, (size_t)wrows * C * 4, st));
            launch_layernorm(x, C, xn, C, d_tok2win, (int)rows, C, blk.n1.w, blk.n1.b, 1e-6f, st);
        } else {
            launch_layernorm(x, C, xn, C, nullptr, (int)rows, C, blk.n1.w, blk.n1.b, 1e-6f, st);
        }
        linear(xn, (int)arows, C, blk.qkv, qkv, 3 * C);
        AttnArgs a;
        a.q = {qkv, 3L * C, hd, nullptr};
        a.k = {qkv + C, 3L * C, hd, nullptr};
        a.v = {qkv + 2 * C, 3L * C, hd, nullptr};
        a.o = ctx;
        a.o_row_stride = C;
        a.o_head_stride = hd;
        a.n_seq = nseq;
        a.L = L;
        a.heads = heads;
        a.kv_heads = heads;
        a.hd = hd;
        a.scale = (float)(1.0 / std::sqrt((double)hd));
        if (blk.use_rel) {
            const int gg = win ? W : g;
            auto rel = win ? std::make_pair<float*, float*>(nullptr, nullptr) : sam_rel(blk, g);
            if (win) rel = sam_rel(blk, W);
            float* rb = wsf("v_relbias", (size_t)nseq * heads * L * (2 * gg));
            launch_sam_relbias(qkv, 3L * C, nseq, gg, gg, heads, hd, rel.first, rel.second, rb, st);
            a.relbias = rb;
            a.rel_h = gg;
            a.rel_w = gg;
        }
        flops_acc_ += 4.0 * nseq * (double)L * L * hd * heads;
        launch_attention(a, st);
        // proj + residual (window_unpartition via row scatter)
        linear(ctx, (int)arows, C, blk.proj, x, C, 0, 1, win ? d_win2tok : nullptr);
        launch_layernorm(x, C, xn, C, nullptr, (int)rows, C, blk.n2.w, blk.n2.b, 1e-6f, st);
        linear(xn, (int)rows, C, blk.fc1, hbuf, hid, ACT_GELU_ERF);
        linear(hbuf, (int)rows, hid, blk.fc2, x, C, 0, 1);
    }
    // neck (sam.rs:503-520) in NHWC
    const int NC = S.neck;
    float* y = wsf("v_neck", (size_t)rows * NC);
    linear(x, (int)rows, C, sam_.neck0, y, NC);
    launch_layernorm(y, NC, y, NC, nullptr, (int)rows, NC, sam_.neck1.w, sam_.neck1.b, 1e-6f, st);
    float* ncols = wsf("v_ncols", (size_t)rows * 9 * NC);
    launch_conv_im2col_nhwc(y, n, g, g, NC, 3, 3, 1, 1, ncols, st);
    linear(ncols, (int)rows, 9 * NC, sam_.neck2, y, NC);
    launch_layernorm(y, NC, y, NC, nullptr, (int)rows, NC, sam_.neck3.w, sam_.neck3.b, 1e-6f, st);
    // downsample (sam.rs:550-575)
    const int g2 = g / 2, g4 = g / 4, c0 = S.out_ch[0], c1 = S.out_ch[1];
    launch_conv_im2col_nhwc(y, n, g, g, NC, 3, 3, 2, 1, ncols, st);
    float* z = wsf("v_net2", (size_t)n * g2 * g2 * c0);
    linear(ncols, n * g2 * g2, 9 * NC, sam_.net2, z, c0);
    float* ncols2 = wsf("v_ncols2", (size_t)n * g4 * g4 * 9 * c0);
    launch_conv_im2col_nhwc(z, n, g2, g2, c0, 3, 3, 2, 1, ncols2, st);
    const int Sq = g4 * g4;
    float* sam_out = wsf("v_samout", (size_t)n * Sq * c1);
    linear(ncols2, n * Sq, 9 * c0, sam_.net3, sam_out, c1);

    // CLIP (clip.rs:165-309) on SAM features
    const int T = Sq + 1, CH = CC.hidden, chd = CH / CC.heads;
    const long crow = (long)n * T;
    float* cx = wsf("c_x", (size_t)crow * CH);
    launch_clip_embed(sam_out, clip_.cls, clip_pos(T), n, Sq, CH, cx, st);
    launch_layernorm(cx, CH, cx, CH, nullptr, (int)crow, CH, clip_.pre.w, clip_.pre.b, 1e-5f, st);
    float* cxn = wsf("c_xn", (size_t)crow * CH);
    float* cqkv = wsf("c_qkv", (size_t)crow * 3 * CH);
    float* cctx = wsf("c_ctx", (size_t)crow * CH);
    float* ch = wsf("c_h", (size_t)crow * CC.ffn);
    for (int l = 0; l < CC.layers; ++l) {
        ClipLayer& cl = clip_.layers[l];
        launch_layernorm(cx, CH, cxn, CH, nullptr, (int)crow, CH, cl.ln1.w, cl.ln1.b, 1e-5f, st);
        linear(cxn, (int)crow, CH, cl.qkv, cqkv, 3 * CH);
        AttnArgs a;
        a.q = {cqkv, 3L * CH, chd, nullptr};
        a.k = {cqkv + CH, 3L * CH, chd, nullptr};
        a.v = {cqkv + 2 * CH, 3L * CH, chd, nullptr};
        a.o = cctx;
        a.o_row_stride = CH;
        a.o_head_stride = chd;
        a.n_seq = n;
        a.L = T;
        a.heads = CC.heads;
        a.kv_heads = CC.heads;
        a.hd = chd;
        a.scale = (float)(1.0 / std::sqrt((double)chd));
        flops_acc_ += 4.0 * n * (double)T * T * chd * CC.heads;
        launch_attention(a, st);
        linear(cctx, (int)crow, CH, cl.out, cx, CH, 0, 1);
        launch_layernorm(cx, CH, cxn, CH, nullptr, (int)crow, CH, cl.ln2.w, cl.ln2.b, 1e-5f, st);
        linear(cxn, (int)crow, CH, cl.fc1, ch, CC.ffn, ACT_QUICK_GELU);
        linear(ch, (int)crow, CC.ffn, cl.fc2, cx, CH, 0, 1);
    }
    // concat + projector
    float* pre = wsf("p_pre", (size_t)n * Sq * (CH + c1));
    launch_concat_clip_sam(cx, sam_out, n, Sq, CH, c1, pre, st);
    float* post = wsf(out, (size_t)n * Sq * cfg_.proj_out);
    linear(pre, n * Sq, CH + c1, proj_, post, cfg_.proj_out);
    return post;
}

std::vector<std::vector<float>> Engine::image_embeddings(const std::vector<const PagePixels*>& pages) {
    std::vector<std::vector<float>> result;
    const int H = cfg_.proj_out;
    for (const PagePixels* p : pages) {
        // one page at a time keeps this helper simple; generate() batches pages.
        float* gimg = p->global_dev && p->dev_ordinal == device_ ? p->global_dev : upload("e_gimg", p->global_chw);
        float* gpost = vision_pass(gimg, 1, p->gsize, "e_gpost");
        const int gs = p->gsize / 64;
        std::vector<float> gh((size_t)gs * gs * H);
        HIP_CHECK(hipMemcpyAsync(gh.data(), gpost, gh.size() * 4, hipMemcpyDeviceToHost, stream_));
        std::vector<float> lh;
        int ls = 0;
        if (p->n_tiles > 0) {
            float* timg = p->tiles_dev && p->dev_ordinal == device_ ? p->tiles_dev : upload("e_timg", p->tiles_chw);
            float* lpost = vision_pass(timg, p->n_tiles, p->tile, "e_lpost");
            ls = p->tile / 64;
            lh.resize((size_t)p->n_tiles * ls * ls * H);
            HIP_CHECK(hipMemcpyAsync(lh.data(), lpost, lh.size() * 4, hipMemcpyDeviceToHost, stream_));
        }
        HIP_CHECK(hipStreamSynchronize(stream_));
        std::vector<float> nl(H), sp(H);
        HIP_CHECK(hipMemcpy(nl.data(), newline_, H * 4, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(sp.data(), separator_, H * 4, hipMemcpyDeviceToHost));
        std::vector<float> rows;
        auto push = [&](const float* r) { rows.insert(rows.end(), r, r + H); };
        if (p->n_tiles > 0) {  // format_local_tokens (model/mod.rs:677-709)
            for (int R = 0; R < p->crop_h * ls; ++R) {
                for (int Cc = 0; Cc < p->crop_w * ls; ++Cc) {
                    int crop = (R / ls) * p->crop_w + (Cc / ls);
                    push(&lh[(((size_t)crop * ls + R % ls) * ls + Cc % ls) * H]);
                }
                push(nl.data());
            }
        }
        for (int R = 0; R < gs; ++R) {  // format_global_tokens (656-675)
            for (int Cc = 0; Cc < gs; ++Cc) push(&gh[((size_t)R * gs + Cc) * H]);
            push(nl.data());
        }
        push(sp.data());
        result.push_back(std::move(rows));
    }
    return result;
}

// ============================================================================ decoder
void Engine::layer_forward_prefill(int l, int T, int B, const int* row_page, const int* row_pos, const long* q_off,
                                   const long* kv_off, const long* o_off, const int* seq_len, int max_len, int Lmax) {
    const LangConfig& L = cfg_.lang;
    DecLayer& d = layers_[l];
    hipStream_t st = stream_;
    const int H = L.hidden, hd = L.head_dim, KVH = L.kv_heads * hd, QKVN = d.qkv.N;
    float* X = wsf("d_x", (size_t)T * H);
    float* XN = wsf("d_xn", (size_t)T * H);
    float* QKV = wsf("d_qkv", (size_t)T * QKVN);
    float* CTX = wsf("d_ctx", (size_t)T * H);
    const long layer_kv = (long)B * page_stride_;
    float* kc = kc_ + (long)l * layer_kv;
    float* vc = vc_ + (long)l * layer_kv;

    launch_rmsnorm(X, H, XN, H, T, H, d.in_norm.w, L.rms_eps, st);
    linear(XN, T, H, d.qkv, QKV, QKVN);
    RopeKvArgs r;
    r.qkv = QKV; r.ld = QKVN; r.rows = T; r.row_page = row_page; r.row_pos = row_pos;
    r.heads = L.heads; r.kv_heads = L.kv_heads; r.hd = hd; r.rope_dim = L.rope_dim; r.use_mla = L.use_mla;
    r.cos = rope_cos_; r.sin = rope_sin_; r.kc = kc; r.vc = vc; r.page_stride = page_stride_; r.head_stride = head_stride_;
    launch_rope_kv(r, st);
    AttnArgs a;
    a.q = {QKV, QKVN, hd, q_off};
    a.k = {kc, hd, head_stride_, kv_off};
    a.v = {vc, hd, head_stride_, kv_off};
    a.o = CTX; a.o_row_stride = H; a.o_head_stride = hd; a.o_seq_off = o_off;
    a.n_seq = B; a.L = max_len; a.seq_len = seq_len;
    a.heads = L.heads; a.kv_heads = L.kv_heads; a.hd = hd;
    a.scale = (float)(1.0 / std::sqrt((double)hd));
    a.causal = 1;
    // the key-piece workspace grows as L^2 (n_seq * heads * sum over query blocks of their pieces * 128 * (hd + 2)
    // floats: 89 MB at 8 x 706 tokens, 2.8 GB at 8 x 4096); above 512 MB the prefill runs the one-block-per-
    // query-block kernel, which needs none
    constexpr size_t kPartCapFloats = (size_t)128 << 20;
    const size_t part_floats = attention_causal_part_floats(B, L.heads, max_len, hd);
    if (part_floats <= kPartCapFloats) {
        a.part_floats = part_floats;
        a.part = wsf("d_attn_part", a.part_floats);
    }
    for (int q = 0; q < B && q < (int)prefill_lens_.size(); ++q)
        flops_acc_ += 2.0 * (double)prefill_lens_[q] * (prefill_lens_[q] + 1) * hd * L.heads;
    launch_attention(a, st);
    (void)Lmax;
    (void)KVH;
    linear(CTX, T, H, d.o, X, H, 0, 1);
    launch_rmsnorm(X, H, XN, H, T, H, d.post_norm.w, L.rms_eps, st);
    if (!d.moe) {
        const int I = L.inter;
        float* G = wsf("d_g", (size_t)T * 2 * I);
        float* HH = wsf("d_hh", (size_t)T * I);
        linear(XN, T, H, d.gu, G, 2 * I);
        launch_silu_mul(G, 2 * I, I, T, HH, I, st);
        linear(HH, T, I, d.down, X, H, 0, 1);
        return;
    }
    // MoE (run_moe, block.rs:1215-1395) with device-side routing
    const int E = L.n_routed, K = L.topk, I = L.moe_inter, TK = T * K;
    float* LOG = wsf("d_log", (size_t)T * E);
    int* IDS = wsi("d_ids", TK);
    float* WTS = wsf("d_wts", TK);
    int* EOFF = wsi("d_eoff", E + 1);
    int* AROW = wsi("d_arow", TK);
    int* APOS = wsi("d_apos", TK);
    linear(XN, T, H, d.router, LOG, E);
    launch_router_topk(LOG, T, E, K, L.scoring == "softmax", L.norm_topk, L.routed_scaling, IDS, WTS, st);
    launch_moe_group(IDS, T, K, E, EOFF, AROW, APOS, nullptr, st);
    float* G = wsf("d_eg", (size_t)TK * 2 * I);
    float* HH = wsf("d_ehh", (size_t)TK * I);
    float* Y = wsf("d_ey", (size_t)TK * H);
    GemmArgs g1;
    g1.M = TK; g1.N = 2 * I; g1.K = H; g1.A = XN; g1.lda = H; g1.a_rows = AROW; g1.W = d.e_gu; g1.ldw = H;
    g1.wdtype = d.e_wdt; g1.w_group_stride = (long)2 * I * H; g1.C = G; g1.ldc = 2 * I;
    g1.group_off = EOFF; g1.groups = E; g1.max_group_rows = T;
    launch_gemm(g1, st);
    flops_acc_ += 2.0 * TK * (2.0 * I) * H + 2.0 * TK * (double)H * I;  // routed gate/up + down (next launch)
    launch_silu_mul(G, 2 * I, I, TK, HH, I, st);
    GemmArgs g2;
    g2.M = TK; g2.N = H; g2.K = I; g2.A = HH; g2.lda = I; g2.W = d.e_d; g2.ldw = I; g2.wdtype = d.e_wdt;
    g2.w_group_stride = (long)H * I; g2.C = Y; g2.ldc = H; g2.group_off = EOFF; g2.groups = E; g2.max_group_rows = T;
    launch_gemm(g2, st);
    float* YS = nullptr;
    if (d.has_shared) {
        const int Is = d.s_d.K;
        float* GS = wsf("d_sg", (size_t)T * 2 * Is);
        float* HS = wsf("d_shh", (size_t)T * Is);
        YS = wsf("d_sy", (size_t)T * H);
        linear(XN, T, H, d.s_gu, GS, 2 * Is);
        launch_silu_mul(GS, 2 * Is, Is, T, HS, Is, st);
        linear(HS, T, Is, d.s_d, YS, H);
    }
    launch_moe_combine(Y, APOS, WTS, YS, T, K, H, X, 1, st);
}

// DSOCR_ROUTER_SWZ=0 (A/B switch, read at every MoE argument build, i.e. per capture): the routing inside gate/up
// reads the row-major router rows instead of their fragment-ordered copy
static bool router_swz_off() {
    const char* e = getenv("DSOCR_ROUTER_SWZ");
    return e && atoi(e) == 0;
}
// DSOCR_MM_SWZ=0 (A/B switch, per capture): 3..8 pages' q/k/v, o_proj and dense gate|up read row-major weights
static bool mm_swz_off() {
    const char* e = getenv("DSOCR_MM_SWZ");
    return e && atoi(e) == 0;
}

// Decode MoE arguments of layer l for B pages (shared by decode_step and profile_decode): the
// layer's weights and the named workspaces; launch_moe_decode (decode.hip) picks the kernels.
MoeDecodeArgs Engine::moe_args(int l, int B, float* X) {
    const LangConfig& L = cfg_.lang;
    DecLayer& d = layers_[l];
    const int H = L.hidden, E = L.n_routed, K = L.topk, I = L.moe_inter, TK = B * K;
    MoeDecodeArgs a;
    a.T = B; a.H = H; a.E = E; a.topk = K; a.I = I;
    a.x = X; a.norm_w = d.post_norm.w; a.eps = L.rms_eps; a.out = X;
    a.router = d.router.W; a.router_wdt = d.router.wdt; a.router_bias = d.router.b;
    a.Wgu = d.e_gu; a.Wd = d.e_d; a.wdtype = d.e_wdt;
    if (d.has_shared) {
        if (d.s_gu.wdt != d.e_wdt) throw std::runtime_error("EINTERNAL: shared/routed expert dtype mismatch");
        a.Is = d.s_d.K; a.sWgu = d.s_gu.W; a.sWd = d.s_d.W; a.hs = wsf("s_shh", (size_t)B * a.Is);
    }
    a.softmax_scoring = L.scoring == "softmax"; a.norm_topk = L.norm_topk; a.scaling = L.routed_scaling;
    a.xn = wsf("s_xn", (size_t)B * H);
    a.xn_router = wsf("s_xn_router", (size_t)B * H);
    a.logits = wsf("s_log", (size_t)B * E);
    a.ids = wsi("s_ids", TK); a.wts = wsf("s_wts", TK);
    a.h = wsf("s_ehh", (size_t)TK * I);
    a.grp = wsi("s_grp", moe_grp_ints(E, B, K));
    a.route_cnt = wsi("s_route_cnt", 16);
    if (B >= 3 && B <= 8) {  // matrix-core grouped kernels: down partials + tickets
        a.dn_part = wsf("s_dnpart", moe_down_mm_part_floats(E, B, K, I, a.Is, H));
        a.dn_tick = wsi("s_dntick", (size_t)H / 64 + 1);  // one ticket per 64-row tile
    }
    if (B <= 8 && d.e_gu_swz && (!d.has_shared || d.s_gu_swz)) {  // fragment-ordered experts
        a.Wgu_swz = d.e_gu_swz; a.Wd_swz = d.e_d_swz; a.sWgu_swz = d.s_gu_swz; a.sWd_swz = d.s_d_swz;
        if (!router_swz_off()) a.router_swz = d.router_swz;
    }
    if (B > 8) {
        a.eoff = wsi("s_eoff", E + 1); a.arow = wsi("s_arow", TK); a.apos = wsi("s_apos", TK);
        a.aw = wsf("s_aw", TK); a.active = wsi("s_active", E); a.n_active = wsi("s_nact", 1);
    }
    return a;
}

bool Engine::persist_ok(int B, int Lmax) {
    // opt-in (DSOCR_PERSIST=1, read per generate): measured slower than the per-layer launch chain on MI355X
    // (43.5 vs 33.5 us per layer), kept as the A/B of the persistent-layer design
    const char* e = getenv("DSOCR_PERSIST");
    if (!e || atoi(e) == 0) return false;
    const LangConfig& L = cfg_.lang;
    if (B != 1 || L.use_mla || L.rope_dim != L.head_dim || L.v_head_dim != L.head_dim || L.n_shared <= 0 ||
        L.topk_method != "greedy" || L.hidden_act != "silu")
        return false;
    if (!dec_persist_shape_ok(L.hidden, L.heads, L.kv_heads, L.head_dim, L.n_routed, L.topk, L.moe_inter,
                              L.n_shared * L.moe_inter, L.inter, Lmax))
        return false;
    for (const DecLayer& d : layers_) {
        if (d.qkv.wdt != WDT_F16 || d.qkv.b || d.o.wdt != WDT_F16 || d.o.b) return false;
        if (d.moe) {
            if (!d.router.W || d.router.wdt != WDT_F16 || d.e_wdt != WDT_F16 || !d.has_shared || d.s_gu.wdt != WDT_F16 ||
                d.s_d.wdt != WDT_F16 || d.s_gu.b || d.s_d.b)
                return false;
        } else if (!d.gu.W || d.gu.wdt != WDT_F16 || d.down.wdt != WDT_F16) {
            return false;
        }
    }
    return dec_persist_resident() != 0;
}

// the persistent decode's weight table: every down projection transposed to [inter][H] (split-K rows), the
// per-layer pointer table on the device, the granule buffer (made once, outside any capture)
void Engine::ensure_persist() {
    if (persist_lw_ || capturing_) return;
    const LangConfig& L = cfg_.lang;
    const int H = L.hidden, E = L.n_routed, I = L.moe_inter;
    std::vector<PersistLayerW> tab(layers_.size());
    for (size_t l = 0; l < layers_.size(); ++l) {
        DecLayer& d = layers_[l];
        PersistLayerW& w = tab[l];
        w.qkv = (const uint16_t*)d.qkv.W;
        w.o = (const uint16_t*)d.o.W;
        w.in_w = d.in_norm.w;
        w.post_w = d.post_norm.w;
        w.moe = d.moe ? 1 : 0;
        if (d.moe) {
            if (!d.e_dT) {
                d.e_dT = dev_alloc((size_t)E * I * H * 2);
                for (int e = 0; e < E; ++e)
                    launch_transpose16((const uint16_t*)d.e_d + (size_t)e * H * I, (uint16_t*)d.e_dT + (size_t)e * I * H, H, I,
                                       stream_);
            }
            const int Is = d.s_d.K;
            if (!d.s_dT) {
                d.s_dT = dev_alloc((size_t)Is * H * 2);
                launch_transpose16(d.s_d.W, d.s_dT, H, Is, stream_);
            }
            w.router = (const uint16_t*)d.router.W;
            w.router_bias = d.router.b;
            w.e_gu = (const uint16_t*)d.e_gu;
            w.e_dT = (const uint16_t*)d.e_dT;
            w.s_gu = (const uint16_t*)d.s_gu.W;
            w.s_dT = (const uint16_t*)d.s_dT;
            w.inter = Is;
        } else {
            if (!d.s_dT) {
                d.s_dT = dev_alloc((size_t)L.inter * H * 2);
                launch_transpose16(d.down.W, d.s_dT, H, L.inter, stream_);
            }
            w.s_gu = (const uint16_t*)d.gu.W;
            w.s_dT = (const uint16_t*)d.s_dT;
            w.inter = L.inter;
        }
    }
    PersistLayerW* dtab = (PersistLayerW*)dev_alloc(tab.size() * sizeof(PersistLayerW));
    HIP_CHECK(hipMemcpyAsync(dtab, tab.data(), tab.size() * sizeof(PersistLayerW), hipMemcpyHostToDevice, stream_));
    persist_g_ = (unsigned long long*)dev_alloc(dec_persist_granules(L.layers) * 8);
    HIP_CHECK(hipStreamSynchronize(stream_));
    persist_lw_ = dtab;
}

// the dense MLP's matrix-core form at 3..8 pages (decode_mm.hip): q/k/v-sized K for gate|up, K % 64 for down
bool Engine::dense_mm_ok(const DecLayer& d, int B) const {
    const LangConfig& L = cfg_.lang;
    DecGemvArgs g1;
    g1.M = B; g1.N = 2 * L.inter; g1.K = L.hidden; g1.ldw = L.hidden;
    DecGemvArgs g2;
    g2.M = B; g2.N = L.hidden; g2.K = L.inter; g2.ldw = L.inter; g2.ldx = L.inter;
    return d.gu.W && d.down.W && dec_mm_ok(g1) && dec_mm_splitk_ok(g2);
}

void Engine::decode_step(int B, int Lmax) {
    // One token for each of B pages: 8 launches per layer (decode.hip).  For B <= 2 the
    // RMSNorms are fused into the consuming GEMV / expert kernels (x normalised on the fly).
    const LangConfig& L = cfg_.lang;
    hipStream_t st = stream_;
    const int H = L.hidden, hd = L.head_dim;
    const bool fuse_norm = B <= 2;
    float* X = wsf("s_x", (size_t)B * H);
    float* XN = wsf("s_xn", (size_t)B * H);
    int* kv_pos = wsi("s_kvpos", B);
    float* CTX = wsf("s_ctx", (size_t)B * H);
    float* part = wsf("s_part", dec_attn_workspace(B, L.heads, hd, Lmax) / 4 + 16);
    if (L.heads % L.kv_heads) throw std::runtime_error("EINVAL: num_attention_heads must be a multiple of num_key_value_heads");
    int* err = wsi("s_err", 4);
    if (B == 1 && persist_active_ && !step_skip_ && !span_rec_) {
        // every layer of the step in one persistent launch (decode_persist.hip)
        DecPersistArgs pa;
        pa.layers = L.layers; pa.lw = persist_lw_; pa.x = X; pa.kv_pos = kv_pos;
        pa.cos = rope_cos_; pa.sin = rope_sin_; pa.kc = kc_; pa.vc = vc_;
        pa.layer_kv = (long)B * page_stride_; pa.head_stride = head_stride_;
        pa.scale = (float)(1.0 / std::sqrt((double)hd)); pa.eps = L.rms_eps;
        pa.softmax_scoring = L.scoring == "softmax"; pa.norm_topk = L.norm_topk; pa.scaling = L.routed_scaling;
        pa.g = persist_g_; pa.err = err;
        if (persist_stamp_mode_ && !persist_ev_.empty() && persist_stamps_) {
            pa.stamps = persist_stamps_;
            pa.stamp_pos0 = persist_stamp_pos0_;
            pa.stamp_cap = persist_stamp_cap_;
            // the launch's own dispatch begin / end (hipExtLaunchKernelGGL events: what rocprofv3's kernel trace
            // reports); the timed generate runs its steps eagerly (events on a dispatch packet cannot be captured)
            prof_events() = ProfEvents{persist_ev_[0], persist_ev_[1]};
            launch_dec_persist(pa, st);
            prof_events() = ProfEvents();
        } else {
            launch_dec_persist(pa, st);
        }
        return;
    }
    // launch spans (set_spans): HIP events on the stream around the launch (dispatch-level duration,
    // what rocprofv3's kernel trace reports) + the in-kernel wave span folded right after it
    auto stamped = [&](int kind, int l, const std::function<void()>& launch, const int* ids, int n_ids) {
        if (!span_rec_ || chain_active_) {  // (chain spans: the launch carries its own slot region)
            launch();
            return;
        }
        hipEvent_t* ev = &span_ev_[((size_t)kind * L.layers + l) * 2];
        const bool events = (span_mode_ & SPAN_EVENTS) != 0, waves = (span_mode_ & SPAN_WAVES) != 0;
        if (events) HIP_CHECK(hipEventRecord(ev[0], st));
        launch();
        if (events) HIP_CHECK(hipEventRecord(ev[1], st));
        // the fold (wave span + the launch's distinct experts): after every launch with wave spans only; an
        // events-only generate runs no extra kernel, so its step is the production chain plus the event
        // markers (bench.py prices its launches with the expert counts of a wave-span generate of the same batch)
        if (waves) launch_span_reduce(span_slots_, span_rec(kind, l), span_step_, span_cap_, ids, n_ids, st);
    };
    for (int l = 0; l < L.layers; ++l) {
        DecLayer& d = layers_[l];
        const int QKVN = d.qkv.N;
        float* QKV = wsf("s_qkv", (size_t)B * QKVN);
        const long layer_kv = (long)B * page_stride_;
        // attention: [norm] qkv -> rope + append + flash-decoding -> o_proj + residual
        DecAttn2Args da;
        da.qkv = QKV; da.ld = QKVN; da.kv_pos = kv_pos; da.B = B; da.heads = L.heads; da.kv_heads = L.kv_heads;
        da.hd = hd; da.rope_dim = L.rope_dim; da.use_mla = L.use_mla; da.max_len = Lmax;
        da.cos = rope_cos_; da.sin = rope_sin_;
        da.kc = kc_ + (long)l * layer_kv; da.vc = vc_ + (long)l * layer_kv;
        da.page_stride = page_stride_; da.head_stride = head_stride_;
        da.scale = (float)(1.0 / std::sqrt((double)hd)); da.part = part; da.o = CTX; da.o_ld = H;
        da.counters = wsi("s_attn_cnt", (size_t)B * L.heads);
        da.err = err;
        da.kv_delay = att_kv_delay();
        da.span = chain_active_ ? chain_slots(l, SPAN_ATTN) : ((span_rec_ && (span_mode_ & SPAN_WAVES)) ? span_slots_ : nullptr);
        // q/k/v projection with the input RMSNorm fused; one page: RoPE in the projection's epilogue, so the
        // attention reads q / k already rotated (B <= 2: the row block-staged; 3..8: dec_gemv_lds / dec_mm)
        DecGemvArgs g;
        g.M = B; g.N = QKVN; g.K = H; g.W = d.qkv.W; g.ldw = H; g.wdtype = d.qkv.wdt; g.bias = d.qkv.b;
        g.y = QKV; g.ldy = QKVN; g.x = X; g.ldx = H; g.norm_w = d.in_norm.w; g.eps = L.rms_eps;
        bool attn_done = false;
        if (B == 1 && !L.use_mla && L.rope_dim == hd) {
            DecRopeEpi re;
            re.kv_pos = kv_pos; re.cos = rope_cos_; re.sin = rope_sin_; re.hd = hd;
            re.rot_rows = (L.heads + L.kv_heads) * hd;
            da.prerot = 1;
            if (qkv_attn_fused() && dec_qkv_attn_ok(g, re, da)) {
                // one launch: the attention blocks stream their K / V chunk beside the projection
                // (s_qkv stays sentinel-filled between launches; SKIP_ATTN, the profile's variant without
                // attention, projects into a scratch row so the hand-off row keeps its sentinels)
                if (step_skip_ & SKIP_ATTN) {
                    g.y = wsf("p_qkv_skip", (size_t)QKVN);
                    launch_dec_qkv_rope(g, re, st);
                } else {
                    stamped(SPAN_ATTN, l, [&] { launch_dec_qkv_attn(g, re, da, st); }, nullptr, 0);
                }
                attn_done = true;
            } else {
                launch_dec_qkv_rope(g, re, st);
            }
        } else if (B <= 8) {
            if (B >= 3 && !mm_swz_off()) g.w_swz = d.qkv_swz;
            launch_dec_gemv(g, st);
        } else {
            launch_rmsnorm(X, H, XN, H, B, H, d.in_norm.w, L.rms_eps, st);
            g.x = XN; g.norm_w = nullptr;
            launch_dec_gemv(g, st);
        }
        if (!attn_done && !(step_skip_ & SKIP_ATTN)) stamped(SPAN_ATTN, l, [&] { launch_dec_attn(da, st); }, nullptr, 0);
        // o_proj + residual
        DecGemvArgs go;
        go.M = B; go.N = H; go.K = L.heads * hd; go.x = CTX; go.ldx = H; go.W = d.o.W; go.ldw = go.K;
        go.wdtype = d.o.wdt; go.bias = d.o.b; go.y = X; go.ldy = H; go.accumulate = 1; go.span = chain_slots(l, SPAN_OPROJ);
        if (B >= 3 && B <= 8 && !mm_swz_off()) go.w_swz = d.o_swz;
        launch_dec_gemv(go, st);
        // MLP / MoE
        if (!d.moe && B >= 3 && B <= 8 && dense_mm_ok(d, B)) {
            // dense MLP (layer 0) on the matrix cores: gate|up with the post-attention RMSNorm fused,
            // SwiGLU, down as a split-K launch accumulating into the residual
            const int I = L.inter;
            float* G = wsf("s_dg", (size_t)B * 2 * I);
            float* HH = wsf("s_dhh", (size_t)B * I);
            DecGemvArgs g1;
            g1.M = B; g1.N = 2 * I; g1.K = H; g1.x = X; g1.ldx = H; g1.norm_w = d.post_norm.w; g1.eps = L.rms_eps;
            g1.W = d.gu.W; g1.ldw = H; g1.wdtype = d.gu.wdt; g1.bias = d.gu.b; g1.y = G; g1.ldy = 2 * I;
            if (!mm_swz_off()) g1.w_swz = d.gu_swz;
            launch_dec_gemv(g1, st);
            launch_silu_mul(G, 2 * I, I, B, HH, I, st);
            DecGemvArgs g2;
            g2.M = B; g2.N = H; g2.K = I; g2.x = HH; g2.ldx = I; g2.W = d.down.W; g2.ldw = I; g2.wdtype = d.down.wdt;
            g2.bias = d.down.b; g2.y = X; g2.ldy = H; g2.accumulate = 1;
            launch_dec_mm_splitk(g2, wsf("s_dpart", dec_mm_splitk_part_floats(H, I)), wsi("s_dtick", dec_mm_splitk_ticks(H)), st);
            continue;
        }
        if (!d.moe) {
            const float* mx = X;
            const float* mnorm = d.post_norm.w;
            if (!fuse_norm) { launch_rmsnorm(X, H, XN, H, B, H, d.post_norm.w, L.rms_eps, st); mx = XN; mnorm = nullptr; }
            MoeDec2Args m;
            m.T = B; m.K = H; m.Hout = H; m.x = mx; m.norm_w = mnorm; m.eps = L.rms_eps; m.out = X;
            m.topk = 0; m.E = 0; m.slots = 0; m.I = 8; m.Is = L.inter;
            m.sWgu = d.gu.W; m.sWd = d.down.W; m.wdtype = d.gu.wdt;
            m.hs = wsf("s_hh", (size_t)B * L.inter);
            m.n_active = wsi("s_nact", 1);
            launch_moe_gateup2(m, st);
            // one page: the down projection split over the 8 waves of a block (moe_down_mix; all of K in flight
            // at once) — moe_down2 walks each 6848-long row in four dependent load rounds
            MoeDec2Args dn = m;
            dn.slot_mode = 1;
            dn.ids = wsi("s_dense_ids", 8);  // no routed segments at topk 0: moe_down_mix reads no id
            if (dn.topk != 0) throw std::logic_error("dense layer with routed experts");
            if (B == 1 && moe_down_mix_ok(dn)) launch_moe_down_mix(dn, st);
            else launch_moe_down2(m, st);
            continue;
        }
        if (!span_rec_) {
            const int parts = MOE_ROUTE | ((step_skip_ & SKIP_GATEUP) ? 0 : MOE_GATEUP) | ((step_skip_ & SKIP_DOWN) ? 0 : MOE_DOWN);
            launch_moe_decode(moe_args(l, B, X), st, parts);
            continue;
        }
        MoeDecodeArgs ma = moe_args(l, B, X);
        ma.route_span = chain_slots(l, SPAN_ROUTER);
        launch_moe_decode(ma, st, MOE_ROUTE);
        ma.span = chain_active_ ? chain_slots(l, SPAN_GATEUP) : ((span_mode_ & SPAN_WAVES) ? span_slots_ : nullptr);
        stamped(SPAN_GATEUP, l, [&] { launch_moe_decode(ma, st, MOE_GATEUP); }, ma.ids, B * ma.topk);
        if (chain_active_) ma.span = chain_slots(l, SPAN_DOWN);
        stamped(SPAN_DOWN, l, [&] { launch_moe_decode(ma, st, MOE_DOWN); }, ma.ids, B * ma.topk);
    }
}

// the screened head's launch arguments for B rows of s_x (workspaces allocated here: call before a graph
// capture): B <= 2 the single-token kernel per page, 3..8 one int8 stream on the matrix cores
LmHeadQ8Args Engine::head_q8_args(int B) {
    const LangConfig& L = cfg_.lang;
    const int H = L.hidden;
    LmHeadQ8Args q;
    q.x = wsf("s_x", (size_t)B * H); q.ldx = H; q.norm_w = final_norm_; q.eps = L.rms_eps;
    q.q = lmq_; q.scale = lmq_scale_; q.bound = lmq_bound_; q.B = B; q.N = L.vocab; q.K = H;
    if (B >= 3) {
        q.qfrag = lmq_frag_; q.qnorm = lmq_qnorm_;
        lmhead_q8mm_grid(L.vocab, H, B, &q.nblk, &q.slot);
    } else {
        lmhead_q8_grid(L.vocab, H, B, &q.nblk, &q.slot);
    }
    q.blk_cnt = wsi("s_blkcnt", (size_t)B * q.nblk); q.blk_t = wsf("s_blkt", (size_t)B * q.nblk);
    q.cand = wsi("s_cand", (size_t)B * q.nblk * q.slot); q.cand_hi = wsf("s_candhi", (size_t)B * q.nblk * q.slot);
    q.xn_out = wsf("s_lmxn", (size_t)B * H);
    return q;
}

void Engine::reserve_head_ws(int B) {
    if (!lmq_ || B > 8 || (B >= 3 && !lmq_frag_)) return;
    (void)head_q8_args(B);
}

// 3..8 pages: fragment-ordered copies of the lm_head and of every MoE layer's experts for the
// matrix-core kernels (decode_mm.hip: every wave weight load one contiguous 1 KiB block; lm_head 6.0 vs
// 4.6 TB/s row-major on MI355X, tools/kbench lm8), made once, outside any capture (HBM: + vocab x hidden
// + the expert weights again, ~5.3 GB of the 288)
void Engine::ensure_mm_weights(int B) {
    if (B > 8 || capturing_) return;
    const LangConfig& L = cfg_.lang;
    if (B >= 3 && !lm_swz_) {
        DecGemvArgs g;
        g.M = B; g.N = L.vocab; g.K = L.hidden; g.ldw = L.hidden;
        if (dec_mm_ok(g)) {
            lm_swz_ = dev_alloc(mm_swizzle_elems(L.vocab, L.hidden) * 2);
            launch_mm_swizzle(lm_head_.W, L.vocab, L.hidden, lm_swz_, stream_);
        }
    }
    // the experts of every MoE layer (routed [E * 2I][H], [E * H][I]; shared [2Is][H], [H][Is]): the
    // grouped matrix-core kernels stream them (3..8 pages)
    const int H = L.hidden, E = L.n_routed, I = L.moe_inter;
    if (B < 3) return;
    // q/k/v, o_proj and the dense gate|up for dec_mm (each wave load one contiguous 1 KiB instead of 64 bytes of
    // 16 rows: tools/mb_bcast.hip)
    auto swz = [&](const Lin& w, void*& out) {
        DecGemvArgs g;
        g.M = B; g.N = w.N; g.K = w.K; g.ldw = w.K;
        if (out || !w.W || (w.wdt != WDT_F16 && w.wdt != WDT_BF16) || !dec_mm_ok(g)) return;
        out = dev_alloc(mm_swizzle_elems(w.N, w.K) * 2);
        launch_mm_swizzle(w.W, w.N, w.K, out, stream_);
    };
    for (DecLayer& d : layers_) {
        swz(d.qkv, d.qkv_swz);
        swz(d.o, d.o_swz);
        if (!d.moe) swz(d.gu, d.gu_swz);
    }
    for (DecLayer& d : layers_) {
        if (!d.moe || d.e_gu_swz || d.e_wdt != WDT_F16 || H % 32 || I % 32) continue;
        d.e_gu_swz = dev_alloc(mm_swizzle_elems(E * 2 * I, H) * 2);
        launch_mm_swizzle(d.e_gu, E * 2 * I, H, d.e_gu_swz, stream_);
        d.e_d_swz = dev_alloc(mm_swizzle_elems(E * H, I) * 2);
        launch_mm_swizzle(d.e_d, E * H, I, d.e_d_swz, stream_);
        if (d.has_shared && d.s_gu.wdt == WDT_F16) {
            const int Is = d.s_d.K;
            d.s_gu_swz = dev_alloc(mm_swizzle_elems(2 * Is, H) * 2);
            launch_mm_swizzle(d.s_gu.W, 2 * Is, H, d.s_gu_swz, stream_);
            d.s_d_swz = dev_alloc(mm_swizzle_elems(H, Is) * 2);
            launch_mm_swizzle(d.s_d.W, H, Is, d.s_d_swz, stream_);
        }
        if (d.router.W && d.router.wdt == WDT_F16 && E % 16 == 0) {
            d.router_swz = dev_alloc(mm_swizzle_elems(E, H) * 2);
            launch_mm_swizzle(d.router.W, E, H, d.router_swz, stream_);
        }
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
}

// one page: q/k/v projection + decode attention as one launch (dec_qkv_attn); DSOCR_QKV_ATTN=0 (A/B
// switch, read once) keeps the two launches
// the fused launch's K / V loads held back behind the projection's weight stream: 150 ticks (1.5 us) from the
// attention block's entry (tools/kbench qkvattn1 sweep 0..300: 12.99 -> 12.49 us at L 1217, 11.36 -> 10.88 at
// L 707; decode layers 417.9 -> 411.6 us per step).  DSOCR_ATT_KV_DELAY (ticks of 10 ns) overrides; 0 = off
int Engine::att_kv_delay() {
    const char* e = getenv("DSOCR_ATT_KV_DELAY");
    return e ? std::max(0, atoi(e)) : 150;
}

bool Engine::qkv_attn_fused() {
    static const bool v = !(getenv("DSOCR_QKV_ATTN") && atoi(getenv("DSOCR_QKV_ATTN")) == 0);
    return v;
}

// screened selection applies (lmhead.hip): int8 copy present, B <= 8 (3..8: the matrix-core form), no
// repetition penalty
// (DSOCR_SCREEN=0 forces the exact lm_head; read per generate call)
bool Engine::screen_applies(int B, float rep_penalty) const {
    if (getenv("DSOCR_SCREEN") && atoi(getenv("DSOCR_SCREEN")) == 0) return false;
    const bool pen = rep_penalty > 0.f && fabsf(rep_penalty - 1.0f) > 1.1920929e-07f;
    return lmq_ && !pen && (B <= 2 || (B <= 8 && lmq_frag_ && lmhead_q8mm_ok(B, cfg_.lang.vocab, cfg_.lang.hidden)));
}

// final norm + lm_head + greedy selection + step bookkeeping for the B decode rows in s_x
void Engine::decode_head(int B, DecSampleArgs& sa, const SampleArgs& pen) {
    const LangConfig& L = cfg_.lang;
    hipStream_t st = stream_;
    const int H = L.hidden;
    float* SX = wsf("s_x", (size_t)B * H);
    if (sa.ban_out) {
        // screened selection: int8 lm_head intervals + running threshold, exact rescoring of the
        // few kept rows — the exact path's token from half the lm_head bytes
        LmHeadQ8Args q = head_q8_args(B);
        q.ban = sa.ban_out; q.ban_ld = sa.ban_ld;
        launch_lmhead_q8(q, st);
        DecSampleArgs ss = sa;
        ss.blk_cnt = q.blk_cnt; ss.blk_t = q.blk_t; ss.cand = q.cand; ss.cand_hi = q.cand_hi; ss.nblk = q.nblk; ss.slot = q.slot;
        ss.w_exact = lm_head_.W; ss.w_exact_wdt = lm_head_.wdt; ss.xn = q.xn_out; ss.K = H;
        if (getenv("DSOCR_SCREEN_STATS")) ss.stats = reinterpret_cast<unsigned long long*>(wsi("s_scrstats", 32));
        launch_dec_sample(ss, st);
        return;
    }
    DecGemvArgs g;
    g.M = B; g.N = L.vocab; g.K = H; g.W = lm_head_.W; g.ldw = H; g.wdtype = lm_head_.wdt; g.bias = lm_head_.b;
    g.y = const_cast<float*>(sa.logits); g.ldy = L.vocab;
    if (B <= 2 || (lm_swz_ && B <= 8)) {  // final RMSNorm fused (B 3..8: dec_mm on the fragment-ordered copy)
        g.x = SX; g.ldx = H; g.norm_w = final_norm_; g.eps = L.rms_eps;
        if (B > 2) g.w_swz = lm_swz_;
    } else {
        float* SXN = wsf("s_xn", (size_t)B * H);
        launch_rmsnorm(SX, H, SXN, H, B, H, final_norm_, L.rms_eps, st);
        g.x = SXN; g.ldx = H;
    }
    launch_dec_gemv(g, st);
    if (trace_) launch_trace_logits(sa.logits, B, L.vocab, sa.ld, sa.out_len, sa.done, trace_, trace_steps_, st);
    launch_rep_penalty(pen, st);
    launch_dec_sample(sa, st);
}

// rand_core 0.6.4 SeedableRng::seed_from_u64 for ChaCha12Rng (rand 0.8.5 StdRng): the 32-byte key
// is filled by PCG32 (state advanced first, XSH-RR output, little-endian words); block counter 0,
// stream 0, empty result buffer (sampling.hip reads this layout)
std::vector<uint32_t> rng_state_from_u64(uint64_t state) {
    std::vector<uint32_t> st(RNG_WORDS, 0u);
    for (int i = 0; i < 8; ++i) {
        state = state * 6364136223846793005ull + 11634580027462260723ull;
        const uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
        const uint32_t rot = (uint32_t)(state >> 59);
        st[RNG_KEY + i] = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    }
    st[RNG_IDX] = 64;
    return st;
}

// ============================================================================ generate
std::vector<std::vector<int64_t>> Engine::generate(const std::vector<GenRequest>& reqs, const GenParams& p, TokenCb cb,
                                                   void* user) {
    using clock = std::chrono::steady_clock;
    const LangConfig& L = cfg_.lang;
    const int B = (int)reqs.size();
    const int H = L.hidden;
    timings_ = Timings();
    timings_.pages = B;
    std::vector<std::vector<int64_t>> out(B);
    if (B == 0) return out;
    if (p.max_new == 0) return out;
    ensure_small(std::max(B, 64));
    hipStream_t st = stream_;
    hipEvent_t ev[6];
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    auto t0 = clock::now();
    HIP_CHECK(hipEventRecord(ev[0], st));
    flops_acc_ = 0;

    // ---------------- 1. vision (compute_image_embeddings, batched over pages)
    std::vector<int> prompt_len(B);
    int max_p = 0;
    long T = 0;
    for (int b = 0; b < B; ++b) {
        prompt_len[b] = (int)reqs[b].ids.size();
        if (prompt_len[b] == 0) throw std::runtime_error("EINVAL: empty prompt");
        max_p = std::max(max_p, prompt_len[b]);
        T += prompt_len[b];
    }
    // group pages by global/tile size
    std::map<int, std::vector<int>> gsz, tsz;
    for (int b = 0; b < B; ++b)
        if (reqs[b].page) {
            gsz[reqs[b].page->gsize].push_back(b);
            if (reqs[b].page->n_tiles > 0) tsz[reqs[b].page->tile].push_back(b);
        }
    // per page: device pointers of global post rows and local post rows
    std::vector<const float*> gpost(B, nullptr), lpost(B, nullptr);
    std::vector<float*> pass_outputs;
    int pass_id = 0;
    // pixels of one size group as one contiguous device batch: device-to-device gathers of
    // HBM-resident pages (dsocr_page_to_device / dsocr_prepare_page_device), host uploads otherwise
    auto gather = [&](const std::vector<int>& pages, bool tiles, size_t n_floats) -> float* {
        const std::string name = "g_img" + std::to_string(pass_id);
        float* d = wsf(name, n_floats);
        size_t off = 0;
        bool host_copy = false;
        for (int b : pages) {
            const PagePixels& pg = *reqs[b].page;
            const size_t nf = tiles ? (size_t)pg.n_tiles * 3 * pg.tile * pg.tile : (size_t)3 * pg.gsize * pg.gsize;
            const float* dev = tiles ? pg.tiles_dev : pg.global_dev;
            const std::vector<float>& host = tiles ? pg.tiles_chw : pg.global_chw;
            if (dev && pg.dev_ordinal == device_)
                HIP_CHECK(hipMemcpyAsync(d + off, dev, nf * 4, hipMemcpyDeviceToDevice, st));
            else if (host.size() == nf) {
                HIP_CHECK(hipMemcpyAsync(d + off, host.data(), nf * 4, hipMemcpyHostToDevice, st));
                host_copy = true;
            }
            else
                throw std::runtime_error("EINVAL: page pixels live on another device");
            off += nf;
        }
        if (off != n_floats) throw std::runtime_error("EINTERNAL: pixel batch size mismatch");
        if (host_copy) HIP_CHECK(hipStreamSynchronize(st));  // host sources may be pageable temporaries
        return d;
    };
    // every pixel batch gathered first, then the passes: odd passes on the second vision stream
    // (DSOCR_VIS_STREAMS=0: all on one stream), joined before the image rows are assembled
    std::vector<float*> g_img, t_img;
    std::vector<int> t_n;
    for (auto& kv : gsz) {
        const int S = kv.first;
        g_img.push_back(gather(kv.second, false, kv.second.size() * 3 * (size_t)S * S));
        ++pass_id;
    }
    for (auto& kv : tsz) {
        const int S = kv.first;
        int n = 0;
        for (int b : kv.second) n += reqs[b].page->n_tiles;
        t_img.push_back(gather(kv.second, true, (size_t)n * 3 * S * S));
        t_n.push_back(n);
        ++pass_id;
    }
    const bool two = vis_streams_on() && gsz.size() + tsz.size() >= 2;
    if (two && !vstream_) {
        HIP_CHECK(hipStreamCreateWithFlags(&vstream_, hipStreamNonBlocking));
        for (auto& e : vis_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (two) {
        HIP_CHECK(hipEventRecord(vis_ev_[0], st));  // pixels gathered
        HIP_CHECK(hipStreamWaitEvent(vstream_, vis_ev_[0], 0));
    }
    int vis_k = 0;
    bool side = false;
    auto run_pass = [&](float* dimg, int n, int S) -> float* {
        const std::string name = "vis_out" + std::to_string(vis_k);
        if (!two || (vis_k++ & 1) == 0) return vision_pass(dimg, n, S, name);
        std::swap(stream_, vstream_);
        ws_prefix_ = "vs1_";
        float* r = nullptr;
        try {
            r = vision_pass(dimg, n, S, name);
        } catch (...) {
            std::swap(stream_, vstream_);
            ws_prefix_.clear();
            throw;
        }
        std::swap(stream_, vstream_);
        ws_prefix_.clear();
        side = true;
        return r;
    };
    {
        size_t gi = 0;
        for (auto& kv : gsz) {
            const int S = kv.first;
            float* post = run_pass(g_img[gi++], (int)kv.second.size(), S);
            const int Sq = (S / 64) * (S / 64);
            for (size_t i = 0; i < kv.second.size(); ++i) gpost[kv.second[i]] = post + (size_t)i * Sq * H;
        }
        size_t ti = 0;
        for (auto& kv : tsz) {
            const int S = kv.first;
            float* post = run_pass(t_img[ti], t_n[ti], S);
            ++ti;
            const int Sq = (S / 64) * (S / 64);
            size_t off = 0;
            for (int b : kv.second) {
                lpost[b] = post + off * Sq * H;
                off += reqs[b].page->n_tiles;
            }
        }
    }
    if (side) {
        HIP_CHECK(hipEventRecord(vis_ev_[1], vstream_));
        HIP_CHECK(hipStreamWaitEvent(st, vis_ev_[1], 0));
    }
    HIP_CHECK(hipEventRecord(ev[1], st));
    timings_.vision_flops = flops_acc_;

    // ---------------- 2. image rows for the injection (model/mod.rs:1208-1239)
    // host image rows of all pages concatenated (kind 1), device vision rows via per-row pointers:
    // we copy them into one contiguous device buffer per kind to keep the assemble kernel simple.
    std::vector<float> host_rows;
    std::vector<long> host_row_base(B, 0);
    for (int b = 0; b < B; ++b)
        if (!reqs[b].page && reqs[b].image_rows) {
            host_row_base[b] = (long)(host_rows.size() / H);
            host_rows.insert(host_rows.end(), reqs[b].image_rows, reqs[b].image_rows + reqs[b].n_image_rows * H);
        }
    // device vision rows are gathered via srcB = one buffer holding every page's [local | global] post rows
    long vis_rows_total = 0;
    std::vector<long> vis_base(B, 0), vis_local_rows(B, 0), vis_global_rows(B, 0);
    for (int b = 0; b < B; ++b)
        if (reqs[b].page) {
            const PagePixels* pg = reqs[b].page;
            vis_base[b] = vis_rows_total;
            vis_local_rows[b] = (long)pg->n_tiles * (pg->tile / 64) * (pg->tile / 64);
            vis_global_rows[b] = (long)(pg->gsize / 64) * (pg->gsize / 64);
            vis_rows_total += vis_local_rows[b] + vis_global_rows[b];
        }
    float* vis_rows = wsf("g_visrows", (size_t)std::max<long>(vis_rows_total, 1) * H);
    for (int b = 0; b < B; ++b)
        if (reqs[b].page) {
            if (vis_local_rows[b])
                HIP_CHECK(hipMemcpyAsync(vis_rows + vis_base[b] * H, lpost[b], vis_local_rows[b] * H * 4,
                                         hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(vis_rows + (vis_base[b] + vis_local_rows[b]) * H, gpost[b],
                                     vis_global_rows[b] * H * 4, hipMemcpyDeviceToDevice, st));
        }
    // image-row sequence of every page (format_local_tokens / format_global_tokens /
    // assemble_artifacts order, model/mod.rs:656-709,879-923): (kind, index) per <image> slot
    std::vector<std::vector<std::pair<int, long>>> img(B);
    for (int b = 0; b < B; ++b) {
        const GenRequest& rq = reqs[b];
        if (rq.page) {
            const PagePixels* pg = rq.page;
            if (pg->n_tiles > 0) {
                const int ls = pg->tile / 64;
                for (int R = 0; R < pg->crop_h * ls; ++R) {
                    for (int Cc = 0; Cc < pg->crop_w * ls; ++Cc) {
                        int crop = (R / ls) * pg->crop_w + (Cc / ls);
                        img[b].push_back({2, vis_base[b] + ((long)crop * ls + R % ls) * ls + Cc % ls});
                    }
                    img[b].push_back({3, 0});
                }
            }
            const int gs = pg->gsize / 64;
            for (int R = 0; R < gs; ++R) {
                for (int Cc = 0; Cc < gs; ++Cc) img[b].push_back({2, vis_base[b] + vis_local_rows[b] + (long)R * gs + Cc});
                img[b].push_back({3, 0});
            }
            img[b].push_back({4, 0});
        } else if (rq.image_rows) {
            for (size_t i = 0; i < rq.n_image_rows; ++i) img[b].push_back({1, host_row_base[b] + (long)i});
        }
        size_t n_mask = 0;
        for (int i = 0; i < prompt_len[b]; ++i) n_mask += (!rq.mask.empty() && rq.mask[i]) ? 1 : 0;
        if (n_mask != img[b].size())
            throw std::runtime_error("EINVAL: prompt/image embedding mismatch: image embeddings provide " +
                                     std::to_string(img[b].size()) + " tokens but mask requires " + std::to_string(n_mask));
        for (int i = 0; i < prompt_len[b]; ++i)
            if ((rq.mask.empty() || !rq.mask[i]) && (rq.ids[i] < 0 || rq.ids[i] >= L.vocab))
                throw std::runtime_error("EINVAL: token id out of bounds for vocab size");
    }
    const int Lmax = max_p + (int)p.max_new + 1;
    ensure_rope(Lmax + 1);
    // KV cache [layers][B][kvh][Lmax][hd] f32 (block.rs:776-789 keeps the cache in f32)
    head_stride_ = (long)Lmax * L.head_dim;
    page_stride_ = (long)L.kv_heads * head_stride_;
    const size_t kv_need = (size_t)L.layers * B * page_stride_ * 4;
    kc_ = wsf("kv_k", kv_need / 4);
    vc_ = wsf("kv_v", kv_need / 4);
    // arrival tickets of the decode-attention combine: zero here, every launch leaves them zero
    HIP_CHECK(hipMemsetAsync(wsi("s_attn_cnt", (size_t)B * L.heads), 0, sizeof(int) * B * L.heads, st));
    HIP_CHECK(hipMemsetAsync(wsi("s_route_cnt", 16), 0, sizeof(int) * 16, st));
    HIP_CHECK(hipMemsetAsync(wsi("s_dntick", (size_t)H / 64 + 1), 0, sizeof(int) * (H / 64 + 1), st));
    {  // decode attention records: sentinel-filled before the first launch (the polling merge refills them)
        const size_t pf = dec_attn_workspace(B, L.heads, L.head_dim, Lmax) / 4 + 16;
        dec_attn_part_init(wsf("s_part", pf), pf * 4, st);
        // the fused q/k/v + attention launch (one page) takes q / k / v by polling this row: sentinel-filled
        const size_t qn = (size_t)B * layers_[0].qkv.N;
        dec_qkv_sentinel_init(wsf("s_qkv", qn), qn, st);
        wsf("p_qkv_skip", qn);  // the profile's variant without attention projects here (allocated before capture)
    }
    HIP_CHECK(hipMemsetAsync(wsi("s_dtick", dec_mm_splitk_ticks(H)), 0, sizeof(int) * dec_mm_splitk_ticks(H), st));
    HIP_CHECK(hipMemsetAsync(wsi("s_err", 4), 0, sizeof(int) * 4, st));  // fused-kernel give-up flag
    // one page: the persistent decode step (its granules: no tag of an earlier generate may match this one's)
    persist_active_ = p.use_cache && persist_ok(B, Lmax);
    if (persist_active_) {
        ensure_persist();
        HIP_CHECK(hipMemsetAsync(persist_g_, 0xff, dec_persist_granules(L.layers) * 8, st));
    }
    const int QKVN = layers_[0].qkv.N;
    float* SX = wsf("s_x", (size_t)B * H);
    float* SXN = wsf("s_xn", (size_t)B * H);
    float* LOGITS = wsf("s_logits", (size_t)B * L.vocab);

    // ---------------- 3. the forward over whole token sequences (DeepseekOcrModel::forward,
    // model/mod.rs:1181-1251): embed + inject (1208-1239), every layer, final norm + lm_head on the
    // last row of each page (the reference projects every position, transformer/model.rs:243-270;
    // only the last row is ever read).  The prefill runs it once on the prompts; use_cache = false
    // (generate_without_cache, model/mod.rs:2051-2283) re-runs it on prompt + generated every step.
    auto forward_rows = [&](const std::vector<int>& lens, const std::vector<std::vector<int>>& extra) {
        long Tn = 0;
        int maxl = 0;
        for (int b = 0; b < B; ++b) { Tn += lens[b]; maxl = std::max(maxl, lens[b]); }
        prefill_lens_ = lens;
        std::vector<int> kind(Tn), index(Tn), row_page(Tn), row_pos(Tn);
        std::vector<long> q_off(B), kv_off(B), o_off(B);
        long r0 = 0;
        for (int b = 0; b < B; ++b) {
            const GenRequest& rq = reqs[b];
            size_t j = 0;
            for (int i = 0; i < lens[b]; ++i) {
                const long r = r0 + i;
                if (i < prompt_len[b] && !rq.mask.empty() && rq.mask[i]) {
                    kind[r] = img[b][j].first;
                    index[r] = (int)img[b][j].second;
                    ++j;
                } else {
                    kind[r] = 0;
                    index[r] = i < prompt_len[b] ? rq.ids[i] : extra[b][i - prompt_len[b]];
                }
                row_page[r] = b;
                row_pos[r] = i;
            }
            q_off[b] = r0 * QKVN;
            kv_off[b] = (long)b * page_stride_;
            o_off[b] = r0 * H;
            r0 += lens[b];
        }
        float* X = wsf("d_x", (size_t)Tn * H);
        int* dk = upload("g_kind", kind);
        int* di = upload("g_index", index);
        float* hr = host_rows.empty() ? nullptr : upload("g_hostrows", host_rows);
        launch_assemble_rows(dk, di, (int)Tn, H, embed_, embed_dt_, hr, vis_rows, newline_, separator_, X, H, st);
        int* d_row_page = upload("g_rowpage", row_page);
        int* d_row_pos = upload("g_rowpos", row_pos);
        long* d_q_off = upload("g_qoff", q_off);
        long* d_kv_off = upload("g_kvoff", kv_off);
        long* d_o_off = upload("g_ooff", o_off);
        int* d_plen = upload("g_plen", lens);
        for (int l = 0; l < L.layers; ++l)
            layer_forward_prefill(l, (int)Tn, B, d_row_page, d_row_pos, d_q_off, d_kv_off, d_o_off, d_plen, maxl, Lmax);
        std::vector<int> last_rows(B), lr_kind(B, 1);
        r0 = 0;
        for (int b = 0; b < B; ++b) { r0 += lens[b]; last_rows[b] = (int)(r0 - 1); }
        int* lk = upload("g_lrkind", lr_kind);
        int* li = upload("g_lrindex", last_rows);
        launch_assemble_rows(lk, li, B, H, nullptr, 0, X, nullptr, nullptr, nullptr, SX, H, st);
        launch_rmsnorm(SX, H, SXN, H, B, H, final_norm_, L.rms_eps, st);
        linear(SXN, B, H, lm_head_, LOGITS, L.vocab);
    };
    HIP_CHECK(hipEventRecord(ev[2], st));
    flops_acc_ = 0;
    std::vector<std::vector<int>> extra(B);
    forward_rows(prompt_len, extra);

    // sampling state: context = prompt ids (+ generated), sampling.rs:34-96
    const long ctx_cap = max_p + (long)p.max_new + 1;
    std::vector<int> ctx((size_t)B * ctx_cap, 0), ctx_len(B), kvpos(B), kvlen(B), zeros(B, 0);
    for (int b = 0; b < B; ++b) {
        for (int i = 0; i < prompt_len[b]; ++i) ctx[(size_t)b * ctx_cap + i] = reqs[b].ids[i];
        ctx_len[b] = prompt_len[b];
        kvpos[b] = prompt_len[b];
        kvlen[b] = prompt_len[b] + 1;
    }
    int* d_ctx = upload("s_ctx_ids", ctx);
    int* d_ctx_len = upload("s_ctx_len", ctx_len);
    int* d_kvpos = wsi("s_kvpos", B);
    int* d_kvlen = wsi("s_kvlen", B);
    HIP_CHECK(hipMemcpyAsync(d_kvpos, kvpos.data(), B * 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_kvlen, kvlen.data(), B * 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int* d_done = upload("s_done", zeros);
    int* d_outlen = upload("s_outlen", zeros);
    int* d_out = wsi("s_out", (size_t)B * p.max_new);
    int* d_tok = wsi("s_tok", B);
    // penalty (applied in place to the logits when != 1) + fused greedy selection
    SampleArgs pen;
    pen.logits = LOGITS; pen.B = B; pen.V = L.vocab; pen.ld = L.vocab; pen.ctx = d_ctx; pen.ctx_cap = ctx_cap;
    pen.ctx_len = d_ctx_len; pen.rep_penalty = p.rep_penalty;
    DecSampleArgs sa;
    sa.logits = LOGITS; sa.B = B; sa.V = L.vocab; sa.ld = L.vocab; sa.ctx = d_ctx; sa.ctx_cap = ctx_cap;
    sa.ctx_len = d_ctx_len; sa.ngram = p.ngram;
    sa.red_blocks = (int)dec_sample_blocks(L.vocab);
    sa.red_val = wsf("s_redv", (size_t)B * sa.red_blocks); sa.red_idx = wsi("s_redi", (size_t)B * sa.red_blocks);
    sa.out_tok = d_tok; sa.out_ids = d_out; sa.out_len = d_outlen; sa.out_cap = (long)p.max_new; sa.done = d_done;
    sa.eos = p.ignore_eos ? -1 : (int)p.eos;
    sa.table = embed_; sa.table_dt = embed_dt_; sa.H = H; sa.x_next = SX; sa.kv_pos = d_kvpos; sa.kv_len = d_kvlen;
    if (p.do_sample) {
        // stochastic selection (sampling.hip): StdRng::seed_from_u64(seed) per page — every page starts
        // from init_rng(seed) like a single-page generate call (model/mod.rs:1917) — or entropy
        sa.do_sample = 1; sa.temperature = p.temperature; sa.top_p = p.top_p; sa.top_k = p.top_k;
        sa.st_ld = L.vocab;
        sa.st_key = reinterpret_cast<uint32_t*>(wsi("s_stkey", (size_t)B * 2 * L.vocab));
        sa.st_idx = wsi("s_stidx", (size_t)B * 2 * L.vocab);
        sa.st_w = reinterpret_cast<double*>(wsf("s_stw", (size_t)B * 2 * L.vocab));
        uint64_t seed = p.seed;
        if (!p.seed_set) {
            std::random_device rd;
            seed = ((uint64_t)rd() << 32) ^ rd();
        }
        const std::vector<uint32_t> st = rng_state_from_u64(seed);
        std::vector<int> all((size_t)B * RNG_WORDS);
        for (int b = 0; b < B; ++b) memcpy(&all[(size_t)b * RNG_WORDS], st.data(), sizeof(uint32_t) * RNG_WORDS);
        sa.rng = reinterpret_cast<uint32_t*>(upload("s_rng", all));
    }
    ensure_mm_weights(B);
    if (!p.do_sample && !p.trace && screen_applies(B, p.rep_penalty)) {
        // the screened head reads the n-gram ban list each selection kernel leaves for the next step
        sa.ban_ld = ctx_cap + 1;
        sa.ban_out = wsi("s_ban", (size_t)B * sa.ban_ld);
        reserve_head_ws(B);
        if (getenv("DSOCR_SCREEN_STATS")) HIP_CHECK(hipMemsetAsync(wsi("s_scrstats", 32), 0, 128, st));
    }
    // parity trace: the raw logits of every step of every page ([B][max_new][V], index = tokens
    // emitted so far), copied before the repetition penalty like the reference's debug dump
    // (crates/infer-deepseek/src/debug.rs) — the exact lm_head runs (no screening) while tracing
    trace_ = p.trace ? wsf("s_trace", (size_t)B * p.max_new * L.vocab) : nullptr;
    trace_steps_ = (long)p.max_new;
    if (trace_) {
        HIP_CHECK(hipMemsetAsync(trace_, 0, sizeof(float) * B * p.max_new * L.vocab, st));
        launch_trace_logits(LOGITS, B, L.vocab, L.vocab, d_outlen, d_done, trace_, trace_steps_, st);
    }
    // the fused selection kernel advances the KV position; after the prefill the first
    // decode position must be P, so start one behind
    launch_rep_penalty(pen, st);
    {
        std::vector<int> pm1(B), lm1(B);
        for (int b = 0; b < B; ++b) { pm1[b] = kvpos[b] - 1; lm1[b] = kvlen[b] - 1; }
        HIP_CHECK(hipMemcpyAsync(d_kvpos, pm1.data(), B * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(d_kvlen, lm1.data(), B * 4, hipMemcpyHostToDevice, st));
        launch_dec_sample(sa, st);
        HIP_CHECK(hipStreamSynchronize(st));
    }
    HIP_CHECK(hipEventRecord(ev[3], st));
    timings_.prefill_flops = flops_acc_;
    std::vector<int> h_done(B), h_outlen(B);
    std::vector<int> h_out;
    size_t steps = 0;
    int* pin_done = nullptr;
    HIP_CHECK(hipHostMalloc((void**)&pin_done, sizeof(int) * (3 * B + 1)));
    // stream callback with the tokens so far (B = 1; model/mod.rs:1980-1982 calls it after every token)
    int streamed = 0;
    auto stream_tokens = [&](int n) {
        if (n <= streamed) return;  // no new token (EOS selected, or the page is done)
        streamed = n;
        std::vector<int> tmp(n);
        if (n) HIP_CHECK(hipMemcpy(tmp.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        std::vector<int64_t> t64(tmp.begin(), tmp.end());
        cb(t64.size(), t64.data(), user);
    };
    auto poll = [&]() {  // done flags, output lengths and the last tokens of every page
        HIP_CHECK(hipMemcpyAsync(pin_done, d_done, B * 4, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipMemcpyAsync(pin_done + B, d_outlen, B * 4, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipMemcpyAsync(pin_done + 2 * B, d_tok, B * 4, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        bool all = true;
        for (int b = 0; b < B; ++b) all &= pin_done[b] != 0;
        return all;
    };
    if (cb && B == 1 && p.max_new > 0) {
        poll();
        if (pin_done[B] > 0) stream_tokens(pin_done[B]);
    }
    if (!p.use_cache) {
        // ---------------- 4'. generate_without_cache (model/mod.rs:2051-2283): every step re-runs the
        // whole forward on prompt + generated tokens (image rows re-injected at the same slots), then
        // the same selection / bookkeeping kernels as the cached loop
        HIP_CHECK(hipEventRecord(ev[4], st));
        std::vector<int> lens = prompt_len;
        for (size_t i = 1; i < p.max_new; ++i) {
            if (poll()) break;
            for (int b = 0; b < B; ++b)
                if (!pin_done[b]) { extra[b].push_back(pin_done[2 * B + b]); ++lens[b]; }
            forward_rows(lens, extra);
            if (trace_) launch_trace_logits(LOGITS, B, L.vocab, L.vocab, d_outlen, d_done, trace_, trace_steps_, st);
            launch_rep_penalty(pen, st);
            launch_dec_sample(sa, st);
            ++steps;
            if (cb && B == 1) {
                poll();
                stream_tokens(pin_done[B]);
            }
        }
        HIP_CHECK(hipEventRecord(ev[5], st));
        HIP_CHECK(hipStreamSynchronize(st));
    } else {
    chain_active_ = false;
    spans_kinds_ = SPAN_KINDS;
    if (span_mode_ == SPAN_CHAIN) {
        span_cap_ = (int)std::max<size_t>(p.max_new, 1) + 1;  // the fold records at (tokens emitted) <= max_new
        const size_t nreg = (size_t)L.layers * SPAN_KINDS_CHAIN;
        span_chain_ = (unsigned long long*)ws("s_span_chain", nreg * SPAN_SLOTS * 16);
        span_chain_rec_ = (unsigned long long*)ws("s_span_chain_rec", (size_t)span_cap_ * nreg * 32);
        span_tmark_ = (unsigned long long*)ws("s_span_tmark", 16);
        span_rec_ = span_chain_rec_;  // (marks the generate as stamped)
        span_step_ = d_outlen;
        chain_active_ = true;
        HIP_CHECK(hipMemsetAsync(span_chain_rec_, 0, (size_t)span_cap_ * nreg * 32, st));
    } else if (span_mode_) {
        span_cap_ = (int)std::max<size_t>(p.max_new, 1);
        const size_t rec_bytes = (size_t)SPAN_KINDS * L.layers * span_cap_ * 4 * 8;
        span_slots_ = (unsigned long long*)ws("s_span_slots", (size_t)SPAN_SLOTS * 16);
        span_rec_ = (unsigned long long*)ws("s_span_rec", rec_bytes);
        span_step_ = d_outlen;
        HIP_CHECK(hipMemsetAsync(span_slots_, 0, (size_t)SPAN_SLOTS * 16, st));
        HIP_CHECK(hipMemsetAsync(span_rec_, 0, rec_bytes, st));
        if (span_ev_.empty()) {
            span_ev_.resize((size_t)SPAN_KINDS * L.layers * 2);
            for (auto& e : span_ev_) HIP_CHECK(hipEventCreate(&e));
        }
        span_ev_ns_.assign((size_t)SPAN_KINDS * L.layers * span_cap_, 0.0);
    }
    // after a stamped step: the dispatch-level duration of every bracketed launch, at the step's index
    auto read_span_events = [&](size_t step) {
        HIP_CHECK(hipEventSynchronize(span_ev_.back()));
        const size_t k = std::min(step, (size_t)span_cap_ - 1);
        for (size_t i = 0; i < (size_t)SPAN_KINDS * L.layers; ++i) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, span_ev_[2 * i], span_ev_[2 * i + 1]) == hipSuccess)
                span_ev_ns_[i * span_cap_ + k] = ms * 1e6;
            else
                (void)hipGetLastError();  // pair not recorded this step (e.g. the dense layer)
        }
    };
    // make sure every decode workspace exists before capture: a dry step allocates them
    // (it writes the step-0 K/V slot, which the real step rewrites), then the state is restored
    decode_step(B, Lmax);
    if (persist_active_) {  // the dry step's granules carry step 1's tags: reset them
        HIP_CHECK(hipMemsetAsync(persist_g_, 0xff, dec_persist_granules(L.layers) * 8, st));
        persist_stamps_host_.clear();
        persist_ev_us_.clear();
        if (persist_stamp_mode_) {
            persist_stamp_pos0_ = kvpos[0];
            persist_stamp_cap_ = (int)p.max_new;
            const size_t n = (size_t)persist_stamp_cap_ * PK_G * L.layers * PK_STAMPS;
            persist_stamps_ = (unsigned long long*)ws("p_pk_stamps", n * 8);
            HIP_CHECK(hipMemsetAsync(persist_stamps_, 0, n * 8, st));
        }
    }
    if (chain_active_) {  // the dry step's stamps must not join step 1's: clear the regions and the marks
        HIP_CHECK(hipMemsetAsync(span_chain_, 0, (size_t)L.layers * SPAN_KINDS_CHAIN * SPAN_SLOTS * 16, st));
        HIP_CHECK(hipMemsetAsync(span_tmark_, 0, 16, st));
    }
    HIP_CHECK(hipMemcpyAsync(d_kvpos, kvpos.data(), B * 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_kvlen, kvlen.data(), B * 4, hipMemcpyHostToDevice, st));
    launch_embed_tokens(embed_, embed_dt_, d_tok, B, H, SX, H, st);
    HIP_CHECK(hipStreamSynchronize(st));

    // ---------------- 4. decode loop (decode.iterative) as a replayed hipGraph
    // DSOCR_NO_GRAPH=1 launches the same kernels eagerly (rocprofv3 kernel tracing of
    // graph replays is unreliable on this stack; kernel durations are unchanged).
    const bool use_graph = !(getenv("DSOCR_NO_GRAPH") && atoi(getenv("DSOCR_NO_GRAPH")) != 0);
    auto step_body = [&]() {
        decode_step(B, Lmax);
        decode_head(B, sa, pen);
        // chain spans: the step's one fold, after the head (the step counter has advanced: record at count - 1)
        if (chain_active_)
            launch_span_chain_fold(span_chain_, L.layers * SPAN_KINDS_CHAIN, span_chain_rec_, span_step_, span_cap_,
                                   span_tmark_, st);
    };
    const bool pk_timed = persist_active_ && persist_stamp_mode_ && !span_rec_;
    if (pk_timed && persist_ev_.empty()) {
        persist_ev_.resize(2);
        for (auto& e : persist_ev_) HIP_CHECK(hipEventCreate(&e));
    }
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    if (use_graph && !pk_timed) {
        capturing_ = true;
        HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        step_body();
        HIP_CHECK(hipStreamEndCapture(st, &graph));
        capturing_ = false;
        HIP_CHECK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
    }

    HIP_CHECK(hipEventRecord(ev[4], st));
    for (size_t i = 1; i < p.max_new; ++i) {
        if (gexec) HIP_CHECK(hipGraphLaunch(gexec, st));
        else step_body();
        if (span_rec_ && (span_mode_ & SPAN_EVENTS)) read_span_events(i);
        if (pk_timed) {  // the persistent launch's dispatch duration (events recorded around it in the step)
            HIP_CHECK(hipEventSynchronize(persist_ev_[1]));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, persist_ev_[0], persist_ev_[1]));
            persist_ev_us_.push_back(ms * 1e3);
        }
        ++steps;
        const bool check = cb != nullptr || (!p.ignore_eos && (i % 8 == 0 || i + 1 == p.max_new));
        if (check) {
            const bool all = poll();
            if (cb && B == 1) stream_tokens(pin_done[B]);
            if (all) break;
        }
    }
    HIP_CHECK(hipEventRecord(ev[5], st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    if (pk_timed) {
        persist_stamps_host_.resize((size_t)persist_stamp_cap_ * PK_G * L.layers * PK_STAMPS);
        HIP_CHECK(hipMemcpy(persist_stamps_host_.data(), persist_stamps_, persist_stamps_host_.size() * 8,
                            hipMemcpyDeviceToHost));
        persist_stamp_mode_ = 0;
    }
    if (chain_active_) {
        const size_t nreg = (size_t)L.layers * SPAN_KINDS_CHAIN;
        std::vector<unsigned long long> dev((size_t)span_cap_ * nreg * 4);
        HIP_CHECK(hipMemcpy(dev.data(), span_chain_rec_, dev.size() * 8, hipMemcpyDeviceToHost));
        spans_host_.assign((size_t)SPAN_KINDS_CHAIN * L.layers * span_cap_ * SPAN_FIELDS, 0);
        // fold at step s's end recorded at index (tokens emitted) = s + 1: shift back to s
        for (int st_ = 1; st_ < span_cap_; ++st_)
            for (int l = 0; l < L.layers; ++l)
                for (int k = 0; k < SPAN_KINDS_CHAIN; ++k) {
                    const unsigned long long* r = &dev[((size_t)st_ * nreg + (size_t)l * SPAN_KINDS_CHAIN + k) * 4];
                    unsigned long long* o = &spans_host_[(((size_t)k * L.layers + l) * span_cap_ + st_ - 1) * SPAN_FIELDS];
                    o[0] = r[0]; o[1] = r[1]; o[3] = r[2];
                }
        spans_steps_ = span_cap_;
        spans_kinds_ = SPAN_KINDS_CHAIN;
        chain_active_ = false;
        span_rec_ = nullptr;
        span_step_ = nullptr;
    } else if (span_rec_) {
        const size_t nrec = (size_t)SPAN_KINDS * L.layers * span_cap_;
        std::vector<unsigned long long> dev(nrec * 4);
        HIP_CHECK(hipMemcpy(dev.data(), span_rec_, dev.size() * 8, hipMemcpyDeviceToHost));
        spans_host_.assign(nrec * SPAN_FIELDS, 0);
        for (size_t r = 0; r < nrec; ++r) {
            for (int f = 0; f < 4; ++f) spans_host_[r * SPAN_FIELDS + f] = dev[r * 4 + f];
            if (span_mode_ & SPAN_EVENTS) spans_host_[r * SPAN_FIELDS + 4] = (unsigned long long)llround(span_ev_ns_[r]);
        }
        spans_steps_ = span_cap_;  // reported with the records it sizes (a throwing generate leaves both)
        // profile_decode runs unstamped; every later generate is stamped again while span_mode_ is set
        span_rec_ = nullptr;
        span_slots_ = nullptr;
        span_step_ = nullptr;
    }
    }  // cached decode loop
    HIP_CHECK(hipHostFree(pin_done));
    {
        int e = 0;
        HIP_CHECK(hipMemcpy(&e, wsi("s_err", 4), sizeof(int), hipMemcpyDeviceToHost));
        if (e) throw std::runtime_error("EINTERNAL: decode hand-off timed out inside a fused kernel");
    }
    if (sa.ban_out && getenv("DSOCR_SCREEN_STATS")) {
        unsigned long long h[16] = {0};
        HIP_CHECK(hipMemcpy(h, wsi("s_scrstats", 32), sizeof(h), hipMemcpyDeviceToHost));
        const double st = h[0] ? (double)h[0] : 1.0;
        fprintf(stderr, "[screen] steps %llu kept/step %.1f survivors/step %.2f phase_us", h[0], h[1] / st, h[2] / st);
        for (int k = 0; k < 7; ++k) fprintf(stderr, " %.2f", h[4 + k] / st / 100.0);  // wall clock: 100 MHz
        fprintf(stderr, "\n");
    }
    h_out.resize((size_t)B * p.max_new);
    HIP_CHECK(hipMemcpy(h_out.data(), d_out, h_out.size() * 4, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(h_outlen.data(), d_outlen, B * 4, hipMemcpyDeviceToHost));
    for (int b = 0; b < B; ++b) out[b].assign(h_out.begin() + (size_t)b * p.max_new, h_out.begin() + (size_t)b * p.max_new + h_outlen[b]);

    timings_.vision_compute_ms = ms_between(ev[0], ev[1]);
    timings_.prefill_ms = ms_between(ev[2], ev[3]);
    timings_.iterative_ms = ms_between(ev[4], ev[5]);
    timings_.generate_ms = ms_between(ev[2], ev[3]) + ms_between(ev[4], ev[5]);
    timings_.steps = steps;
    if (trace_ && p.trace)
        HIP_CHECK(hipMemcpy(p.trace, trace_, sizeof(float) * B * p.max_new * L.vocab, hipMemcpyDeviceToHost));
    trace_ = nullptr;
    last_B_ = B;
    last_Lmax_ = Lmax;
    (void)t0;
    for (auto& e : ev) (void)hipEventDestroy(e);
    return out;
}

Engine::DecodeProfile Engine::profile_decode(int iters) {
    DecodeProfile prof;
    const LangConfig& L = cfg_.lang;
    const int B = last_B_, Lmax = last_Lmax_;
    if (B == 0 || Lmax == 0) throw std::runtime_error("EINVAL: run a generate() first");
    const int H = L.hidden, hd = L.head_dim;
    hipStream_t st = stream_;
    std::vector<int> kvpos(B);
    HIP_CHECK(hipMemcpy(kvpos.data(), wsi("s_kvpos", B), B * 4, hipMemcpyDeviceToHost));
    // the replays re-run the last decoded position (pos - 1): its K/V slot is rewritten with the same values
    std::vector<int> pm1(B);
    long keys = 0;
    for (int b = 0; b < B; ++b) { pm1[b] = std::max(0, kvpos[b] - 1); keys += pm1[b] + 1; }
    int* d_pos = wsi("p_kvpos", B);
    HIP_CHECK(hipMemcpy(d_pos, pm1.data(), B * 4, hipMemcpyHostToDevice));
    prof.tokens = B;
    prof.kv_len = pm1[0] + 1;
    {
        const size_t qn = (size_t)B * layers_[0].qkv.N;
        HIP_CHECK(hipMemsetAsync(wsf("p_qkv_attn", qn), 0, qn * 4, st));
    }
    // the replays rewrite the K / V slot of pos - 1 in every layer (the attention replays from a scratch
    // row): keep those slots and put them back after the attention replays and at the end, so the
    // step-graph replays and any later use of the engine state see the cache the generate left
    const size_t slot_w = (size_t)hd * 4, n_slots = (size_t)L.layers * B * 2;
    float* kv_saved = wsf("p_kv_saved", n_slots * L.kv_heads * hd);
    auto kv_slots = [&](bool restore) {
        for (int l = 0; l < L.layers; ++l)
            for (int b = 0; b < B; ++b)
                for (int kv = 0; kv < 2; ++kv) {
                    float* base = (kv ? vc_ : kc_) + (long)l * B * page_stride_ + (long)b * page_stride_ + (long)pm1[b] * hd;
                    float* keep = kv_saved + (((size_t)l * B + b) * 2 + kv) * L.kv_heads * hd;
                    if (restore)
                        HIP_CHECK(hipMemcpy2DAsync(base, head_stride_ * 4, keep, slot_w, slot_w, L.kv_heads, hipMemcpyDeviceToDevice, st));
                    else
                        HIP_CHECK(hipMemcpy2DAsync(keep, slot_w, base, head_stride_ * 4, slot_w, L.kv_heads, hipMemcpyDeviceToDevice, st));
                }
    };
    kv_slots(false);
    // n back-to-back launches captured in one hipGraph, replayed between two events on the
    // engine stream: per-launch time = span / n = device time + the dependent-kernel boundary
    // (eager launches go host-bound below ~3.5 us per kernel, MI355X_MICROARCH.md
    // graph-replay-floor, so they cannot time the short decode kernels)
    // Two figures per kernel:
    //  * avg_us: every launch carries its own start / stop events on its dispatch packet
    //    (hipExtLaunchKernelGGL through DSOCR_LAUNCH: the begin / end timestamps rocprofv3's kernel
    //    trace reports), eager, one launch at a time — the figure the committed rocprof summaries
    //    corroborate;
    //  * replay_us: n launches back to back in one hipGraph replay, span / n - the kernel inside a
    //    dependent chain as the decode loop runs it (duration + the ~1.2 us kernel boundary, minus
    //    whatever startup the chained dispatch hides).
    auto timed = [&](KernelProfile& kp, int n, const std::function<void(int)>& body) {
        body(0);  // warm (code objects, TLB) and every workspace allocated before capture
        // the events are destroyed on every exit, the EINTERNAL / HIP-error throws below included
        struct EventSet {
            std::vector<hipEvent_t> v;
            ~EventSet() {
                for (auto& e : v)
                    if (e) (void)hipEventDestroy(e);
            }
        } evs;
        evs.v.assign(2 * n, nullptr);
        std::vector<hipEvent_t>& ev = evs.v;
        for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
        for (int i = 0; i < n; ++i) {
            prof_events() = ProfEvents{ev[2 * i], ev[2 * i + 1]};  // the body's first launch times itself
            body(i);
            if (prof_events().start) {  // the body launched nothing through DSOCR_LAUNCH: bracket it
                prof_events() = ProfEvents();
                throw std::runtime_error("EINTERNAL: profiled body made no instrumented launch");
            }
        }
        HIP_CHECK(hipEventSynchronize(ev[2 * n - 1]));
        double sum = 0;
        for (int i = 0; i < n; ++i) sum += ms_between(ev[2 * i], ev[2 * i + 1]);
        kp.avg_us = 1000.0 * sum / n;
        kp.launches = n;
        if (getenv("DSOCR_NO_GRAPH") && atoi(getenv("DSOCR_NO_GRAPH")) != 0) return;
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        hipGraph_t graph = nullptr;
        hipGraphExec_t gexec = nullptr;
        capturing_ = true;
        HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < n; ++i) body(i);
        HIP_CHECK(hipStreamEndCapture(st, &graph));
        capturing_ = false;
        HIP_CHECK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
        HIP_CHECK(hipGraphLaunch(gexec, st));  // warm replay
        HIP_CHECK(hipEventRecord(e0, st));
        HIP_CHECK(hipGraphLaunch(gexec, st));
        HIP_CHECK(hipEventRecord(e1, st));
        HIP_CHECK(hipEventSynchronize(e1));
        kp.replay_us = 1000.0 * ms_between(e0, e1) / n;
        (void)hipGraphExecDestroy(gexec);
        (void)hipGraphDestroy(graph);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    };
    std::vector<int> moe_layers;
    for (int l = 0; l < L.layers; ++l)
        if (layers_[l].moe) moe_layers.push_back(l);
    if (!moe_layers.empty()) {
        const int E = L.n_routed, K = L.topk, I = L.moe_inter, TK = B * K;
        std::vector<int> ids(TK);
        HIP_CHECK(hipMemcpy(ids.data(), wsi("s_ids", TK), TK * 4, hipMemcpyDeviceToHost));
        std::vector<char> seen(E, 0);
        for (int v : ids)
            if (v >= 0 && v < E && !seen[v]) { seen[v] = 1; ++prof.experts_touched; }
        const float* Xc = wsf("s_x", (size_t)B * H);
        // replay on a scratch copy of the residual stream so the engine state is untouched
        float* Xs = wsf("p_x", (size_t)B * H);
        HIP_CHECK(hipMemcpyAsync(Xs, Xc, (size_t)B * H * 4, hipMemcpyDeviceToDevice, st));
        // the gate/up and down launches of decode_step's dispatch (launch_moe_decode), replayed
        // alone on the routing state the last step left (logits, normalised rows, expert groups)
        auto args = [&](int l) { return moe_args(l, B, Xs); };
        const int n = iters * (int)moe_layers.size();
        moe_decode_kernel_names(args(moe_layers[0]), &prof.gateup_kernel, &prof.down_kernel);
        // rotating over the layers (~55 MB each) defeats the 256 MB Infinity Cache
        timed(prof.moe_gateup, n, [&](int i) { launch_moe_decode(args(moe_layers[i % moe_layers.size()]), st, MOE_GATEUP); });
        timed(prof.moe_down, n, [&](int i) { launch_moe_decode(args(moe_layers[i % moe_layers.size()]), st, MOE_DOWN); });
        const DecLayer& d0 = layers_[moe_layers[0]];
        const double Is = d0.has_shared ? d0.s_d.K : 0;
        const double touched = (double)prof.experts_touched;
        prof.moe_gateup.bytes = (touched * 2.0 * I + 2.0 * Is) * H * 2.0   // fp16 gate+up rows
                                + (double)B * H * 4 + (double)(TK * I + B * Is) * 4;  // x in, h out
        prof.moe_gateup.flops = 2.0 * (TK * 2.0 * I + B * 2.0 * Is) * H;
        prof.moe_down.bytes = (touched * I + Is) * H * 2.0 + (double)(TK * I + B * Is) * 4 + 2.0 * B * H * 4;
        prof.moe_down.flops = 2.0 * (TK * (double)I + B * Is) * H;
    }
    {
        const int QKVN = layers_[0].qkv.N;
        float* part = wsf("s_part", dec_attn_workspace(B, L.heads, hd, Lmax) / 4 + 16);
        float* CTX = wsf("p_ctx", (size_t)B * H);
        const int n = iters * L.layers;
        timed(prof.attention, n, [&](int i) {
            const int l = i % L.layers;
            DecAttn2Args da;
            // a scratch q/k/v row (zeros): s_qkv holds the fused launch's sentinels, and the replays
            // rewrite the K / V slot of pos - 1 from this row
            da.qkv = wsf("p_qkv_attn", (size_t)B * QKVN); da.ld = QKVN; da.kv_pos = d_pos; da.B = B; da.heads = L.heads;
            da.kv_heads = L.kv_heads; da.hd = hd; da.rope_dim = L.rope_dim; da.use_mla = L.use_mla; da.max_len = Lmax;
            da.cos = rope_cos_; da.sin = rope_sin_;
            da.kc = kc_ + (long)l * B * page_stride_; da.vc = vc_ + (long)l * B * page_stride_;
            da.page_stride = page_stride_; da.head_stride = head_stride_;
            da.scale = (float)(1.0 / std::sqrt((double)hd)); da.part = part; da.o = CTX; da.o_ld = H;
            da.err = wsi("s_err", 4);
            da.counters = wsi("s_attn_cnt", (size_t)B * L.heads);
            launch_dec_attn(da, st);
        });
        kv_slots(true);
        // K and V of every attended key (f32 cache) + q/k/v row + context out
        prof.attention.bytes = (double)keys * L.kv_heads * hd * 4.0 * 2.0 + (double)B * (QKVN + H) * 4.0;
        prof.attention.flops = 4.0 * keys * L.heads * hd;
    }
    {
        float* LG = wsf("p_logits", (size_t)B * L.vocab);
        const float* SX = wsf("s_x", (size_t)B * H);
        float* SXN = wsf("p_xn", (size_t)B * H);
        ensure_mm_weights(B);
        const bool fused = B <= 2 || (lm_swz_ && B <= 8);
        if (!fused) launch_rmsnorm(SX, H, SXN, H, B, H, final_norm_, L.rms_eps, st);
        timed(prof.lm_head, iters, [&](int) {
            DecGemvArgs g;
            g.M = B; g.N = L.vocab; g.K = H; g.W = lm_head_.W; g.ldw = H; g.wdtype = lm_head_.wdt; g.bias = lm_head_.b;
            g.y = LG; g.ldy = L.vocab;
            if (fused) {
                g.x = SX; g.ldx = H; g.norm_w = final_norm_; g.eps = L.rms_eps;
                if (B > 2) g.w_swz = lm_swz_;
            } else { g.x = SXN; g.ldx = H; }
            launch_dec_gemv(g, st);
        });
        prof.lm_head.bytes = (double)L.vocab * H * 2.0 + (double)B * (L.vocab + H) * 4.0;
        prof.lm_head.flops = 2.0 * B * (double)L.vocab * H;
        if (screen_applies(B, 1.0f)) {
            // screened head: int8 lm_head + selection (no bookkeeping, no ban: side-effect free)
            const LmHeadQ8Args q = head_q8_args(B);
            DecSampleArgs ss;
            ss.B = B; ss.V = L.vocab; ss.ld = L.vocab; ss.ctx = wsi("p_sctx", 64); ss.ctx_cap = 64;
            ss.ctx_len = wsi("p_ctxlen", B); ss.ngram = 0; ss.out_tok = wsi("p_tok", B);
            ss.blk_cnt = q.blk_cnt; ss.blk_t = q.blk_t; ss.cand = q.cand; ss.cand_hi = q.cand_hi; ss.nblk = q.nblk;
            ss.slot = q.slot; ss.w_exact = lm_head_.W; ss.w_exact_wdt = lm_head_.wdt; ss.xn = q.xn_out; ss.K = H;
            HIP_CHECK(hipMemsetAsync(ss.ctx_len, 0, B * 4, st));
            timed(prof.lm_head_screened, iters, [&](int) {
                launch_lmhead_q8(q, st);
                launch_dec_sample(ss, st);
            });
            prof.lm_head_screened.bytes = (double)L.vocab * H + (double)L.vocab * 8.0 + (double)B * H * 4.0;
            prof.lm_head_screened.flops = 2.0 * B * (double)L.vocab * H;
        }
    }
    {
        // attention-side GEMVs of every layer, replayed on scratch outputs
        const int QKVN = layers_[0].qkv.N;
        const float* SX = wsf("s_x", (size_t)B * H);
        float* Y = wsf("p_qkv", (size_t)B * QKVN);
        float* XO = wsf("p_xo", (size_t)B * H);
        const int n = iters * L.layers;
        const bool fuse_norm = B <= 2;
        timed(prof.qkv, n, [&](int i) {
            const DecLayer& d = layers_[i % L.layers];
            DecGemvArgs g;
            g.M = B; g.N = QKVN; g.K = H; g.W = d.qkv.W; g.ldw = H; g.wdtype = d.qkv.wdt; g.bias = d.qkv.b;
            g.y = Y; g.ldy = QKVN; g.x = SX; g.ldx = H;
            if (fuse_norm) { g.norm_w = d.in_norm.w; g.eps = L.rms_eps; }
            launch_dec_gemv(g, st);
        });
        prof.qkv.bytes = (double)QKVN * H * 2.0 + (double)B * (H + QKVN) * 4.0;
        prof.qkv.flops = 2.0 * B * (double)QKVN * H;
        timed(prof.o_proj, n, [&](int i) {
            const DecLayer& d = layers_[i % L.layers];
            DecGemvArgs go;
            go.M = B; go.N = H; go.K = L.heads * hd; go.x = SX; go.ldx = H; go.W = d.o.W; go.ldw = go.K;
            go.wdtype = d.o.wdt; go.bias = d.o.b; go.y = XO; go.ldy = H; go.accumulate = 0;
            launch_dec_gemv(go, st);
        });
        prof.o_proj.bytes = (double)H * L.heads * hd * 2.0 + (double)B * 2 * H * 4.0;
        prof.o_proj.flops = 2.0 * B * (double)H * L.heads * hd;
        std::vector<int> moe_l;
        for (int l = 0; l < L.layers; ++l)
            if (layers_[l].moe) moe_l.push_back(l);
        if (!moe_l.empty() && moe_decode_route_launch(moe_args(moe_l[0], B, XO))) {
            // the routing launches of the dispatch ([RMSNorm +] router GEMV [+ routing / grouping]; none when the
            // gate/up launch routes itself)
            timed(prof.router, iters * (int)moe_l.size(), [&](int i) {
                MoeDecodeArgs ma = moe_args(moe_l[i % moe_l.size()], B, XO);
                ma.x = SX;
                launch_moe_decode(ma, st, MOE_ROUTE);
            });
            prof.router.bytes = (double)L.n_routed * H * 2.0 + (double)B * (H + L.n_routed) * 4.0;
            prof.router.flops = 2.0 * B * (double)L.n_routed * H;
        }
    }
    if (!(getenv("DSOCR_NO_GRAPH") && atoi(getenv("DSOCR_NO_GRAPH")) != 0)) {
        // every decoder layer of one step as one hipGraph (what the decode loop replays, minus
        // lm_head and selection); the residual stream is restored at the head of each replay and
        // the KV slot written is the next free position (past every generated token)
        float* X = wsf("s_x", (size_t)B * H);
        float* X0 = wsf("p_x0", (size_t)B * H);
        HIP_CHECK(hipMemcpyAsync(X0, X, (size_t)B * H * 4, hipMemcpyDeviceToDevice, st));
        decode_step(B, Lmax);  // every workspace exists before capture
        // the step graph, and the same graph without one kernel's launches: the difference per launch is
        // that kernel's in-context cost (its dispatch and its place in the dependent chain included)
        auto step_us = [&](int skip) {
            hipGraph_t g = nullptr;
            hipGraphExec_t ge = nullptr;
            step_skip_ = skip;
            capturing_ = true;
            HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            HIP_CHECK(hipMemcpyAsync(X, X0, (size_t)B * H * 4, hipMemcpyDeviceToDevice, st));
            decode_step(B, Lmax);
            HIP_CHECK(hipStreamEndCapture(st, &g));
            capturing_ = false;
            step_skip_ = 0;
            HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            const int n = std::max(8, iters * 4);
            hipEvent_t e0, e1;
            HIP_CHECK(hipEventCreate(&e0));
            HIP_CHECK(hipEventCreate(&e1));
            HIP_CHECK(hipGraphLaunch(ge, st));
            HIP_CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < n; ++i) HIP_CHECK(hipGraphLaunch(ge, st));
            HIP_CHECK(hipEventRecord(e1, st));
            HIP_CHECK(hipEventSynchronize(e1));
            const double us = 1000.0 * ms_between(e0, e1) / n;
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
            return us;
        };
        int n_moe = 0;
        for (const DecLayer& d : layers_) n_moe += d.moe ? 1 : 0;
        double full = step_us(0);
        const double no_gu = n_moe ? step_us(SKIP_GATEUP) : full;
        const double no_dn = n_moe ? step_us(SKIP_DOWN) : full;
        const double no_at = step_us(SKIP_ATTN);
        full = 0.5 * (full + step_us(0));  // bracket the variants: replay-to-replay drift averages out
        prof.layers_step.avg_us = full;
        prof.layers_step.launches = std::max(8, iters * 4);
        if (n_moe) {
            prof.moe_gateup.ctx_us = (full - no_gu) / n_moe;
            prof.moe_down.ctx_us = (full - no_dn) / n_moe;
        }
        prof.attention.ctx_us = (full - no_at) / L.layers;
        HIP_CHECK(hipMemcpyAsync(X, X0, (size_t)B * H * 4, hipMemcpyDeviceToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    kv_slots(true);
    HIP_CHECK(hipStreamSynchronize(st));
    return prof;
}

}  // namespace dsocr
