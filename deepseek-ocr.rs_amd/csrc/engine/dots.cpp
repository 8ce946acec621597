// dots.ocr vision tower (BASELINE configs[3]).  Reference: crates/infer-dots/src/vision/dots_vit.rs
// (DotsVisionModel::load 25-77, forward 80-96; block / attention / SwiGLU / merger 305-686) and
// vision/preprocess.rs (preprocess_image 103-145, smart_resize 244-279).
#include "dots.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>

#include "../common/host_util.hpp"
#include "engine.hpp"
#include "host_ops.hpp"

namespace dsocr {

void launch_dots_rmsnorm(const void* x, int in_f32, long rows, int D, const float* w, float eps, void* y, hipStream_t s);
void launch_dots_layernorm(const void* x, long rows, int D, const float* w, const float* b, float eps, void* y,
                           hipStream_t s);
void launch_dots_swiglu(const void* gu, long N, int I, void* h, hipStream_t s);
void launch_dots_rope_qk(const void* qkv, long N, int heads, int hd, const float* cos_t, const float* sin_t, void* out,
                         hipStream_t s);
void launch_dots_gelu(void* x, long n, hipStream_t s);
void launch_dots_to_bf16(const float* x, long N, int D, long ldi, void* y, int ldo, hipStream_t s);
void launch_dots_bf16_to_f32(const void* x, long n, float* y, hipStream_t s);

DotsConfig parse_dots_config(const Json& root) {
    DotsConfig c;
    const Json& v = root.has("vision_config") ? root["vision_config"] : root;
    auto geti = [&](const char* k, int def) { return v.has(k) ? (int)v[k].as_int() : def; };
    c.embed = geti("embed_dim", c.embed);
    c.hidden = geti("hidden_size", c.embed);
    c.inter = geti("intermediate_size", c.inter);
    c.layers = geti("num_hidden_layers", c.layers);
    c.heads = geti("num_attention_heads", c.heads);
    c.channels = geti("num_channels", c.channels);
    c.patch = geti("patch_size", c.patch);
    c.merge = geti("spatial_merge_size", c.merge);
    c.temporal = geti("temporal_patch_size", c.temporal);
    if (v.has("rms_norm_eps")) c.eps = v["rms_norm_eps"].as_double();
    if (v.has("use_bias")) c.use_bias = v["use_bias"].as_bool();
    if (v.has("post_norm")) c.post_norm = v["post_norm"].as_bool();
    if (v.has("is_causal") && v["is_causal"].as_bool())
        throw std::runtime_error("EINVAL: causal dots vision attention is not supported (the reference runs it bidirectional)");
    const Json& p = root["preprocessor_config"];
    if (p.has("min_pixels")) c.min_pixels = p["min_pixels"].as_int();
    if (p.has("max_pixels")) c.max_pixels = p["max_pixels"].as_int();
    for (int i = 0; i < 3; ++i) {
        if (p.has("image_mean")) c.mean[i] = (float)p["image_mean"][i].as_double();
        if (p.has("image_std")) c.stdv[i] = (float)p["image_std"][i].as_double();
    }
    if (p.has("patch_size") && p["patch_size"].as_int() != c.patch)
        throw std::runtime_error("EINVAL: preprocessor patch_size differs from the vision config");
    if (root.has("weight_prefix")) c.prefix = root["weight_prefix"].as_string();
    const int hd = c.heads > 0 ? c.embed / c.heads : 0;
    if (c.heads <= 0 || c.embed % c.heads) throw std::runtime_error("EINVAL: embed_dim not divisible by num_heads");
    if (hd % 4) throw std::runtime_error("EINVAL: vision head dim must be divisible by 4");  // dots_vit.rs:700
    if (hd != 64 && hd != 128) throw std::runtime_error("EINVAL: the dots attention kernel supports head_dim 64 / 128");
    if (c.temporal != 1) throw std::runtime_error("EINVAL: temporal_patch_size > 1 (video frames) not supported");
    if (c.embed % 64 || c.inter % 64) throw std::runtime_error("EINVAL: embed_dim / intermediate_size must be multiples of 64");
    return c;
}

// preprocess.rs:244-279 (f64 arithmetic, Rust round = half away from zero)
void dots_smart_resize(long height, long width, long factor, long min_pixels, long max_pixels, long* rh, long* rw) {
    const double f = (double)std::max(factor, 1L);
    double h = (double)std::max(height, 1L), w = (double)std::max(width, 1L);
    auto rnd = [](double x) { return std::round(x); };
    if (h < f) { w = rnd((w * f) / h); h = f; }
    if (w < f) { h = rnd((h * f) / w); w = f; }
    const double aspect = std::max(h, w) / std::min(h, w);
    if (aspect > 200.0) throw std::runtime_error("EINVAL: aspect ratio exceeds limit");
    double hb = rnd(h / f) * f, wb = rnd(w / f) * f;
    const double area = hb * wb;
    const double maxp = (double)std::max(max_pixels, 1L), minp = (double)std::max(min_pixels, 1L);
    if (area > maxp) {
        const double beta = std::sqrt((h * w) / maxp);
        hb = std::floor((h / beta) / f) * f;
        wb = std::floor((w / beta) / f) * f;
    } else if (area < minp) {
        const double beta = std::sqrt(minp / (h * w));
        hb = std::ceil((h * beta) / f) * f;
        wb = std::ceil((w * beta) / f) * f;
    }
    if (hb < f || wb < f) throw std::runtime_error("EINVAL: degenerate smart_resize target");
    *rh = (long)hb;
    *rw = (long)wb;
}

DotsPatches dots_preprocess(const DotsConfig& c, const uint8_t* rgb, int w, int h) {
    if (!rgb || w <= 0 || h <= 0) throw std::runtime_error("EINVAL: empty image");
    DotsPatches out;
    long rh, rw;
    dots_smart_resize(h, w, (long)c.patch * c.merge, c.min_pixels, c.max_pixels, &rh, &rw);
    std::vector<uint8_t> resized;
    const uint8_t* src = rgb;
    if (rh != h || rw != w) {
        resized.resize((size_t)rh * rw * 3);
        resize_catmull_rom_fir(rgb, w, h, resized.data(), (int)rw, (int)rh);
        src = resized.data();
    }
    const int P = c.patch, M = c.merge;
    const int gh = (int)rh / P, gw = (int)rw / P;
    if (gh % M || gw % M) throw std::runtime_error("EINVAL: patch grid not divisible by the merge size");
    out.grid_t = 1;
    out.grid_h = gh;
    out.grid_w = gw;
    out.resized_h = (int)rh;
    out.resized_w = (int)rw;
    const int K = 3 * P * P;
    out.data.resize((size_t)gh * gw * K);
    const float rescale = 1.0f / 255.0f;
    size_t n = 0;
    for (int bh = 0; bh < gh / M; ++bh)
        for (int bw = 0; bw < gw / M; ++bw)
            for (int ih = 0; ih < M; ++ih)
                for (int iw = 0; iw < M; ++iw, ++n) {
                    const int y0 = (bh * M + ih) * P, x0 = (bw * M + iw) * P;
                    float* dst = out.data.data() + n * K;
                    for (int ch = 0; ch < 3; ++ch)
                        for (int py = 0; py < P; ++py)
                            for (int px = 0; px < P; ++px) {
                                const float v = (float)src[((size_t)(y0 + py) * rw + (x0 + px)) * 3 + ch];
                                const float scaled = v * rescale;
                                dst[(ch * P + py) * P + px] = (scaled - c.mean[ch]) / c.stdv[ch];
                            }
                }
    return out;
}

namespace {
// DSOCR_DOTS_PV_PLANES (A/B switch, read per layer): the attention's P.V on 3 bf16 planes of p (default: every
// product exact in the f32 accumulator, the reference's f32 probs.matmul(v), dots_vit.rs:402-409 / 584-589) or 2
// (opt-in: 16 significant bits of p, <= 2^-17 relative per probability, 2^-8 below the block output's bf16 rounding)
int dots_pv_planes() {
    const char* e = getenv("DSOCR_DOTS_PV_PLANES");
    return (e && atoi(e) == 2) ? 2 : 3;
}
std::string read_text(const std::string& p) {
    std::ifstream f(p);
    if (!f) throw std::runtime_error("ENOENT: cannot read config " + p);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}
}  // namespace

void* DotsVision::dev_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) throw std::runtime_error("ENOMEM: hipMalloc(" + std::to_string(bytes) + ")");
    allocs_.push_back(p);
    return p;
}

void* DotsVision::ws(const std::string& name, size_t bytes) {
    auto it = ws_.find(name);
    if (it != ws_.end() && it->second.second >= bytes) return it->second.first;
    if (it != ws_.end()) {
        HIP_CHECK(hipStreamSynchronize(stream_));
        HIP_CHECK(hipFree(it->second.first));
    }
    void* p = nullptr;
    const size_t cap = bytes + bytes / 8 + 256;
    if (hipMalloc(&p, cap) != hipSuccess) throw std::runtime_error("ENOMEM: workspace " + name);
    ws_[name] = {p, cap};
    return p;
}

DotsVision::DotsVision(const std::string& config_path, const std::string& weights_path, uint64_t seed, int device)
    : device_(device) {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) throw std::runtime_error("EDEVICE: no HIP device with ordinal " + std::to_string(device));
    HIP_CHECK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        throw std::runtime_error(std::string("EDEVICE: device is ") + prop.gcnArchName + ", engine is built for gfx950");
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    c_ = parse_dots_config(Json::parse(read_text(config_path)));
    std::unique_ptr<SafeTensors> st;
    if (!weights_path.empty()) st.reset(new SafeTensors(weights_path));
    const std::string& pre = c_.prefix;
    auto has = [&](const std::string& name) { return st ? st->has(pre + name) : synth_has(pre + name); };
    // bf16 bits of a tensor (the checkpoint is bf16; f32 tensors are rounded RNE, f16 refused)
    auto bits = [&](const std::string& name, size_t numel) {
        std::vector<uint16_t> b(numel);
        const std::string full = pre + name;
        if (!st) {
            synth_bf16(full, seed, numel, b.data());
            return b;
        }
        const StTensor& t = st->get(full);
        if ((size_t)t.numel() != numel)
            throw std::runtime_error("EINVAL: shape mismatch for `" + full + "`: " + std::to_string(t.numel()) + " vs " +
                                     std::to_string(numel));
        if (t.dtype == "BF16") std::memcpy(b.data(), t.data, numel * 2);
        else if (t.dtype == "F32")
            for (size_t i = 0; i < numel; ++i) b[i] = f32_to_bf16_rne(((const float*)t.data)[i]);
        else throw std::runtime_error("EINVAL: dots tensor `" + full + "` has dtype " + t.dtype + " (BF16 / F32 expected)");
        return b;
    };
    auto up16 = [&](const std::vector<uint16_t>& v) {
        void* p = dev_alloc(v.size() * 2);
        HIP_CHECK(hipMemcpy(p, v.data(), v.size() * 2, hipMemcpyHostToDevice));
        return p;
    };
    auto upf = [&](const std::string& name, size_t numel) -> float* {
        std::vector<uint16_t> b = bits(name, numel);
        std::vector<float> f(numel);
        for (size_t i = 0; i < numel; ++i) f[i] = bf16_to_f32(b[i]);
        float* p = (float*)dev_alloc(numel * 4);
        HIP_CHECK(hipMemcpy(p, f.data(), numel * 4, hipMemcpyHostToDevice));
        return p;
    };
    const int D = c_.embed, I = c_.inter, P = c_.patch;
    // patch embed conv [D][C][P][P] as a [D][C*P*P] linear, K zero-padded to a multiple of 64
    patch_k_ = c_.channels * P * P;
    patch_kp_ = (patch_k_ + 63) / 64 * 64;
    {
        std::vector<uint16_t> w = bits("patch_embed.patchifier.proj.weight", (size_t)D * patch_k_);
        std::vector<uint16_t> wp((size_t)D * patch_kp_, 0);
        for (int o = 0; o < D; ++o) std::memcpy(&wp[(size_t)o * patch_kp_], &w[(size_t)o * patch_k_], patch_k_ * 2);
        patch_w_ = up16(wp);
        if (has("patch_embed.patchifier.proj.bias")) patch_b_ = upf("patch_embed.patchifier.proj.bias", D);
        patch_norm_ = upf("patch_embed.patchifier.norm.weight", D);
    }
    {
        const char* e = getenv("DSOCR_DOTS_SWIGLU_FUSE");
        swiglu_fused_ = (!e || atoi(e) != 0) && I % 32 == 0 && D % 32 == 0;
        const char* r = getenv("DSOCR_DOTS_ROPE_FUSE");
        rope_fused_ = (!r || atoi(r) != 0) && D % c_.heads == 0 && D / c_.heads == 128 && D % 128 == 0 && D % 32 == 0;
    }
    // [fc1 | fc3] rows (or bias entries) -> per 32: fc1 32b..32b+31, fc3 32b..32b+31 (the fused epilogue's pairs)
    auto pair32 = [&](std::vector<uint16_t>& v, size_t row) {
        if (!swiglu_fused_) return;
        std::vector<uint16_t> o(v.size());
        for (int b = 0; b < I / 32; ++b)
            for (int k = 0; k < 32; ++k) {
                std::copy_n(v.begin() + (size_t)(32 * b + k) * row, row, o.begin() + (size_t)(64 * b + k) * row);
                std::copy_n(v.begin() + (size_t)(I + 32 * b + k) * row, row, o.begin() + (size_t)(64 * b + 32 + k) * row);
            }
        v.swap(o);
    };
    for (int l = 0; l < c_.layers; ++l) {
        Block b;
        const std::string bp = "blocks." + std::to_string(l) + ".";
        b.n1 = upf(bp + "norm1.weight", D);
        b.n2 = upf(bp + "norm2.weight", D);
        b.qkv = up16(bits(bp + "attn.qkv.weight", (size_t)3 * D * D));
        b.proj = up16(bits(bp + "attn.proj.weight", (size_t)D * D));
        std::vector<uint16_t> f13 = bits(bp + "mlp.fc1.weight", (size_t)I * D);
        std::vector<uint16_t> f3 = bits(bp + "mlp.fc3.weight", (size_t)I * D);
        f13.insert(f13.end(), f3.begin(), f3.end());
        pair32(f13, (size_t)D);
        b.fc13 = up16(f13);
        b.fc2 = up16(bits(bp + "mlp.fc2.weight", (size_t)D * I));
        if (c_.use_bias) {
            if (has(bp + "attn.qkv.bias")) b.b_qkv = upf(bp + "attn.qkv.bias", 3 * D);
            if (has(bp + "attn.proj.bias")) b.b_proj = upf(bp + "attn.proj.bias", D);
            if (has(bp + "mlp.fc1.bias") != has(bp + "mlp.fc3.bias"))
                throw std::runtime_error("EINVAL: fc1 / fc3 biases must both exist or both be absent");
            if (has(bp + "mlp.fc1.bias")) {
                std::vector<uint16_t> a = bits(bp + "mlp.fc1.bias", I), c3 = bits(bp + "mlp.fc3.bias", I);
                a.insert(a.end(), c3.begin(), c3.end());
                pair32(a, 1);
                std::vector<float> f(a.size());
                for (size_t i = 0; i < a.size(); ++i) f[i] = bf16_to_f32(a[i]);
                b.b_fc13 = (float*)dev_alloc(f.size() * 4);
                HIP_CHECK(hipMemcpy(b.b_fc13, f.data(), f.size() * 4, hipMemcpyHostToDevice));
            }
            if (has(bp + "mlp.fc2.bias")) b.b_fc2 = upf(bp + "mlp.fc2.bias", D);
        }
        blocks_.push_back(b);
    }
    if (c_.post_norm) post_norm_ = upf("post_trunk_norm.weight", D);
    const int G = D * c_.merge * c_.merge;
    ln_w_ = upf("merger.ln_q.weight", D);
    ln_b_ = upf("merger.ln_q.bias", D);
    m0_ = up16(bits("merger.mlp.0.weight", (size_t)G * G));
    m0_b_ = upf("merger.mlp.0.bias", G);
    m2_ = up16(bits("merger.mlp.2.weight", (size_t)c_.hidden * G));
    m2_b_ = upf("merger.mlp.2.bias", c_.hidden);
    HIP_CHECK(hipDeviceSynchronize());
}

DotsVision::~DotsVision() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (auto& kv : ws_) (void)hipFree(kv.second.first);
    for (void* p : allocs_) (void)hipFree(p);
    if (stream_) (void)hipStreamDestroy(stream_);
}

void DotsVision::gemm(const void* A, long lda, int M, int N, int K, const void* W, const float* bias, void* C, long ldc,
                      int accumulate, int swiglu) {
    GemmBf16Args g;
    g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.W = W; g.ldw = K; g.bias = bias;
    g.C = reinterpret_cast<float*>(C); g.ldc = ldc; g.accumulate = accumulate; g.out_bf16 = 1; g.swiglu = swiglu;
    launch_gemm_bf16(g, stream_);
}

void DotsVision::embed_device(const float* d_patches, int gt, int gh, int gw, float* d_out) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    hipStream_t st = stream_;
    const int D = c_.embed, I = c_.inter, H = c_.heads, hd = D / H, M = c_.merge, G = D * M * M;
    if (gh % M || gw % M) throw std::runtime_error("EINVAL: grid not divisible by the merge size");
    const long per = (long)gh * gw, N = (long)gt * per, groups = N / (M * M);
    // rotary table (VisionRotaryEmbedding::build_embeddings, dots_vit.rs:717-735): per token
    // [h * inv_freq | w * inv_freq] (f32), cos / sin correctly rounded, duplicated to [t | t].  A function of
    // the grid alone: built on the host once per grid shape and kept on the device (2.7 M double cos / sin
    // per 2044 px page took ~30 ms of host time ahead of the page's first kernel)
    const int rope = hd / 2, axis = rope / 2;
    float* d_cos = (float*)ws("d_cos", (size_t)N * hd * 4);
    float* d_sin = (float*)ws("d_sin", (size_t)N * hd * 4);
    if (rope_key_[0] != gt || rope_key_[1] != gh || rope_key_[2] != gw) {
        std::vector<float> inv(axis);
        for (int i = 0; i < axis; ++i) inv[i] = 1.0f / std::pow(10000.0f, (float)(2 * i) / (float)rope);
        std::vector<float> cs((size_t)N * hd), sn((size_t)N * hd);
        long n = 0;
        for (int f = 0; f < gt; ++f)
            for (int bh = 0; bh < gh / M; ++bh)
                for (int bw = 0; bw < gw / M; ++bw)
                    for (int ih = 0; ih < M; ++ih)
                        for (int iw = 0; iw < M; ++iw, ++n) {
                            const float hp = (float)(bh * M + ih), wp = (float)(bw * M + iw);
                            for (int j = 0; j < rope; ++j) {
                                const float a = j < axis ? hp * inv[j] : wp * inv[j - axis];
                                const float c = (float)std::cos((double)a), s = (float)std::sin((double)a);
                                cs[n * hd + j] = cs[n * hd + rope + j] = c;
                                sn[n * hd + j] = sn[n * hd + rope + j] = s;
                            }
                        }
        HIP_CHECK(hipMemcpyAsync(d_cos, cs.data(), cs.size() * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(d_sin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));  // the host vectors go out of scope
        rope_key_[0] = gt; rope_key_[1] = gh; rope_key_[2] = gw;
    }

    void* X = ws("d_x", (size_t)N * D * 2);
    void* XN = ws("d_xn", (size_t)N * D * 2);
    void* QKV = ws("d_qkv", (size_t)N * 3 * D * 2);
    void* QKVr = rope_fused_ ? nullptr : ws("d_qkvr", (size_t)N * 3 * D * 2);
    void* CTXb = ws("d_ctxb", (size_t)N * D * 2);
    void* GU = swiglu_fused_ ? nullptr : ws("d_gu", (size_t)N * 2 * I * 2);
    void* HB = ws("d_h", (size_t)N * I * 2);
    void* PB = ws("d_pb", (size_t)N * patch_kp_ * 2);
    hipEvent_t ev[4];
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(ev[0], st));
    // patch embed (DotsPatchEmbed::forward 256-261): pixels in the model dtype, conv as a GEMM, + bias, RMSNorm
    launch_dots_to_bf16(d_patches, N, patch_k_, patch_k_, PB, patch_kp_, st);
    gemm(PB, patch_kp_, (int)N, D, patch_kp_, patch_w_, patch_b_, X, D, 0);
    launch_dots_rmsnorm(X, 0, N, D, patch_norm_, (float)c_.eps, X, st);
    HIP_CHECK(hipEventRecord(ev[1], st));
    float attn_ms = 0.f;
    hipEvent_t a0, a1;
    HIP_CHECK(hipEventCreate(&a0));
    HIP_CHECK(hipEventCreate(&a1));
    for (int l = 0; l < c_.layers; ++l) {
        const Block& b = blocks_[l];
        // DotsVisionBlock::forward (305-315) / VisionAttention::forward (364-431)
        launch_dots_rmsnorm(X, 0, N, D, b.n1, (float)c_.eps, XN, st);
        // the rotary of q / k in the q|k|v GEMM's epilogue (rope_fused_) or by dots_rope8 into QKVr below
        const bool rope_in_gemm = rope_fused_;
        if (rope_in_gemm) {
            GemmBf16Args g;
            g.M = (int)N; g.N = 3 * D; g.K = D; g.A = XN; g.lda = D; g.W = b.qkv; g.ldw = D; g.bias = b.b_qkv;
            g.C = reinterpret_cast<float*>(QKV); g.ldc = 3 * D; g.out_bf16 = 1;
            g.rope_cos = d_cos; g.rope_sin = d_sin; g.rope_cols = 2 * D;
            launch_gemm_bf16(g, st);
        } else {
            gemm(XN, D, (int)N, 3 * D, D, b.qkv, b.b_qkv, QKV, 3 * D, 0);
        }
        const bool timed = l < time_layers;
        const float scale = (float)(1.0 / std::sqrt((double)hd));
        // bf16 matrix cores with the same f32 math (attention_bf16.hip): rotated q / k stay bf16
        // (exactly the reference's rounding), the context is written as the bf16 tensor it becomes
        // rotated q / k into QKVr; v is read where the qkv GEMM wrote it
        if (!rope_in_gemm) launch_dots_rope_qk(QKV, N, H, hd, d_cos, d_sin, QKVr, st);
        const uint16_t* QK = (const uint16_t*)(rope_in_gemm ? QKV : QKVr);
        AttnBf16Args a;
        a.q = QK; a.k = QK + D; a.v = (const uint16_t*)QKV + 2 * D;
        a.q_rs = a.k_rs = a.v_rs = 3L * D; a.q_hs = a.k_hs = a.v_hs = hd;
        a.o = CTXb; a.o_rs = D; a.o_hs = hd; a.o_bf16 = 1;
        a.n_seq = gt; a.L = (int)per; a.heads = H; a.kv_heads = H; a.hd = hd; a.scale = scale;
        a.pv_planes = dots_pv_planes();
        if (timed) prof_events() = ProfEvents{a0, a1};  // the launch's own dispatch timestamps
        launch_attention_bf16(a, st);
        if (timed) {
            HIP_CHECK(hipEventSynchronize(a1));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, a0, a1));
            attn_ms += ms;
        }
        gemm(CTXb, D, (int)N, D, D, b.proj, b.b_proj, X, D, 1);
        launch_dots_rmsnorm(X, 0, N, D, b.n2, (float)c_.eps, XN, st);
        if (swiglu_fused_) {  // h straight from the GEMM epilogue (bitwise the same as the two launches)
            gemm(XN, D, (int)N, 2 * I, D, b.fc13, b.b_fc13, HB, I, 0, 1);
        } else {
            gemm(XN, D, (int)N, 2 * I, D, b.fc13, b.b_fc13, GU, 2 * I, 0);
            launch_dots_swiglu(GU, N, I, HB, st);
        }
        gemm(HB, I, (int)N, D, I, b.fc2, b.b_fc2, X, D, 1);
    }
    HIP_CHECK(hipEventRecord(ev[2], st));
    if (post_norm_) launch_dots_rmsnorm(X, 0, N, D, post_norm_, (float)c_.eps, X, st);
    // PatchMerger::forward (676-686): LayerNorm, [groups][D*M*M] view, Linear + gelu, Linear
    launch_dots_layernorm(X, N, D, ln_w_, ln_b_, 1e-6f, XN, st);
    void* P0 = ws("d_m0", (size_t)groups * G * 2);
    gemm(XN, G, (int)groups, G, G, m0_, m0_b_, P0, G, 0);
    launch_dots_gelu(P0, groups * (long)G, st);
    void* OUT = ws("d_mout", (size_t)groups * c_.hidden * 2);
    gemm(P0, G, (int)groups, c_.hidden, G, m2_, m2_b_, OUT, c_.hidden, 0);
    launch_dots_bf16_to_f32(OUT, groups * (long)c_.hidden, d_out, st);
    HIP_CHECK(hipEventRecord(ev[3], st));
    HIP_CHECK(hipEventSynchronize(ev[3]));
    HIP_CHECK(hipGetLastError());
    auto ms = [](hipEvent_t x, hipEvent_t y) { float m = 0.f; (void)hipEventElapsedTime(&m, x, y); return (double)m; };
    t_.patch_ms = ms(ev[0], ev[1]);
    t_.blocks_ms = ms(ev[1], ev[2]);
    t_.merger_ms = ms(ev[2], ev[3]);
    t_.attention_ms = attn_ms;
    t_.tokens = N;
    t_.groups = groups;
    t_.total_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    for (auto& e : ev) (void)hipEventDestroy(e);
    (void)hipEventDestroy(a0);
    (void)hipEventDestroy(a1);
}

std::vector<float> DotsVision::embed(const DotsPatches& p) {
    const long N = (long)p.grid_t * p.grid_h * p.grid_w;
    if ((long)p.data.size() != N * patch_k_) throw std::runtime_error("EINVAL: patch tensor size mismatch");
    const long groups = N / (c_.merge * c_.merge);
    float* d_p = (float*)ws("h_patches", p.data.size() * 4);
    float* d_o = (float*)ws("h_out", (size_t)groups * c_.hidden * 4);
    HIP_CHECK(hipMemcpyAsync(d_p, p.data.data(), p.data.size() * 4, hipMemcpyHostToDevice, stream_));
    embed_device(d_p, p.grid_t, p.grid_h, p.grid_w, d_o);
    std::vector<float> out((size_t)groups * c_.hidden);
    HIP_CHECK(hipMemcpy(out.data(), d_o, out.size() * 4, hipMemcpyDeviceToHost));
    return out;
}

}  // namespace dsocr
