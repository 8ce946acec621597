// Engine: device-resident DeepSeek-OCR (SAM + CLIP + projector + DeepSeek-V2 MoE
// decoder) orchestrating the gfx950 kernels.  One engine per GPU; pages are
// batched inside an engine and sharded across GPUs by the caller (one process per
// GPU, no collectives: SURVEY §8e).
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/kernels.hpp"
#include "config.hpp"

namespace dsocr {

#define HIP_CHECK(x)                                                                                   \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess)                                                                          \
            throw std::runtime_error(std::string("EDEVICE: ") + #x + ": " + hipGetErrorString(_e));    \
    } while (0)

struct Lin {
    void* W = nullptr;
    int wdt = WDT_BF16;
    int N = 0, K = 0;
    float* b = nullptr;
};
struct Ln {
    float* w = nullptr;
    float* b = nullptr;
};

struct SamBlock {
    Ln n1, n2;
    Lin qkv, proj, fc1, fc2;
    bool global = false;
    int rel_len = 0;                       // rows of the stored rel tables (2*tokens-1)
    std::vector<float> relh, relw;         // host copies [rel_len][hd]
    std::map<int, std::pair<float*, float*>> rel_dev;  // grid -> resized device tables
    bool use_rel = false;
};
struct SamW {
    Lin patch;
    bool has_pos = false;
    int pos_grid = 0;
    std::vector<float> pos_host;           // [C][grid][grid]
    std::map<int, float*> pos_dev;         // grid -> [grid*grid][C]
    std::vector<SamBlock> blocks;
    Lin neck0, neck2, net2, net3;
    Ln neck1, neck3;
};
struct ClipLayer {
    Ln ln1, ln2;
    Lin qkv, out, fc1, fc2;
};
struct ClipW {
    float* cls = nullptr;
    std::vector<float> pos_host;           // [seq+1][C]
    std::map<int, float*> pos_dev;         // tokens -> [tokens][C]
    Ln pre;
    std::vector<ClipLayer> layers;
};
struct DecLayer {
    Ln in_norm, post_norm;
    Lin qkv, o;
    bool moe = false;
    Lin gu, down;                 // dense MLP (layer 0) [2I][H], [H][I]
    Lin router;                   // [E][H]
    float* router_bias = nullptr; // e_score_correction_bias
    void* e_gu = nullptr;         // [E][2Im][H]
    void* e_d = nullptr;          // [E][H][Im]
    int e_wdt = WDT_F16;
    bool has_shared = false;
    Lin s_gu, s_d;                // [2Is][H], [H][Is]
    // fragment-ordered copies for the 3..8-page matrix-core kernels (Engine::ensure_mm_weights)
    void* e_gu_swz = nullptr; void* e_d_swz = nullptr; void* s_gu_swz = nullptr; void* s_d_swz = nullptr;
    void* router_swz = nullptr;  // fragment-ordered router rows (3..8 pages: the routing inside gate/up)
    void* qkv_swz = nullptr; void* o_swz = nullptr; void* gu_swz = nullptr;  // ... q/k/v, o_proj, dense gate|up
    // the persistent one-page decode (decode_persist.hip): down projections transposed to [inter][H] rows
    void* e_dT = nullptr;         // routed [E][Im][H]
    void* s_dT = nullptr;         // shared [Is][H] (MoE) / dense [I][H]
};

struct PagePixels {
    int base = 1024, tile = 640;
    bool crop = true;
    int crop_w = 1, crop_h = 1;
    std::vector<float> global_chw;  // [3][G][G]
    int gsize = 0;
    std::vector<float> tiles_chw;   // [n][3][T][T]
    int n_tiles = 0;
    size_t n_image_tokens = 0;
    // optional device-resident copies (dsocr_page_to_device): generate() then reads the pixels
    // from HBM (device-to-device gather) instead of uploading the host arrays
    float* global_dev = nullptr;
    float* tiles_dev = nullptr;
    int dev_ordinal = -1;
    ~PagePixels();
};

struct Timings {
    double vision_prepare_ms = 0, vision_compute_ms = 0, prefill_ms = 0, iterative_ms = 0, generate_ms = 0;
    size_t steps = 0, pages = 0;
    // algorithmic f32 FLOPs of the stage (linears 2 M N K, attention 4 L_q L_k d per head; causal
    // prefill counts the lower triangle): the MFMA roofline's numerator
    double vision_flops = 0, prefill_flops = 0;
};

struct GenRequest {
    std::vector<int> ids;
    std::vector<uint8_t> mask;
    const PagePixels* page = nullptr;
    const float* image_rows = nullptr;
    size_t n_image_rows = 0;
};
struct GenParams {
    size_t max_new = 512;
    float rep_penalty = 1.f;
    int ngram = 20;
    long eos = -1;
    bool ignore_eos = false;
    // sampling (do_sample && temperature > 0, sampling.rs:67-86); rng = init_rng(seed) per call
    bool do_sample = false;
    double temperature = 0.0, top_p = -1.0;
    long top_k = 0;
    bool seed_set = false;
    uint64_t seed = 0;
    bool use_cache = true;  // false: generate_without_cache (model/mod.rs:2051-2283)
    float* trace = nullptr; // host [B][max_new][vocab]: raw logits of every step (parity hook)
};
typedef void (*TokenCb)(size_t, const int64_t*, void*);
// rand_core seed_from_u64 for rand 0.8.5 StdRng, in the layout sampling.hip reads (RNG_WORDS words)
std::vector<uint32_t> rng_state_from_u64(uint64_t seed);

class Engine {
  public:
    Engine(const std::string& config_path, const std::string& weights_path, int device, int dtype, uint64_t seed,
           const std::string& snapshot_path = "");
    ~Engine();

    const ModelConfig& cfg() const { return cfg_; }
    // vision embeddings of pages (host output rows per page concatenated)
    std::vector<std::vector<float>> image_embeddings(const std::vector<const PagePixels*>& pages);
    // batched generate; returns generated ids per page
    std::vector<std::vector<int64_t>> generate(const std::vector<GenRequest>& reqs, const GenParams& p, TokenCb cb,
                                               void* user);
    Timings last_timings() const { return timings_; }
    // Replays the decode MoE grouped GEMV (routed experts, gate/up + down) of every MoE
    // layer on the last decode step's routing, timing each launch pair with HIP events.
    struct KernelProfile {
        double avg_us = 0, bytes = 0, flops = 0;
        int launches = 0;
        double replay_us = 0;
        double ctx_us = 0;  // in-context marginal cost per launch (step graph with / without it)
    };
    struct DecodeProfile {
        KernelProfile moe_gateup, moe_down, attention, lm_head, qkv, o_proj, router, layers_step, lm_head_screened;
        int experts_touched = 0, tokens = 0, kv_len = 0;
        const char* gateup_kernel = "";  // kernels the dispatch picked at this batch size
        const char* down_kernel = "";
    };
    DecodeProfile profile_decode(int iters);
    // In-context launch spans (diagnostics, off by default): while on, every decode step of a generate
    // records per layer the (first wave entry, last wave exit) of its MoE gate/up, MoE down and
    // attention launches, with the distinct experts the MoE launches streamed (WaveSpan +
    // span_reduce_kernel; one extra fold launch after each stamped launch, inside the replayed graph).
    // SPAN_CHAIN (alone): no fold or event between launches; the gate/up, down, attention, o_proj and router
    // launches of every layer stamp their own slot region and one fold runs at the end of each step, so the
    // step is the production chain plus the waves' slot stores: exit(k) - exit(k - 1) is a launch's
    // dispatch-level duration (its boundary included, as a back-to-back rocprofv3 kernel-trace record)
    enum SpanKind : int { SPAN_GATEUP = 0, SPAN_DOWN = 1, SPAN_ATTN = 2, SPAN_KINDS = 3, SPAN_OPROJ = 3, SPAN_ROUTER = 4,
                          SPAN_KINDS_CHAIN = 5 };
    static constexpr int SPAN_FIELDS = 5;
    enum SpanMode : int { SPAN_WAVES = 1, SPAN_EVENTS = 2, SPAN_CHAIN = 4 };  // bit mask; 0 = off
    void set_spans(int mode) { span_mode_ = (mode & SPAN_CHAIN) ? SPAN_CHAIN : mode & (SPAN_WAVES | SPAN_EVENTS); }
    int span_kinds() const { return spans_kinds_; }
    // [kind][layer][step][SPAN_FIELDS] u64 {entry, exit (100 MHz wall clock), distinct experts, waves,
    // dispatch duration in ns (HIP events recorded around the launch inside the replayed graph)} of the
    // last generate with spans on; step = tokens emitted before the step (1 .. steps - 1 are decode steps)
    const std::vector<unsigned long long>& spans() const { return spans_host_; }
    int span_steps() const { return spans_steps_; }  // the steps of spans_host_ (set with it)
    hipStream_t stream() const { return stream_; }
    // persistent decode diagnostics: mode 1 = the next generate times every persistent launch with HIP events
    // and records the phase clocks (PK_STAMPS per workgroup and layer) of its decode steps; read them after it
    void set_persist_stamps(int mode) { persist_stamp_mode_ = mode; }
    bool persist_used() const { return persist_active_; }
    const std::vector<unsigned long long>& persist_stamps() const { return persist_stamps_host_; }
    const std::vector<double>& persist_launch_us() const { return persist_ev_us_; }
    void upload_page(PagePixels& pg);
    void prepare_page_device(const uint8_t* rgb, int w, int h, PagePixels& px);

  private:
    // ---- loading
    void load_weights(const std::string& path, uint64_t seed, const std::string& snapshot_path);
    // ---- workspace
    void* ws(const std::string& name, size_t bytes);
    float* wsf(const std::string& name, size_t n) { return (float*)ws(name, n * sizeof(float)); }
    int* wsi(const std::string& name, size_t n) { return (int*)ws(name, n * sizeof(int)); }
    long* wsl(const std::string& name, size_t n) { return (long*)ws(name, n * sizeof(long)); }
    template <typename T>
    T* upload(const std::string& name, const std::vector<T>& v) {
        // host vectors are often temporaries: stage them in a per-name pinned buffer and copy
        // asynchronously (each name is uploaded at most once per generate(), which ends with a
        // stream synchronisation, so a staging buffer is never rewritten while in flight)
        const size_t bytes = v.size() * sizeof(T);
        T* p = (T*)ws(name, bytes + 16);
        if (!v.empty()) {
            void* h = pinned(name, bytes);
            std::memcpy(h, v.data(), bytes);
            HIP_CHECK(hipMemcpyAsync(p, h, bytes, hipMemcpyHostToDevice, stream_));
        }
        return p;
    }
    void* pinned(const std::string& name, size_t bytes);
    // ---- compute pieces
    void linear(const float* x, int M, int ldx, const Lin& l, float* y, int ldy, int act = 0, int accumulate = 0,
                const int* c_rows = nullptr);
    float* sam_pos(int g);
    std::pair<float*, float*> sam_rel(SamBlock& b, int g);
    float* clip_pos(int tokens);
    // runs SAM+CLIP+projector on n images of size S; returns device rows [n*(S/64)^2][H] in buffer `out`
    float* vision_pass(const float* imgs, int n, int S, const std::string& out);
    void prefill(int B, const std::vector<int>& rows_per_page, const float* x0, int Lmax);
    void decode_step(int B, int Lmax);
    // one page: every decoder layer of a step as one persistent launch (decode_persist.hip) when the model's
    // shape and dtypes fit it, all 256 workgroups are resident and DSOCR_PERSIST=1 (opt-in)
    bool persist_ok(int B, int Lmax);
    void ensure_persist();
    MoeDecodeArgs moe_args(int l, int B, float* X);
    void decode_head(int B, DecSampleArgs& sa, const SampleArgs& pen);
    void reserve_head_ws(int B);
    LmHeadQ8Args head_q8_args(int B);
    bool screen_applies(int B, float rep_penalty) const;
    void layer_forward_prefill(int l, int T, int B, const int* row_page, const int* row_pos, const long* q_off,
                               const long* kv_off, const long* o_off, const int* seq_len, int max_len, int Lmax);

    ModelConfig cfg_;
    int device_ = 0;
    int dtype_ = 1;
    hipStream_t stream_ = nullptr;
    // the page batch's second vision pass (tiles beside the global views) runs on vstream_ with its own
    // workspaces (ws_prefix_): the two towers' small CLIP / norm kernels fill each other's idle CUs
    hipStream_t vstream_ = nullptr;
    hipEvent_t vis_ev_[2] = {nullptr, nullptr};
    std::string ws_prefix_;
    std::vector<void*> allocations_;
    std::map<std::string, std::pair<void*, size_t>> ws_;
    bool capturing_ = false;

    SamW sam_;
    ClipW clip_;
    Lin proj_;
    float* newline_ = nullptr;
    float* separator_ = nullptr;
    void* embed_ = nullptr;
    int embed_dt_ = WDT_F16;
    std::vector<DecLayer> layers_;
    float* final_norm_ = nullptr;
    Lin lm_head_;
    void* lm_swz_ = nullptr;         // lm_head in dec_mm fragment order (3..8 pages; made on first use)
    void ensure_mm_weights(int B);
    bool dense_mm_ok(const DecLayer& d, int B) const;
    void* lmq_ = nullptr;            // int8 [vocab][hidden] screening copy of lm_head
    float* lmq_scale_ = nullptr;     // per-row scale
    float* lmq_bound_ = nullptr;     // per-row error-bound factor (times ||x||)
    float* lmq_qnorm_ = nullptr;     // per-row s ||Q|| (3..8 pages: the token rows' int8 representation error)
    void* lmq_frag_ = nullptr;       // the int8 rows in the int8 matrix cores' fragment order (3..8 pages)
    float* rope_cos_ = nullptr;
    float* rope_sin_ = nullptr;
    int rope_cap_ = 0;
    float* ones_ = nullptr;
    int* iota_ = nullptr;
    int small_cap_ = 0;
    // kv cache
    float* kc_ = nullptr;
    float* vc_ = nullptr;
    size_t kv_bytes_ = 0;
    long page_stride_ = 0, head_stride_ = 0;
    Timings timings_;
    double flops_acc_ = 0;  // FLOPs issued by linear() / attention since the last stage mark
    std::vector<int> prefill_lens_;  // rows per page of the prefill being issued
    int last_B_ = 0;
    std::map<std::string, std::pair<void*, size_t>> pinned_;
    std::map<std::pair<int, int>, std::pair<int*, int*>> winmaps_;  // (n, grid) -> tok2win, win2tok
    int last_Lmax_ = 0;
    float* trace_ = nullptr;  // device logits trace of the running generate (parity hook)
    int span_mode_ = 0;
    // profile_decode: launches decode_step leaves out (the with / without step-graph differences)
    enum StepSkip : int { SKIP_GATEUP = 1, SKIP_DOWN = 2, SKIP_ATTN = 4 };
    int step_skip_ = 0;
    static bool qkv_attn_fused();
    static int att_kv_delay();
    unsigned long long* span_slots_ = nullptr;  // device [SPAN_SLOTS][2]
    unsigned long long* span_rec_ = nullptr;    // device [SPAN_KINDS][layers][span_cap_][4]
    const int* span_step_ = nullptr;            // device step counter (out_len of page 0)
    int span_cap_ = 0;
    std::vector<unsigned long long> spans_host_;
    int spans_steps_ = 0;
    std::vector<hipEvent_t> span_ev_;           // [SPAN_KINDS][layers][2]
    std::vector<double> span_ev_ns_;            // [SPAN_KINDS][layers][span_cap_]
    int spans_kinds_ = SPAN_KINDS;
    bool chain_active_ = false;                 // a SPAN_CHAIN generate is running
    unsigned long long* span_chain_ = nullptr;  // device [layers * SPAN_KINDS_CHAIN][SPAN_SLOTS][2]
    unsigned long long* span_chain_rec_ = nullptr;  // device [span_cap_][layers * SPAN_KINDS_CHAIN][4]
    unsigned long long* span_tmark_ = nullptr;  // device [2]
    unsigned long long* chain_slots(int layer, int kind) const {
        return chain_active_ ? span_chain_ + ((size_t)layer * SPAN_KINDS_CHAIN + kind) * SPAN_SLOTS * 2 : nullptr;
    }
    unsigned long long* span_rec(int kind, int layer) const {
        return span_rec_ + ((size_t)kind * cfg_.lang.layers + layer) * span_cap_ * 4;
    }
    long trace_steps_ = 0;
    bool persist_active_ = false;               // this generate's decode steps run dec_persist
    PersistLayerW* persist_lw_ = nullptr;       // device [layers]
    unsigned long long* persist_g_ = nullptr;   // granules [dec_persist_granules(layers)]
    unsigned long long* persist_stamps_ = nullptr;  // device phase clocks of the last stamped step (optional)
    int persist_stamp_mode_ = 0;                // 1: the next generate records stamps of its decode steps
    int persist_stamp_pos0_ = 0, persist_stamp_cap_ = 0;
    std::vector<unsigned long long> persist_stamps_host_;
    std::vector<hipEvent_t> persist_ev_;        // [steps][2] HIP events around each persistent launch (timing mode)
    std::vector<double> persist_ev_us_;

    void* dev_alloc(size_t bytes);
    void ensure_rope(int len);
    void ensure_small(int n);
};

}  // namespace dsocr
