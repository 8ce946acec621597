// dots.ocr vision tower on one GPU (BASELINE configs[3]: "dots-ocr bf16 high-res 2048px page"):
// DotsVisionModel (crates/infer-dots/src/vision/dots_vit.rs) with its preprocessing
// (vision/preprocess.rs), the reference's bf16 semantics, gfx950 kernels (gemm_bf16 with the
// bf16-output epilogue, dots.hip, the f32 flash attention).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "../common/json.hpp"
#include "../kernels/kernels.hpp"

namespace dsocr {

struct DotsConfig {
    // DotsVisionConfig (infer-dots/src/config/mod.rs:9-26)
    int embed = 1536, hidden = 1536, inter = 4224, layers = 42, heads = 12, channels = 3, patch = 14, merge = 2,
        temporal = 1;
    double eps = 1e-5;
    bool use_bias = false, post_norm = true;
    // DotsPreprocessConfig (vision/preprocess.rs:11-19; defaults = the upstream preprocessor_config.json)
    long min_pixels = 3136, max_pixels = 11289600;
    float mean[3] = {0.48145466f, 0.4578275f, 0.40821073f}, stdv[3] = {0.26862954f, 0.26130258f, 0.27577711f};
    std::string prefix = "vision_tower.";
};
DotsConfig parse_dots_config(const Json& j);

// smart_resize (preprocess.rs:244-279)
void dots_smart_resize(long height, long width, long factor, long min_pixels, long max_pixels, long* rh, long* rw);

struct DotsPatches {
    std::vector<float> data;  // [N][3 * p * p] in merge-group order (patches_from_normalised)
    int grid_t = 1, grid_h = 0, grid_w = 0;
    int resized_h = 0, resized_w = 0;
};
// preprocess_image (preprocess.rs:103-145): smart_resize, resize (fast_image_resize's Catmull-Rom
// convolution restated, host_ops.hpp resize_catmull_rom_fir; parity unpinned), normalise, patches in
// merge-group order
DotsPatches dots_preprocess(const DotsConfig& c, const uint8_t* rgb, int w, int h);

struct DotsTimings {
    double total_ms = 0, patch_ms = 0, blocks_ms = 0, attention_ms = 0, merger_ms = 0;
    long tokens = 0, groups = 0;
};

class DotsVision {
  public:
    DotsVision(const std::string& config_path, const std::string& weights_path, uint64_t seed, int device);
    ~DotsVision();
    const DotsConfig& cfg() const { return c_; }
    // DotsVisionModel::forward for one image: [groups][hidden] (bf16 values as f32) into `out`
    std::vector<float> embed(const DotsPatches& p);
    // the same on patches already in device memory (bench: inputs resident in HBM)
    void embed_device(const float* d_patches, int grid_t, int grid_h, int grid_w, float* d_out);
    DotsTimings last_timings() const { return t_; }
    // per-layer attention time measured with events (first `layers` blocks; 0 = timing off)
    int time_layers = 0;

  private:
    struct Block {
        float* n1 = nullptr;
        float* n2 = nullptr;
        void* qkv = nullptr;   // bf16 [3D][D]
        void* proj = nullptr;  // bf16 [D][D]
        void* fc13 = nullptr;  // bf16 [2I][D] = [fc1 | fc3], or per 32 rows [fc1 32 | fc3 32] when swiglu_fused_
        void* fc2 = nullptr;   // bf16 [D][I]
        float *b_qkv = nullptr, *b_proj = nullptr, *b_fc13 = nullptr, *b_fc2 = nullptr;
    };
    void* ws(const std::string& name, size_t bytes);
    void* dev_alloc(size_t bytes);
    void gemm(const void* A, long lda, int M, int N, int K, const void* W, const float* bias, void* C, long ldc,
              int accumulate, int swiglu = 0);
    // fc1|fc3 GEMM with the SwiGLU in its epilogue (DSOCR_DOTS_SWIGLU_FUSE, default on; needs I % 32, D % 32)
    bool swiglu_fused_ = false;
    // q / k rotary in the q|k|v GEMM's epilogue (DSOCR_DOTS_ROPE_FUSE, default on; needs 128-dim heads)
    bool rope_fused_ = false;

    DotsConfig c_;
    int device_ = 0;
    hipStream_t stream_ = nullptr;
    std::vector<void*> allocs_;
    std::map<std::string, std::pair<void*, size_t>> ws_;
    long rope_key_[3] = {-1, -1, -1};  // (gt, gh, gw) of the rotary table now in d_cos / d_sin
    void* patch_w_ = nullptr;  // bf16 [D][Kp] (K = 3 p p zero-padded to a multiple of 64)
    int patch_k_ = 0, patch_kp_ = 0;
    float* patch_b_ = nullptr;
    float* patch_norm_ = nullptr;
    std::vector<Block> blocks_;
    float* post_norm_ = nullptr;
    float *ln_w_ = nullptr, *ln_b_ = nullptr;
    void* m0_ = nullptr;
    float* m0_b_ = nullptr;
    void* m2_ = nullptr;
    float* m2_b_ = nullptr;
    DotsTimings t_;
};

}  // namespace dsocr
