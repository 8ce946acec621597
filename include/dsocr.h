/*
 * dsocr.h — C ABI of the MI355X-native DeepSeek-OCR page engine (gfx950).
 *
 * Drop-in boundary for the reference's `OcrEngine` (TimmyOVO/deepseek-ocr.rs,
 * crates/core/src/inference.rs:189-209) and its loader `load_model`
 * (crates/infer-deepseek/src/model/mod.rs:90-115).  A Rust FFI crate (or the
 * Python mirror in deepseek-ocr.rs_amd/dsocr) binds these symbols; see
 * INTEGRATION.md.  Plain C types only: no torch, no C++ types.
 *
 * Ownership: the caller owns every host buffer it passes; the engine owns its
 * device memory.  An engine handle is Send-not-Sync like the reference engine
 * (server/src/state.rs:22 keeps one behind a Mutex): one thread at a time.
 * Errors: every call returns a dsocr_status; dsocr_last_error() gives the
 * thread-local message.  DSOCR_EINVAL maps to the reference server's HTTP 400
 * ("prompt formatting failed" / "prompt/image embedding mismatch",
 * server/src/generation.rs:108-118), everything else to 500.
 */
#ifndef DSOCR_H
#define DSOCR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    DSOCR_OK = 0,
    DSOCR_EINVAL = 1,    /* bad arguments / prompt-image mismatch (reference: anyhow context -> 400) */
    DSOCR_ENOENT = 2,    /* missing file or tensor */
    DSOCR_EDEVICE = 3,   /* HIP runtime failure / no gfx950 device */
    DSOCR_ENOMEM = 4,    /* device allocation failed */
    DSOCR_EINTERNAL = 5  /* anything else (-> 500) */
} dsocr_status;

/* Reference `Precision` (core/src/runtime.rs:15-19).  F16 = the reference's GPU default:
 * decoder weights rounded bf16->f16, f32 compute. */
typedef enum { DSOCR_F32 = 0, DSOCR_F16 = 1, DSOCR_BF16 = 2 } dsocr_dtype;

typedef struct dsocr_engine dsocr_engine;
typedef struct dsocr_page_pixels dsocr_page_pixels;

/* ModelLoadArgs (core/src/inference.rs:178-186). weights_path == NULL selects the
 * deterministic synthetic checkpoint (seeded, real tensor names/shapes). */
typedef struct {
    const char* config_path;
    const char* weights_path;
    const char* snapshot_path; /* optional .dsq snapshot (crates/dsq): its Q4_K / Q6_K / Q8_0 / float linears
                                  replace the checkpoint's, decoded to fp16 on the GPU at load (dtype must be
                                  DSOCR_F16); NULL = none */
    int device_ordinal;
    dsocr_dtype dtype;
    uint64_t synthetic_seed;
} dsocr_load_args;

/* VisionSettings (core/src/inference.rs:13-18). */
typedef struct {
    uint32_t base_size;
    uint32_t image_size;
    int crop_mode;
} dsocr_vision_settings;

/* DecodeParameters (core/src/inference.rs:21-79) + generation options (model/mod.rs:177-218). */
typedef struct {
    size_t max_new_tokens;
    int do_sample;               /* sampling iff do_sample && temperature > 0 (sampling.rs:67), else greedy */
    double temperature;
    double top_p;                /* active in [0, 1) (apply_top_p); otherwise unset */
    size_t top_k;                /* 0: unset */
    float repetition_penalty;    /* 1.0: off */
    size_t no_repeat_ngram_size; /* 0 or 1: off (reference default 20) */
    uint64_t seed;               /* StdRng::seed_from_u64(seed) when has_seed, else entropy */
    int use_cache;               /* 0: generate_without_cache (model/mod.rs:2051-2283): the whole forward re-runs
                                    on prompt + generated tokens every step (same ids, O(n^2) work) */
    int64_t eos_token_id;        /* < 0: none (reference: config eos_token_id) */
    int ignore_eos;              /* benchmark mode: always produce max_new_tokens */
    int has_seed;                /* DecodeParameters::seed is Some */
} dsocr_decode_params;

/* stream callback: invoked after each generated token (model/mod.rs:1980-1982). */
typedef void (*dsocr_stream_cb)(size_t n_generated, const int64_t* tokens, void* user);

/* One page of a batched generate call. */
typedef struct {
    const int64_t* input_ids;      /* [prompt_len], BOS first (build_prompt_tokens) */
    const uint8_t* image_mask;     /* [prompt_len], 1 on <image> slots; may be NULL if no image */
    size_t prompt_len;
    const dsocr_page_pixels* page; /* if non-NULL the vision tower runs on device for this page */
    const float* image_rows;       /* else: host image embeddings [n_image_rows][hidden] (or NULL) */
    size_t n_image_rows;
} dsocr_request;

typedef struct {
    int64_t* out_ids; /* caller buffer, capacity max_new_tokens */
    size_t cap;
    size_t n_out;
    dsocr_status status;
} dsocr_result;

/* Stage times of the last call, named after the reference Timer events
 * (model/mod.rs:1871,1924,1975,2464,2498). */
typedef struct {
    double vision_prepare_ms;     /* vision.prepare_inputs (host, this call's pages) */
    double vision_compute_ms;     /* vision.compute_embeddings */
    double decode_prefill_ms;     /* decode.prefill */
    double decode_iterative_ms;   /* decode.iterative */
    double decode_generate_ms;    /* decode.generate */
    size_t decode_steps;          /* decode forwards executed */
    size_t pages;
    double vision_flops;          /* algorithmic f32 FLOPs of vision.compute_embeddings (linears 2MNK, */
    double prefill_flops;         /* attention 4 Lq Lk d per head, causal: lower triangle) and of decode.prefill */
} dsocr_timings;

/* ---- engine lifecycle (load_model, model/mod.rs:90-115; DeepseekOcrModel::load 946-1105) */
dsocr_status dsocr_engine_load(const dsocr_load_args* args, dsocr_engine** out);
void dsocr_engine_free(dsocr_engine* e);
const char* dsocr_last_error(void);
/* hidden size (image-row width), vocab, eos id, layers */
dsocr_status dsocr_engine_info(const dsocr_engine* e, size_t* hidden, size_t* vocab, int64_t* eos_token_id,
                               size_t* num_layers);

/* ---- host preprocessing a1-a3 (build_global_view 2308-2330, dynamic_preprocess_with_params
 *      preprocess.rs:67-138, image_to_tensor 2332-2347).  rgb: HWC uint8. */
dsocr_status dsocr_prepare_page(const uint8_t* rgb, uint32_t width, uint32_t height,
                                const dsocr_vision_settings* vs, dsocr_page_pixels** out);
/* a1-a3 on the GPU of `e` (vision/resample.rs + preprocess.rs + model/mod.rs:2295-2347, the same
 * results as dsocr_prepare_page bit for bit): only the RGB8 bytes cross PCIe, the f32 CHW tensors
 * are produced in HBM.  The page's pixels are device-resident only (dsocr_page_pixels_view returns
 * NULL arrays; dsocr_page_read_device copies them back). */
dsocr_status dsocr_prepare_page_device(dsocr_engine* e, const uint8_t* rgb, uint32_t w, uint32_t h,
                                       const dsocr_vision_settings* vs, dsocr_page_pixels** out);
dsocr_status dsocr_page_read_device(const dsocr_page_pixels* p, float* global_out /* [3][G][G] */,
                                    float* tiles_out /* [n_tiles][3][T][T] or NULL */);
void dsocr_page_free(dsocr_page_pixels* p);
/* Stage the page's preprocessed pixels in the engine's device memory (HBM) once, e.g. ahead of
 * a timed or latency-critical generate; later calls gather them device-to-device.  The device
 * copy is owned by the page (freed by dsocr_page_free).  Reference counterpart: none (the
 * reference re-uploads every tensor per call, model/mod.rs:2332-2347). */
dsocr_status dsocr_page_to_device(dsocr_engine* e, dsocr_page_pixels* p);
/* crop grid (w,h), tile count, and the number of <image> slots build_image_placeholders emits */
dsocr_status dsocr_page_info(const dsocr_page_pixels* p, uint32_t* crop_w, uint32_t* crop_h, uint32_t* n_tiles,
                             size_t* n_image_tokens);
/* normalised CHW f32 views: global [3][S][S], tiles [n][3][T][T] (NULL if none) */
dsocr_status dsocr_page_pixels_view(const dsocr_page_pixels* p, const float** global_chw, uint32_t* global_size,
                                    const float** tiles_chw, uint32_t* tile_size);

/* ---- compute_image_embeddings (model/mod.rs:1276-1314): rows [n][hidden] per page,
 *      concatenated into `out` (capacity cap_rows); rows_per_page[i] receives each count. */
dsocr_status dsocr_image_embeddings(dsocr_engine* e, const dsocr_page_pixels* const* pages, size_t n_pages,
                                    float* out, size_t cap_rows, size_t* rows_per_page);

/* ---- generate (model/mod.rs:1870-2048), batch-1 semantics per page */
dsocr_status dsocr_generate(dsocr_engine* e, const dsocr_request* req, const dsocr_decode_params* params,
                            dsocr_stream_cb cb, void* user, int64_t* out_ids, size_t cap, size_t* n_out);
/* B pages at once (vision batched, prefill batched, decode batched); each result equals dsocr_generate. */
dsocr_status dsocr_generate_batch(dsocr_engine* e, size_t n, const dsocr_request* reqs,
                                  const dsocr_decode_params* params, dsocr_result* results);
dsocr_status dsocr_last_timings(const dsocr_engine* e, dsocr_timings* t);
/* Parity hook: dsocr_generate_batch plus the raw logits (before repetition penalty and n-gram ban) of
 * every step of every page, logits_out [n][max_new_tokens][vocab] host f32, step s = the logits the
 * s-th generated token was selected from (step 0 = the prefill's last row).  The reference's
 * counterparts: the cli-debug top-2 logits dump (crates/infer-deepseek/src/debug.rs:17-21,
 * model/mod.rs:1937-1949) and the teacher-forcing logits its baseline tests compare
 * (tests/baseline.rs:1108).  Selection runs on the exact lm_head while tracing (the screened head
 * never forms the full logits; its ids equal the exact head's).  logits_cap = capacity of logits_out in
 * floats; DSOCR_EINVAL (nothing written) when n * max_new_tokens * vocab exceeds it. */
dsocr_status dsocr_generate_trace(dsocr_engine* e, size_t n, const dsocr_request* reqs,
                                  const dsocr_decode_params* params, dsocr_result* results, float* logits_out,
                                  size_t logits_cap);

/* Decode-kernel profile (bench roofline): replays the dominant decode kernels of the
 * last generate() call on its final routing / KV state, each timed with HIP events on
 * the engine stream.  avg_us = mean duration of one launch; bytes / flops = algorithmic
 * HBM traffic / work of one launch (fp16 weights touched + f32 activations / KV reads). */
typedef struct dsocr_kernel_profile {
    double avg_us;     /* one launch between its own pair of events (the begin-to-end rocprofv3 reports) */
    double bytes;
    double flops;
    int launches;
    double replay_us;  /* per launch in a back-to-back hipGraph replay (incl. the kernel boundary) */
    double ctx_us;     /* in context: (one decode step's layers replayed as a hipGraph - the same graph without this
                          launch in any layer) / its launches per step, i.e. what it costs inside the real step
                          chain, its own dispatch included (MoE gate/up, MoE down, attention; else 0) */
} dsocr_kernel_profile;
typedef struct dsocr_decode_profile {
    dsocr_kernel_profile moe_gateup;  /* decode MoE gate/up launch(es) of one layer (routed + shared): the kernel
                                         the dispatch picks at this batch size, named in moe_gateup_kernel */
    dsocr_kernel_profile moe_down;    /* routed + shared down + combine + residual (moe_down_kernel) */
    dsocr_kernel_profile attention;   /* dec_attn_kernel (RoPE / KV append / flash-decoding / combine): one layer */
    dsocr_kernel_profile lm_head;     /* exact lm_head over the 129280 x 1280 rows: dec_gemv_stream (1-2 pages) or
                                         the matrix-core dec_mm on the fragment-ordered copy (3-8 pages) */
    int experts_touched;              /* routed experts active in the replayed step (per layer, summed / layers) */
    int tokens;                       /* pages in the batch */
    int kv_len;                       /* keys attended by page 0 */
    dsocr_kernel_profile qkv;         /* RMSNorm + fused q/k/v projection, one layer (dec_qkv_rope with RoPE in the
                                         epilogue at 1 page, dec_gemv at 2, dec_mm at 3-8) */
    dsocr_kernel_profile o_proj;      /* o_proj + residual, one layer (dec_gemv at 1-2 pages, dec_mm at 3-8) */
    dsocr_kernel_profile router;      /* MoE router: dec_gemv logits at 1-2 pages (the mix kernels rank-select),
                                         dec_route_grp (RMSNorm + logits + top-k + expert records) at 3-8 */
    dsocr_kernel_profile layers_step; /* every decoder layer of one decode step, replayed as one hipGraph */
    dsocr_kernel_profile lm_head_screened; /* int8 screened lm_head + exact rescoring selection (B <= 8, no penalty;
                                              3..8: one int8 stream on the int8 matrix cores) */
    const char* moe_gateup_kernel;    /* static strings: kernel names of the two MoE entries above */
    const char* moe_down_kernel;
} dsocr_decode_profile;
dsocr_status dsocr_profile_decode(dsocr_engine* e, int iters, dsocr_decode_profile* out);

/* In-context launch spans (diagnostics for the roofline line; no reference counterpart).  mode is a bit
 * mask, 0 = off: 1 = wave spans (every wave of the MoE gate/up (kind 0), MoE down (1) and attention (2)
 * launches writes its entry / exit s_memrealtime (100 MHz) to a slot, a one-block fold launch after each
 * keeps the first entry / last exit), 2 = HIP events recorded on the stream around those launches inside
 * the replayed step graph (the dispatch-level duration rocprofv3's kernel trace reports; read back after
 * every step; no extra kernel runs, so the step is the production chain plus the event markers), 4 (alone)
 * = chain spans: the gate/up, down, attention, o_proj (kind 3) and router (kind 4) launches of every layer
 * stamp their waves into their own slot regions and ONE fold launch runs at the end of each step (no fold
 * or event between launches), so exit(launch) - exit(previous launch) is the launch's dispatch-level
 * duration with its boundary, as rocprofv3 records a back-to-back dispatch; kinds = 5 then.  Mode 1
 * also records the distinct experts each MoE launch streamed (mode 2 alone leaves that field 0).  The decode steps
 * of every following generate are recorded; dsocr_engine_spans copies the last such generate's records,
 * [kinds][layers][steps][5] uint64 {entry, exit, distinct experts, waves, event duration ns}, into out
 * (cap = capacity in uint64; DSOCR_EINVAL if short; out NULL: only the dimensions are returned);
 * step s = tokens emitted before the step, decode steps are 1 .. steps - 1, unused entries are 0. */
dsocr_status dsocr_engine_set_spans(dsocr_engine* e, int mode);
dsocr_status dsocr_engine_spans(const dsocr_engine* e, uint64_t* out, size_t cap, size_t* kinds, size_t* layers,
                                size_t* steps);

/* ---- one-page persistent decode (decode_persist.hip; no reference counterpart: the reference's decode step is
 * Candle's per-op launches, model/mod.rs:1977-2034).  At B = 1 every decoder layer of a step runs as ONE
 * persistent launch when DSOCR_PERSIST=1 and the model's shape and dtypes fit it (opt-in: measured slower than
 * the per-layer launch chain).
 * dsocr_engine_set_persist_stamps(e, 1): the next generate times each persistent launch with HIP events and
 * records its phase clocks; dsocr_engine_persist_info then returns whether the last generate used the persistent
 * launch (*used), the launch durations in us (durations[cap_d], *n_launches) and the phase clocks
 * [steps][256 workgroups][layers][9] uint64 (s_memrealtime, 100 MHz) of its decode steps (stamps[cap_s],
 * *n_stamps; step i = position prompt_len + i).  NULL arrays: sizes only. */
dsocr_status dsocr_engine_set_persist_stamps(dsocr_engine* e, int mode);
dsocr_status dsocr_engine_persist_info(const dsocr_engine* e, int* used, double* durations, size_t cap_d,
                                       size_t* n_launches, uint64_t* stamps, size_t cap_s, size_t* n_stamps);

/* ---- device helpers for tests / tooling (plain pointers; no torch) */
dsocr_status dsocr_device_count(int* n);
dsocr_status dsocr_dev_alloc(size_t bytes, void** ptr);
dsocr_status dsocr_dev_free(void* ptr);
dsocr_status dsocr_memcpy_h2d(void* dst, const void* src, size_t bytes);
dsocr_status dsocr_memcpy_d2h(void* dst, const void* src, size_t bytes);
dsocr_status dsocr_dev_sync(void);
/* host: deterministic synthetic bf16 weights (same recipe as oracle/synth.c) */
dsocr_status dsocr_synth_bf16(const char* name, uint64_t seed, uint64_t n, uint16_t* out);
/* host: Pillow-exact bicubic resize (vision/resample.rs:101-160), RGB8 HWC */
dsocr_status dsocr_resize_bicubic(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw,
                                  uint32_t dh);
/* fast_image_resize Convolution(CatmullRom) on RGB8 HWC (host; the dots.ocr and PaddleOCR-VL preprocessing resize,
 * crates/infer-paddleocr/src/vision/preprocess.rs:223-243, infer-dots vision/preprocess.rs) */
dsocr_status dsocr_resize_catmull_rom(const uint8_t* src, uint32_t sw, uint32_t sh, uint8_t* dst, uint32_t dw,
                                      uint32_t dh);

/* ---- kernel-level entry points (device pointers, default stream) for parity tests */
/* C[M][N] = act(A[M][K] . W[N][K]^T + bias) (+ C if accumulate); wdtype 0 = bf16, 1 = f16 */
dsocr_status dsocr_k_gemm(int M, int N, int K, const float* A, const void* W, int wdtype, const float* bias, float* C,
                          int act, int accumulate);
/* Vision / prefill linear (sam.rs:656-701, clip.rs:418-447; block.rs linears) on the fused split kernel:
 * f32 A [M][K], 16-bit W [N][K] (wdtype 0 bf16: 3 bf16 planes of A; 1 f16: W split into hi / lo bf16 too,
 * 5 products), C = act(A W^T + bias) (+ C), exact f32 products; splits <= 0 picks the engine's split-K. */
dsocr_status dsocr_k_gemm_f32a(int M, int N, int K, const float* A, const void* W, int wdtype, const float* bias,
                               float* C, int act, int accumulate, int splits);
/* Routed-expert linear of the prefill (block.rs:1215-1395 applies expert e to the rows that picked it):
 * group g owns gathered rows group_off[g] .. group_off[g+1] (device array), row r reads A row
 * a_rows ? a_rows[r] : r and writes C row c_rows ? c_rows[r] : r (-1 drops it), weights W + g * w_group_stride
 * ([N][K] 16-bit), bias + g * bias_group_stride.  kernel 0: the engine's dispatch (launch_gemm); 1 / 2: the
 * grouped kernel with 32- / 128-row tiles whatever the rows per group. */
dsocr_status dsocr_k_gemm_grouped(int M, int N, int K, const float* A, int lda, const int* a_rows, const void* W,
                                  int wdtype, long long w_group_stride, const float* bias, long long bias_group_stride,
                                  float* C, int ldc, const int* c_rows, int act, int accumulate, const int* group_off,
                                  int groups, int max_group_rows, int kernel);
/* Decode linear (transformer/block.rs attention / MLP projections at seq_len 1): y[M][N] =
 * act(xn . W^T + bias) (+ y), xn = rmsnorm(x; norm_w, eps) when norm_w != NULL (block.rs:24-29), else x. */
dsocr_status dsocr_k_gemv(int M, int N, int K, const float* x, const float* norm_w, float eps, const void* W,
                          int wdtype, const float* bias, float* y, int act, int accumulate);
/* Long-K decode linear for 1..8 rows on the matrix cores (the dense layer-0 down projection of the
 * 3..8-page decode, K = 6848): y[M][N] (+)= x . W^T + bias, split-K with an in-launch ordered sum. */
dsocr_status dsocr_k_gemv_splitk(int M, int N, int K, const float* x, const void* W, int wdtype, const float* bias,
                                 float* y, int accumulate);
dsocr_status dsocr_k_layernorm(int rows, int cols, const float* x, const float* w, const float* b, float eps,
                               float* y);
/* DSQ record payload (device bytes, crates/dsq/src/lib.rs:60-110 dtype codes 0/1/8/12/14/16) ->
 * fp16 [out_dim][in_dim] on the device; replaces dsq-runtime's qtensor_from_ggml + QMatMul for the
 * dequant-on-load path (crates/dsq-runtime/src/lib.rs:336-366). */
dsocr_status dsocr_k_dsq_dequant(int qtype, const void* src, size_t src_bytes, size_t out_dim, size_t in_dim,
                                 void* out_f16);
dsocr_status dsocr_k_rmsnorm(int rows, int cols, const float* x, const float* w, float eps, float* y);
/* softmax(scale * q.k^T [+ SAM decomposed rel-pos] [causal]) . v over n_seq uniform sequences of L
 * rows; q,k,v,o are [n_seq*L][heads*hd]; relh/relw (optional) are the resized [2g-1][hd] tables of
 * a gh x gw grid (gh*gw == L). */
dsocr_status dsocr_k_attention(int n_seq, int L, int heads, int hd, float scale, int causal, const float* q,
                               const float* k, const float* v, float* o, const float* relh, const float* relw, int gh,
                               int gw);
/* Bidirectional attention over bf16 values with f32 math on the bf16 matrix cores (the dots.ocr ViT,
 * dots_vit.rs:433-498): qkv bf16 [n_seq*L][ld] holding q | k | v (heads*hd each) per row; o [n_seq*L][o_ld]
 * f32 (o_bf16 = 0) or bf16 (o_bf16 = 1, RNE). */
dsocr_status dsocr_k_attention_bf16(int n_seq, int L, int heads, int hd, float scale, const void* qkv, long ld,
                                    void* o, long o_ld, int o_bf16);
/* Decode attention step (block.rs:608-789 at seq_len 1, rope block.rs:1403-1471): for page b the
 * token at position pos = kv_pos[b] has its q / k rotated (cos/sin tables [max_len][rope_dim]; prerot != 0:
 * the q / k rows of qkv are already rotated), k and v appended to the f32 cache [B][kv_heads][max_len][hd]
 * at pos, then o[b] = softmax(scale * q.K[:pos+1]^T) . V[:pos+1].  qkv: [B][(heads + 2 kv_heads) * hd];
 * o: [B][heads*hd]. */
dsocr_status dsocr_k_decode_attention(int B, int heads, int kv_heads, int hd, int rope_dim, int max_len, float scale,
                                      const float* qkv, const float* cos, const float* sin, float* kc, float* vc,
                                      const int* kv_pos, float* o, int prerot);
/* One page's decode attention sub-layer as the engine runs it (block.rs:446-804 at seq_len 1): RMSNorm +
 * q/k/v projection (Wqkv [3H][H], 16-bit) with RoPE in the epilogue, K/V append at kv_pos[s], softmax
 * attention over positions 0..kv_pos[s], for `steps` launches back to back (x [steps][H], kv_pos [steps],
 * o [steps][H]).  fused != 0: the one-launch form (dec_qkv_attn: attention blocks poll the q/k/v row, which
 * must enter the first launch filled with DSOCR_HANDOFF_SENTINEL words and is left so by every launch);
 * fused == 0 or the residency rule refusing it: projection and attention as two launches.  *used_fused
 * reports which ran.  128-dim MHA heads only.  Device pointers. */
#define DSOCR_HANDOFF_SENTINEL 0x7FBADBADu
dsocr_status dsocr_k_qkv_attention(int fused, int steps, int H, int heads, int hd, int max_len, float scale,
                                   float eps, const float* x, const float* norm_w, const void* Wqkv, int wdtype,
                                   const float* cos, const float* sin, float* kc, float* vc, const int* kv_pos,
                                   float* qkv_row, float* o, int* used_fused);
/* Residency rule of the polled in-launch hand-offs (pure host decision, no device call): 1 when
 * waiting_blocks (blocks that may spin on blocks of the same grid) < usable slots = (min(api, 8), one fewer
 * where the occupancy API may over-admit) x cus; else 0 (the engine then launches the non-polling form). */
int dsocr_k_poll_wait_fits(long waiting_blocks, int api_blocks_per_cu, int cus);
/* Decode MoE layer (the north-star kernel chain, block.rs:1215-1395): [RMSNorm] + router GEMV +
 * softmax top-k + grouping + grouped SwiGLU experts + shared experts + weighted combine,
 * out[T][H] += moe(xn), xn = rmsnorm(x; norm_w, eps) if norm_w != NULL else x.  Runs exactly the
 * engine's decode dispatch for T tokens (the same launches Engine::decode_step issues).
 * Wgu: [E][2I][H] (gate rows then up rows), Wd: [E][H][I], router [E][H], shared Wgu [2Is][H],
 * shared Wd [H][Is] (shared may be NULL), all 16-bit (wdtype). */
dsocr_status dsocr_k_moe(int T, int H, int E, int topk, int I, int Is, const float* x, const float* norm_w,
                         float eps, const void* router,
                         const void* Wgu, const void* Wd, const void* sWgu, const void* sWd, int wdtype,
                         int norm_topk, float scaling, float* out, int* topk_ids_out, float* topk_w_out);
/* Kernel names launch_moe_decode picks for a decode MoE of T tokens (static strings), e.g. the bench's
 * roofline label: "moe_gateup_mix_kernel" at T = 1, "moe_gateup_grp_kernel" at T = 3..8. */
dsocr_status dsocr_k_moe_kernels(int T, int H, int E, int topk, int I, int Is, int has_norm, const char** gateup,
                                 const char** down);
/* Screened greedy selection (the engine's decode head at B <= 2 without repetition penalty): the
 * int8 copy of W (bf16 [V][K], quantised as at engine load) gives every row an interval that holds
 * the exact logit, the surviving rows are rescored with the exact kernel's arithmetic; out_tok[b] =
 * the first-index argmax of rmsnorm(x_b; norm_w, eps) . W^T over the rows not in page b's ban list
 * (ban [B][ban_ld]: count then tokens, or NULL), as argmax_index (sampling.rs:104-118). */
dsocr_status dsocr_k_lmhead_screened(int B, int V, int K, const float* x, const float* norm_w, float eps,
                                     const void* W, const int* ban, int ban_ld, int* out_tok);
/* Greedy selection with repetition penalty + n-gram ban (sampling.rs:34-158) over B rows of V
 * logits; ctx [B][ctx_cap] int32 with ctx_len[B]. */
dsocr_status dsocr_k_sample_greedy(int B, int V, float* logits, const int* ctx, int ctx_cap, const int* ctx_len,
                                   int ngram, float rep_penalty, int* out_tok);
/* Stochastic selection (select_token_id's do_sample branch: top-k, top-p, WeightedIndex over rand's
 * StdRng seeded by seed_from_u64(seed)) on device logits [B][V] after the repetition penalty and the
 * n-gram ban; `draws` successive selections on the same logits with the RNG state carried over
 * (out_tok [draws][B]).  Device pointers, like dsocr_k_sample_greedy. */
dsocr_status dsocr_k_sample_stoch(int B, int V, float* logits, const int* ctx, int ctx_cap, const int* ctx_len,
                                  int ngram, float rep_penalty, double temperature, size_t top_k, double top_p,
                                  uint64_t seed, int draws, int* out_tok);

/* ---- dots.ocr vision tower (BASELINE configs[3]; crates/infer-dots/src/vision/dots_vit.rs
 *      DotsVisionModel::load / forward, vision/preprocess.rs preprocess_image).  The tower runs in the
 *      reference's bf16 semantics (every op's output rounded to bf16; attention scores / softmax /
 *      probs.V in f32).  config_path: the dots config.json (its `vision_config`, plus an optional
 *      `preprocessor_config` object with the preprocessor_config.json fields); weights_path NULL
 *      selects the seeded synthetic checkpoint (tensor names `vision_tower.*`). */
typedef struct dsocr_dots dsocr_dots;
dsocr_status dsocr_dots_load(const char* config_path, const char* weights_path, uint64_t synthetic_seed, int device,
                             dsocr_dots** out);
void dsocr_dots_free(dsocr_dots* d);
dsocr_status dsocr_dots_info(const dsocr_dots* d, size_t* hidden, size_t* embed_dim, size_t* layers, size_t* patch_dim);
/* preprocess_image (host): RGB8 HWC -> patches [N][3*p*p] in merge-group order; grid_thw = (t, h, w) */
dsocr_status dsocr_dots_preprocess(const char* config_path, const uint8_t* rgb, uint32_t width, uint32_t height,
                                   float* patches, size_t cap_patches, size_t* n_patches, uint32_t* grid_thw);
/* preprocess + tower for one page: out [groups][hidden] f32 (bf16 values), groups = N / merge^2 */
dsocr_status dsocr_dots_embed(dsocr_dots* d, const uint8_t* rgb, uint32_t width, uint32_t height, float* out,
                              size_t cap_rows, size_t* n_rows, uint32_t* grid_thw);
/* tower on device-resident patches (device pointers; the bench's inputs-in-HBM form); the first
 * time_attention_layers layers' attention launches are timed alone (0: no per-layer sync) */
dsocr_status dsocr_dots_embed_device(dsocr_dots* d, const float* patches, uint32_t grid_t, uint32_t grid_h,
                                     uint32_t grid_w, float* out, int time_attention_layers);
typedef struct {
    double total_ms, patch_ms, blocks_ms, attention_ms, merger_ms;
    size_t tokens, groups;
} dsocr_dots_timings;
dsocr_status dsocr_dots_last_timings(const dsocr_dots* d, dsocr_dots_timings* t);

#ifdef __cplusplus
}
#endif
#endif /* DSOCR_H */
