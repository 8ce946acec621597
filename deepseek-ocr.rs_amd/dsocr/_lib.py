"""ctypes binding of include/dsocr.h (the C ABI).  Loads the in-tree
deepseek-ocr.rs_amd/lib/libdsocr.so and fails loudly if it is missing: there is
no CPU fallback in the product path."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libdsocr.so")

OK, EINVAL, ENOENT, EDEVICE, ENOMEM, EINTERNAL = range(6)
STATUS_NAMES = {0: "OK", 1: "EINVAL", 2: "ENOENT", 3: "EDEVICE", 4: "ENOMEM", 5: "EINTERNAL"}
DTYPES = {"f32": 0, "f16": 1, "bf16": 2}


class DsocrError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status
        self.message = message


class LoadArgs(C.Structure):
    _fields_ = [("config_path", C.c_char_p), ("weights_path", C.c_char_p), ("snapshot_path", C.c_char_p),
                ("device_ordinal", C.c_int), ("dtype", C.c_int), ("synthetic_seed", C.c_uint64)]


class VisionSettingsC(C.Structure):
    _fields_ = [("base_size", C.c_uint32), ("image_size", C.c_uint32), ("crop_mode", C.c_int)]


class DecodeParamsC(C.Structure):
    _fields_ = [("max_new_tokens", C.c_size_t), ("do_sample", C.c_int), ("temperature", C.c_double),
                ("top_p", C.c_double), ("top_k", C.c_size_t), ("repetition_penalty", C.c_float),
                ("no_repeat_ngram_size", C.c_size_t), ("seed", C.c_uint64), ("use_cache", C.c_int),
                ("eos_token_id", C.c_int64), ("ignore_eos", C.c_int), ("has_seed", C.c_int)]


class RequestC(C.Structure):
    _fields_ = [("input_ids", C.POINTER(C.c_int64)), ("image_mask", C.POINTER(C.c_uint8)),
                ("prompt_len", C.c_size_t), ("page", C.c_void_p), ("image_rows", C.POINTER(C.c_float)),
                ("n_image_rows", C.c_size_t)]


class ResultC(C.Structure):
    _fields_ = [("out_ids", C.POINTER(C.c_int64)), ("cap", C.c_size_t), ("n_out", C.c_size_t),
                ("status", C.c_int)]


class TimingsC(C.Structure):
    _fields_ = [("vision_prepare_ms", C.c_double), ("vision_compute_ms", C.c_double),
                ("decode_prefill_ms", C.c_double), ("decode_iterative_ms", C.c_double),
                ("decode_generate_ms", C.c_double), ("decode_steps", C.c_size_t), ("pages", C.c_size_t),
                ("vision_flops", C.c_double), ("prefill_flops", C.c_double)]


class KernelProfileC(C.Structure):
    _fields_ = [("avg_us", C.c_double), ("bytes", C.c_double), ("flops", C.c_double), ("launches", C.c_int),
                ("replay_us", C.c_double), ("ctx_us", C.c_double)]


class DecodeProfileC(C.Structure):
    _fields_ = [("moe_gateup", KernelProfileC), ("moe_down", KernelProfileC), ("attention", KernelProfileC),
                ("lm_head", KernelProfileC), ("experts_touched", C.c_int), ("tokens", C.c_int), ("kv_len", C.c_int),
                ("qkv", KernelProfileC), ("o_proj", KernelProfileC), ("router", KernelProfileC),
                ("layers_step", KernelProfileC), ("lm_head_screened", KernelProfileC),
                ("moe_gateup_kernel", C.c_char_p), ("moe_down_kernel", C.c_char_p)]


class DotsTimingsC(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("patch_ms", C.c_double), ("blocks_ms", C.c_double),
                ("attention_ms", C.c_double), ("merger_ms", C.c_double), ("tokens", C.c_size_t), ("groups", C.c_size_t)]


STREAM_CB = C.CFUNCTYPE(None, C.c_size_t, C.POINTER(C.c_int64), C.c_void_p)

# every symbol include/dsocr.h declares (tests check the library exports all of them)
EXPORTS = [
    "dsocr_engine_load", "dsocr_engine_free", "dsocr_last_error", "dsocr_engine_info", "dsocr_prepare_page",
    "dsocr_page_free", "dsocr_page_to_device", "dsocr_page_info", "dsocr_page_pixels_view", "dsocr_image_embeddings", "dsocr_generate",
    "dsocr_generate_batch", "dsocr_last_timings", "dsocr_profile_decode", "dsocr_device_count", "dsocr_dev_alloc", "dsocr_dev_free",
    "dsocr_memcpy_h2d", "dsocr_memcpy_d2h", "dsocr_dev_sync", "dsocr_synth_bf16", "dsocr_resize_bicubic",
    "dsocr_k_gemm", "dsocr_k_gemm_f32a", "dsocr_k_gemm_grouped", "dsocr_k_gemv", "dsocr_k_layernorm", "dsocr_k_rmsnorm", "dsocr_k_attention", "dsocr_k_decode_attention", "dsocr_k_moe",
    "dsocr_k_sample_greedy", "dsocr_k_sample_stoch", "dsocr_k_dsq_dequant", "dsocr_prepare_page_device", "dsocr_page_read_device",
    "dsocr_generate_trace", "dsocr_k_moe_kernels", "dsocr_k_lmhead_screened",
    "dsocr_dots_load", "dsocr_dots_free", "dsocr_dots_info", "dsocr_dots_preprocess", "dsocr_dots_embed",
    "dsocr_dots_embed_device", "dsocr_dots_last_timings", "dsocr_k_attention_bf16", "dsocr_k_gemv_splitk",
    "dsocr_engine_set_spans", "dsocr_engine_spans", "dsocr_k_qkv_attention", "dsocr_k_poll_wait_fits",
    "dsocr_engine_set_persist_stamps", "dsocr_engine_persist_info",
    "dsocr_resize_catmull_rom",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DsocrError(EINTERNAL, f"libdsocr.so not built at {LIB_PATH}; run `python deepseek-ocr.rs_amd/build.py`")
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, u32, f32, i64 = C.c_void_p, C.c_size_t, C.c_int, C.c_uint32, C.c_float, C.c_int64
    L.dsocr_last_error.restype = C.c_char_p
    L.dsocr_engine_load.argtypes = [C.POINTER(LoadArgs), C.POINTER(vp)]
    L.dsocr_engine_free.argtypes = [vp]
    L.dsocr_engine_free.restype = None
    L.dsocr_engine_info.argtypes = [vp, C.POINTER(sz), C.POINTER(sz), C.POINTER(i64), C.POINTER(sz)]
    L.dsocr_prepare_page.argtypes = [vp, u32, u32, C.POINTER(VisionSettingsC), C.POINTER(vp)]
    L.dsocr_page_free.argtypes = [vp]
    L.dsocr_prepare_page_device.argtypes = [vp, vp, u32, u32, C.POINTER(VisionSettingsC), C.POINTER(vp)]
    L.dsocr_page_read_device.argtypes = [vp, vp, vp]
    L.dsocr_page_free.restype = None
    L.dsocr_page_to_device.argtypes = [vp, vp]
    L.dsocr_page_info.argtypes = [vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32), C.POINTER(sz)]
    L.dsocr_page_pixels_view.argtypes = [vp, C.POINTER(vp), C.POINTER(u32), C.POINTER(vp), C.POINTER(u32)]
    L.dsocr_image_embeddings.argtypes = [vp, C.POINTER(vp), sz, vp, sz, C.POINTER(sz)]
    L.dsocr_generate.argtypes = [vp, C.POINTER(RequestC), C.POINTER(DecodeParamsC), STREAM_CB, vp, vp, sz,
                                 C.POINTER(sz)]
    L.dsocr_generate_batch.argtypes = [vp, sz, C.POINTER(RequestC), C.POINTER(DecodeParamsC), C.POINTER(ResultC)]
    L.dsocr_generate_trace.argtypes = [vp, sz, C.POINTER(RequestC), C.POINTER(DecodeParamsC), C.POINTER(ResultC), vp,
                                       sz]
    L.dsocr_k_attention_bf16.argtypes = [i32, i32, i32, i32, f32, vp, C.c_long, vp, C.c_long, i32]
    L.dsocr_dots_load.argtypes = [C.c_char_p, C.c_char_p, C.c_uint64, i32, C.POINTER(vp)]
    L.dsocr_dots_free.argtypes = [vp]
    L.dsocr_dots_free.restype = None
    L.dsocr_dots_info.argtypes = [vp, C.POINTER(sz), C.POINTER(sz), C.POINTER(sz), C.POINTER(sz)]
    L.dsocr_dots_preprocess.argtypes = [C.c_char_p, vp, u32, u32, vp, sz, C.POINTER(sz), C.POINTER(u32)]
    L.dsocr_dots_embed.argtypes = [vp, vp, u32, u32, vp, sz, C.POINTER(sz), C.POINTER(u32)]
    L.dsocr_dots_embed_device.argtypes = [vp, vp, u32, u32, u32, vp, i32]
    L.dsocr_dots_last_timings.argtypes = [vp, C.POINTER(DotsTimingsC)]
    L.dsocr_k_lmhead_screened.argtypes = [i32, i32, i32, vp, vp, f32, vp, vp, i32, vp]
    L.dsocr_k_moe_kernels.argtypes = [i32, i32, i32, i32, i32, i32, i32, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)]
    L.dsocr_last_timings.argtypes = [vp, C.POINTER(TimingsC)]
    L.dsocr_profile_decode.argtypes = [vp, i32, C.POINTER(DecodeProfileC)]
    L.dsocr_engine_set_spans.argtypes = [vp, i32]
    L.dsocr_engine_spans.argtypes = [vp, vp, sz, C.POINTER(sz), C.POINTER(sz), C.POINTER(sz)]
    L.dsocr_engine_set_persist_stamps.argtypes = [vp, i32]
    L.dsocr_engine_persist_info.argtypes = [vp, C.POINTER(i32), vp, sz, C.POINTER(sz), vp, sz, C.POINTER(sz)]
    L.dsocr_device_count.argtypes = [C.POINTER(i32)]
    L.dsocr_dev_alloc.argtypes = [sz, C.POINTER(vp)]
    L.dsocr_dev_free.argtypes = [vp]
    L.dsocr_memcpy_h2d.argtypes = [vp, vp, sz]
    L.dsocr_memcpy_d2h.argtypes = [vp, vp, sz]
    L.dsocr_synth_bf16.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, vp]
    L.dsocr_resize_bicubic.argtypes = [vp, u32, u32, vp, u32, u32]
    L.dsocr_resize_catmull_rom.argtypes = [vp, u32, u32, vp, u32, u32]
    L.dsocr_k_gemm.argtypes = [i32, i32, i32, vp, vp, i32, vp, vp, i32, i32]
    L.dsocr_k_gemm_f32a.argtypes = [i32, i32, i32, vp, vp, i32, vp, vp, i32, i32, i32]
    L.dsocr_k_gemm_grouped.argtypes = [i32, i32, i32, vp, i32, vp, vp, i32, C.c_longlong, vp, C.c_longlong, vp, i32, vp, i32,
                                       i32, vp, i32, i32, i32]
    L.dsocr_k_gemv.argtypes = [i32, i32, i32, vp, vp, f32, vp, i32, vp, vp, i32, i32]
    L.dsocr_k_gemv_splitk.argtypes = [i32, i32, i32, vp, vp, i32, vp, vp, i32]
    L.dsocr_k_layernorm.argtypes = [i32, i32, vp, vp, vp, f32, vp]
    L.dsocr_k_rmsnorm.argtypes = [i32, i32, vp, vp, f32, vp]
    L.dsocr_k_dsq_dequant.argtypes = [i32, vp, sz, sz, sz, vp]
    L.dsocr_k_attention.argtypes = [i32, i32, i32, i32, f32, i32, vp, vp, vp, vp, vp, vp, i32, i32]
    L.dsocr_k_decode_attention.argtypes = [i32, i32, i32, i32, i32, i32, f32, vp, vp, vp, vp, vp, vp, vp, i32]
    L.dsocr_k_qkv_attention.argtypes = [i32, i32, i32, i32, i32, i32, f32, f32, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp,
                                        vp, C.POINTER(i32)]
    L.dsocr_k_poll_wait_fits.argtypes = [C.c_long, i32, i32]
    L.dsocr_k_moe.argtypes = [i32, i32, i32, i32, i32, i32, vp, vp, f32, vp, vp, vp, vp, vp, i32, i32, f32, vp, vp, vp]
    L.dsocr_k_sample_greedy.argtypes = [i32, i32, vp, vp, i32, vp, i32, f32, vp]
    L.dsocr_k_sample_stoch.argtypes = [i32, i32, vp, vp, i32, vp, i32, f32, C.c_double, C.c_size_t, C.c_double,
                                       C.c_uint64, i32, vp]
    _lib = L
    return L


def check(status: int):
    if status != OK:
        msg = lib().dsocr_last_error()
        raise DsocrError(status, msg.decode() if msg else "")
