"""Oracle: config resolution (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates crates/infer-deepseek/src/config/mod.rs (serde defaults and the
nested-language merge), SamBackboneParams::from_backbone_cfg (vision/sam.rs:40-112),
ClipVisionParams::from_backbone (vision/clip.rs:35-52) and should_use_moe
(transformer/weights.rs:609-619).
"""
from __future__ import annotations

import copy
import json
from dataclasses import dataclass, field


def _merge_missing(target, fallback):
    """config/mod.rs:330-365 merge_missing."""
    if isinstance(target, dict):
        if isinstance(fallback, dict):
            for k, fv in fallback.items():
                if k in target:
                    if target[k] is None:
                        target[k] = copy.deepcopy(fv)
                    else:
                        target[k] = _merge_missing(target[k], fv)
                else:
                    target[k] = copy.deepcopy(fv)
        return target
    if isinstance(target, list):
        if isinstance(fallback, list) and len(target) == 0:
            return copy.deepcopy(fallback)
        return target
    if target is None:
        return copy.deepcopy(fallback)
    return target


# serde defaults, config/mod.rs:144-240 + 287-328
_LANG_DEFAULTS = dict(
    ep_size=1, routed_scaling_factor=1.0, moe_layer_freq=1, norm_topk_prob=False,
    aux_loss_alpha=0.001, seq_aux=True, hidden_act="silu", initializer_range=0.02,
    rms_norm_eps=1e-6, use_cache=True, pretraining_tp=1, tie_word_embeddings=False,
    rope_theta=10000.0, attention_bias=False, attention_dropout=0.0, use_mla=True,
)

_LANG_KEYS = {
    "vocab_size", "hidden_size", "intermediate_size", "moe_intermediate_size", "num_hidden_layers",
    "num_attention_heads", "num_key_value_heads", "n_shared_experts", "n_routed_experts", "ep_size",
    "routed_scaling_factor", "kv_lora_rank", "q_lora_rank", "qk_rope_head_dim", "v_head_dim",
    "qk_nope_head_dim", "topk_method", "n_group", "topk_group", "num_experts_per_tok",
    "moe_layer_freq", "moe_layer_freq_override", "first_k_dense_replace", "norm_topk_prob",
    "scoring_func", "aux_loss_alpha", "seq_aux", "hidden_act", "max_position_embeddings",
    "initializer_range", "rms_norm_eps", "use_cache", "pad_token_id", "bos_token_id",
    "eos_token_id", "pretraining_tp", "tie_word_embeddings", "rope_theta", "rope_scaling",
    "attention_bias", "attention_dropout", "use_mla", "torch_dtype", "lm_head", "rm_head",
}


@dataclass
class LangCfg:
    raw: dict

    def __getattr__(self, k):
        raw = self.__dict__["raw"]
        if k in raw:
            return raw[k]
        if k in _LANG_DEFAULTS:
            return _LANG_DEFAULTS[k]
        return None

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads


def resolved_language_config(cfg: dict) -> LangCfg:
    """DeepseekOcrConfig::resolved_language_config, config/mod.rs:70-92."""
    top = {k: v for k, v in cfg.items() if k in _LANG_KEYS}
    has_top = "vocab_size" in top and "hidden_size" in top
    lc = cfg.get("language_config")
    if lc is not None:
        primary = {k: v for k, v in lc.items() if k not in ("architectures", "auto_map")}
    elif has_top:
        primary = copy.deepcopy(top)
    else:
        raise ValueError("language configuration missing (neither language_config nor top-level defaults provided)")
    if has_top:
        primary = _merge_missing(primary, top)
    if lc is not None and lc.get("moe_layer_freq_override") is not None:
        primary["moe_layer_freq"] = lc["moe_layer_freq_override"]
    return LangCfg(primary)


def should_use_moe(lang: LangCfg, layer_idx: int) -> bool:
    """transformer/weights.rs:609-619."""
    n = lang.n_routed_experts or 0
    if n == 0:
        return False
    if layer_idx < (lang.first_k_dense_replace or 0):
        return False
    return layer_idx % lang.moe_layer_freq == 0


@dataclass
class SamParams:
    """vision/sam.rs:40-112 (window 14, neck 256, mlp_ratio 4, eps 1e-6 are fixed there)."""
    image_size: int = 1024
    patch_size: int = 16
    embed_dim: int = 768
    depth: int = 12
    num_heads: int = 12
    window_size: int = 14
    neck_channels: int = 256
    out_channels: list = field(default_factory=lambda: [512, 1024])
    global_attn_indexes: list = field(default_factory=lambda: [2, 5, 8, 11])
    mlp_ratio: float = 4.0
    norm_eps: float = 1e-6


def sam_params(cfg: dict) -> SamParams:
    vis = cfg.get("vision_config") or {}
    b = (vis.get("width") or {}).get("sam_vit_b")
    if b is None:
        raise ValueError("sam_vit_b vision backbone missing from config")
    p = SamParams()
    p.image_size = vis.get("image_size") or b.get("image_size") or 1024
    p.patch_size = b.get("patch_size") or 16
    p.embed_dim = b.get("width") or 768
    p.depth = b.get("layers") or 12
    p.num_heads = b.get("heads") or 12
    if b.get("downsample_channels"):
        p.out_channels = list(b["downsample_channels"])
    if b.get("global_attn_indexes") is not None:
        p.global_attn_indexes = list(b["global_attn_indexes"])
    return p


@dataclass
class ClipParams:
    hidden_size: int
    num_layers: int
    num_heads: int
    ffn_hidden_size: int
    image_size: int
    patch_size: int
    seq_length: int
    eps: float = 1e-5


def clip_params(cfg: dict) -> ClipParams:
    """vision/clip.rs:25-52."""
    c = ((cfg.get("vision_config") or {}).get("width") or {}).get("clip-l-14-224")
    if c is None:
        raise ValueError("clip-l-14-224 vision backbone missing from config")
    h = c["width"]
    return ClipParams(hidden_size=h, num_layers=c["layers"], num_heads=c["heads"], ffn_hidden_size=4 * h,
                      image_size=c["image_size"], patch_size=c["patch_size"],
                      seq_length=(c["image_size"] // c["patch_size"]) ** 2)


def projector_params(cfg: dict) -> dict:
    p = cfg.get("projector_config")
    if p is None:
        raise ValueError("projector_config missing from DeepseekOcrConfig")
    if p.get("projector_type") != "linear":
        raise ValueError(f"unsupported projector_type `{p.get('projector_type')}`")
    return p


def load(path) -> dict:
    with open(path) as f:
        return json.load(f)
