// Model configuration resolved exactly like the reference:
//   DeepseekOcrConfig::resolved_language_config (config/mod.rs:70-92, serde defaults 287-328)
//   SamBackboneParams::from_backbone_cfg (vision/sam.rs:40-112)
//   ClipVisionParams::from_backbone (vision/clip.rs:35-52)
//   should_use_moe (transformer/weights.rs:609-619)
#pragma once
#include <cmath>
#include <string>
#include <vector>

#include "../common/json.hpp"

namespace dsocr {

struct LangConfig {
    int vocab = 0, hidden = 0, inter = 0, moe_inter = 0, layers = 0, heads = 0, kv_heads = 0;
    int n_shared = 0, n_routed = 0, topk = 0, first_dense = 0, moe_freq = 1;
    bool norm_topk = false, use_mla = true, attention_bias = false;
    float routed_scaling = 1.f, rms_eps = 1e-6f, rope_theta = 10000.f;
    int rope_dim = 0, head_dim = 0, v_head_dim = 0;
    std::string scoring = "softmax", topk_method = "greedy", hidden_act = "silu";
    long eos = -1, bos = 0;
    bool has_lora = false;
    bool moe_layer(int l) const {
        if (n_routed <= 0) return false;
        if (l < first_dense) return false;
        return l % moe_freq == 0;
    }
};

struct SamConfig {
    int image_size = 1024, patch = 16, dim = 768, depth = 12, heads = 12, window = 14, neck = 256;
    std::vector<int> out_ch{512, 1024};
    std::vector<int> global_idx{2, 5, 8, 11};
    float mlp_ratio = 4.f;
    bool is_global(int b) const {
        for (int g : global_idx) if (g == b) return true;
        return false;
    }
};

struct ClipConfig {
    int hidden = 1024, layers = 24, heads = 16, ffn = 4096, image_size = 224, patch = 14, seq = 256;
};

struct ModelConfig {
    LangConfig lang;
    SamConfig sam;
    ClipConfig clip;
    int proj_in = 2048, proj_out = 1280;
    std::string proj_type = "linear";
};

inline void merge_missing(Json& target, const Json& fallback) {
    if (target.kind == Json::Object) {
        if (fallback.kind != Json::Object) return;
        for (auto& kv : fallback.obj) {
            auto it = target.obj.find(kv.first);
            if (it == target.obj.end()) target.obj[kv.first] = kv.second;
            else if (it->second.is_null()) it->second = kv.second;
            else merge_missing(it->second, kv.second);
        }
    } else if (target.kind == Json::Array) {
        if (fallback.kind == Json::Array && target.arr.empty()) target = fallback;
    } else if (target.is_null()) {
        target = fallback;
    }
}

inline ModelConfig resolve_config(const Json& cfg) {
    static const char* lang_keys[] = {
        "vocab_size", "hidden_size", "intermediate_size", "moe_intermediate_size", "num_hidden_layers",
        "num_attention_heads", "num_key_value_heads", "n_shared_experts", "n_routed_experts", "ep_size",
        "routed_scaling_factor", "kv_lora_rank", "q_lora_rank", "qk_rope_head_dim", "v_head_dim",
        "qk_nope_head_dim", "topk_method", "n_group", "topk_group", "num_experts_per_tok", "moe_layer_freq",
        "moe_layer_freq_override", "first_k_dense_replace", "norm_topk_prob", "scoring_func", "hidden_act",
        "max_position_embeddings", "rms_norm_eps", "bos_token_id", "eos_token_id", "rope_theta", "attention_bias",
        "use_mla", "torch_dtype"};
    Json top;
    top.kind = Json::Object;
    for (auto k : lang_keys)
        if (cfg.obj.count(k)) top.obj[k] = cfg.obj.at(k);
    const bool has_top = top.has("vocab_size") && top.has("hidden_size");
    Json L;
    if (cfg.has("language_config")) L = cfg["language_config"];
    else if (has_top) L = top;
    else throw std::runtime_error("EINVAL: language configuration missing (neither language_config nor top-level defaults provided)");
    if (has_top) merge_missing(L, top);
    if (cfg.has("language_config") && cfg["language_config"].has("moe_layer_freq_override"))
        L.obj["moe_layer_freq"] = cfg["language_config"]["moe_layer_freq_override"];

    ModelConfig m;
    LangConfig& l = m.lang;
    l.vocab = (int)L["vocab_size"].as_int();
    l.hidden = (int)L["hidden_size"].as_int();
    l.inter = (int)L["intermediate_size"].as_int();
    l.moe_inter = (int)L["moe_intermediate_size"].as_int(0);
    l.layers = (int)L["num_hidden_layers"].as_int();
    l.heads = (int)L["num_attention_heads"].as_int();
    l.kv_heads = L.has("num_key_value_heads") ? (int)L["num_key_value_heads"].as_int() : l.heads;
    l.n_shared = (int)L["n_shared_experts"].as_int(0);
    l.n_routed = (int)L["n_routed_experts"].as_int(0);
    l.topk = (int)L["num_experts_per_tok"].as_int(0);
    l.first_dense = (int)L["first_k_dense_replace"].as_int(0);
    l.moe_freq = L.has("moe_layer_freq") ? (int)L["moe_layer_freq"].as_int() : 1;
    l.norm_topk = L["norm_topk_prob"].as_bool(false);
    l.use_mla = L.has("use_mla") ? L["use_mla"].as_bool(true) : true;
    l.attention_bias = L["attention_bias"].as_bool(false);
    l.routed_scaling = L.has("routed_scaling_factor") ? (float)L["routed_scaling_factor"].as_double() : 1.f;
    l.rms_eps = L.has("rms_norm_eps") ? (float)L["rms_norm_eps"].as_double() : 1e-6f;
    l.rope_theta = L.has("rope_theta") ? (float)L["rope_theta"].as_double() : 10000.f;
    l.scoring = L.has("scoring_func") ? L["scoring_func"].as_string() : "softmax";
    l.topk_method = L.has("topk_method") ? L["topk_method"].as_string() : "greedy";
    l.hidden_act = L.has("hidden_act") ? L["hidden_act"].as_string() : "silu";
    l.eos = L.has("eos_token_id") ? L["eos_token_id"].as_int() : -1;
    l.bos = L.has("bos_token_id") ? L["bos_token_id"].as_int() : 0;
    l.has_lora = L.has("q_lora_rank") || L.has("kv_lora_rank");
    if (l.hidden <= 0 || l.heads <= 0 || l.hidden % l.heads) throw std::runtime_error("EINVAL: bad hidden/heads");
    l.head_dim = l.hidden / l.heads;
    int rd = L.has("qk_rope_head_dim") ? (int)L["qk_rope_head_dim"].as_int() : l.head_dim;
    l.rope_dim = rd == 0 ? l.head_dim : rd;
    int vd = L.has("v_head_dim") ? (int)L["v_head_dim"].as_int() : 0;
    l.v_head_dim = vd == 0 ? l.head_dim : vd;

    const Json& vis = cfg["vision_config"];
    const Json& sb = vis["width"]["sam_vit_b"];
    if (sb.is_null()) throw std::runtime_error("EINVAL: sam_vit_b vision backbone missing from config");
    SamConfig& s = m.sam;
    s.image_size = vis.has("image_size") ? (int)vis["image_size"].as_int() : (sb.has("image_size") ? (int)sb["image_size"].as_int() : 1024);
    s.patch = sb.has("patch_size") ? (int)sb["patch_size"].as_int() : 16;
    s.dim = sb.has("width") ? (int)sb["width"].as_int() : 768;
    s.depth = sb.has("layers") ? (int)sb["layers"].as_int() : 12;
    s.heads = sb.has("heads") ? (int)sb["heads"].as_int() : 12;
    if (sb.has("downsample_channels")) {
        s.out_ch.clear();
        for (auto& v : sb["downsample_channels"].arr) s.out_ch.push_back((int)v.as_int());
    }
    if (sb.has("global_attn_indexes")) {
        s.global_idx.clear();
        for (auto& v : sb["global_attn_indexes"].arr) s.global_idx.push_back((int)v.as_int());
    }
    const Json& cb = vis["width"]["clip-l-14-224"];
    if (cb.is_null()) throw std::runtime_error("EINVAL: clip-l-14-224 vision backbone missing from config");
    ClipConfig& c = m.clip;
    c.hidden = (int)cb["width"].as_int();
    c.heads = (int)cb["heads"].as_int();
    c.layers = (int)cb["layers"].as_int();
    c.patch = (int)cb["patch_size"].as_int();
    c.image_size = (int)cb["image_size"].as_int();
    c.ffn = 4 * c.hidden;
    c.seq = (c.image_size / c.patch) * (c.image_size / c.patch);
    const Json& pc = cfg["projector_config"];
    if (pc.is_null()) throw std::runtime_error("EINVAL: projector_config missing from DeepseekOcrConfig");
    m.proj_type = pc["projector_type"].as_string();
    if (m.proj_type != "linear") throw std::runtime_error("EINVAL: unsupported projector_type `" + m.proj_type + "`");
    m.proj_in = (int)pc["input_dim"].as_int();
    m.proj_out = (int)pc["n_embed"].as_int();
    if (m.proj_out != l.hidden) throw std::runtime_error("EINVAL: projector n_embed mismatches language hidden size");
    if (s.out_ch.size() != 2) throw std::runtime_error("EINVAL: expected exactly two downsample stages");
    return m;
}

}  // namespace dsocr
