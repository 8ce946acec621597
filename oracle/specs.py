"""Oracle: the tensor names/shapes the reference loads for a config
(TEST INFRASTRUCTURE).  Restates the VarBuilder lookups of transformer/weights.rs:164-606,
vision/sam.rs:143-184 + 636-924, vision/clip.rs:73-484 and model/mod.rs:258-307."""
import numpy as np  # noqa: F401


def tensor_names(cfg):
    """Every tensor the reference loads for this config (names/shapes as in weights.rs, sam.rs, clip.rs)."""
    from oracle.config import clip_params, resolved_language_config, sam_params, should_use_moe
    L = resolved_language_config(cfg)
    S = sam_params(cfg)
    Cp = clip_params(cfg)
    t = {}
    sp = "model.sam_model."
    t[sp + "patch_embed.proj.weight"] = (S.embed_dim, 3, S.patch_size, S.patch_size)
    t[sp + "patch_embed.proj.bias"] = (S.embed_dim,)
    g = S.image_size // S.patch_size
    t[sp + "pos_embed"] = (1, g, g, S.embed_dim)
    hd = S.embed_dim // S.num_heads
    for b in range(S.depth):
        p = f"{sp}blocks.{b}."
        for nn in ("norm1", "norm2"):
            t[p + nn + ".weight"] = (S.embed_dim,)
            t[p + nn + ".bias"] = (S.embed_dim,)
        t[p + "attn.qkv.weight"] = (3 * S.embed_dim, S.embed_dim)
        t[p + "attn.qkv.bias"] = (3 * S.embed_dim,)
        t[p + "attn.proj.weight"] = (S.embed_dim, S.embed_dim)
        t[p + "attn.proj.bias"] = (S.embed_dim,)
        tokens = g if b in S.global_attn_indexes else S.window_size
        t[p + "attn.rel_pos_h"] = (2 * tokens - 1, hd)
        t[p + "attn.rel_pos_w"] = (2 * tokens - 1, hd)
        hid = int(S.embed_dim * S.mlp_ratio)
        t[p + "mlp.fc1.weight"] = (hid, S.embed_dim)
        t[p + "mlp.fc1.bias"] = (hid,)
        t[p + "mlp.fc2.weight"] = (S.embed_dim, hid)
        t[p + "mlp.fc2.bias"] = (S.embed_dim,)
    nc = S.neck_channels
    t[sp + "neck.0.weight"] = (nc, S.embed_dim, 1, 1)
    t[sp + "neck.1.weight"] = (nc,)
    t[sp + "neck.1.bias"] = (nc,)
    t[sp + "neck.2.weight"] = (nc, nc, 3, 3)
    t[sp + "neck.3.weight"] = (nc,)
    t[sp + "neck.3.bias"] = (nc,)
    t[sp + "net_2.weight"] = (S.out_channels[0], nc, 3, 3)
    t[sp + "net_3.weight"] = (S.out_channels[1], S.out_channels[0], 3, 3)
    cp = "model.vision_model."
    C = Cp.hidden_size
    t[cp + "embeddings.class_embedding"] = (C,)
    t[cp + "embeddings.position_embedding.weight"] = (Cp.seq_length + 1, C)
    t[cp + "pre_layrnorm.weight"] = (C,)
    t[cp + "pre_layrnorm.bias"] = (C,)
    for l in range(Cp.num_layers):
        p = f"{cp}transformer.layers.{l}."
        for nn in ("layer_norm1", "layer_norm2"):
            t[p + nn + ".weight"] = (C,)
            t[p + nn + ".bias"] = (C,)
        t[p + "self_attn.qkv_proj.weight"] = (3 * C, C)
        t[p + "self_attn.qkv_proj.bias"] = (3 * C,)
        t[p + "self_attn.out_proj.weight"] = (C, C)
        t[p + "self_attn.out_proj.bias"] = (C,)
        t[p + "mlp.fc1.weight"] = (4 * C, C)
        t[p + "mlp.fc1.bias"] = (4 * C,)
        t[p + "mlp.fc2.weight"] = (C, 4 * C)
        t[p + "mlp.fc2.bias"] = (C,)
    pc = cfg["projector_config"]
    t["model.projector.layers.weight"] = (pc["n_embed"], pc["input_dim"])
    t["model.projector.layers.bias"] = (pc["n_embed"],)
    t["model.image_newline"] = (pc["n_embed"],)
    t["model.view_seperator"] = (pc["n_embed"],)
    H = L.hidden_size
    t["model.embed_tokens.weight"] = (L.vocab_size, H)
    for l in range(L.num_hidden_layers):
        p = f"model.layers.{l}."
        t[p + "input_layernorm.weight"] = (H,)
        t[p + "post_attention_layernorm.weight"] = (H,)
        for pr in ("q_proj", "k_proj", "v_proj", "o_proj"):
            t[p + f"self_attn.{pr}.weight"] = (H, H)
        if should_use_moe(L, l):
            E, I = L.n_routed_experts, L.moe_intermediate_size
            t[p + "mlp.gate.weight"] = (E, H)
            for e in range(E):
                t[p + f"mlp.experts.{e}.gate_proj.weight"] = (I, H)
                t[p + f"mlp.experts.{e}.up_proj.weight"] = (I, H)
                t[p + f"mlp.experts.{e}.down_proj.weight"] = (H, I)
            Is = I * L.n_shared_experts
            t[p + "mlp.shared_experts.gate_proj.weight"] = (Is, H)
            t[p + "mlp.shared_experts.up_proj.weight"] = (Is, H)
            t[p + "mlp.shared_experts.down_proj.weight"] = (H, Is)
        else:
            I = L.intermediate_size
            t[p + "mlp.gate_proj.weight"] = (I, H)
            t[p + "mlp.up_proj.weight"] = (I, H)
            t[p + "mlp.down_proj.weight"] = (H, I)
    t["model.norm.weight"] = (H,)
    t["lm_head.weight"] = (L.vocab_size, H)
    return t
