"""Independent cross-check of the CPU oracle against HF ``transformers`` (5.15, offline) modules
of the same architecture family — the DeepSeek-OCR-2 text decoder (MHA + dense layer 0 +
DeepSeekMoE with shared experts, softmax greedy router, rotate_half RoPE) and its SAM-ViTDet
encoder (windowed / global attention with decomposed rel-pos, neck, stride-2 downsample) —
instantiated from config objects with the oracle's seeded synthetic weights (no download).

This pins the oracle's decoder and SAM arithmetic to a second, independent implementation
(the reference itself cannot run here: SURVEY §8c).  Tolerances: f32 end to end, different
reduction orders -> relative 2e-4 on logits / SAM features.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
M = pytest.importorskip("transformers.models.deepseek_ocr2.modeling_deepseek_ocr2")
Cfg = pytest.importorskip("transformers.models.deepseek_ocr2.configuration_deepseek_ocr2")

from oracle.config import resolved_language_config, sam_params, should_use_moe  # noqa: E402
from oracle.decoder import Decoder  # noqa: E402
from oracle.vision import Sam  # noqa: E402
from oracle.weights import Weights  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = os.path.join(ROOT, "deepseek-ocr.rs_amd", "dsocr", "configs", "tiny.json")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32))


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-6, np.max(np.abs(b))))


def test_decoder_matches_transformers_deepseek_text_model():
    cfg = json.load(open(TINY))
    W = Weights(seed=11, dtype="f16")  # decoder weights f16-rounded, as the engine / oracle use them
    dec = Decoder(cfg, W)
    L = dec.lang
    n_layers = L.num_hidden_layers
    tc = Cfg.DeepseekOcr2TextConfig(
        vocab_size=L.vocab_size, hidden_size=L.hidden_size, intermediate_size=L.intermediate_size,
        moe_intermediate_size=L.moe_intermediate_size, num_hidden_layers=n_layers,
        num_attention_heads=L.num_attention_heads, num_key_value_heads=dec.nkv,
        n_routed_experts=L.n_routed_experts, n_shared_experts=L.n_shared_experts,
        num_experts_per_tok=L.num_experts_per_tok, topk_method="greedy", routed_scaling_factor=1.0,
        rms_norm_eps=L.rms_norm_eps, max_position_embeddings=4096,
        rope_parameters={"rope_type": "default", "rope_theta": float(L.rope_theta)},
        mlp_layer_types=["sparse" if should_use_moe(L, i) else "dense" for i in range(n_layers)])
    tc._attn_implementation = "eager"
    model = M.DeepseekOcr2TextModel(tc).eval()
    H, I, Im, E = L.hidden_size, L.intermediate_size, L.moe_intermediate_size, L.n_routed_experts
    g = lambda n, s: _t(W.get(n, s))
    sd = {"embed_tokens.weight": g("model.embed_tokens.weight", (L.vocab_size, H)),
          "norm.weight": g("model.norm.weight", (H,))}
    for li in range(n_layers):
        p, q = f"model.layers.{li}.", f"layers.{li}."
        for n in ("q_proj", "k_proj", "v_proj", "o_proj"):
            sd[q + f"self_attn.{n}.weight"] = g(p + f"self_attn.{n}.weight", (H, H))
        sd[q + "input_layernorm.weight"] = g(p + "input_layernorm.weight", (H,))
        sd[q + "post_attention_layernorm.weight"] = g(p + "post_attention_layernorm.weight", (H,))
        if should_use_moe(L, li):
            sd[q + "mlp.gate.weight"] = g(p + "mlp.gate.weight", (E, H))
            sd[q + "mlp.experts.gate_up_proj"] = torch.stack(
                [torch.cat([g(p + f"mlp.experts.{e}.gate_proj.weight", (Im, H)),
                            g(p + f"mlp.experts.{e}.up_proj.weight", (Im, H))]) for e in range(E)])
            sd[q + "mlp.experts.down_proj"] = torch.stack(
                [g(p + f"mlp.experts.{e}.down_proj.weight", (H, Im)) for e in range(E)])
            Is = Im * L.n_shared_experts
            for n, s in (("gate_proj", (Is, H)), ("up_proj", (Is, H)), ("down_proj", (H, Is))):
                sd[q + f"mlp.shared_experts.{n}.weight"] = g(p + f"mlp.shared_experts.{n}.weight", s)
        else:
            for n, s in (("gate_proj", (I, H)), ("up_proj", (I, H)), ("down_proj", (H, I))):
                sd[q + f"mlp.{n}.weight"] = g(p + f"mlp.{n}.weight", s)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and all("rotary" in m for m in missing), (missing, unexpected)

    ids = np.random.default_rng(3).integers(2, L.vocab_size, 37)
    emb = dec.embed(ids)
    dec.reset()
    ref = dec.forward(emb, last_only=False)                     # oracle logits [S, V]
    with torch.no_grad():
        hid = model(inputs_embeds=_t(emb)[None]).last_hidden_state[0].numpy()
    got = hid @ W.get("lm_head.weight", (L.vocab_size, H)).T
    assert _rel(got, ref) < 2e-4, _rel(got, ref)
    assert np.array_equal(np.argmax(got, -1), np.argmax(ref, -1))
    # incremental decode through the oracle's KV cache equals the full causal pass
    dec.reset()
    dec.forward(emb[:-1])
    last = dec.forward(emb[-1:])
    assert _rel(last[0], ref[-1]) < 2e-5


def test_sam_matches_transformers_sam_encoder():
    cfg = json.load(open(TINY))
    W = Weights(seed=12, dtype="f16")
    sam = Sam(cfg, W)
    p = sam.p
    sc = Cfg.DeepseekOcr2SamVisionConfig(
        hidden_size=p.embed_dim, output_channels=p.neck_channels, num_hidden_layers=p.depth,
        num_attention_heads=p.num_heads, image_size=p.image_size, patch_size=p.patch_size, hidden_act="gelu",
        layer_norm_eps=p.norm_eps, qkv_bias=True, mlp_ratio=p.mlp_ratio, window_size=p.window_size,
        global_attn_indexes=list(p.global_attn_indexes), downsample_channels=list(p.out_channels))
    sc._attn_implementation = "eager"
    enc = M.DeepseekOcr2SamVisionEncoder(sc).eval()
    pre = "model.sam_model."
    C, t = p.embed_dim, p.image_size // p.patch_size
    g = lambda n, s: _t(W.get(pre + n, s))
    nc = p.neck_channels
    c0, c1 = p.out_channels
    sd = {"patch_embed.projection.weight": g("patch_embed.proj.weight", (C, 3, p.patch_size, p.patch_size)),
          "patch_embed.projection.bias": g("patch_embed.proj.bias", (C,)),
          "pos_embed": g("pos_embed", (1, t, t, C)),
          "neck.conv1.weight": g("neck.0.weight", (nc, C, 1, 1)),
          "neck.layer_norm1.weight": g("neck.1.weight", (nc,)), "neck.layer_norm1.bias": g("neck.1.bias", (nc,)),
          "neck.conv2.weight": g("neck.2.weight", (nc, nc, 3, 3)),
          "neck.layer_norm2.weight": g("neck.3.weight", (nc,)), "neck.layer_norm2.bias": g("neck.3.bias", (nc,)),
          "proj.conv1.weight": g("net_2.weight", (c0, nc, 3, 3)), "proj.conv2.weight": g("net_3.weight", (c1, c0, 3, 3))}
    hid = int(C * p.mlp_ratio)
    for b in range(p.depth):
        s, q = f"blocks.{b}.", f"layers.{b}."
        tok = t if b in p.global_attn_indexes else p.window_size
        hd = C // p.num_heads
        sd.update({q + "layer_norm1.weight": g(s + "norm1.weight", (C,)), q + "layer_norm1.bias": g(s + "norm1.bias", (C,)),
                   q + "layer_norm2.weight": g(s + "norm2.weight", (C,)), q + "layer_norm2.bias": g(s + "norm2.bias", (C,)),
                   q + "attn.qkv.weight": g(s + "attn.qkv.weight", (3 * C, C)), q + "attn.qkv.bias": g(s + "attn.qkv.bias", (3 * C,)),
                   q + "attn.proj.weight": g(s + "attn.proj.weight", (C, C)), q + "attn.proj.bias": g(s + "attn.proj.bias", (C,)),
                   q + "attn.rel_pos_h": g(s + "attn.rel_pos_h", (2 * tok - 1, hd)),
                   q + "attn.rel_pos_w": g(s + "attn.rel_pos_w", (2 * tok - 1, hd)),
                   q + "mlp.lin1.weight": g(s + "mlp.fc1.weight", (hid, C)), q + "mlp.lin1.bias": g(s + "mlp.fc1.bias", (hid,)),
                   q + "mlp.lin2.weight": g(s + "mlp.fc2.weight", (C, hid)), q + "mlp.lin2.bias": g(s + "mlp.fc2.bias", (C,))})
    missing, unexpected = enc.load_state_dict(sd, strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    rng = np.random.default_rng(4)
    for size in (p.image_size, (p.image_size * 5) // 8):   # native grid, and a resized (tile) grid
        img = rng.uniform(-1, 1, (1, 3, size, size)).astype(np.float32)
        ref = sam.forward(img)                                  # NHWC
        with torch.no_grad():
            got = enc(pixel_values=_t(img)).last_hidden_state.permute(0, 2, 3, 1).numpy()
        assert got.shape == ref.shape
        assert _rel(got, ref) < 2e-4, (size, _rel(got, ref))


def test_clip_matches_transformers_clip_encoder():
    """CLIP-L transformer stack (pre_layrnorm + pre-LN layers, quick-GELU) against transformers'
    CLIPVisionTransformer pieces, fed the oracle's SAM-feature token embeddings (the DeepSeek-OCR
    CLIP takes SAM features instead of its own patch conv: clip.rs:165-236)."""
    from transformers.models.clip import configuration_clip as CC, modeling_clip as CM
    from oracle.vision import Clip
    cfg = json.load(open(TINY))
    W = Weights(seed=13, dtype="f16")
    clip = Clip(cfg, W)
    p = clip.p
    C = p.hidden_size
    vc = CC.CLIPVisionConfig(hidden_size=C, intermediate_size=p.ffn_hidden_size, num_hidden_layers=p.num_layers,
                             num_attention_heads=p.num_heads, image_size=p.image_size, patch_size=p.patch_size,
                             hidden_act="quick_gelu", layer_norm_eps=p.eps)
    vc._attn_implementation = "eager"
    vt = CM.CLIPVisionModel(vc).eval()
    g = lambda n, s: _t(clip.g(n, s))
    sd = {"pre_layrnorm.weight": g("pre_layrnorm.weight", (C,)), "pre_layrnorm.bias": g("pre_layrnorm.bias", (C,))}
    for li in range(p.num_layers):
        s, q = f"transformer.layers.{li}.", f"encoder.layers.{li}."
        qkv_w, qkv_b = clip.g(s + "self_attn.qkv_proj.weight", (3 * C, C)), clip.g(s + "self_attn.qkv_proj.bias", (3 * C,))
        for j, n in enumerate(("q_proj", "k_proj", "v_proj")):
            sd[q + f"self_attn.{n}.weight"] = _t(qkv_w[j * C:(j + 1) * C])
            sd[q + f"self_attn.{n}.bias"] = _t(qkv_b[j * C:(j + 1) * C])
        for n, hn in (("self_attn.out_proj", "self_attn.out_proj"), ("layer_norm1", "layer_norm1"),
                      ("layer_norm2", "layer_norm2")):
            sd[q + hn + ".weight"] = g(s + n + ".weight", (C, C) if "proj" in n else (C,))
            sd[q + hn + ".bias"] = g(s + n + ".bias", (C,))
        sd[q + "mlp.fc1.weight"] = g(s + "mlp.fc1.weight", (p.ffn_hidden_size, C))
        sd[q + "mlp.fc1.bias"] = g(s + "mlp.fc1.bias", (p.ffn_hidden_size,))
        sd[q + "mlp.fc2.weight"] = g(s + "mlp.fc2.weight", (C, p.ffn_hidden_size))
        sd[q + "mlp.fc2.bias"] = g(s + "mlp.fc2.bias", (C,))
    vm = getattr(vt, "vision_model", vt)  # the module holding pre_layrnorm / encoder
    missing, unexpected = vm.load_state_dict(sd, strict=False)
    assert not unexpected and all(m.startswith(("embeddings.", "post_layernorm.")) for m in missing), missing
    rng = np.random.default_rng(5)
    for grid in (int(round(p.seq_length ** 0.5)), 4):        # native 16x16 grid and a resized one
        sam_feat = rng.standard_normal((2, grid, grid, C)).astype(np.float32)
        ref = clip.forward(sam_feat)
        cls = np.broadcast_to(clip.g("embeddings.class_embedding", (C,)), (2, 1, C))
        emb = np.concatenate([cls, sam_feat.reshape(2, grid * grid, C)], 1) + clip.pos(grid * grid + 1)[None]
        with torch.no_grad():
            got = vm.encoder(inputs_embeds=vm.pre_layrnorm(_t(emb))).last_hidden_state.numpy()
        assert _rel(got, ref) < 2e-4, (grid, _rel(got, ref))
