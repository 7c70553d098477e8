"""Model geometry presets (HF `Wav2Vec2Config` key names) and frame-length arithmetic.

The shapes follow the public HF configs of facebook/wav2vec2-base-960h and
facebook/wav2vec2-large-960h-lv60 ("Model shapes"); key names are the
ones `transformers.Wav2Vec2Config` uses (configuration_wav2vec2.py:165-219).
"""
from __future__ import annotations

import copy
import json
import os
from typing import List

_BASE = dict(
    hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
    vocab_size=32, conv_dim=[512] * 7, conv_kernel=[10, 3, 3, 3, 3, 2, 2], conv_stride=[5, 2, 2, 2, 2, 2, 2],
    conv_bias=False, feat_extract_norm="group", do_stable_layer_norm=False,
    num_conv_pos_embeddings=128, num_conv_pos_embedding_groups=16, layer_norm_eps=1e-5,
)

_LARGE = dict(_BASE, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
              conv_bias=True, feat_extract_norm="layer", do_stable_layer_norm=True)

# Tiny geometries used for the committed golden vectors (tests/golden/make_golden.py).
_TINY_GROUP = dict(_BASE, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                   conv_dim=[32] * 7, num_conv_pos_embeddings=16, num_conv_pos_embedding_groups=4)
_TINY_LAYER = dict(_TINY_GROUP, conv_bias=True, feat_extract_norm="layer", do_stable_layer_norm=True)

PRESETS = {
    "facebook/wav2vec2-base-960h": _BASE,
    "wav2vec2-base": _BASE,
    "facebook/wav2vec2-large-960h-lv60": _LARGE,
    "facebook/wav2vec2-large-960h-lv60-self": _LARGE,
    "wav2vec2-large": _LARGE,
    "tiny-group": _TINY_GROUP,
    "tiny-layer": _TINY_LAYER,
}


def get_config(name_or_path: str) -> dict:
    """Preset by model name, or a local HF checkpoint directory's config.json."""
    if name_or_path in PRESETS:
        return copy.deepcopy(PRESETS[name_or_path])
    cfg_file = os.path.join(name_or_path, "config.json")
    if os.path.isfile(cfg_file):
        with open(cfg_file) as f:
            raw = json.load(f)
        cfg = copy.deepcopy(_BASE)
        for k in cfg:
            if k in raw:
                cfg[k] = raw[k]
        return cfg
    raise KeyError(f"unknown model '{name_or_path}': not a preset and no config.json found")


def frame_lengths(cfg: dict, n_samples: int) -> List[int]:
    """Conv output length per feature-encoder layer: L_i = floor((L_{i-1} - k_i)/s_i) + 1."""
    out, L = [], int(n_samples)
    for k, s in zip(cfg["conv_kernel"], cfg["conv_stride"]):
        L = (L - k) // s + 1
        out.append(L)
    return out


def num_frames(cfg: dict, n_samples: int) -> int:
    return frame_lengths(cfg, n_samples)[-1]


def param_shapes(cfg: dict):
    """(name, shape) of every Wav2Vec2ForCTC state_dict entry, in state_dict order."""
    H, C = cfg["hidden_size"], cfg["conv_dim"]
    out = [("wav2vec2.masked_spec_embed", (H,))]
    group = cfg["feat_extract_norm"] == "group"
    for i, (c, k) in enumerate(zip(C, cfg["conv_kernel"])):
        cin = 1 if i == 0 else C[i - 1]
        b = f"wav2vec2.feature_extractor.conv_layers.{i}."
        out.append((b + "conv.weight", (c, cin, k)))
        if cfg["conv_bias"]:
            out.append((b + "conv.bias", (c,)))
        if (group and i == 0) or not group:
            out += [(b + "layer_norm.weight", (c,)), (b + "layer_norm.bias", (c,))]
    fp = "wav2vec2.feature_projection."
    out += [(fp + "layer_norm.weight", (C[-1],)), (fp + "layer_norm.bias", (C[-1],)),
            (fp + "projection.weight", (H, C[-1])), (fp + "projection.bias", (H,))]
    K, G = cfg["num_conv_pos_embeddings"], cfg["num_conv_pos_embedding_groups"]
    pc = "wav2vec2.encoder.pos_conv_embed.conv."
    out += [(pc + "bias", (H,)), (pc + "parametrizations.weight.original0", (1, 1, K)),
            (pc + "parametrizations.weight.original1", (H, H // G, K))]
    out += [("wav2vec2.encoder.layer_norm.weight", (H,)), ("wav2vec2.encoder.layer_norm.bias", (H,))]
    F_ = cfg["intermediate_size"]
    for li in range(cfg["num_hidden_layers"]):
        lp = f"wav2vec2.encoder.layers.{li}."
        for pr in ("k_proj", "v_proj", "q_proj", "out_proj"):
            out += [(lp + f"attention.{pr}.weight", (H, H)), (lp + f"attention.{pr}.bias", (H,))]
        out += [(lp + "layer_norm.weight", (H,)), (lp + "layer_norm.bias", (H,)),
                (lp + "feed_forward.intermediate_dense.weight", (F_, H)),
                (lp + "feed_forward.intermediate_dense.bias", (F_,)),
                (lp + "feed_forward.output_dense.weight", (H, F_)),
                (lp + "feed_forward.output_dense.bias", (H,)),
                (lp + "final_layer_norm.weight", (H,)), (lp + "final_layer_norm.bias", (H,))]
    out += [("lm_head.weight", (cfg["vocab_size"], H)), ("lm_head.bias", (cfg["vocab_size"],))]
    return out
