"""Seeded synthetic Wav2Vec2ForCTC weights, and loading of local HF checkpoints.

Pretrained checkpoints are not reachable offline, so benches and
parity tests run on weights drawn here.  Every tensor comes from its own
`numpy.random.default_rng([seed, crc32(name)])` stream, so the draw is
bit-identical on every machine and independent of tensor order.
"""
from __future__ import annotations

import math
import os
import zlib
from typing import Dict

import numpy as np

from .config import param_shapes

DEFAULT_SEED = 20260415


def synth_weights(cfg: dict, seed: int = DEFAULT_SEED, blank_bias: float = 1.0) -> Dict[str, np.ndarray]:
    """name -> float32 array with fan-in scaled normals, perturbed norm affines.

    `blank_bias` is added to lm_head.bias[0] (the CTC blank, vocab.json `<pad>`=0)
    so that both blank and non-blank frames occur.
    """
    out: Dict[str, np.ndarray] = {}
    for name, shape in param_shapes(cfg):
        rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
        n = rng.standard_normal(shape)
        leaf = name.rsplit(".", 1)[-1]
        if name.endswith("masked_spec_embed"):
            a = rng.uniform(size=shape)
        elif "layer_norm" in name and leaf == "weight":
            a = 1.0 + 0.1 * n
        elif "layer_norm" in name and leaf == "bias":
            a = 0.1 * n
        elif leaf == "original0":                      # pos-conv weight_norm magnitude per tap
            H = cfg["hidden_size"]
            G = cfg["num_conv_pos_embedding_groups"]
            K = cfg["num_conv_pos_embeddings"]
            a = math.sqrt(H * (H // G) / ((H // G) * K)) * (1.0 + 0.1 * n)
        elif leaf == "original1":
            a = n
        elif leaf == "bias":
            a = 0.02 * n
        else:                                          # conv / linear weight: N(0, 1/fan_in) (x2 for conv+GELU)
            fan_in = int(np.prod(shape[1:]))
            gain = 2.0 if "conv_layers" in name else 1.0
            a = n * math.sqrt(gain / fan_in)
        out[name] = np.ascontiguousarray(a, dtype=np.float32)
    out["lm_head.bias"][0] += np.float32(blank_bias)
    return out


LEGACY_NAMES = (("weight_g", "parametrizations.weight.original0"),
                ("weight_v", "parametrizations.weight.original1"))


def remap_legacy(sd: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Checkpoints saved before torch's parametrized weight_norm name the positional conv's
    weight-norm tensors `weight_g` / `weight_v`; HF maps them to `parametrizations.weight.original0/1`
    on load.  Applied to every checkpoint format."""
    for old, new in LEGACY_NAMES:
        key = "wav2vec2.encoder.pos_conv_embed.conv." + old
        if key in sd:
            sd["wav2vec2.encoder.pos_conv_embed.conv." + new] = sd.pop(key)
    return sd


def load_hf_checkpoint(path: str) -> Dict[str, np.ndarray]:
    """state_dict of a LOCAL HF checkpoint dir (safetensors preferred; torch files weights_only)."""
    st = os.path.join(path, "model.safetensors")
    if os.path.isfile(st):
        from safetensors.numpy import load_file
        return remap_legacy({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in load_file(st).items()})
    pt = os.path.join(path, "pytorch_model.bin")
    if os.path.isfile(pt):
        import torch
        sd = torch.load(pt, map_location="cpu", weights_only=True)
        return remap_legacy({k: v.float().numpy() for k, v in sd.items()})
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path}")
