"""Module tree of `Wav2Vec2ForCTC` and the reference's `collect_params` walk over it (row A6, A9).

The reference driver prints every `model.named_modules()` name while collecting the trainable tensors
(`/root/reference/main.py:79-80`) and then prints the collected `param_names` list (`main.py:312-314`).
The engine computes the same list from the geometry alone: the tree below restates the HF module layout
(`transformers/models/wav2vec2/modeling_wav2vec2.py`: `Wav2Vec2ForCTC`, `Wav2Vec2Model`,
`Wav2Vec2FeatureEncoder` with its `GroupNorm` / `NoLayerNorm` / `LayerNorm` conv layers,
`Wav2Vec2FeatureProjection`, `Wav2Vec2Encoder[StableLayerNorm]`, `Wav2Vec2PositionalConvEmbedding` with
torch's weight-norm parametrization, `Wav2Vec2EncoderLayer[StableLayerNorm]`), in registration order,
with each module's own parameters.  `tests/test_host.py` checks it against `tests/golden/g8_collect_params.json`,
which the reference's own `collect_params` produced on transformers' model (`tests/golden/make_golden.py g8`).
"""
from __future__ import annotations

from typing import List, Tuple

# (name, is_layer_norm, own parameter names in registration order)
Module = Tuple[str, bool, List[str]]


def named_modules(cfg: dict) -> List[Module]:
    """`Wav2Vec2ForCTC(cfg).named_modules()` in order (pre-order, registration order)."""
    out: List[Module] = [("", False, []), ("wav2vec2", False, ["masked_spec_embed"])]
    fe = "wav2vec2.feature_extractor"
    out += [(fe, False, []), (fe + ".conv_layers", False, [])]
    group = cfg["feat_extract_norm"] == "group"
    conv_p = ["weight", "bias"] if cfg["conv_bias"] else ["weight"]
    for i in range(len(cfg["conv_dim"])):
        b = f"{fe}.conv_layers.{i}"
        out += [(b, False, []), (b + ".conv", False, conv_p)]
        if group:
            if i == 0:   # Wav2Vec2GroupNormConvLayer: conv, activation, layer_norm (nn.GroupNorm)
                out += [(b + ".activation", False, []), (b + ".layer_norm", False, ["weight", "bias"])]
            else:        # Wav2Vec2NoLayerNormConvLayer: conv, activation
                out += [(b + ".activation", False, [])]
        else:            # Wav2Vec2LayerNormConvLayer: conv, layer_norm (nn.LayerNorm), activation
            out += [(b + ".layer_norm", True, ["weight", "bias"]), (b + ".activation", False, [])]
    fp = "wav2vec2.feature_projection"
    out += [(fp, False, []), (fp + ".layer_norm", True, ["weight", "bias"]),
            (fp + ".projection", False, ["weight", "bias"]), (fp + ".dropout", False, [])]
    en = "wav2vec2.encoder"
    pc = en + ".pos_conv_embed"
    out += [(en, False, []), (pc, False, []), (pc + ".conv", False, ["bias"]),
            (pc + ".conv.parametrizations", False, []),
            (pc + ".conv.parametrizations.weight", False, ["original0", "original1"]),
            (pc + ".conv.parametrizations.weight.0", False, []),
            (pc + ".padding", False, []), (pc + ".activation", False, []),
            (en + ".layer_norm", True, ["weight", "bias"]), (en + ".dropout", False, []),
            (en + ".layers", False, [])]
    for li in range(cfg["num_hidden_layers"]):
        lb = f"{en}.layers.{li}"
        at, ff = lb + ".attention", lb + ".feed_forward"
        out += [(lb, False, []), (at, False, [])]
        out += [(f"{at}.{p}", False, ["weight", "bias"]) for p in ("k_proj", "v_proj", "q_proj", "out_proj")]
        out += [(lb + ".dropout", False, []), (lb + ".layer_norm", True, ["weight", "bias"]), (ff, False, []),
                (ff + ".intermediate_dropout", False, []), (ff + ".intermediate_dense", False, ["weight", "bias"]),
                (ff + ".intermediate_act_fn", False, []), (ff + ".output_dense", False, ["weight", "bias"]),
                (ff + ".output_dropout", False, []), (lb + ".final_layer_norm", True, ["weight", "bias"])]
    out += [("dropout", False, []), ("lm_head", False, ["weight", "bias"])]
    return out


def _named_parameters(mods: List[Module], i: int) -> List[str]:
    """`mods[i].named_parameters()` (recursive, the module's own first, then its subtree), as the full
    dotted names the reference appends (`f"{nm}.{np}"`, main.py:93)."""
    nm = mods[i][0]
    out = []
    for m2, _, ps in mods[i:]:
        if m2 != nm and not (nm == "" or m2.startswith(nm + ".")):
            break
        out += [f"{m2}.{p}" if m2 else p for p in ps]
    return out


def collect_params(cfg: dict, bias_only: bool = False, train_feature: bool = False, train_LN: bool = True
                   ) -> Tuple[List[str], List[str]]:
    """(printed module names, param_names) of reference `collect_params` (main.py:62-103) with
    `train_all` False (out of the engine's scope).  param_names lists a tensor once per module whose walk
    reaches it, so feature-encoder tensors repeat (the Adam multiplicity)."""
    mods = named_modules(cfg)
    printed, names = [], []
    trainable = ["bias"] if bias_only else ["weight", "bias"]
    for i, (nm, is_ln, ps) in enumerate(mods):
        printed.append(nm)
        if train_LN and is_ln:
            names += [f"{nm}.{p}" for p in ps if p in trainable]
        if train_feature:
            parts = nm.split(".")
            if len(parts) > 1 and parts[1] in ("feature_extractor", "feature_projection"):
                names += _named_parameters(mods, i)
    return printed, names
