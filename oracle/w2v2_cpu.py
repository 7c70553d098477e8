"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

PyTorch-CPU functional restatement of the reference's SUTA adapt loop:

  * Wav2Vec2ForCTC forward  — HF transformers 5.15.0
    `models/wav2vec2/modeling_wav2vec2.py` (cited as HF:<line>):
      conv feature encoder       HF:254-323, 409-419
      feature projection         HF:422-434
      positional conv embedding  HF:326-379
      encoder (post-LN, base)    HF:667-726 with layers HF:591-608
      encoder (stable-LN, large) HF:741-802 with layers HF:631-654
      attention                  HF:466-548 (+ eager_attention_forward HF:437-463)
      lm_head                    HF:1700
  * SUTA loss                — reference main.py:26-60 and 181-203
  * trainable-entry list     — reference main.py:62-103 (`collect_params`),
                               with its duplicate listing of nested modules
  * AdamW step               — torch 2.10 optim/adam.py:347-548 single-tensor
                               path: a tensor listed k times is stepped k times
                               per `optimizer.step()` with the same gradient
  * episodic adapt loop      — reference main.py:319-402 (vanilla forward,
                               then `steps` x forward_and_adapt main.py:172-215)
  * SDPL pseudo-label loss   — reference main_SDPL.py:143-209 (torch CPU CTCLoss
                               on the time-log-softmax; target = greedy transcript)

Parameters are a dict keyed by the HF `state_dict()` names; the config is a dict
with HF `Wav2Vec2Config` key names.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

PFX = "wav2vec2."


def frame_lengths(cfg: dict, n_samples: int) -> List[int]:
    """Conv output length per layer, L_i = floor((L_{i-1} - k_i) / s_i) + 1 (torch Conv1d, no padding)."""
    out = []
    L = n_samples
    for k, s in zip(cfg["conv_kernel"], cfg["conv_stride"]):
        L = (L - k) // s + 1
        out.append(L)
    return out


def pos_conv_weight(p: Dict[str, torch.Tensor]) -> torch.Tensor:
    """weight_norm(dim=2): w = g * v / ||v||, norm over dims (0, 1) for every tap k (HF:337-341)."""
    g = p[PFX + "encoder.pos_conv_embed.conv.parametrizations.weight.original0"]
    v = p[PFX + "encoder.pos_conv_embed.conv.parametrizations.weight.original1"]
    nrm = torch.linalg.vector_norm(v, dim=(0, 1), keepdim=True)
    return g * (v / nrm)


def forward(p: Dict[str, torch.Tensor], cfg: dict, x: torch.Tensor) -> torch.Tensor:
    """Wav2Vec2ForCTC(x).logits for x of shape (B, N) float32; eval mode (dropouts inactive)."""
    eps = cfg.get("layer_norm_eps", 1e-5)
    nconv = len(cfg["conv_dim"])
    group = cfg["feat_extract_norm"] == "group"
    h = x[:, None, :]
    for i in range(nconv):
        base = PFX + f"feature_extractor.conv_layers.{i}."
        h = F.conv1d(h, p[base + "conv.weight"], p.get(base + "conv.bias"), stride=cfg["conv_stride"][i])
        if group and i == 0:                       # HF:319-323 GroupNorm(C groups, C channels)
            C = h.shape[1]
            h = F.group_norm(h, C, p[base + "layer_norm.weight"], p[base + "layer_norm.bias"], eps=1e-5)
        elif not group:                            # HF:291-299 LayerNorm over channels (default eps 1e-5)
            h = F.layer_norm(h.transpose(1, 2), (h.shape[1],), p[base + "layer_norm.weight"],
                             p[base + "layer_norm.bias"], eps=1e-5).transpose(1, 2)
        h = F.gelu(h)
    h = h.transpose(1, 2)                          # (B, T, C)   HF:1340
    fp = PFX + "feature_projection."
    h = F.layer_norm(h, (h.shape[-1],), p[fp + "layer_norm.weight"], p[fp + "layer_norm.bias"], eps=eps)
    h = F.linear(h, p[fp + "projection.weight"], p[fp + "projection.bias"])     # HF:429-434

    # positional conv embedding HF:360-368: conv(pad K//2, groups) -> drop last frame (even K) -> GELU
    K = cfg["num_conv_pos_embeddings"]
    w = pos_conv_weight(p)
    pc = F.conv1d(h.transpose(1, 2), w, p[PFX + "encoder.pos_conv_embed.conv.bias"], padding=K // 2,
                  groups=cfg["num_conv_pos_embedding_groups"])
    if K % 2 == 0:
        pc = pc[:, :, :-1]
    h = h + F.gelu(pc).transpose(1, 2)
    enc = PFX + "encoder."
    H = cfg["hidden_size"]
    stable = cfg["do_stable_layer_norm"]
    if not stable:                                 # HF:689-691
        h = F.layer_norm(h, (H,), p[enc + "layer_norm.weight"], p[enc + "layer_norm.bias"], eps=eps)
    for li in range(cfg["num_hidden_layers"]):
        lp = enc + f"layers.{li}."
        if stable:                                 # HF:631-654 pre-LN
            a = _attention(p, lp, cfg, F.layer_norm(h, (H,), p[lp + "layer_norm.weight"],
                                                     p[lp + "layer_norm.bias"], eps=eps))
            h = h + a
            h = h + _ffn(p, lp, F.layer_norm(h, (H,), p[lp + "final_layer_norm.weight"],
                                              p[lp + "final_layer_norm.bias"], eps=eps))
        else:                                      # HF:591-608 post-LN
            h = h + _attention(p, lp, cfg, h)
            h = F.layer_norm(h, (H,), p[lp + "layer_norm.weight"], p[lp + "layer_norm.bias"], eps=eps)
            h = h + _ffn(p, lp, h)
            h = F.layer_norm(h, (H,), p[lp + "final_layer_norm.weight"], p[lp + "final_layer_norm.bias"], eps=eps)
    if stable:                                     # HF:791
        h = F.layer_norm(h, (H,), p[enc + "layer_norm.weight"], p[enc + "layer_norm.bias"], eps=eps)
    return F.linear(h, p["lm_head.weight"], p["lm_head.bias"])                    # HF:1700


def _attention(p, lp, cfg, h):
    """softmax(Q K^T * d^-0.5) V over heads, biases on q/k/v/out (HF:500-548, 437-463)."""
    B, T, H = h.shape
    nh = cfg["num_attention_heads"]
    d = H // nh
    ap = lp + "attention."
    q = F.linear(h, p[ap + "q_proj.weight"], p[ap + "q_proj.bias"]).view(B, T, nh, d).transpose(1, 2)
    k = F.linear(h, p[ap + "k_proj.weight"], p[ap + "k_proj.bias"]).view(B, T, nh, d).transpose(1, 2)
    v = F.linear(h, p[ap + "v_proj.weight"], p[ap + "v_proj.bias"]).view(B, T, nh, d).transpose(1, 2)
    s = torch.matmul(q, k.transpose(2, 3)) * (d ** -0.5)
    a = torch.matmul(torch.softmax(s, dim=-1), v).transpose(1, 2).reshape(B, T, H)
    return F.linear(a, p[ap + "out_proj.weight"], p[ap + "out_proj.bias"])


def _ffn(p, lp, h):
    fp = lp + "feed_forward."
    u = F.gelu(F.linear(h, p[fp + "intermediate_dense.weight"], p[fp + "intermediate_dense.bias"]))
    return F.linear(u, p[fp + "output_dense.weight"], p[fp + "output_dense.bias"])


# ----------------------------------------------------------------------------------------------
# collect_params restatement (reference main.py:62-103)
# ----------------------------------------------------------------------------------------------
def module_tree(cfg: dict) -> List[Tuple[str, str, List[str]]]:
    """(module_name, kind, direct-param names) in Wav2Vec2ForCTC.named_modules() order.

    kind is 'ln' for nn.LayerNorm modules, else 'other'.  Only modules that own
    parameters (directly or through children) matter for collect_params.
    """
    mods: List[Tuple[str, str, List[str]]] = []
    group = cfg["feat_extract_norm"] == "group"
    bias = cfg.get("conv_bias", False)
    mods.append(("", "other", []))
    mods.append(("wav2vec2", "other", ["masked_spec_embed"]))
    mods.append(("wav2vec2.feature_extractor", "other", []))
    mods.append(("wav2vec2.feature_extractor.conv_layers", "other", []))
    for i in range(len(cfg["conv_dim"])):
        b = f"wav2vec2.feature_extractor.conv_layers.{i}"
        mods.append((b, "other", []))
        mods.append((b + ".conv", "other", ["weight"] + (["bias"] if bias else [])))
        if group and i == 0:
            mods.append((b + ".layer_norm", "other", ["weight", "bias"]))       # nn.GroupNorm
        elif not group:
            mods.append((b + ".layer_norm", "ln", ["weight", "bias"]))
    mods.append(("wav2vec2.feature_projection", "other", []))
    mods.append(("wav2vec2.feature_projection.layer_norm", "ln", ["weight", "bias"]))
    mods.append(("wav2vec2.feature_projection.projection", "other", ["weight", "bias"]))
    mods.append(("wav2vec2.encoder", "other", []))
    mods.append(("wav2vec2.encoder.layer_norm", "ln", ["weight", "bias"]))
    for li in range(cfg["num_hidden_layers"]):
        b = f"wav2vec2.encoder.layers.{li}"
        mods.append((b + ".layer_norm", "ln", ["weight", "bias"]))
        mods.append((b + ".final_layer_norm", "ln", ["weight", "bias"]))
    return mods


def trainable_entries(cfg: dict, bias_only=False, train_feature=False, train_LN=True) -> List[str]:
    """Ordered list of parameter names as `collect_params` appends them (duplicates included).

    main.py:79-94: for each module m in named_modules(): if m is nn.LayerNorm and
    train_LN, append its weight/bias (bias only with --bias_only); if the module
    name's 2nd dotted component is feature_extractor/feature_projection and
    train_feature, append ALL its parameters recursively (named_parameters()).
    `train_all` is not restated (out of scope for the engine).
    """
    mods = module_tree(cfg)
    names_with_params = [(m, k, [f"{m}.{q}" if m else q for q in ps]) for m, k, ps in mods]
    out: List[str] = []
    for nm, kind, _ in mods:
        if train_LN and kind == "ln":
            for q in (["bias"] if bias_only else ["weight", "bias"]):
                out.append(f"{nm}.{q}")
        if train_feature:
            parts = nm.split(".")
            if len(parts) > 1 and parts[1] in ("feature_extractor", "feature_projection"):
                for m2, _, ps in names_with_params:          # recursive named_parameters()
                    if m2 == nm or m2.startswith(nm + "."):
                        out.extend(ps)
    return out


def multiplicity(entries: Sequence[str]) -> Dict[str, int]:
    mult: Dict[str, int] = {}
    for e in entries:
        mult[e] = mult.get(e, 0) + 1
    return mult


# ----------------------------------------------------------------------------------------------
# SUTA loss (reference main.py:26-60, 181-203)
# ----------------------------------------------------------------------------------------------
def softmax_entropy(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    return -(x.softmax(dim) * x.log_softmax(dim)).sum(dim)                      # main.py:26-28


def suta_loss(logits: torch.Tensor, em_coef: float, reweight: bool, temp: float, non_blank: bool,
              div_coef: float = 0.0) -> torch.Tensor:
    """loss = em*E + (1-em)*MCC (+ div*D) for logits (1, T, V); batch 1 only (main.py:30-44 squeezes)."""
    z = logits / temp
    loss = logits.new_zeros(())
    if em_coef > 0:
        ent = softmax_entropy(z)                                                 # (1, T)
        if non_blank:
            mask = logits.argmax(-1) != 0                                        # main.py:183-184
            loss = loss + ent[mask].mean() * em_coef                             # main.py:190
        else:
            loss = loss + ent.mean() * em_coef                                   # main.py:193
    if 1 - em_coef > 0:
        p = z.softmax(-1).squeeze(0)                                             # main.py:31-32
        V = p.shape[-1]
        if reweight:                                                             # main.py:33-37
            w = softmax_entropy(z).detach().squeeze(0)
            w = 1 + torch.exp(-w)
            w = z.shape[1] * w / w.sum()
            C = (p * w[:, None]).t().mm(p)
        else:
            C = p.t().mm(p)                                                      # main.py:39
        C = C / C.sum(dim=1)                                                     # main.py:41 (column j / s_j)
        loss = loss + (C.sum() - torch.trace(C)) / V * (1 - em_coef)             # main.py:42 (class_num = V = 32)
    if div_coef > 0:                                                             # main.py:46-60, 201-203
        cls = logits.squeeze(0).mean(0)[1:]
        loss = loss + (-softmax_entropy(cls, 0)) * div_coef
    return loss


# ----------------------------------------------------------------------------------------------
# SDPL objective (reference main_SDPL.py:143-209)
# ----------------------------------------------------------------------------------------------
SPECIAL_IDS = (1, 2, 3)  # <s>, </s>, <unk>: decoded as several characters -> the reference's vocab lookup raises


def pseudo_label_target(ids: Sequence[int]) -> List[int]:
    """processor.batch_decode(argmax)[0] mapped back through vocab.json (main_SDPL.py:194-200): collapse
    repeats, drop blank 0, '|' (4) <-> ' ', strip() -> leading/trailing delimiters dropped."""
    out, prev = [], None
    for i in ids:
        i = int(i)
        if i == prev:
            continue
        prev = i
        if i != 0:
            out.append(i)
    while out and out[0] == 4:
        out.pop(0)
    while out and out[-1] == 4:
        out.pop()
    if any(i in SPECIAL_IDS for i in out):
        raise KeyError("special token in the pseudo-label transcript (reference vocab lookup fails)")
    return out


def pseudo_labeling_loss(logits: torch.Tensor) -> torch.Tensor:
    """nn.CTCLoss(blank=0)(outputs.log_softmax(1).transpose(1, 0), target) (main_SDPL.py:192-209): the
    log-softmax is over TIME (dim 1 of (1, T, V)); reduction 'mean' divides by the target length."""
    target = pseudo_label_target(logits.argmax(-1)[0].tolist())
    logp = logits.log_softmax(1).transpose(1, 0)                                 # (T, 1, V)
    return F.ctc_loss(logp, torch.tensor(target, dtype=torch.int32), torch.tensor([logp.shape[0]]),
                      torch.tensor([len(target)]), blank=0, reduction="mean", zero_infinity=False)


def sdpl_loss(logits: torch.Tensor, em_coef: float, reweight: bool, temp: float, non_blank: bool,
              pl_coef: float, div_coef: float = 0.0) -> torch.Tensor:
    """loss * (1 - pl_coef) + pseudo_labeling_loss * pl_coef (main_SDPL.py:180)."""
    return suta_loss(logits, em_coef, reweight, temp, non_blank, div_coef) * (1 - pl_coef) + \
        pseudo_labeling_loss(logits) * pl_coef


# ----------------------------------------------------------------------------------------------
# AdamW single-tensor path with duplicate-entry multiplicity
# ----------------------------------------------------------------------------------------------
class AdamState:
    def __init__(self, names: Sequence[str], params: Dict[str, torch.Tensor]):
        self.step = {n: 0 for n in names}
        self.m = {n: torch.zeros_like(params[n]) for n in names}
        self.v = {n: torch.zeros_like(params[n]) for n in names}


def adam_step(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor], state: AdamState,
              entries: Sequence[str], lr: float, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0) -> None:
    """One optimizer.step(): iterate the entry list in order (adam.py:389-548).

    Each entry: step += 1; param *= 1 - lr*wd; m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g^2;
    denom = sqrt(v)/sqrt(1-b2^t) + eps; param -= lr/(1-b1^t) * m/denom.
    """
    b1, b2 = betas
    with torch.no_grad():
        for n in entries:
            g = grads[n]
            p = params[n]
            state.step[n] += 1
            t = state.step[n]
            if weight_decay != 0:
                p.mul_(1 - lr * weight_decay)
            state.m[n].lerp_(g, 1 - b1)
            state.v[n].mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1 = 1 - b1 ** t
            bc2 = 1 - b2 ** t
            step_size = lr / bc1
            denom = (state.v[n].sqrt() / math.sqrt(bc2)).add_(eps)
            p.addcdiv_(state.m[n], denom, value=-step_size)


def sgd_step(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor], entries: Sequence[str],
             lr: float) -> None:
    """One torch.optim.SGD(params, lr, weight_decay=0).step() (main.py:18; sgd.py _single_tensor_sgd at momentum 0):
    param.add_(grad, alpha=-lr) once per entry, in list order (a tensor listed k times moves k times)."""
    with torch.no_grad():
        for n in entries:
            params[n].add_(grads[n], alpha=-lr)


def step_lr(lr: float, gamma: float, step_size: int, i: int) -> float:
    """The lr StepLR (main.py:20-21: eval(scheduler)(optimizer, step_size=1, gamma=0.7)) leaves in the param group
    after i scheduler steps (main.py:207-208): the group lr times gamma, in double, at every step count that is a
    multiple of step_size (lr_scheduler.py StepLR.get_lr, chained form).  step_size 0: no scheduler."""
    if step_size <= 0:
        return lr
    for e in range(1, i + 1):
        if e % step_size == 0:
            lr = lr * gamma
    return lr


class OptCarry:
    """Optimizer / scheduler state carried from one utterance to the next in non-episodic runs (the reference
    never restores it then, main.py:327-328): the adapted tensors, Adam moments and the optimizer step count."""

    def __init__(self):
        self.params = None
        self.state = None
        self.nstep = 0


# ----------------------------------------------------------------------------------------------
# Episodic SUTA on one utterance (reference main.py:327-398 + forward_and_adapt main.py:172-215)
# ----------------------------------------------------------------------------------------------
def run_suta(params0: Dict[str, torch.Tensor], cfg: dict, x: torch.Tensor, steps: int, *, lr=2e-5, temp=2.5,
             em_coef=0.3, reweight=True, non_blank=True, div_coef=0.0, train_feature=True, bias_only=False,
             record: Sequence[int] = None, pl_coef: float = 0.0, opt: str = "AdamW", lr_step_size: int = 0,
             lr_gamma: float = 0.7, carry: OptCarry = None) -> Tuple[Dict[int, torch.Tensor], Dict[str, torch.Tensor]]:
    """Returns ({r: logits after r updates} for r in record (0 = vanilla), final trainable tensors).

    Uses the minimal schedule (S+1 forwards, S backwards): the re-inference forward of
    step i (main.py:212-214) equals the grad forward of step i+1 (same params, same x).
    opt: 'AdamW' / 'Adam' (identical at weight decay 0) or 'SGD' (main.py:9-18); lr_step_size > 0: StepLR
    (main.py:20-21).  carry: non-episodic state from the previous utterance (None = episodic reset).
    """
    if record is None:
        record = list(range(steps + 1))
    if opt not in ("AdamW", "Adam", "SGD"):
        raise ValueError(opt)
    entries = trainable_entries(cfg, bias_only=bias_only, train_feature=train_feature)
    uniq = list(dict.fromkeys(entries))
    if carry is not None and carry.params is not None:
        params, state = carry.params, carry.state
    else:
        params = {k: v.detach().clone() for k, v in params0.items()}
        state = AdamState(uniq, params)
    nstep = carry.nstep if carry is not None else 0
    out: Dict[int, torch.Tensor] = {}
    for i in range(steps + 1):
        for n in uniq:
            params[n].requires_grad_(True)
        logits = forward(params, cfg, x)
        if i in record:
            out[i] = logits.detach().clone()
        if i == steps:
            break
        if pl_coef > 0:  # SDPL (main_SDPL.py:143-186)
            loss = sdpl_loss(logits, em_coef, reweight, temp, non_blank, pl_coef, div_coef)
        else:
            loss = suta_loss(logits, em_coef, reweight, temp, non_blank, div_coef)
        grads = torch.autograd.grad(loss, [params[n] for n in uniq])
        lr_i = step_lr(lr, lr_gamma, lr_step_size, nstep)
        if opt == "SGD":
            sgd_step(params, dict(zip(uniq, grads)), entries, lr_i)
        else:
            adam_step(params, dict(zip(uniq, grads)), state, entries, lr_i)
        nstep += 1
    if carry is not None:
        for n in uniq:
            params[n].requires_grad_(False)
        carry.params, carry.state, carry.nstep = params, state, nstep
    return out, {n: params[n].detach().clone() for n in uniq}


def normalize_wave(x):
    """HF Wav2Vec2FeatureExtractor.zero_mean_unit_var_norm (feature_extraction_wav2vec2.py:78-97), float32."""
    import numpy as np
    x = np.asarray(x, dtype=np.float32)
    return (x - x.mean()) / np.sqrt(x.var() + 1e-7)
