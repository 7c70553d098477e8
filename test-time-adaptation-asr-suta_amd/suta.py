"""`forward_and_adapt`-compatible drop-in for the reference driver ("Callers").

The reference adapts one utterance with (`/root/reference/main.py:302-348`):

    model = Wav2Vec2ForCTC.from_pretrained(asr).eval().cuda()
    model = configure_model(model)
    params, param_names = collect_params(model, bias_only, train_feature, train_all, train_LN)
    optimizer, scheduler = setup_optimizer(params, opt, lr, scheduler=scheduler)
    if episodic:
        model_state, optimizer_state, scheduler_state = copy_model_and_optimizer(model, optimizer, scheduler)
    ...
        if episodic:
            model, optimizer, scheduler = load_model_and_optimizer(model, optimizer, model_state,
                                                                   optimizer_state, scheduler_state)
        with torch.no_grad():
            outputs = model(input_values).logits
        for i in range(steps):
            outputs = forward_and_adapt(input_values, model, optimizer, em_coef, reweight, temp, non_blank,
                                        scheduler, div_coef)

Every name in that block exists here with the reference's signature and argument meaning, so the loop runs
unchanged after `from suta_amd.suta import *`.  The objects are thin handles on one libsuta engine (one GPU,
one utterance slot): `model(x).logits` is `suta_forward`, `forward_and_adapt` is `suta_step_ex` (grad forward,
fused entropy + MCC (+ div) loss, hand-written backward, AdamW / SGD with the reference's `collect_params`
multiplicities and StepLR, then the no-grad re-forward unless `repeat_inference=False`), and
`load_model_and_optimizer` with the snapshot `copy_model_and_optimizer` took at setup is `suta_reset`.  There
is no CPU fallback: without `libsuta.so` every call raises.

Limits (each raises rather than computing something else):
  * one utterance per call (batch 1): the reference's `mcc_loss` squeezes dim 0 (main.py:32), so a batch of
    several utterances is not a reference computation; the batched engine calls (`SutaEngine.adapt` /
    `adapt_varlen`) adapt many utterances, each as if alone;
  * `train_all=True` / `train_LN=False` (main.py:62-103 with those flags; no script uses them);
  * a state snapshot taken after adaptation started: the engine restores the pristine state only, which is
    the one snapshot the reference takes (main.py:310-311);
  * the scheduler must be passed to every `forward_and_adapt` of an episode or to none of them (the engine
    derives the step's lr from the optimizer steps since the last reset).
"""
from __future__ import annotations

import types
from typing import List, Optional

import numpy as np

from .engine import OPTIMIZERS, SutaEngine, SutaHParams
from .modules import collect_params as _collect_names
from .modules import named_modules as _named_modules

__all__ = ["Wav2Vec2ForCTC", "configure_model", "collect_params", "setup_optimizer", "copy_model_and_optimizer",
           "load_model_and_optimizer", "forward_and_adapt"]


class Wav2Vec2ForCTC:
    """`Wav2Vec2ForCTC(...).eval().cuda()` stand-in: the frozen encoder and one utterance slot of a libsuta
    engine on GPU `device`.  `model(x)` returns an object whose `.logits` is a (1, T, vocab) float32 tensor on
    x's device (the reference calls it under `torch.no_grad()`, main.py:331-332)."""

    def __init__(self, cfg: dict, weights: dict, device: int = 0, max_samples: int = 600000):
        self.config = dict(cfg)
        self._weights = weights
        self.device = device
        self.engine = SutaEngine(cfg, weights, device=device, max_batch=1, max_samples=max_samples)
        self._generation = 0      # bumped by every reset: identifies the pristine state
        self._steps = 0           # optimizer steps since the last reset
        self.last_loss = float("nan")   # SUTA loss of the last forward_and_adapt

    @classmethod
    def from_pretrained(cls, asr: str, synthetic_weights: bool = False, device: int = 0,
                        max_samples: int = 600000) -> "Wav2Vec2ForCTC":
        """A local checkpoint directory or HF-cache entry (offline); `synthetic_weights` falls back to the seeded
        weights of that geometry (suta_amd.main.load_model)."""
        from .main import load_model
        cfg, weights = load_model(asr, synthetic_weights)
        return cls(cfg, weights, device=device, max_samples=max_samples)

    # --- nn.Module surface the reference loop touches -------------------------------------------------
    def eval(self):
        return self

    def cuda(self, device=None):
        return self

    def requires_grad_(self, flag: bool = True):
        return self

    def zero_grad(self, set_to_none: bool = True):
        """Gradients live in the engine and are consumed by the step that made them (main.py:209)."""

    def named_modules(self):
        """(name, module) pairs in `Wav2Vec2ForCTC.named_modules()` order; the modules are descriptors
        (SimpleNamespace: is_layer_norm, parameter names), enough for collect_params' walk."""
        for name, is_ln, ps in _named_modules(self.config):
            yield name, types.SimpleNamespace(is_layer_norm=is_ln, parameter_names=list(ps))

    def state_dict(self) -> dict:
        """Frozen tensors as loaded, trainable tensors as currently adapted (torch tensors, HF names)."""
        import torch
        out = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in self._weights.items()}
        for n in self.engine.trainable_names():
            out[n] = torch.from_numpy(self.engine.get_param(0, n))
        return out

    def __call__(self, x):
        _check_batch1(x)
        logits = self.engine.forward(x, normalize=False)
        return types.SimpleNamespace(logits=_as_like(logits, x))

    forward = __call__

    def close(self):
        self.engine.close()

    def _reset(self):
        self.engine.reset()
        self._generation += 1
        self._steps = 0


class _Param:
    """One `collect_params` entry: the tensor's HF name; `.data` reads the slot's current value."""

    def __init__(self, model: Wav2Vec2ForCTC, name: str):
        self.model, self.name = model, name
        self.requires_grad = True

    @property
    def data(self):
        import torch
        return torch.from_numpy(self.model.engine.get_param(0, self.name))

    def __repr__(self):
        return f"Parameter({self.name})"


class _ParamList(list):
    """collect_params' `params`, remembering the flags the engine needs (multiplicity per tensor)."""
    model: Wav2Vec2ForCTC
    bias_only: bool
    train_feature: bool


def configure_model(model: Wav2Vec2ForCTC) -> Wav2Vec2ForCTC:
    """main.py:167-170: the encoder is frozen by construction (only collect_params' tensors adapt)."""
    return model.requires_grad_(False)


def collect_params(model: Wav2Vec2ForCTC, bias_only=False, train_feature=False, train_all=False, train_LN=True):
    """main.py:62-103: prints every module name, returns (params, names) with a tensor listed once per module
    whose walk reaches it (feature-encoder tensors repeat: the engine's Adam multiplicity)."""
    if train_all:
        raise NotImplementedError("collect_params(train_all=True): full-model adaptation is outside the engine's "
                                  "scope (DESIGN.md section 7)")
    if not train_LN:
        raise NotImplementedError("collect_params(train_LN=False): the engine always adapts the LayerNorm tensors "
                                  "(every script passes train_LN=True, main.py:265)")
    printed, names = _collect_names(model.config, bias_only=bias_only, train_feature=train_feature)
    for nm in printed:
        print(nm)
    params = _ParamList(_Param(model, n) for n in names)
    params.model, params.bias_only, params.train_feature = model, bool(bias_only), bool(train_feature)
    return params, names


class SutaOptimizer:
    """setup_optimizer's optimizer: AdamW / Adam (identical at the reference's weight decay 0) or SGD over the
    collected tensors.  The update itself runs inside forward_and_adapt (main.py:206), on the device."""

    def __init__(self, params: _ParamList, name: str, lr: float, betas, weight_decay: float):
        self.params, self.name = params, name
        self.base_lr, self.betas, self.weight_decay = float(lr), tuple(betas), float(weight_decay)
        self.param_groups = [{"params": list(params), "lr": float(lr), "betas": tuple(betas),
                              "weight_decay": float(weight_decay), "initial_lr": float(lr)}]
        self.scheduler: Optional[SutaStepLR] = None
        self.unscheduled_steps = 0

    def zero_grad(self, set_to_none: bool = True):
        pass

    def step(self, closure=None):
        raise RuntimeError("the SUTA update runs inside forward_and_adapt (suta_step_ex); there is no separate "
                           "gradient to apply")

    def state_dict(self):
        return {"name": self.name, "param_groups": [dict(g, params=[p.name for p in g["params"]])
                                                    for g in self.param_groups]}


class SutaStepLR:
    """torch.optim.lr_scheduler.StepLR(optimizer, step_size, gamma) (main.py:20-21): stepped by forward_and_adapt
    after each optimizer step (main.py:207-208); the engine applies the same chained lr * gamma products."""

    def __init__(self, optimizer: SutaOptimizer, step_size: int = 1, gamma: float = 0.7):
        if int(step_size) < 1:
            raise ValueError("StepLR step_size must be >= 1")
        self.optimizer, self.step_size, self.gamma = optimizer, int(step_size), float(gamma)
        self.last_epoch = 0
        optimizer.scheduler = self

    def get_last_lr(self) -> List[float]:
        return [self.optimizer.param_groups[0]["lr"]]

    def step(self):
        """Advance the host mirror of the lr (the device lr table is indexed by the engine's step count)."""
        self.last_epoch += 1
        g = self.optimizer.param_groups[0]
        if self.last_epoch % self.step_size == 0:
            g["lr"] = g["lr"] * self.gamma

    def state_dict(self):
        return {"step_size": self.step_size, "gamma": self.gamma, "last_epoch": self.last_epoch}


def setup_optimizer(params, opt_name="AdamW", lr=1e-4, beta=0.9, weight_decay=0., scheduler=None, step_size=1,
                    gamma=0.7):
    """main.py:8-23.  `scheduler` is the reference's string (eval'd there, resolved without eval here: it must
    name torch.optim.lr_scheduler.StepLR, the one scheduler that call constructs)."""
    import torch
    if not isinstance(params, _ParamList):
        raise TypeError("setup_optimizer expects the params returned by suta_amd.suta.collect_params")
    if opt_name not in OPTIMIZERS:
        raise NotImplementedError(f"optimizer {opt_name!r}: the engine implements {sorted(OPTIMIZERS)}")
    print(f"[INFO]    optimizer: {getattr(torch.optim, opt_name)}")
    print(f"[INFO]    scheduler: {scheduler}")
    betas = (beta, 0.999) if opt_name == "Adam" else (0.9, 0.999)   # AdamW / SGD: torch defaults
    SutaHParams(optimizer=opt_name, weight_decay=weight_decay).to_c()   # refuses what the engine cannot do
    opt = SutaOptimizer(params, opt_name, lr, betas, weight_decay)
    if scheduler is None:
        return opt, None
    from .main import resolve_scheduler
    try:
        resolve_scheduler(scheduler)
    except SystemExit as e:
        raise NotImplementedError(str(e)) from None
    return opt, SutaStepLR(opt, step_size=step_size, gamma=gamma)


class _Snapshot:
    """What copy_model_and_optimizer returns: the engine's pristine state (its generation number)."""

    def __init__(self, model: Wav2Vec2ForCTC, what: str):
        self.generation, self.what = model._generation, what


def copy_model_and_optimizer(model: Wav2Vec2ForCTC, optimizer: SutaOptimizer, scheduler=None):
    """main.py:137-145.  The engine keeps one pristine copy of the trainable tensors (P0) and treats the moments
    as zero at step 0, so the snapshot is a token for that state; it can be taken while the model is pristine
    (before any forward_and_adapt since setup or the last restore), which is where the reference takes it."""
    if model._steps != 0:
        raise NotImplementedError("copy_model_and_optimizer after adaptation: the engine restores the pristine "
                                  "state only (the reference snapshots right after setup_optimizer, main.py:310-311)")
    ms, os_ = _Snapshot(model, "model"), _Snapshot(model, "optimizer")
    return (ms, os_, _Snapshot(model, "scheduler")) if scheduler is not None else (ms, os_, None)


def load_model_and_optimizer(model: Wav2Vec2ForCTC, optimizer: SutaOptimizer, model_state, optimizer_state,
                             scheduler_state):
    """main.py:147-155: restores the trainable tensors, the optimizer moments and step counts, and the scheduler
    (suta_reset).  Returns (model, optimizer, scheduler) -- the scheduler the optimizer was set up with."""
    if not isinstance(model_state, _Snapshot) or not isinstance(optimizer_state, _Snapshot):
        raise TypeError("load_model_and_optimizer expects the states copy_model_and_optimizer returned")
    model._reset()
    optimizer.param_groups[0]["lr"] = optimizer.base_lr
    optimizer.unscheduled_steps = 0
    sch = optimizer.scheduler
    if sch is not None:
        sch.last_epoch = 0
    return model, optimizer, sch


def forward_and_adapt(x, model, optimizer, em_coef=0.9, reweight=False, temp=1., not_blank=True, scheduler=None,
                      div_coef=0, repeat_inference=True, skip_short_thd=None):
    """main.py:172-215: one SUTA step on utterance x (1, n_samples) -- grad forward, loss
    em_coef * masked entropy (+ (1 - em_coef) * MCC) (+ div_coef * div), backward, optimizer step, scheduler step,
    then the no-grad re-forward whose logits are returned (`repeat_inference=False`: the grad forward's logits).
    `skip_short_thd` is accepted and unused, as in the reference."""
    if not isinstance(optimizer, SutaOptimizer) or optimizer.params.model is not model:
        raise TypeError("forward_and_adapt expects the optimizer setup_optimizer built on this model's params")
    _check_batch1(x)
    if scheduler is not None and scheduler is not optimizer.scheduler:
        raise ValueError("scheduler was not built by setup_optimizer for this optimizer")
    if scheduler is not None and optimizer.unscheduled_steps:
        raise NotImplementedError("a scheduler passed after steps taken without it in the same episode")
    g = optimizer.param_groups[0]
    hp = SutaHParams(lr=optimizer.base_lr if scheduler is not None else g["lr"], temp=float(temp),
                     em_coef=float(em_coef), div_coef=float(div_coef), reweight=bool(reweight),
                     non_blank=bool(not_blank), train_feature=optimizer.params.train_feature,
                     bias_only=optimizer.params.bias_only, episodic=False, betas=optimizer.betas,
                     weight_decay=optimizer.weight_decay, optimizer=optimizer.name,
                     lr_step_size=scheduler.step_size if scheduler is not None else 0,
                     lr_gamma=scheduler.gamma if scheduler is not None else 0.7)
    dev_ptr, out_t = None, None
    if getattr(x, "is_cuda", False):
        import torch
        if x.device.index not in (None, model.device):
            raise ValueError(f"input on {x.device}, engine on cuda:{model.device}")
        T = model.engine.num_frames(int(x.shape[-1]))
        out_t = torch.empty((1, T, model.engine.V), dtype=torch.float32, device=x.device)
        dev_ptr = out_t.data_ptr()
    out, loss = model.engine.step_ex(x, hp, repeat_inference=repeat_inference, logits_device_ptr=dev_ptr)
    model._steps += 1
    model.last_loss = float(loss[0])
    if scheduler is not None:
        scheduler.step()
    else:
        optimizer.unscheduled_steps += 1
    return out_t if out_t is not None else _as_like(out, x)


def _check_batch1(x):
    shape = tuple(x.shape)
    if len(shape) == 2 and shape[0] != 1:
        raise ValueError(f"input of shape {shape}: one utterance per call (the reference's mcc_loss squeezes the "
                         "batch dimension, main.py:32); adapt many utterances with SutaEngine.adapt_varlen")
    if len(shape) not in (1, 2):
        raise ValueError(f"input of shape {shape}: expected (1, n_samples)")


def _as_like(a: np.ndarray, x):
    """numpy result -> torch tensor on x's device (numpy in, numpy out)."""
    if isinstance(x, np.ndarray):
        return a
    import torch
    t = torch.from_numpy(a)
    return t.to(x.device) if getattr(x, "is_cuda", False) else t
