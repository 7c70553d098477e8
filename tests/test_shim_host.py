"""CPU tier: the host logic of the forward_and_adapt shim (suta_amd/suta.py) with a stand-in engine.

The stand-in records the suta_hparams each forward_and_adapt hands to suta_step_ex; the checks are that the
reference's positional arguments land in the right fields (main.py:172-173, 348), that the optimizer / scheduler
handles follow setup_optimizer (main.py:8-23) -- including the per-step lr the reference's driver loop observed
(g9 `lrs`, produced by the reference itself) -- and that what the engine cannot do raises.  The GPU parity of the
same loop is tests/test_gpu_shim.py.
"""
import contextlib
import io
import os

import numpy as np
import pytest
import torch

from suta_amd import suta as S
from suta_amd.config import get_config

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class FakeEngine:
    V = 32

    def __init__(self, cfg, weights, device=0, max_batch=1, max_samples=600000):
        self.calls, self.resets = [], 0

    def num_frames(self, n):
        return (n - 400) // 320 + 1

    def forward(self, x, normalize=False):
        return np.zeros((1, self.num_frames(x.shape[-1]), 32), np.float32)

    def step_ex(self, x, hp, repeat_inference=True, normalize=False, logits_device_ptr=None):
        self.calls.append((hp, repeat_inference))
        return np.full((1, self.num_frames(x.shape[-1]), 32), len(self.calls), np.float32), np.zeros(1, np.float32)

    def reset(self):
        self.resets += 1

    def trainable_names(self):
        return []

    def close(self):
        pass


@pytest.fixture
def fake(monkeypatch):
    monkeypatch.setattr(S, "SutaEngine", FakeEngine)


def _setup(opt_name="AdamW", lr=5e-4, sched=None, preset="tiny-group", **kw):
    cfg = get_config(preset)
    model = S.configure_model(S.Wav2Vec2ForCTC(cfg, {}).eval().cuda())
    with contextlib.redirect_stdout(io.StringIO()) as out:
        params, names = S.collect_params(model, kw.get("bias_only", False), kw.get("train_feature", True), False,
                                         True)
        opt, sch = S.setup_optimizer(params, opt_name, lr, scheduler=sched)
    return model, params, names, opt, sch, out.getvalue()


def test_positional_arguments_reach_the_engine(fake):
    model, params, names, opt, sch, log = _setup(bias_only=True, train_feature=False)
    assert log.splitlines()[0] == ""                       # collect_params prints the root module name first
    assert "[INFO]    optimizer: <class 'torch.optim.adamw.AdamW'>" in log
    x = torch.zeros(1, 8000)
    out = S.forward_and_adapt(x, model, opt, 0.4, True, 2.0, False, sch, 0.1)     # main.py:348 order
    hp, rep = model.engine.calls[-1]
    assert (hp.em_coef, hp.reweight, hp.temp, hp.non_blank, hp.div_coef) == (0.4, True, 2.0, False, 0.1)
    assert (hp.lr, hp.optimizer, hp.lr_step_size, hp.bias_only, hp.train_feature, hp.episodic) == \
        (5e-4, "AdamW", 0, True, False, False)
    assert rep is True and tuple(out.shape) == (1, 24, 32) and isinstance(out, torch.Tensor)
    S.forward_and_adapt(x, model, opt, 0.4, True, 2.0, False, sch, 0.1, False)
    assert model.engine.calls[-1][1] is False                # repeat_inference
    # defaults of the reference signature: em_coef 0.9, reweight False, temp 1, not_blank True, div 0
    S.forward_and_adapt(x, model, opt)
    hp, _ = model.engine.calls[-1]
    assert (hp.em_coef, hp.reweight, hp.temp, hp.non_blank, hp.div_coef) == (0.9, False, 1.0, True, 0.0)


@pytest.mark.parametrize("variant", ["steplr_group", "sgd_steplr_layer", "steplr_group_nonepisodic", "sgd_group"])
def test_scheduler_lr_sequence_matches_reference_loop(fake, variant):
    """The lr the reference loop read before each step (g9 `lrs`, main.py:20-21 / 207-208) equals the shim's host
    mirror; the engine gets the base lr and the StepLR constants, restored by load_model_and_optimizer."""
    z = np.load(os.path.join(G, f"g9_sched_{variant}.npz"), allow_pickle=False)
    sched = None if str(z["scheduler"]) == "None" else str(z["scheduler"])
    model, params, names, opt, sch, _ = _setup(str(z["opt"]), float(z["lr"]), sched,
                                               "tiny-layer" if "layer" in variant else "tiny-group")
    assert list(names) == [str(n) for n in z["entries"]]     # collect_params multiplicities (reference output)
    episodic = bool(z["episodic"])
    states = S.copy_model_and_optimizer(model, opt, sch) if episodic else None
    for n in (8000, 12345):
        if episodic:
            model, opt, sch = S.load_model_and_optimizer(model, opt, *states)
        lrs = []
        for i in range(int(z["steps"])):
            lrs.append(opt.param_groups[0]["lr"])
            S.forward_and_adapt(torch.zeros(1, 8000), model, opt, 0.3, True, 2.5, True, sch, 0.0)
            hp = model.engine.calls[-1][0]
            assert hp.lr == float(z["lr"]) and hp.lr_step_size == (1 if sched else 0) and hp.lr_gamma == 0.7
            assert hp.optimizer == str(z["opt"])
        assert np.array_equal(np.array(lrs, np.float64), z[f"N{n}/lrs"])
    assert model.engine.resets == (2 if episodic else 0)


def test_refusals(fake):
    cfg = get_config("tiny-group")
    model = S.Wav2Vec2ForCTC(cfg, {})
    with contextlib.redirect_stdout(io.StringIO()):
        with pytest.raises(NotImplementedError):
            S.collect_params(model, False, True, True, True)          # train_all
        with pytest.raises(NotImplementedError):
            S.collect_params(model, False, True, False, False)        # train_LN=False
        params, _ = S.collect_params(model, False, True)
        with pytest.raises(NotImplementedError):
            S.setup_optimizer(params, "RMSprop", 1e-4)
        with pytest.raises(NotImplementedError):
            S.setup_optimizer(params, "AdamW", 1e-4, scheduler="torch.optim.lr_scheduler.ExponentialLR")
        with pytest.raises(ValueError):
            S.setup_optimizer(params, "SGD", 1e-4, weight_decay=0.1)  # torch would add wd * p; the engine does not
        with pytest.raises(TypeError):
            S.setup_optimizer([], "AdamW", 1e-4)
        opt, sch = S.setup_optimizer(params, "AdamW", 1e-4)
    with pytest.raises(ValueError):
        S.forward_and_adapt(torch.zeros(2, 8000), model, opt)          # one utterance per call (main.py:32)
    states = S.copy_model_and_optimizer(model, opt, sch)
    S.forward_and_adapt(torch.zeros(1, 8000), model, opt)
    with pytest.raises(NotImplementedError):
        S.copy_model_and_optimizer(model, opt, sch)                    # only the pristine state is restorable
    S.load_model_and_optimizer(model, opt, *states)
    assert model._steps == 0 and model.engine.resets == 1
    with pytest.raises(RuntimeError):
        opt.step()                                                     # the update is inside forward_and_adapt
