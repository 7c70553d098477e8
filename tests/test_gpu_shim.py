"""GPU tier: the `forward_and_adapt`-compatible shim (suta_amd/suta.py) replaying the reference driver loop.

Each test runs the reference's own loop body (`/root/reference/main.py:305-348`: configure_model, collect_params,
setup_optimizer, copy_model_and_optimizer, load_model_and_optimizer, the no-grad vanilla forward and
`forward_and_adapt(input_values, model, optimizer, em_coef, reweight, temp, non_blank, scheduler, div_coef)` called
positionally) with the shim's objects, against the goldens that loop produced on transformers' model
(tests/golden/make_golden.py g3 / g9).  Every call goes through libsuta's C ABI (suta_forward, suta_step_ex,
suta_reset).  Tolerances: logits within tests/parity.logits_tol(lr) = 2e-5 + 0.2 lr, adapted tensors by
tests/parity.assert_params_close (Adam budget) / assert_sgd_params_close.
"""
import ast
import contextlib
import io
import os

import numpy as np
import pytest
import torch

from suta_amd import suta as S
from suta_amd.config import get_config
from suta_amd.weights import synth_weights
from tests.parity import assert_params_close, assert_sgd_params_close, logits_tol

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _setup(preset, opt_name, lr, sched, bias_only=False, train_feature=True, device_input=False):
    """main.py:303-311 with the shim's objects."""
    cfg = get_config(preset)
    model = S.Wav2Vec2ForCTC(cfg, synth_weights(cfg)).eval().cuda()
    model = S.configure_model(model)
    with contextlib.redirect_stdout(io.StringIO()) as out:
        params, names = S.collect_params(model, bias_only, train_feature, False, True)
        opt, sch = S.setup_optimizer(params, opt_name, lr, scheduler=sched)
    assert "[INFO]    optimizer:" in out.getvalue()
    return model, params, names, opt, sch


@pytest.mark.parametrize("variant", ["steplr_group", "steplr_layer", "sgd_group", "sgd_steplr_layer",
                                     "steplr_group_nonepisodic"])
def test_reference_loop_through_shim_matches_g9(variant):
    """g9: the reference loop with StepLR and / or SGD, episodic and not (state, moments and the scheduler's
    step count carried into the second utterance)."""
    z = _load(f"g9_sched_{variant}.npz")
    preset = "tiny-layer" if "layer" in variant else "tiny-group"
    opt_name, lr, sched, episodic, steps = (str(z["opt"]), float(z["lr"]), str(z["scheduler"]), bool(z["episodic"]),
                                            int(z["steps"]))
    sched = None if sched == "None" else sched
    model, params, names, optimizer, scheduler = _setup(preset, opt_name, lr, sched)
    assert list(names) == [str(n) for n in z["entries"]]
    if episodic:                                                              # main.py:310-311
        model_state, optimizer_state, scheduler_state = S.copy_model_and_optimizer(model, optimizer, scheduler)
    prev = {k: v.copy() for k, v in synth_weights(get_config(preset)).items()}
    for n in (8000, 12345):
        x = torch.from_numpy(z[f"N{n}/x"])[None]
        if episodic:                                                          # main.py:327-328
            model, optimizer, scheduler = S.load_model_and_optimizer(model, optimizer, model_state, optimizer_state,
                                                                     scheduler_state)
        with torch.no_grad():
            outputs = model(x).logits                                         # main.py:331-332
        np.testing.assert_allclose(outputs[0].numpy(), z[f"N{n}/logits"][0], rtol=0, atol=logits_tol(lr))
        lrs = []
        for i in range(steps):                                                # main.py:347-348
            lrs.append(optimizer.param_groups[0]["lr"])
            outputs = S.forward_and_adapt(x, model, optimizer, 0.3, True, 2.5, True, scheduler, 0.0)
            np.testing.assert_allclose(outputs[0].numpy(), z[f"N{n}/logits"][i + 1], rtol=0, atol=logits_tol(5e-4),
                                       err_msg=f"{variant} N{n} step {i + 1}")
        assert np.array_equal(np.array(lrs, np.float64), z[f"N{n}/lrs"])    # the host lr mirror == torch's
        sd = model.state_dict()
        for key in z.files:
            if key.startswith(f"N{n}/final/"):
                name = key[len(f"N{n}/final/"):]
                got = sd[name].numpy()
                if opt_name == "SGD":
                    assert_sgd_params_close(got, z[key], prev[name], name=name)
                else:
                    assert_params_close(got, z[key], lr, steps * (1 if episodic else 2), name=name)
        if not episodic:
            prev = {k[len(f"N{n}/final/"):]: z[k] for k in z.files if k.startswith(f"N{n}/final/")}
    model.close()


@pytest.mark.parametrize("variant", ["group", "layer_lr5e-4", "group_biasonly", "group_lnonly", "group_em1"])
def test_reference_loop_through_shim_matches_g3(variant):
    """g3: 10 steps of the reference loop per variant (post-LN / stable-LN, LN-only, bias-only, em 1 + div),
    the input a cuda tensor as in the reference (`input_values.cuda()`): logits come back on the device."""
    z = _load(f"g3_tiny_{variant}.npz")
    h = ast.literal_eval(str(z["hp_json"]))
    preset = "tiny-group" if variant.startswith("group") else "tiny-layer"
    model, params, names, optimizer, scheduler = _setup(preset, "AdamW", h["lr"], None, bias_only=h["bias_only"],
                                                        train_feature=h["train_feature"])
    model_state, optimizer_state, scheduler_state = S.copy_model_and_optimizer(model, optimizer, scheduler)
    for n in (8000, 12345):
        x = torch.from_numpy(z[f"N{n}/x"])[None].cuda()
        model, optimizer, scheduler = S.load_model_and_optimizer(model, optimizer, model_state, optimizer_state,
                                                                 scheduler_state)
        ref = z[f"N{n}/logits"]
        with torch.no_grad():
            outputs = model(x).logits
        assert outputs.is_cuda
        np.testing.assert_allclose(outputs[0].cpu().numpy(), ref[0], rtol=0, atol=logits_tol(h["lr"]))
        for i in range(10):
            outputs = S.forward_and_adapt(x, model, optimizer, h["em"], h["rw"], h["temp"], h["nb"], scheduler,
                                          h["div"])
            assert outputs.is_cuda and outputs.shape == (1, ref.shape[1], ref.shape[2])
            np.testing.assert_allclose(outputs[0].cpu().numpy(), ref[i + 1], rtol=0, atol=logits_tol(h["lr"]),
                                       err_msg=f"{variant} N{n} step {i + 1}")
            assert np.isfinite(model.last_loss) or h["nb"]
        sd = model.state_dict()
        for key in z.files:
            if key.startswith(f"N{n}/final/"):
                name = key[len(f"N{n}/final/"):]
                assert_params_close(sd[name].numpy(), z[key], h["lr"], 10, name=name)
    model.close()


def test_repeat_inference_false_returns_grad_forward_logits():
    """forward_and_adapt(..., repeat_inference=False) (main.py:211-215) returns the logits the loss was taken on:
    step i's grad forward runs on the tensors step i - 1 left, so it equals step i - 1's re-inference bitwise
    (same kernels, same inputs), and step 0's equals the vanilla forward."""
    model, params, names, optimizer, scheduler = _setup("tiny-group", "AdamW", 5e-4, None)
    states = S.copy_model_and_optimizer(model, optimizer, scheduler)
    x = torch.from_numpy(_load("g3_tiny_group_lr5e-4.npz")["N8000/x"])[None]
    S.load_model_and_optimizer(model, optimizer, *states)
    vanilla = model(x).logits
    rep = [S.forward_and_adapt(x, model, optimizer, 0.3, True, 2.5, True, None, 0.0) for _ in range(3)]
    S.load_model_and_optimizer(model, optimizer, *states)
    grad_fw = [S.forward_and_adapt(x, model, optimizer, 0.3, True, 2.5, True, None, 0.0, False) for _ in range(4)]
    assert torch.equal(grad_fw[0], vanilla)
    for i in range(3):
        assert torch.equal(grad_fw[i + 1], rep[i]), i
    with pytest.raises(ValueError):
        S.forward_and_adapt(torch.zeros(2, 8000), model, optimizer, 0.3, True, 2.5, True, None, 0.0)
    with pytest.raises(NotImplementedError):   # the engine restores the pristine state only
        S.copy_model_and_optimizer(model, optimizer, scheduler)
    model.close()
