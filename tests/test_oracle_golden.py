"""Pin the CPU oracle (oracle/) against golden vectors made by the reference's own code.

Fixtures: tests/golden/make_golden.py (reference main.py imported with a jiwer stub).
"""
import ast
import os

import numpy as np
import pytest
import torch

from oracle import w2v2_cpu as W
from oracle.suta_loss_np import suta_loss_and_grad
from suta_amd.config import get_config
from suta_amd.weights import synth_weights
from tests.parity import (assert_params_close, assert_sgd_params_close, logits_tol, same_pseudo_labels,
                          sdpl_logits_tol)

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_g1_closed_form_loss_grad_matches_reference():
    z = _load("g1_loss_grad.npz")
    for case in z["cases"]:
        L = z[f"{case}/logits"]
        temp, em, rw, nb, div = z[f"{case}/hp"]
        loss, g = suta_loss_and_grad(L, temp, em, bool(rw), bool(nb), div)
        ref_g = z[f"{case}/grad_f64"]
        ref_loss = float(z[f"{case}/loss_f64"])
        np.testing.assert_allclose(g, ref_g, rtol=1e-9, atol=1e-14, err_msg=case)
        if np.isnan(ref_loss):
            assert np.isnan(loss), case
        else:
            assert abs(loss - ref_loss) <= 1e-10 * max(1, abs(ref_loss)), case
        # the fp32 reference grad is within fp32 rounding of the exact one
        np.testing.assert_allclose(z[f"{case}/grad_f32"], ref_g, rtol=0, atol=max(2e-6 * np.abs(ref_g).max(), 1e-8), err_msg=case)


def test_g1_allblank_is_nan_loss_finite_grad():
    z = _load("g1_loss_grad.npz")
    assert np.isnan(float(z["allblank_T49/loss_f32"]))
    assert np.isfinite(z["allblank_T49/grad_f32"]).all()


def test_g1_torch_restatement_matches_reference():
    z = _load("g1_loss_grad.npz")
    for case in z["cases"]:
        L = torch.tensor(z[f"{case}/logits"][None], dtype=torch.float64, requires_grad=True)
        temp, em, rw, nb, div = z[f"{case}/hp"]
        loss = W.suta_loss(L, em, bool(rw), temp, bool(nb), div)
        loss.backward()
        np.testing.assert_allclose(L.grad[0].numpy(), z[f"{case}/grad_f64"], rtol=1e-12, atol=1e-15, err_msg=case)


def test_g2_adam_multiplicity():
    z = _load("g2_adam_mult.npz")
    for k in range(1, 6):
        p = {"w": torch.from_numpy(z["p0"].copy())}
        st = W.AdamState(["w"], p)
        for s in range(3):
            W.adam_step(p, {"w": torch.from_numpy(z["grads"][s].copy())}, st, ["w"] * k, lr=1e-3)
            np.testing.assert_array_equal(p["w"].numpy(), z[f"k{k}"][s], err_msg=f"k={k} step={s}")


def test_collect_params_multiplicity_base():
    """96 entries / 63 unique / 4 633 856 elements for base + --train_feature."""
    cfg = get_config("wav2vec2-base")
    e = W.trainable_entries(cfg, train_feature=True)
    shapes = dict(__import__("suta_amd.config", fromlist=["param_shapes"]).param_shapes(cfg))
    assert len(e) == 96
    u = list(dict.fromkeys(e))
    assert len(u) == 63
    assert sum(int(np.prod(shapes[n])) for n in u) == 4633856
    m = W.multiplicity(e)
    assert m["wav2vec2.feature_extractor.conv_layers.3.conv.weight"] == 4
    assert m["wav2vec2.feature_extractor.conv_layers.0.layer_norm.bias"] == 4
    assert m["wav2vec2.feature_projection.layer_norm.weight"] == 3
    assert m["wav2vec2.feature_projection.projection.weight"] == 2
    assert m["wav2vec2.encoder.layers.5.final_layer_norm.bias"] == 1


@pytest.mark.parametrize("variant", ["group", "group_lr5e-4", "layer", "layer_lr5e-4", "group_lnonly",
                                     "group_biasonly", "group_em1"])
def test_g3_tiny_suta_oracle_matches_reference(variant):
    z = _load(f"g3_tiny_{variant}.npz")
    preset = "tiny-group" if variant.startswith("group") else "tiny-layer"
    cfg = get_config(preset)
    sd = synth_weights(cfg)
    from tests.golden.make_golden import weights_digest  # noqa
    assert weights_digest(sd) == str(z["weights_sha256"]), "seeded weight generator drifted"
    hp = ast.literal_eval(str(z["hp_json"]))
    entries = W.trainable_entries(cfg, bias_only=hp["bias_only"], train_feature=hp["train_feature"])
    assert entries == [str(s) for s in z["entries"]]
    params = {k: torch.from_numpy(v) for k, v in sd.items()}
    for n in (8000, 12345):
        x = torch.from_numpy(z[f"N{n}/x"])[None]
        out, final = W.run_suta(params, cfg, x, 10, lr=hp["lr"], temp=hp["temp"], em_coef=hp["em"],
                                reweight=hp["rw"], non_blank=hp["nb"], div_coef=hp["div"],
                                train_feature=hp["train_feature"], bias_only=hp["bias_only"])
        ref = z[f"N{n}/logits"]
        for i in range(11):
            np.testing.assert_allclose(out[i][0].numpy(), ref[i], rtol=0, atol=logits_tol(hp["lr"]), err_msg=f"{variant} N{n} step {i}")
        for k, v in final.items():
            assert_params_close(v.numpy(), z[f"N{n}/final/{k}"], hp["lr"], 10, name=k)


@pytest.mark.slow
@pytest.mark.parametrize("n", [16000])
def test_g4_base_oracle_matches_reference(n):
    path = os.path.join(G, f"g4_base_{n}.npz")
    if not os.path.exists(path):
        pytest.skip("g4 fixture missing")
    z = _load(f"g4_base_{n}.npz")
    cfg = get_config("wav2vec2-base")
    sd = synth_weights(cfg)
    params = {k: torch.from_numpy(v) for k, v in sd.items()}
    from tests.golden.make_golden import wave
    x = torch.from_numpy(wave(n, 0 if n == 16000 else 1))[None]
    steps = [int(s) for s in z["steps"]]
    out, final = W.run_suta(params, cfg, x, 10, record=steps)
    for j, s in enumerate(steps):
        np.testing.assert_allclose(out[s][0].numpy(), z["logits"][j], rtol=0, atol=5e-5, err_msg=f"step {s}")
    for k, v in final.items():
        idx = z[f"final/{k}/idx"]
        assert_params_close(v.numpy().reshape(-1)[idx], z[f"final/{k}/val"], 2e-5, 10, max_frac=0.05, name=k)


@pytest.mark.slow
def test_g7_large_oracle_matches_reference():
    """large-960h-lv60 geometry (layer-norm conv stack, conv bias, stable LN), 20 SUTA steps."""
    z = _load("g7_large_16000.npz")
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    params = {k: torch.from_numpy(v) for k, v in sd.items()}
    from tests.golden.make_golden import wave
    x = torch.from_numpy(wave(16000, 7))[None]
    steps = [int(s) for s in z["steps"]]
    out, final = W.run_suta(params, cfg, x, 20, record=steps)
    for j, s in enumerate(steps):
        np.testing.assert_allclose(out[s][0].numpy(), z["logits"][j], rtol=0, atol=5e-5, err_msg=f"step {s}")
    for k, v in final.items():
        idx = z[f"final/{k}/idx"]
        assert_params_close(v.numpy().reshape(-1)[idx], z[f"final/{k}/val"], 2e-5, 20, max_frac=0.05, name=k)


# ---------------------------------------------------------------------------------------------
# SDPL (reference main_SDPL.py:143-209): g6 fixtures
# ---------------------------------------------------------------------------------------------
def test_g6_sdpl_target_matches_reference_transcript():
    from suta_amd.decode import VOCAB
    z = _load("g6_sdpl_loss.npz")
    for case in z["cases"]:
        ids = z[f"{case}/logits"].argmax(-1)
        tgt = W.pseudo_label_target(ids)
        text = str(z[f"{case}/transcript"])
        assert "".join(" " if VOCAB[i] == "|" else VOCAB[i] for i in tgt) == text, case


def test_g6_sdpl_torch_restatement_matches_reference():
    z = _load("g6_sdpl_loss.npz")
    for case in z["cases"]:
        temp, em, rw, nb, pl = z[f"{case}/hp"]
        L = torch.tensor(z[f"{case}/logits"][None], dtype=torch.float64, requires_grad=True)
        loss = W.sdpl_loss(L, em, bool(rw), temp, bool(nb), pl)
        loss.backward()
        ref = z[f"{case}/grad_f64"]
        np.testing.assert_allclose(L.grad[0].numpy(), ref, rtol=1e-9, atol=1e-12, err_msg=case)
        rl = float(z[f"{case}/loss_f64"])
        assert (np.isnan(rl) and np.isnan(loss.item())) or abs(loss.item() - rl) <= 1e-9 * max(1, abs(rl)), case


@pytest.mark.parametrize("variant", ["group", "layer"])
def test_g6_sdpl_tiny_oracle_matches_reference(variant):
    z = _load(f"g6_sdpl_tiny_{variant}.npz")
    cfg = get_config(f"tiny-{variant}")
    sd = synth_weights(cfg, blank_bias=0.0)
    sd["lm_head.bias"][1:4] -= 30.0
    params = {k: torch.from_numpy(v) for k, v in sd.items()}
    lr = float(z["lr"])
    x = torch.from_numpy(z["N8000/x"])[None]
    out, final = W.run_suta(params, cfg, x, 5, lr=lr, em_coef=1.0, reweight=False, non_blank=True, pl_coef=1.0)
    for i in range(6):
        np.testing.assert_allclose(out[i][0].numpy(), z["N8000/logits"][i], rtol=0, atol=sdpl_logits_tol(lr, i),
                                   err_msg=f"step {i}")
        assert np.mean(out[i][0].numpy().argmax(-1) == z["N8000/logits"][i].argmax(-1)) >= 0.9
    for key in z.files:
        if key.startswith("N8000/final/"):
            name = key[len("N8000/final/"):]
            assert_params_close(final[name].numpy(), z[key], lr, 5, max_frac=1.0, name=name, factor=2.0)


# ---------------------------------------------------------------------------------------------
# --scheduler StepLR / --opt SGD (reference main.py:8-23, 147-155, 207-208): g9 fixtures
# ---------------------------------------------------------------------------------------------
G9_VARIANTS = ["steplr_group", "steplr_layer", "sgd_group", "sgd_steplr_layer", "steplr_group_nonepisodic"]


def g9_hparams(z):
    """(opt, lr, lr_step_size, episodic, steps) of a g9 fixture: the reference's setup_optimizer passes
    step_size 1 and gamma 0.7 to the scheduler (main.py:8, 21)."""
    return (str(z["opt"]), float(z["lr"]), 1 if str(z["scheduler"]) != "None" else 0, bool(z["episodic"]),
            int(z["steps"]))


def test_step_lr_matches_reference_lr_sequence():
    z = _load("g9_sched_steplr_group_nonepisodic.npz")
    lrs = np.concatenate([z["N8000/lrs"], z["N12345/lrs"]])   # one scheduler across both utterances
    got = [W.step_lr(float(z["lr"]), 0.7, 1, i) for i in range(len(lrs))]
    assert np.array_equal(np.array(got, np.float64), lrs)
    z = _load("g9_sched_steplr_group.npz")                   # episodic: restored per utterance
    assert np.array_equal(z["N8000/lrs"], z["N12345/lrs"])


@pytest.mark.parametrize("variant", G9_VARIANTS)
def test_g9_scheduler_sgd_oracle_matches_reference(variant):
    z = _load(f"g9_sched_{variant}.npz")
    cfg = get_config("tiny-layer" if "layer" in variant else "tiny-group")
    sd = synth_weights(cfg)
    from tests.golden.make_golden import weights_digest  # noqa
    assert weights_digest(sd) == str(z["weights_sha256"]), "seeded weight generator drifted"
    assert W.trainable_entries(cfg, train_feature=True) == [str(s) for s in z["entries"]]
    opt, lr, ss, episodic, steps = g9_hparams(z)
    params = {k: torch.from_numpy(v) for k, v in sd.items()}
    carry = None if episodic else W.OptCarry()
    prev = {k: v.copy() for k, v in sd.items()}
    for n in (8000, 12345):
        x = torch.from_numpy(z[f"N{n}/x"])[None]
        out, final = W.run_suta(params, cfg, x, steps, lr=lr, opt=opt, lr_step_size=ss, carry=carry)
        for i in range(steps + 1):
            np.testing.assert_allclose(out[i][0].numpy(), z[f"N{n}/logits"][i], rtol=0, atol=logits_tol(5e-4),
                                       err_msg=f"{variant} N{n} step {i}")
        for k, v in final.items():
            ref = z[f"N{n}/final/{k}"]
            if opt == "SGD":
                assert_sgd_params_close(v.numpy(), ref, prev[k], name=k)
            else:
                assert_params_close(v.numpy(), ref, lr, steps * (1 if episodic else 2), name=k)
        if not episodic:
            prev = {k: z[f"N{n}/final/{k}"] for k in final}
