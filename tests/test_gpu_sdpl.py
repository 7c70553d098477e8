"""GPU tier: the SDPL objective (reference main_SDPL.py:143-209) in libsuta.

Fixtures g6_* come from the reference's own main_SDPL.forward_and_adapt (tests/golden/make_golden.py).
Tolerances: loss-and-grad kernel within 4x the reference's own fp32-vs-fp64 deviation (at least
5e-6 * max|g|); adapted logits within tests/parity.sdpl_logits_tol (the pseudo-label gradient of
every class outside the label is pure rounding noise that Adam amplifies, see there), greedy ids
agreeing on >= 90 % of frames, adapted tensors within the Adam step budget.
"""
import os

import numpy as np
import pytest

from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights
from tests.parity import assert_params_close, same_pseudo_labels, sdpl_logits_tol

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_ENG = {}


def sdpl_weights(cfg):
    sd = synth_weights(cfg, blank_bias=0.0)
    sd["lm_head.bias"][1:4] -= 30.0  # as the fixtures: keep <s>, </s>, <unk> off the greedy path
    return sd


def engine(preset, max_batch=2):
    key = (preset, max_batch)
    if key not in _ENG:
        cfg = get_config(preset)
        _ENG[key] = (SutaEngine(cfg, sdpl_weights(cfg), max_batch=max_batch), cfg)
    return _ENG[key]


def test_sdpl_loss_kernel_matches_reference():
    eng, _ = engine("tiny-group")
    z = np.load(os.path.join(G, "g6_sdpl_loss.npz"), allow_pickle=False)
    for case in z["cases"]:
        L = z[f"{case}/logits"]
        temp, em, rw, nb, pl = z[f"{case}/hp"]
        hp = SutaHParams(temp=float(temp), em_coef=float(em), reweight=bool(rw), non_blank=bool(nb), pl_coef=float(pl))
        d, loss = eng.loss_grad(L, hp)
        ref = z[f"{case}/grad_f64"]
        own = np.abs(z[f"{case}/grad_f32"] - ref).max()
        tol = max(4 * own, 5e-6 * np.abs(ref).max())  # fp32 noise on the (exactly 0) non-label classes
        np.testing.assert_allclose(d[0], ref, rtol=0, atol=tol, err_msg=str(case))
        rl = float(z[f"{case}/loss_f64"])
        if np.isnan(rl):
            assert np.isnan(loss[0]), case
        else:
            assert abs(loss[0] - rl) <= 2e-5 * max(1.0, abs(rl)), (case, loss[0], rl)


@pytest.mark.parametrize("variant", ["group", "layer"])
def test_sdpl_tiny_adaptation_tracks_reference(variant):
    z = np.load(os.path.join(G, f"g6_sdpl_tiny_{variant}.npz"), allow_pickle=False)
    eng, cfg = engine(f"tiny-{variant}")
    lr = float(z["lr"])
    hp = SutaHParams(lr=lr, em_coef=1.0, reweight=False, non_blank=True, pl_coef=1.0)
    compared = 0
    for n in (8000, 12345):
        logits, ids, T = eng.adapt(z[f"N{n}/x"], 5, hp, record=list(range(6)))
        ours = [logits[i][0] for i in range(6)]
        ref = z[f"N{n}/logits"]
        for i in range(6):
            if not same_pseudo_labels(ours, ref, i):
                break  # a greedy flip changed the CTC target: the runs adapt toward different labels
            np.testing.assert_allclose(ours[i], ref[i], rtol=0, atol=sdpl_logits_tol(lr, i),
                                       err_msg=f"{variant} N{n} step {i}")
            assert np.mean(ids[i][0] == ref[i].argmax(-1)) >= 0.9, (variant, n, i)
            compared += 1
        if same_pseudo_labels(ours, ref, 5):
            for key in z.files:
                if key.startswith(f"N{n}/final/"):
                    name = key[len(f"N{n}/final/"):]
                    assert_params_close(eng.get_param(0, name), z[key], lr, 5, max_frac=1.0, name=name, factor=2.0)
    assert compared >= 8  # most of the 12 recorded steps share the reference's pseudo labels


def test_sdpl_ragged_batch_equals_single_runs():
    eng, cfg = engine("tiny-group", max_batch=3)
    hp = SutaHParams(lr=1e-4, em_coef=1.0, reweight=False, pl_coef=1.0)
    waves = [synth.wave(n, 80 + i) for i, n in enumerate((9000, 12001, 8000))]
    lv, iv, tv = eng.adapt_varlen(waves, 3, hp, record=[0, 3])
    for b, w in enumerate(waves):
        l1, _, t1 = eng.adapt(w, 3, hp, record=[0, 3])
        assert tv[b] == t1
        np.testing.assert_allclose(lv[3][b], l1[3][0], rtol=0, atol=sdpl_logits_tol(1e-4, 3))


def test_sdpl_special_token_in_pseudo_label_raises():
    cfg = get_config("tiny-group")
    sd = synth_weights(cfg, blank_bias=0.0)
    sd["lm_head.bias"][3] += 50.0  # every frame decodes to <unk>
    eng = SutaEngine(cfg, sd, max_batch=1)
    with pytest.raises(RuntimeError, match="special token"):
        eng.adapt(synth.wave(8000, 1), 1, SutaHParams(pl_coef=1.0), record=[1])
    eng.close()
