"""GPU tier: libsuta (HIP, gfx950) against the committed reference goldens and the CPU oracle.

Every call goes through the C ABI (include/suta.h) via the ctypes binding.
Tolerances (stated per test):
  * fused loss-and-grad vs reference autograd (float64 golden): |d| <= 2e-6 * max|g| + 1e-9
  * adapted logits vs reference: tests/parity.logits_tol(lr) = 2e-5 + 0.2*lr absolute
  * adapted tensors: tests/parity.assert_params_close (Adam sign-flip budget)
"""
import ast
import os

import numpy as np
import pytest
import torch

from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights
from tests.parity import assert_params_close, assert_sgd_params_close, logits_tol

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_ENGINES = {}


PRECISIONS = ["fp32", "fp32-split-bf16"]


def engine(preset, max_batch=4, blank_bias=1.0, precision="fp32"):
    key = (preset, max_batch, blank_bias)
    if key not in _ENGINES:
        cfg = get_config(preset)
        _ENGINES[key] = (SutaEngine(cfg, synth_weights(cfg, blank_bias=blank_bias), max_batch=max_batch), cfg)
    _ENGINES[key][0].set_precision(precision)
    return _ENGINES[key]


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_loss_kernel_matches_reference_autograd():
    eng, _ = engine("tiny-group")
    z = _load("g1_loss_grad.npz")
    for case in z["cases"]:
        L = z[f"{case}/logits"]
        temp, em, rw, nb, div = z[f"{case}/hp"]
        hp = SutaHParams(temp=float(temp), em_coef=float(em), reweight=bool(rw), non_blank=bool(nb), div_coef=float(div))
        d, loss = eng.loss_grad(L, hp)
        ref = z[f"{case}/grad_f64"]
        np.testing.assert_allclose(d[0], ref, rtol=0, atol=2e-6 * np.abs(ref).max() + 1e-9, err_msg=str(case))
        rl = float(z[f"{case}/loss_f64"])
        if np.isnan(rl):
            assert np.isnan(loss[0]), case
        else:
            assert abs(loss[0] - rl) <= 1e-5 * max(1.0, abs(rl)), (case, loss[0], rl)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("variant", ["group", "group_lr5e-4", "layer", "layer_lr5e-4", "group_lnonly",
                                     "group_biasonly", "group_em1"])
def test_tiny_suta_matches_reference(variant, precision):
    z = _load(f"g3_tiny_{variant}.npz")
    preset = "tiny-group" if variant.startswith("group") else "tiny-layer"
    eng, cfg = engine(preset, precision=precision)
    h = ast.literal_eval(str(z["hp_json"]))
    hp = SutaHParams(lr=h["lr"], temp=h["temp"], em_coef=h["em"], reweight=h["rw"], non_blank=h["nb"],
                     div_coef=h["div"], train_feature=h["train_feature"], bias_only=h["bias_only"])
    for n in (8000, 12345):
        x = z[f"N{n}/x"]
        logits, ids, T = eng.adapt(x, 10, hp, record=list(range(11)))
        ref = z[f"N{n}/logits"]
        for i in range(11):
            np.testing.assert_allclose(logits[i][0], ref[i], rtol=0, atol=logits_tol(h["lr"]),
                                       err_msg=f"{variant} N{n} step {i}")
            np.testing.assert_array_equal(ids[i][0], logits[i][0].argmax(-1))
        for key in z.files:
            if key.startswith(f"N{n}/final/"):
                name = key[len(f"N{n}/final/"):]
                assert_params_close(eng.get_param(0, name), z[key], h["lr"], 10, name=name)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("n", [16000, 32000])
def test_base_suta_matches_reference(n, precision):
    z = _load(f"g4_base_{n}.npz")
    eng, cfg = engine("wav2vec2-base", precision=precision)
    x = synth.wave(n, 0 if n == 16000 else 1)
    steps = [int(s) for s in z["steps"]]
    logits, ids, T = eng.adapt(x, 10, SutaHParams(), record=steps)
    for j, s in enumerate(steps):
        np.testing.assert_allclose(logits[s][0], z["logits"][j], rtol=0, atol=5e-5, err_msg=f"step {s}")
    for key in z.files:
        if key.startswith("final/") and key.endswith("/idx"):
            name = key[len("final/"):-len("/idx")]
            got = eng.get_param(0, name).reshape(-1)[z[key]]
            assert_params_close(got, z[f"final/{name}/val"], 2e-5, 10, max_frac=0.05, name=name)


@pytest.mark.parametrize("precision", PRECISIONS)
def test_base_forward_matches_oracle_8s(precision):
    """Vanilla logits at the bench length (8 s, T = 399) against the CPU oracle."""
    from oracle import w2v2_cpu as W
    eng, cfg = engine("wav2vec2-base", precision=precision)
    x = synth.wave(128000, 3)
    eng.reset()
    got = eng.forward(x)[0]
    sd = synth_weights(cfg)
    with torch.no_grad():
        ref = W.forward({k: torch.from_numpy(v) for k, v in sd.items()}, cfg, torch.from_numpy(x)[None])[0].numpy()
    np.testing.assert_allclose(got, ref, rtol=0, atol=5e-5)


@pytest.mark.parametrize("n", [400, 719, 720, 1041])
def test_shortest_inputs_match_oracle(n):
    """Edge lengths of the conv stack: N = 400 is the shortest input with a frame (T = 1; the receptive
    field), 719/720 straddle T = 1 -> 2, 1041 gives T = 3.  Two SUTA steps (scripts' lr) against the CPU
    oracle, with the base-size tolerance of test_base_suta_matches_reference."""
    from oracle import w2v2_cpu as W
    eng, cfg = engine("wav2vec2-base")
    sd = synth_weights(cfg)
    x = synth.wave(n, 11)
    logits, ids, T = eng.adapt(x, 2, SutaHParams(), record=[0, 1, 2])
    assert T == (n - 400) // 320 + 1
    ref, _ = W.run_suta({k: torch.from_numpy(v) for k, v in sd.items()}, cfg, torch.from_numpy(x)[None], 2,
                        record=[0, 1, 2])
    for r in (0, 1, 2):
        np.testing.assert_allclose(logits[r][0], ref[r][0].numpy(), rtol=0, atol=5e-5,
                                   err_msg=f"N{n} step {r}")


def test_longest_input_matches_oracle():
    """The reference truncates every utterance to 600 000 samples (data.py, 37.5 s, T = 1874): the
    engine's maximum size.  One SUTA step against the CPU oracle at that length."""
    from oracle import w2v2_cpu as W
    eng, cfg = engine("wav2vec2-base")
    sd = synth_weights(cfg)
    x = synth.wave(600000, 12)
    logits, ids, T = eng.adapt(x, 1, SutaHParams(), record=[0, 1])
    assert T == 1874
    ref, _ = W.run_suta({k: torch.from_numpy(v) for k, v in sd.items()}, cfg, torch.from_numpy(x)[None], 1,
                        record=[0, 1])
    for r in (0, 1):
        np.testing.assert_allclose(logits[r][0], ref[r][0].numpy(), rtol=0, atol=5e-5, err_msg=f"step {r}")
    with pytest.raises(Exception):
        eng.adapt(synth.wave(600001, 12), 1, SutaHParams(), record=[1])


def test_raw_wave_normalisation_on_device():
    eng, cfg = engine("tiny-group")
    raw = synth.raw_wave(9000, 5)
    eng.reset()
    a = eng.forward(raw, normalize=True)
    b = eng.forward(synth.normalize(raw), normalize=False)
    np.testing.assert_allclose(a, b, rtol=0, atol=2e-5)


def test_step_api_equals_adapt_schedule():
    """Reference schedule (suta_step: 2 forwards/step) == minimal schedule (suta_adapt)."""
    eng, cfg = engine("tiny-group")
    x = synth.wave(10000, 7)
    hp = SutaHParams(lr=5e-4)
    logits, _, _ = eng.adapt(x, 3, hp, record=[3])
    eng.reset()
    for _ in range(3):
        out, loss = eng.step(x, hp)
    np.testing.assert_allclose(out[0], logits[3][0], rtol=0, atol=1e-6)
    assert np.isfinite(loss).all()


def test_batch_equals_independent_runs():
    eng, cfg = engine("tiny-group", max_batch=4)
    xs = synth.batch(11000, 3, start=20)
    hp = SutaHParams(lr=5e-4)
    lb, ib, _ = eng.adapt(xs, 5, hp, record=[0, 5])
    for b in range(3):
        l1, _, _ = eng.adapt(xs[b], 5, hp, record=[0, 5])
        np.testing.assert_allclose(lb[5][b], l1[5][0], rtol=0, atol=logits_tol(5e-4))
        np.testing.assert_allclose(lb[0][b], l1[0][0], rtol=0, atol=1e-5)


def test_split_precision_tracks_exact_fp32_8s():
    """Both GEMM modes are fp32-accurate: 10-step adapted logits agree to fp32 noise."""
    eng, cfg = engine("wav2vec2-base")
    x = synth.wave(128000, 4)
    a, _, _ = eng.adapt(x, 10, SutaHParams(), record=[0, 10])
    eng.set_precision("fp32-split-bf16")
    b, _, _ = eng.adapt(x, 10, SutaHParams(), record=[0, 10])
    eng.set_precision("fp32")
    for r in (0, 10):
        np.testing.assert_allclose(b[r], a[r], rtol=0, atol=5e-5)


@pytest.mark.parametrize("precision", PRECISIONS)
def test_bitwise_deterministic(precision):
    eng, cfg = engine("wav2vec2-base", precision=precision)
    x = synth.wave(32000, 9)
    a, _, _ = eng.adapt(x, 3, SutaHParams(), record=[3])
    b, _, _ = eng.adapt(x, 3, SutaHParams(), record=[3])
    assert np.array_equal(a[3], b[3])


@pytest.mark.parametrize("preset,n", [("tiny-group", 11000), ("wav2vec2-base", 32000)])
def test_graph_replay_equals_eager(preset, n):
    """suta_adapt captures its whole loop (slot reset, vanilla forward, S x (backward + Adam + forward),
    recorded logits and greedy ids) as one graph and replays it: bitwise == eager, incl. final tensors."""
    eng, cfg = engine(preset)
    x = synth.batch(n, 2, start=90)
    hp = SutaHParams(lr=5e-4)
    names = eng.trainable_names()
    eng.set_graphs(False)
    a, ia, _ = eng.adapt(x, 4, hp, record=[1, 2, 4])
    assert eng.graph_stats()["last"] == "eager"
    pa = [{k: eng.get_param(b, k) for k in names} for b in range(2)]
    eng.set_graphs(True)
    g0 = eng.graph_stats()
    b, ib, _ = eng.adapt(x, 4, hp, record=[1, 2, 4])   # same key as the eager call: captured, then launched
    g1 = eng.graph_stats()
    c, ic, _ = eng.adapt(x, 4, hp, record=[1, 2, 4])   # replayed
    g2 = eng.graph_stats()
    assert g1["last"] == "captured" and g1["captures"] == g0["captures"] + 1 and g1["launches"] == g0["launches"] + 1
    assert g2["last"] == "replayed" and g2["captures"] == g1["captures"] and g2["launches"] == g1["launches"] + 1
    pc = [{k: eng.get_param(u, k) for k in names} for u in range(2)]
    for r in (1, 2, 4):
        assert np.array_equal(a[r], b[r]) and np.array_equal(a[r], c[r]), r
        assert np.array_equal(ia[r], ib[r]) and np.array_equal(ia[r], ic[r]), r
    for u in range(2):
        for k in names:
            assert np.array_equal(pa[u][k], pc[u][k]), (u, k)
    # a different record set is a different key: eager first, then its own graph
    d, _, _ = eng.adapt(x, 4, hp, record=[0, 3])
    e2, _, _ = eng.adapt(x, 4, hp, record=[0, 3])
    for r in (0, 3):
        assert np.array_equal(d[r], e2[r]), r


def test_non_episodic_graph_replay_equals_eager():
    """Non-episodic calls carry the adapted tensors and the Adam state (moments, step counter) from one
    call to the next (reference main.py:323-348 without --episodic).  Three calls with one key, run with
    graphs off and with graphs on (the second and third replayed): logits, greedy ids and final tensors
    bitwise equal, and a following suta_step (which reads the carried Adam moments and step) too."""
    cfg = get_config("tiny-group")
    sd = synth_weights(cfg)
    xs = [synth.batch(11000, 2, start=120 + 2 * i) for i in range(3)]
    hp = SutaHParams(lr=5e-4, episodic=False)
    runs = []
    for graphs in (False, True):
        eng = SutaEngine(cfg, sd, device=0, max_batch=2)
        eng.set_graphs(graphs)
        outs = [eng.adapt(x, 3, hp, record=[0, 1, 3]) for x in xs]
        names = eng.trainable_names()
        finals = [{k: eng.get_param(b, k) for k in names} for b in range(2)]
        nxt, loss = eng.step(xs[0], hp)
        after = [{k: eng.get_param(b, k) for k in names} for b in range(2)]
        runs.append((outs, finals, nxt, loss, after))
        eng.close()
    (oa, fa, na, la, aa), (ob, fb, nb, lb, ab) = runs
    for (l1, i1, _), (l2, i2, _) in zip(oa, ob):
        for r in (0, 1, 3):
            assert np.array_equal(l1[r], l2[r]) and np.array_equal(i1[r], i2[r]), r
    assert np.array_equal(na, nb) and np.array_equal(la, lb)
    for u in range(2):
        for k in fa[u]:
            assert np.array_equal(fa[u][k], fb[u][k]) and np.array_equal(aa[u][k], ab[u][k]), (u, k)
    assert any(not np.array_equal(fa[0][k], aa[0][k]) for k in fa[0])   # the step moved the tensors


def test_episodic_reset_restores_pristine_tensors():
    eng, cfg = engine("tiny-layer")
    sd = synth_weights(cfg)
    eng.adapt(synth.wave(9000, 1), 2, SutaHParams(lr=1e-3), record=[])
    eng.reset()
    for name in eng.trainable_names():
        assert np.array_equal(eng.get_param(0, name), sd[name]), name


@pytest.mark.parametrize("preset", ["wav2vec2-base", "tiny-layer"])
@pytest.mark.parametrize("tf,bo", [(True, False), (False, False), (True, True)])
def test_multiplicity_matches_collect_params(preset, tf, bo):
    from oracle import w2v2_cpu as W
    eng, cfg = engine(preset)
    mult = W.multiplicity(W.trainable_entries(cfg, bias_only=bo, train_feature=tf))
    for name in eng.trainable_names():
        assert eng.param_info(name, tf, bo)[0] == mult.get(name, 0), name
    for name in mult:
        assert eng.param_info(name, tf, bo)[0] == mult[name], name


def test_all_blank_utterance_keeps_finite_params():
    """K = 0 non-blank frames: reference loss is NaN but the gradient stays finite."""
    eng, cfg = engine("tiny-group", blank_bias=60.0)
    x = synth.wave(8000, 2)
    logits, ids, _ = eng.adapt(x, 2, SutaHParams(lr=5e-4), record=[0, 2])
    assert (ids[0] == 0).all()
    out, loss = eng.step(x, SutaHParams(lr=5e-4))
    assert np.isnan(loss).all()
    for name in eng.trainable_names():
        assert np.isfinite(eng.get_param(0, name)).all(), name


@pytest.mark.parametrize("n", [32000, 128000, 240000])
def test_fused_attention_equals_unfused(n, monkeypatch):
    """The flash attention kernels (forward: online softmax, ctx + LSE; backward: P recomputed, dQ/dK/dV,
    exact fp32 MFMA) against the S-GEMM / softmax / PV-GEMM path that stores P: 3 SUTA steps, ragged
    pair included (keys past an utterance's length get probability 0 in both); T = 99, 399, 749."""
    cfg = get_config("wav2vec2-base")
    sd = synth_weights(cfg)
    monkeypatch.setenv("SUTA_ATTN_FUSED", "0")
    ref_eng = SutaEngine(cfg, sd, max_batch=2, max_samples=n)
    monkeypatch.setenv("SUTA_ATTN_FUSED", "1")
    eng, _ = engine("wav2vec2-base")
    x = synth.wave(n, 21)
    a, _, _ = ref_eng.adapt(x, 3, SutaHParams(), record=[0, 3])
    b, _, _ = eng.adapt(x, 3, SutaHParams(), record=[0, 3])
    for r in (0, 3):
        np.testing.assert_allclose(b[r], a[r], rtol=0, atol=2e-5, err_msg=f"step {r}")
    waves = [synth.wave(n, 22), synth.wave(n * 3 // 5, 23)]
    a, _, _ = ref_eng.adapt_varlen(waves, 2, SutaHParams(), record=[2])
    b, _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[2])
    for u in range(2):
        np.testing.assert_allclose(b[2][u], a[2][u], rtol=0, atol=2e-5, err_msg=f"ragged utterance {u}")
    ref_eng.close()


def test_posconv_kernel_equals_gemm_path(monkeypatch):
    """The dedicated positional-conv kernel (forward: bias + GELU + residual, pre-activation stored;
    backward: transposed conv + residual, ragged padding rows zeroed) against the conv-A GEMM path."""
    cfg = get_config("wav2vec2-base")
    sd = synth_weights(cfg)
    monkeypatch.setenv("SUTA_POSCONV", "0")
    ref_eng = SutaEngine(cfg, sd, max_batch=2, max_samples=128000)
    monkeypatch.delenv("SUTA_POSCONV")
    eng, _ = engine("wav2vec2-base")
    x = synth.wave(128000, 31)
    a, _, _ = ref_eng.adapt(x, 3, SutaHParams(), record=[0, 3])
    b, _, _ = eng.adapt(x, 3, SutaHParams(), record=[0, 3])
    for r in (0, 3):
        np.testing.assert_allclose(b[r], a[r], rtol=0, atol=2e-5, err_msg=f"step {r}")
    for name in eng.trainable_names():
        if "conv_layers.0" in name or "feature_projection" in name:
            assert_params_close(eng.get_param(0, name), ref_eng.get_param(0, name), 2e-5, 3, name=name)
    waves = [synth.wave(51234, 32), synth.wave(20000, 33)]
    a, _, _ = ref_eng.adapt_varlen(waves, 2, SutaHParams(), record=[2])
    b, _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[2])
    for u in range(2):
        np.testing.assert_allclose(b[2][u], a[2][u], rtol=0, atol=2e-5, err_msg=f"ragged utterance {u}")
    ref_eng.close()


def test_branch_free_gelu_equals_erff_gelu(monkeypatch):
    """Exact fp32 mode, wav2vec2-base shapes: the branch-free GELU / GELU' (common.h gelu_fast, erfc fractional error
    < 1.2e-7) of the conv0 + GroupNorm front-end (default) against the erff forms (SUTA_FAST_GELU=0, read per launch;
    the oracle parity tests pin the default end to end).  Ragged pair, 3 steps: logits within
    logits_tol, adapted tensors within the Adam budget."""
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=48000)
    eng.set_graphs(False)
    waves = [synth.wave(48000, 98), synth.wave(30400, 99)]
    names = eng.trainable_names()
    out, par = {}, {}
    for fg in ("1", "0"):
        monkeypatch.setenv("SUTA_FAST_GELU", fg)
        out[fg], _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        par[fg] = [{n: eng.get_param(b, n) for n in names} for b in range(2)]
    eng.close()
    for u in range(2):
        for r in (0, 3):
            np.testing.assert_allclose(out["1"][r][u], out["0"][r][u], rtol=0, atol=logits_tol(2e-5),
                                       err_msg=f"step {r} utt {u}")
        for n in names:
            assert_params_close(par["1"][u][n], par["0"][u][n], 2e-5, 3, name=f"utt {u} {n}")


@pytest.mark.parametrize("variant", ["steplr_group", "steplr_layer", "sgd_group", "sgd_steplr_layer",
                                     "steplr_group_nonepisodic"])
def test_scheduler_and_sgd_match_reference(variant):
    """--scheduler torch.optim.lr_scheduler.StepLR (lr * 0.7^i, restored by the episodic reset) and --opt SGD
    against the reference driver loop's own runs (g9, main.py:308-348): logits after every step within
    logits_tol, adapted tensors within the Adam budget (AdamW) or the SGD bound; the non-episodic variant carries
    tensors, moments and the scheduler's step count into the second utterance."""
    from tests.test_oracle_golden import g9_hparams
    z = _load(f"g9_sched_{variant}.npz")
    preset = "tiny-layer" if "layer" in variant else "tiny-group"
    cfg = get_config(preset)
    sd = synth_weights(cfg)
    opt, lr, ss, episodic, steps = g9_hparams(z)
    eng = SutaEngine(cfg, sd, max_batch=1)
    hp = SutaHParams(lr=lr, optimizer=opt, lr_step_size=ss, episodic=episodic)
    prev = {k: v.copy() for k, v in sd.items()}
    for n in (8000, 12345):
        logits, ids, T = eng.adapt(z[f"N{n}/x"], steps, hp, record=list(range(steps + 1)))
        for i in range(steps + 1):
            np.testing.assert_allclose(logits[i][0], z[f"N{n}/logits"][i], rtol=0, atol=logits_tol(5e-4),
                                       err_msg=f"{variant} N{n} step {i}")
        for key in z.files:
            if key.startswith(f"N{n}/final/"):
                name = key[len(f"N{n}/final/"):]
                if opt == "SGD":
                    assert_sgd_params_close(eng.get_param(0, name), z[key], prev[name], name=name)
                else:
                    assert_params_close(eng.get_param(0, name), z[key], lr, steps * (1 if episodic else 2), name=name)
        if not episodic:
            prev = {k[len(f"N{n}/final/"):]: z[k] for k in z.files if k.startswith(f"N{n}/final/")}
    eng.close()
