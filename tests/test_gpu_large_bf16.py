"""GPU tier: the large-960h-lv60 geometry and the bf16 GEMM mode (BASELINE.json config C4).

* large (layer-norm feature encoder, conv bias, stable pre-LN encoder, H = 1024, 24 layers) in the
  fp32 modes against the reference's own 20-step SUTA run (golden g7): logits within 5e-5 absolute
  (measured 7.6e-6 at step 20), adapted tensors by tests/parity.assert_params_close.
* bf16 mode (every GEMM operand rounded to bf16, fp32 accumulation; the reference has no bf16 path):
  against the fp32 reference goldens and the exact-fp32 engine, tests/parity.assert_bf16_close
  (logits within 6 % of max |ref|; greedy ids agreeing on >= 90 % of frames on the 24-frame tiny
  configs, >= 97 % on base / large).
"""
import ast
import os

import numpy as np
import pytest

from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights
from tests.parity import BF16_LOGITS_RTOL_BASE, BF16_LOGITS_RTOL_LARGE, assert_bf16_close, assert_params_close, logits_tol

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_ENGINES = {}


def engine(preset, precision, max_samples=128000):
    if preset not in _ENGINES:
        cfg = get_config(preset)
        _ENGINES[preset] = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=max_samples)
    _ENGINES[preset].set_precision(precision)
    return _ENGINES[preset]


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _g7_wave():
    from tests.golden.make_golden import wave
    return wave(16000, 7)


@pytest.mark.parametrize("precision", ["fp32", "fp32-split-bf16"])
def test_large_suta_matches_reference(precision):
    z = _load("g7_large_16000.npz")
    eng = engine("wav2vec2-large", precision)
    steps = [int(s) for s in z["steps"]]
    logits, ids, T = eng.adapt(_g7_wave(), 20, SutaHParams(), record=steps)
    for j, s in enumerate(steps):
        np.testing.assert_allclose(logits[s][0], z["logits"][j], rtol=0, atol=5e-5, err_msg=f"step {s}")
    for key in z.files:
        if key.startswith("final/") and key.endswith("/idx"):
            name = key[len("final/"):-len("/idx")]
            got = eng.get_param(0, name).reshape(-1)[z[key]]
            assert_params_close(got, z[f"final/{name}/val"], 2e-5, 20, max_frac=0.05, name=name)


@pytest.mark.parametrize("variant", ["group", "group_lr5e-4", "layer", "layer_lr5e-4"])
def test_bf16_tiny_tracks_reference(variant):
    z = _load(f"g3_tiny_{variant}.npz")
    eng = engine("tiny-group" if variant.startswith("group") else "tiny-layer", "bf16")
    h = ast.literal_eval(str(z["hp_json"]))
    hp = SutaHParams(lr=h["lr"], temp=h["temp"], em_coef=h["em"], reweight=h["rw"], non_blank=h["nb"],
                     div_coef=h["div"], train_feature=h["train_feature"], bias_only=h["bias_only"])
    for n in (8000, 12345):
        logits, ids, T = eng.adapt(z[f"N{n}/x"], 10, hp, record=list(range(11)))
        for i in (0, 1, 5, 10):
            assert_bf16_close(logits[i][0], z[f"N{n}/logits"][i], 0.9, f"{variant} N{n} step {i}")
            np.testing.assert_array_equal(ids[i][0], logits[i][0].argmax(-1))


def test_bf16_large_tracks_reference():
    z = _load("g7_large_16000.npz")
    eng = engine("wav2vec2-large", "bf16")
    steps = [int(s) for s in z["steps"]]
    logits, _, _ = eng.adapt(_g7_wave(), 20, SutaHParams(), record=steps)
    for j, s in enumerate(steps):
        assert_bf16_close(logits[s][0], z["logits"][j], 0.97, f"large step {s}", rtol=BF16_LOGITS_RTOL_LARGE)


def test_bf16_base_tracks_reference_and_fp32_8s():
    z = _load("g4_base_16000.npz")
    eng = engine("wav2vec2-base", "bf16")
    steps = [int(s) for s in z["steps"]]
    logits, _, _ = eng.adapt(synth.wave(16000, 0), 10, SutaHParams(), record=steps)
    for j, s in enumerate(steps):
        assert_bf16_close(logits[s][0], z["logits"][j], 0.97, f"base N16000 step {s}", rtol=BF16_LOGITS_RTOL_BASE)
    x = synth.wave(128000, 4)
    b, _, _ = eng.adapt(x, 10, SutaHParams(), record=[0, 10])
    eng.set_precision("fp32")
    a, _, _ = eng.adapt(x, 10, SutaHParams(), record=[0, 10])
    for r in (0, 10):
        assert_bf16_close(b[r][0], a[r][0], 0.97, f"base 8 s step {r} vs exact fp32", rtol=BF16_LOGITS_RTOL_BASE)


def test_bf16_batch_equals_single_and_deterministic():
    eng = engine("wav2vec2-base", "bf16")
    xs = synth.batch(32000, 2, start=40)
    lb, _, _ = eng.adapt(xs, 3, SutaHParams(), record=[3])
    l1, _, _ = eng.adapt(xs[1], 3, SutaHParams(), record=[3])
    l2, _, _ = eng.adapt(xs[1], 3, SutaHParams(), record=[3])
    assert np.array_equal(l1[3][0], l2[3][0])
    # batch and single runs choose different split-K / tile schedules: fp32 summation-order noise
    # flips bf16 roundings downstream, so they agree to bf16 (not fp32) tolerance
    assert_bf16_close(lb[3][1], l1[3][0], 0.97, "batch slot 1 vs single", rtol=BF16_LOGITS_RTOL_BASE)


def test_bf16_planes_equal_fp32_staged_path(monkeypatch):
    """The bf16-plane linears (default) and the fp32-staged bf16 kernels (SUTA_BF16_PLANES=0) round the same
    operands the same way (RNE to bf16, fp32 accumulation): they agree to bf16 tolerance, and each rerun
    is bitwise identical."""
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    x = synth.batch(32000, 2, start=60)
    out = {}
    for planes in ("1", "0"):
        monkeypatch.setenv("SUTA_BF16_PLANES", planes)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        a, _, _ = eng.adapt(x, 3, SutaHParams(), record=[0, 3])
        b, _, _ = eng.adapt(x, 3, SutaHParams(), record=[0, 3])
        assert np.array_equal(a[3], b[3]), planes
        out[planes] = a
        eng.close()
    for r in (0, 3):
        for u in range(2):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"planes vs fp32-staged step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE)


def test_bf16_flash_images_equal_fp32_image_kernels(monkeypatch):
    """bf16 mode's flash kernels stage K / V / Q / dO / dS / K^T as bf16 LDS images (default) instead of
    fp32 images converted per MFMA operand (SUTA_FLASH_BF16_IMG=0).  Same RNE roundings, same MFMA order
    in the forward: step-0 logits bitwise equal; after backward steps only the dQ partial's summation
    order differs, so adapted logits agree to bf16 tolerance.  Ragged pair, T = 399 and 239."""
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=128000)
    eng.set_precision("bf16")
    waves = [synth.wave(128000, 70), synth.wave(76800, 71)]
    out = {}
    for img in ("1", "0"):
        monkeypatch.setenv("SUTA_FLASH_BF16_IMG", img)
        out[img], _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
    eng.close()
    for u in range(2):
        assert np.array_equal(out["1"][0][u], out["0"][0][u]), f"step 0 utt {u}"
        assert_bf16_close(out["1"][3][u], out["0"][3][u], 0.97, f"bf16 images step 3 utt {u}",
                          rtol=BF16_LOGITS_RTOL_LARGE)


def test_bf16_posconv_kernel_equals_conv_a_path(monkeypatch):
    """posconv_bf16_kernel (config C4's positional conv, 16 groups of 64 channels, 128 taps) against the
    conv-A GEMM path it replaces (SUTA_POSCONV=0): the same bf16 operand rounding with fp32 accumulation
    in another order (fp32 noise that flips bf16 roundings downstream, as between any two bf16 schedules),
    so both agree within the bf16 tolerance, and reruns are bitwise identical; a ragged batch covers the
    backward's zeroed padding rows.  (test_bf16_large_tracks_reference pins the kernel against the fp32
    reference goldens.)"""
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    monkeypatch.setenv("SUTA_POSCONV", "0")
    ref = SutaEngine(cfg, sd, max_batch=2, max_samples=64000)
    monkeypatch.delenv("SUTA_POSCONV")
    eng = SutaEngine(cfg, sd, max_batch=2, max_samples=64000)
    ref.set_precision("bf16")
    eng.set_precision("bf16")
    x = synth.wave(48000, 41)
    a, _, _ = ref.adapt(x, 3, SutaHParams(), record=[0, 3])
    b, _, _ = eng.adapt(x, 3, SutaHParams(), record=[0, 3])
    b2, _, _ = eng.adapt(x, 3, SutaHParams(), record=[0, 3])
    assert np.array_equal(b[3], b2[3])
    for r in (0, 3):
        assert_bf16_close(b[r][0], a[r][0], 0.97, f"step {r}", rtol=BF16_LOGITS_RTOL_LARGE)
    waves = [synth.wave(40000, 42), synth.wave(23000, 43)]
    a, _, _ = ref.adapt_varlen(waves, 2, SutaHParams(), record=[2])
    b, _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[2])
    for u in range(2):
        assert_bf16_close(b[2][u], a[2][u], 0.97, f"ragged utterance {u}", rtol=BF16_LOGITS_RTOL_LARGE)
    ref.close()
    eng.close()


def test_bf16_hbx_slice_ring_kernel_bitwise_equals_128_tile(monkeypatch):
    """gemm_hbx_kernel (256 x 256 tile, 32-deep slice ring, v_mfma_f32_32x32x16_bf16) forced on every bf16-plane linear
    (SUTA_HBX=2: every epilogue class -- bias / residual, bias + GELU + bf16 pre-activation, GELU' -- small grids and
    edge tiles of a ragged pair: 198 and 124 rows of a 256-row tile), in every epilogue form (SUTA_HBX_T=1: C^T
    accumulators, row-per-lane 16-B stores; 2: the same staged through LDS into whole-line stores; 0: the
    column-per-lane form) and main loop (SUTA_HBX_FORM=2: four-phase 64-deep K-tiles, staggered wave groups; 3 the same
    with three half-tiles of DMA in flight and one wait per K-tile; 4 form 3 on v_mfma_f32_16x16x32_bf16 with the
    accumulators remapped to the C^T layout through LDS, round 6; 1 the four phases in lockstep; 0 the 32-deep slice
    ring), against the 128 x 128 kernel (SUTA_HBX=0),
    all without split-K (SUTA_SPLITK=0: a split sums k in another order): the same MFMA products in the same k order, so
    logits and adapted tensors are bitwise equal; and the large model's 20-step SUTA against the reference goldens g7
    (bf16 tolerance).  Reference main.py:181,205."""
    monkeypatch.setenv("SUTA_SPLITK", "0")
    z = _load("g7_large_16000.npz")
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    steps = [int(s) for s in z["steps"]]
    waves = [synth.wave(32000, 82), synth.wave(20000, 83)]
    out, params = {}, {}
    for mode, tr, form in (("0", "1", "2"), ("2", "1", "2"), ("2", "2", "2"), ("2", "2", "3"), ("2", "2", "4"),
                           ("2", "2", "1"), ("2", "2", "0"), ("2", "0", "2")):
        monkeypatch.setenv("SUTA_HBX", mode)
        monkeypatch.setenv("SUTA_HBX_T", tr)
        monkeypatch.setenv("SUTA_HBX_FORM", form)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        if mode == "2" and tr == "2" and form == "2":
            eng.set_census(True)
            logits, _, _ = eng.adapt(_g7_wave(), 20, SutaHParams(), record=steps)
            census = eng.get_census()
            eng.set_census(False)
            assert any(k.startswith("hbx 256x256 ") for k in census), census
            for j, s in enumerate(steps):
                assert_bf16_close(logits[s][0], z["logits"][j], 0.97, f"hbx large step {s}", rtol=BF16_LOGITS_RTOL_LARGE)
        key = mode + tr + form
        out[key], _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        params[key] = {n: eng.get_param(1, n) for n in eng.trainable_names()}
        eng.close()
    for key in ("212", "222", "223", "224", "221", "220", "202"):
        for r in (0, 3):
            for u in range(2):
                assert np.array_equal(out[key][r][u], out["012"][r][u]), (key, r, u)
        for n, v in params[key].items():
            assert np.array_equal(v, params["012"][n]), (key, n)


def test_bf16_fused_delta_bitwise_equals_separate_pass(monkeypatch):
    """The flash backward's row term delta = rowsum(dctx * ctx) computed in the dctx GEMM's C^T epilogue (EPI_DELTA,
    gemm_hbx; the fp32 dctx is then not written) against the separate attn_delta_kernel pass (SUTA_FUSED_DELTA=0):
    the epilogue sums in the kernel's order (4-column fma dots, then its xor tree), so logits and adapted tensors are
    bitwise equal.  wav2vec2-large in bf16 mode on a ragged pair, hbx forced on the small grid (SUTA_HBX=2)."""
    monkeypatch.setenv("SUTA_SPLITK", "0")
    monkeypatch.setenv("SUTA_HBX", "2")
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    waves = [synth.wave(32000, 86), synth.wave(20000, 87)]
    out, params, delta_launches = {}, {}, {}
    for fd in ("1", "0"):
        monkeypatch.setenv("SUTA_FUSED_DELTA", fd)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        eng.set_census(True)
        out[fd], _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        census = eng.get_census()
        eng.set_census(False)
        # the census's "epi <kernel> <tile> <flags>" entries: EPI_DELTA (256) alone on the 256 x 256 kernel
        delta_launches[fd] = sum(v for k, v in census.items() if k.startswith("epi hbx 256x256 ") and k.endswith(" 256"))
        params[fd] = {n: eng.get_param(1, n) for n in eng.trainable_names()}
        eng.close()
    assert delta_launches["1"] == 3 * cfg["num_hidden_layers"], delta_launches   # one dctx GEMM per layer-backward
    assert delta_launches["0"] == 0, delta_launches
    for r in (0, 3):
        for u in range(2):
            assert np.array_equal(out["1"][r][u], out["0"][r][u]), (r, u)
    for n, v in params["1"].items():
        assert np.array_equal(v, params["0"][n]), n


def test_bf16_epilogue_gelu_as_equals_erff(monkeypatch):
    """The bf16-plane GEMM epilogues' GELU / GELU' (common.h gelu2_bf16ep / dgelu2_bf16ep: Abramowitz & Stegun 7.1.28
    erf, |error| <= 3e-7, packed fp32, default) against erff (SUTA_FAST_GELU=0), wav2vec2-large in bf16 mode: the
    outputs are bf16 planes, so the two agree to bf16 tolerance (greedy ids >= 97 %)."""
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    waves = [synth.wave(32000, 84), synth.wave(20000, 85)]
    out = {}
    for fg in ("1", "0"):
        monkeypatch.setenv("SUTA_FAST_GELU", fg)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        out[fg], _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        eng.close()
    for r in (0, 3):
        for u in range(2):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"A&S GELU vs erff step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE)


@pytest.mark.parametrize("preset", ["wav2vec2-base", "wav2vec2-large"])
def test_flash_fwd_plane_kernel_equals_row_kernel(monkeypatch, preset):
    """flash_fwd_bf16p_kernel (Q / K / V read from the QKV GEMM's bf16 plane, V^T by transposed LDS reads;
    default in bf16 mode) against flash_fwd_bf16_kernel (fp32 rows rounded in the kernel,
    SUTA_FLASH_FWD_PLANE=0): the same RNE-rounded operands; the exponent argument is one fma instead of a
    multiply and a subtraction, so probabilities differ by fp32 rounding and the adapted logits agree to
    the bf16 tolerance.  Ragged pair (T = 399 and 239: a partial last key tile, both 32-key halves of it
    masked differently), reruns bitwise identical."""
    cfg = get_config(preset)
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=128000)
    eng.set_precision("bf16")
    eng.set_graphs(False)  # eager: a replayed graph would keep the kernels it was captured with
    waves = [synth.wave(128000, 80), synth.wave(76800, 81)]
    out = {}
    for plane in ("1", "0"):
        monkeypatch.setenv("SUTA_FLASH_FWD_PLANE", plane)
        a, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        b, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        for u in range(2):
            assert np.array_equal(a[3][u], b[3][u]), (plane, u)
        out[plane] = a
    eng.close()
    for r in (0, 3):
        for u in range(2):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"plane fwd step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE)


@pytest.mark.parametrize("preset", ["wav2vec2-base", "wav2vec2-large"])
def test_flash_bwd_plane_kernel_equals_row_kernel(monkeypatch, preset):
    """flash_bwd_bf16p_kernel (Q / K / V from the qkv bf16 plane, dO from the plane the out-projection's
    input-gradient GEMM writes, dV^T / dK^T operands by transposed LDS reads; default in bf16 mode) against
    flash_bwd_bf16_kernel (fp32 rows rounded in the kernel, transposed LDS images; SUTA_FLASH_BWD_PLANE=0):
    the same RNE-rounded operands, the exponent argument one fma instead of a multiply and a subtraction
    -> adapted logits and tensors agree to the bf16 tolerance; the step-0 logits (no backward yet) are
    bitwise equal; reruns bitwise identical.  Ragged pair (T = 399 / 239: masked keys and rows)."""
    cfg = get_config(preset)
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=128000)
    eng.set_precision("bf16")
    eng.set_graphs(False)  # eager: a replayed graph would keep the kernels it was captured with
    waves = [synth.wave(128000, 82), synth.wave(76800, 83)]
    out = {}
    for plane in ("1", "0"):
        monkeypatch.setenv("SUTA_FLASH_BWD_PLANE", plane)
        a, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 1, 3])
        b, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 1, 3])
        for u in range(2):
            assert np.array_equal(a[3][u], b[3][u]), (plane, u)
        out[plane] = a
    eng.close()
    for u in range(2):
        assert np.array_equal(out["1"][0][u], out["0"][0][u]), u
        for r in (1, 3):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"plane bwd step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_fused_conv_layernorm_backward_equals_separate_passes(monkeypatch, precision):
    """wav2vec2-large's layer-norm conv stack: the LayerNorm backward that also sums the conv bias gradients
    and conv0's weight gradient (default) against the separate column-sum passes and the conv0 weight-gradient
    GEMM (SUTA_FUSED_CONV_LN=0).  The same sums in another fixed order (fp32; the GEMM rounded its operands to
    bf16 in bf16 mode, the fused sum does not): fp32 logits within logits_tol, adapted conv tensors by the
    Adam budget; bf16 to the bf16 tolerance.  Ragged pair (padding rows carry zero gradient)."""
    cfg = get_config("wav2vec2-large")
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=48000)
    eng.set_precision(precision)
    waves = [synth.wave(48000, 90), synth.wave(30400, 91)]
    names = [n for n in eng.trainable_names() if "feature_extractor" in n]
    out, par = {}, {}
    for fused in ("1", "0"):
        monkeypatch.setenv("SUTA_FUSED_CONV_LN", fused)
        eng.set_graphs(False)
        out[fused], _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[1, 3])
        par[fused] = [{n: eng.get_param(b, n) for n in names} for b in range(2)]
    eng.close()
    for u in range(2):
        for r in (1, 3):
            if precision == "fp32":
                np.testing.assert_allclose(out["1"][r][u], out["0"][r][u], rtol=0, atol=logits_tol(2e-5),
                                           err_msg=f"step {r} utt {u}")
            else:
                assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"step {r} utt {u}", rtol=BF16_LOGITS_RTOL_LARGE)
        if precision == "fp32":
            for n in names:
                assert_params_close(par["1"][u][n], par["0"][u][n], 2e-5, 3, name=f"utt {u} {n}")


def test_conv_stack_on_bf16_planes_equals_fp32_staged(monkeypatch):
    """wav2vec2-large's conv stack in bf16 mode: the forward conv GEMMs on bf16 planes (activation planes written
    by the conv LayerNorms, per-slot transposed bf16 weights rebuilt after each AdamW step; default) against the
    fp32-staged one-plane kernels (SUTA_CONV_PLANES=0).  The same RNE-rounded operands, another accumulation
    order: adapted logits agree to the bf16 tolerance; reruns bitwise identical.  Ragged pair."""
    cfg = get_config("wav2vec2-large")
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=48000)
    eng.set_precision("bf16")
    eng.set_graphs(False)  # eager: a replayed graph would keep the kernels it was captured with
    waves = [synth.wave(48000, 92), synth.wave(30400, 93)]
    out = {}
    for cp in ("1", "0"):
        monkeypatch.setenv("SUTA_CONV_PLANES", cp)
        a, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        b, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        for u in range(2):
            assert np.array_equal(a[3][u], b[3][u]), (cp, u)
        out[cp] = a
    eng.close()
    for r in (0, 3):
        for u in range(2):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"conv planes step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE)


@pytest.mark.parametrize("model", ["wav2vec2-large", "wav2vec2-base"])
def test_ffn_preactivation_bf16_equals_fp32(monkeypatch, model):
    """bf16 mode: the FFN pre-activation u stored in bf16 by the FFN1 GEMM epilogue and read back in bf16 by the
    FFN2 input gradient's gelu' (default) against u kept in fp32 (SUTA_PRE_BF16=0).  Stable-LN (large) and
    post-LN (base) layer paths, ragged pair: adapted logits agree to the bf16 tolerance; reruns bitwise."""
    cfg = get_config(model)
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=48000)
    eng.set_precision("bf16")
    eng.set_graphs(False)  # eager: a replayed graph would keep the kernels it was captured with
    waves = [synth.wave(48000, 94), synth.wave(30400, 95)]
    out = {}
    for pb in ("1", "0"):
        monkeypatch.setenv("SUTA_PRE_BF16", pb)
        a, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        b, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        for u in range(2):
            assert np.array_equal(a[3][u], b[3][u]), (pb, u)
        out[pb] = a
    eng.close()
    rtol = BF16_LOGITS_RTOL_LARGE if model == "wav2vec2-large" else BF16_LOGITS_RTOL_BASE
    for u in range(2):
        np.testing.assert_array_equal(out["1"][0][u], out["0"][0][u])  # step 0: the forward does not read u
        assert_bf16_close(out["1"][3][u], out["0"][3][u], 0.97, f"pre bf16 step 3 utt {u}", rtol=rtol)


@pytest.mark.parametrize("switch", ["SUTA_CONV_Z_BF16", "SUTA_DY_PLANES"])
def test_bf16_storage_of_conv_outputs_and_dy_equals_fp32_storage(monkeypatch, switch):
    """bf16 mode, wav2vec2-large: (SUTA_CONV_Z_BF16) the conv stack's outputs z_i and activation gradients da_i
    stored in bf16 by conv0 / the conv GEMM epilogues and read widened by the conv LayerNorms, and (SUTA_DY_PLANES)
    the stable-LN backward's dy written by the QKV / FFN1 input-gradient GEMMs as bf16 planes -- torch autocast's
    bf16 conv / matmul outputs and gradients (default) -- against fp32 storage (=0).  Ragged pair: adapted logits
    agree to the bf16 tolerance, reruns are bitwise identical, step 0 is bitwise equal for the backward-only switch."""
    cfg = get_config("wav2vec2-large")
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=48000)
    eng.set_precision("bf16")
    eng.set_graphs(False)  # eager: a replayed graph would keep the kernels it was captured with
    waves = [synth.wave(48000, 96), synth.wave(30400, 97)]
    out = {}
    for on in ("1", "0"):
        monkeypatch.setenv(switch, on)
        a, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        b, _, _ = eng.adapt_varlen(waves, 3, SutaHParams(), record=[0, 3])
        for u in range(2):
            assert np.array_equal(a[3][u], b[3][u]), (on, u)
        out[on] = a
    eng.close()
    for u in range(2):
        if switch == "SUTA_DY_PLANES":
            np.testing.assert_array_equal(out["1"][0][u], out["0"][0][u])  # the forward is unchanged
        for r in (0, 3):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"{switch} step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE)


def test_batched_gemm_without_off32_epilogue_falls_back(monkeypatch):
    """A batched (Z > 1) GEMM -- the conv stack's per-utterance forward -- that the 256 x 256 kernel cannot take for
    want of the 32-bit-offset epilogue (SUTA_EPI_FAST=0 here; an operand over 4 GiB in general) runs on the 128 x 128
    kernel instead of failing (the dispatcher decides with p.off32 known).  wav2vec2-large in bf16 mode, the 256 x 256
    kernel forced onto every eligible GEMM (SUTA_HBX=2), no split-K, ragged pair: the default run puts the batched conv
    forward on hbx, the SUTA_EPI_FAST=0 run on hb, and logits and adapted tensors are bitwise equal (the 256 x 256
    forms are bitwise the 128 x 128 kernel; the general epilogue applies the fast one's operations in its order)."""
    monkeypatch.setenv("SUTA_SPLITK", "0")
    monkeypatch.setenv("SUTA_HBX", "2")
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    waves = [synth.wave(32000, 76), synth.wave(20000, 77)]
    out, params, batched_hbx = {}, {}, {}
    for fast in ("1", "0"):
        monkeypatch.setenv("SUTA_EPI_FAST", fast)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        eng.set_census(True)
        out[fast], _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[0, 2])
        census = eng.get_census()
        eng.set_census(False)
        batched_hbx[fast] = sum(v for k, v in census.items() if k.startswith("hbx ") and " z=2 " in k)
        params[fast] = {n: eng.get_param(1, n) for n in eng.trainable_names()}
        eng.close()
    assert batched_hbx["1"] > 0 and batched_hbx["0"] == 0, batched_hbx
    for r in (0, 2):
        for u in range(2):
            assert np.array_equal(out["1"][r][u], out["0"][r][u]), (r, u)
    for n, v in params["1"].items():
        assert np.array_equal(v, params["0"][n]), n


@pytest.mark.parametrize("form", ["2", "3", "4"])
def test_conv_input_gradients_on_256_tile_bitwise(monkeypatch, form):
    """The layer-norm conv stack's input gradients (conv-A rows m + seg - pad, per-tap weight segments; config C4's
    conv-seg GEMMs, one per output-row residue, Z = batch) on the four-phase 256 x 256 kernel's CONV form (per-segment
    row validity and weight-slice jumps in the DMA pointers; SUTA_HBP_CONV=1, default) against the 128 x 128 kernel
    (SUTA_HBP_CONV=0): the same MFMA products in the same k order, so logits and adapted tensors are bitwise equal.
    wav2vec2-large in bf16 mode, a ragged pair (per-utterance valid rows), the 256 x 256 kernel forced onto the small
    grids (SUTA_HBX=2), no split-K, in the staggered main loops (SUTA_HBX_FORM 2, 3 and 4: 16x16x32 MFMAs)."""
    monkeypatch.setenv("SUTA_SPLITK", "0")
    monkeypatch.setenv("SUTA_HBX", "2")
    monkeypatch.setenv("SUTA_HBX_FORM", form)
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    waves = [synth.wave(32000, 74), synth.wave(20000, 75)]
    out, params, conv = {}, {}, {}
    for hc in ("1", "0"):
        monkeypatch.setenv("SUTA_HBP_CONV", hc)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        eng.set_census(True)
        out[hc], _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[0, 2])
        census = eng.get_census()
        eng.set_census(False)
        conv[hc] = {k: v for k, v in census.items() if k.endswith(" conv-seg")}
        params[hc] = {n: eng.get_param(1, n) for n in eng.trainable_names()}
        eng.close()
    assert conv["1"] and all(k.startswith("hbx 256x256 ") for k in conv["1"]), conv["1"]
    assert conv["0"] and all(k.startswith("hb 128x128 ") for k in conv["0"]), conv["0"]
    for r in (0, 2):
        for u in range(2):
            assert np.array_equal(out["1"][r][u], out["0"][r][u]), (r, u)
    for n, v in params["1"].items():
        assert np.array_equal(v, params["0"][n]), n


def test_conv_weight_gradients_on_256_tile_tn_form_bitwise(monkeypatch):
    """The layer-norm conv stack's weight gradients dW_i = im2col(a_{i-1})^T dz_i (MN-contiguous bf16 planes, Z = batch;
    config C4's former gemm_hbt_kernel GEMMs) on the four-phase 256 x 256 kernel's TN form (transposed LDS reads of
    [k][m] images, K tails read from the zero page; SUTA_HBT4=2 forces it onto the small test grids) against the
    128 x 128 hbt kernel (SUTA_HBT4=0), no split-K: the same products summed in the same k order, so logits and adapted
    tensors (the conv weights among them) are bitwise equal.  wav2vec2-large in bf16 mode, a ragged pair."""
    monkeypatch.setenv("SUTA_SPLITK", "0")
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    waves = [synth.wave(32000, 76), synth.wave(20000, 77)]
    out, params, dw = {}, {}, {}
    for h4 in ("2", "0"):
        monkeypatch.setenv("SUTA_HBT4", h4)
        eng = SutaEngine(cfg, sd, max_batch=2, max_samples=32000)
        eng.set_precision("bf16")
        eng.set_census(True)
        out[h4], _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[0, 2])
        census = eng.get_census()
        eng.set_census(False)
        dw[h4] = [k for k in census if k.startswith("hbt")]
        params[h4] = {n: eng.get_param(1, n) for n in eng.trainable_names()}
        eng.close()
    assert dw["2"] and all(k.startswith("hbt4 256x256 ") for k in dw["2"]), dw["2"]
    assert dw["0"] and all(k.startswith("hbt 128x128 ") for k in dw["0"]), dw["0"]
    for r in (0, 2):
        for u in range(2):
            assert np.array_equal(out["2"][r][u], out["0"][r][u]), (r, u)
    for n, v in params["2"].items():
        assert np.array_equal(v, params["0"][n]), n


@pytest.mark.parametrize("model", ["wav2vec2-large", "wav2vec2-base"])
def test_bf16_plane_flash_backward_ragged_edges(monkeypatch, model):
    """The bf16-plane flash backward (key-major dS image read back transposed for dQ, row-permuted Q / dO images, dQ
    partials in fragment order transposed by flash_dq_reduce_frag, dK / dV staged through LDS into whole-row stores;
    round 6) against the fp32-row bf16 kernel (SUTA_FLASH_BWD_PLANE=0: row-layout partials, flash_dq_reduce) on a
    ragged batch with T = 399 (13 key groups: two key blocks, a half-empty last query tile), 262 (keys past the
    length inside a wave) and 49 (one query tile): logits within the bf16 tolerance after 1 and 2 steps, the step-0
    logits bitwise equal, reruns bitwise identical."""
    cfg = get_config(model)
    sd = synth_weights(cfg)
    waves = [synth.wave(n, 70 + i) for i, n in enumerate((128000, 84000, 16000))]
    out = {}
    for plane in ("1", "0"):
        monkeypatch.setenv("SUTA_FLASH_BWD_PLANE", plane)
        eng = SutaEngine(cfg, sd, max_batch=3, max_samples=128000)
        eng.set_precision("bf16")
        a, _, t = eng.adapt_varlen(waves, 2, SutaHParams(), record=[0, 1, 2])
        b, _, _ = eng.adapt_varlen(waves, 2, SutaHParams(), record=[0, 1, 2])
        eng.close()
        assert list(t) == [399, 262, 49]
        for u in range(3):
            assert np.array_equal(a[2][u], b[2][u]), (plane, u)
        out[plane] = a
    for u in range(3):
        assert np.array_equal(out["1"][0][u], out["0"][0][u]), u
        for r in (1, 2):
            assert_bf16_close(out["1"][r][u], out["0"][r][u], 0.97, f"{model} plane bwd step {r} utt {u}",
                              rtol=BF16_LOGITS_RTOL_LARGE if model == "wav2vec2-large" else BF16_LOGITS_RTOL_BASE)
