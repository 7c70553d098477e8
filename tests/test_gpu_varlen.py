"""GPU tier: ragged batches (suta_adapt_varlen).

The reference adapts one utterance per forward_and_adapt (main.py:327-398), so a ragged batch must
give every utterance the result of running it alone: no padding frame may enter a statistic
(GroupNorm over time, softmax keys, positional-conv padding, loss means) or a gradient sum.
Tolerances: tests/parity.logits_tol(lr) on logits (batched vs single runs differ only by fp32
summation order), tests/parity.assert_params_close on the adapted tensors.
"""
import numpy as np
import pytest

from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights
from tests.parity import assert_params_close, logits_tol

pytestmark = pytest.mark.gpu

_ENG = {}


def engine(preset, max_batch=4):
    key = (preset, max_batch)
    if key not in _ENG:
        cfg = get_config(preset)
        _ENG[key] = (SutaEngine(cfg, synth_weights(cfg), max_batch=max_batch), cfg)
    return _ENG[key]


def _check_against_singles(eng, waves, steps, hp, record, normalize=False):
    lv, iv, tv = eng.adapt_varlen(waves, steps, hp, record=record, normalize=normalize)
    finals = [{n: eng.get_param(b, n) for n in eng.trainable_names()} for b in range(len(waves))]
    for b, w in enumerate(waves):
        l1, i1, t1 = eng.adapt(w, steps, hp, record=record, normalize=normalize)
        assert tv[b] == t1
        for r in record:
            np.testing.assert_allclose(lv[r][b], l1[r][0], rtol=0, atol=logits_tol(hp.lr), err_msg=f"utt {b} step {r}")
            assert np.mean(iv[r][b] == i1[r][0]) > 0.99
        for n in eng.trainable_names():
            assert_params_close(finals[b][n], eng.get_param(0, n), hp.lr, steps, name=f"utt {b} {n}")


@pytest.mark.parametrize("preset", ["tiny-group", "tiny-layer"])
def test_ragged_batch_equals_single_runs_tiny(preset):
    eng, cfg = engine(preset)
    waves = [synth.wave(n, 40 + i) for i, n in enumerate((12345, 8000, 10007, 9600))]
    _check_against_singles(eng, waves, 5, SutaHParams(lr=5e-4), [0, 1, 5])


def test_ragged_batch_equals_single_runs_base():
    eng, cfg = engine("wav2vec2-base", max_batch=3)
    waves = [synth.wave(n, 50 + i) for i, n in enumerate((32000, 17003, 24480))]
    _check_against_singles(eng, waves, 3, SutaHParams(), [0, 3])


def test_ragged_batch_raw_waveforms_normalized_on_device():
    eng, cfg = engine("tiny-group")
    waves = [synth.raw_wave(n, 60 + i) for i, n in enumerate((9000, 11111))]
    _check_against_singles(eng, waves, 2, SutaHParams(lr=5e-4), [0, 2], normalize=True)


def test_equal_lengths_take_the_uniform_path_bitwise():
    eng, cfg = engine("tiny-group")
    xs = synth.batch(10000, 3, start=70)
    hp = SutaHParams(lr=5e-4)
    lu, _, _ = eng.adapt(xs, 3, hp, record=[3])
    lv, _, tv = eng.adapt_varlen(list(xs), 3, hp, record=[3])
    for b in range(3):
        assert np.array_equal(lv[3][b], lu[3][b])


def test_ragged_rejects_bad_lengths():
    eng, cfg = engine("tiny-group")
    with pytest.raises(RuntimeError):
        eng.adapt_varlen(np.zeros((2, 8000), np.float32), 1, SutaHParams(), record=[1], lengths=[8000, 9000])
    with pytest.raises(RuntimeError):
        eng.adapt_varlen([np.zeros(8000, np.float32), np.zeros(100, np.float32)], 1, SutaHParams(), record=[1])
