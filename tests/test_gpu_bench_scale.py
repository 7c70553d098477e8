"""GPU tier: parity at the bench's own scale and on the replayed (hipGraph) ragged path.

* The headline layout exactly as bench.py runs it: bench.BATCH (164) x 128 000-sample utterances x 10 SUTA
  steps in one suta_adapt call, scripts/LS.sh flags, record steps 0/1/3/5/10, greedy ids only (bench.py's timed
  key: want_logits False).  As in the bench, the first call of the key runs eagerly (the census is taken on it),
  the second captures the loop and launches it, the third REPLAYS it (suta_get_graph_stats asserts each mode).
  The replayed call's greedy ids and adapted tensors must equal, bitwise, those of an eager call on the same
  batch that also copies out logits (replay == eager); that eager call's first / middle / last slots are
  compared with the CPU oracle (oracle/w2v2_cpu.run_suta): logits within 5e-5 absolute (the base-size
  tolerance of tests/test_gpu_parity.py), adapted tensors by tests/parity.assert_params_close.  The batch is
  imported from bench.py, so a change of the bench's batch moves this pin with it; the launch census asserts
  the grids that batch reaches (B x 399 rows -> ceil(B*399/128) row tiles of the linears, Z = B conv GEMMs).
* Config C4 at bench.C4_BATCH likewise (bf16, 20 steps): replay == eager bitwise, eager against the exact-fp32
  engine and the oracle.
* Ragged batches that share a quantised layout but differ in per-utterance lengths: the second call
  replays the captured step with new lengths (device-side length buffers); it must equal single runs
  and the eager (graphs off) execution bitwise.
* Ragged batches with T > 512 frames (long utterances: the attention path for long keys plus
  ragged masks) against single runs; the minimal-length utterance (T = 1) beside a long one.
"""
import numpy as np
import pytest
import torch

import bench
from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights
from tests.parity import assert_params_close, logits_tol

pytestmark = pytest.mark.gpu

BENCH_RECORD = bench.RECORD   # [0, 1, 3, 5, 10]


def _slots(B):
    return sorted({0, B // 2, B - 1})


def _row_tiles(B, T, tile=128):
    return -(-(B * T) // tile)


def _timed_mode_equals_eager(eng, warm, x, S, hp, rec, slots):
    """bench.py's call sequence on one key (ids only): eager warm-up, capture + launch, replay -- then an eager call
    with logits on the same batch.  Asserts the loop modes, and that the replayed call's ids and adapted tensors
    equal the eager call's bitwise.  Returns (eager logits, eager ids, T, census of the first (eager) call)."""
    names = eng.trainable_names()
    eng.set_census(True)
    eng.adapt(warm, S, hp, record=rec, want_logits=False)                        # bench warm-up: a new key, eager
    census = eng.get_census()
    eng.set_census(False)
    assert eng.graph_stats()["last"] == "eager"
    eng.adapt(x, S, hp, record=rec, want_logits=False)                           # 1st timed call: capture + launch
    g1 = eng.graph_stats()
    assert g1["last"] == "captured", g1
    _, ids_r, T = eng.adapt(x, S, hp, record=rec, want_logits=False)             # later timed calls: replay
    g2 = eng.graph_stats()
    assert g2["last"] == "replayed" and g2["captures"] == g1["captures"] and g2["launches"] == g1["launches"] + 1, g2
    par_r = {b: {n: eng.get_param(b, n) for n in names} for b in slots}
    logits, ids, T2 = eng.adapt(x, S, hp, record=rec)                            # logits wanted: a new key, eager
    assert eng.graph_stats()["last"] == "eager" and T2 == T
    for r in rec:
        assert np.array_equal(ids_r[r], ids[r]), f"replayed ids != eager ids at step {r}"
    for b in slots:
        for n in names:
            assert np.array_equal(par_r[b][n], eng.get_param(b, n)), f"replayed != eager: slot {b} {n}"
    return logits, ids, T, census


def test_bench_layout_matches_oracle():
    """reference main.py:347-348 (S x forward_and_adapt per utterance) at the bench's batch, in the bench's timed
    execution mode (graph replay), pinned bitwise to an eager call that is checked against the oracle."""
    from oracle import w2v2_cpu as W
    import os
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    cfg = get_config("wav2vec2-base")
    sd = synth_weights(cfg)
    B, N, S = bench.BATCH, 128000, 10
    eng = SutaEngine(cfg, sd, device=0, max_batch=B, max_samples=N)
    hp = SutaHParams()
    warm = torch.from_numpy(synth.batch(N, B, start=0)).cuda()
    x = synth.batch(N, B, start=B)          # bench.py's first timed batch at --warmup 1
    logits, ids, T, census = _timed_mode_equals_eager(eng, warm, torch.from_numpy(x).cuda(), S, hp, BENCH_RECORD,
                                                      _slots(B))
    assert T == 399
    txt = "\n".join(f"{k}: {v}" for k, v in sorted(census.items()))
    gy = _row_tiles(B, T)
    for gx in (6, 18, 24):   # N = 768 (out-proj, FFN2, their dX), 2304 (QKV), 3072 (FFN1, dX of FFN2)
        assert any(k.startswith("grid glds 128x128 ") and f" gx={gx} gy={gy} z=1 " in k for k in census), (gx, gy, txt)
    assert any(k.startswith(("glds ", "f32 ")) and f" z={B} " in k for k in census), txt   # per-utterance conv GEMMs
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    for slot in _slots(B):
        ref, final = W.run_suta(sdt, cfg, torch.from_numpy(x[slot])[None], S, record=[0, 1, 5, 10])
        for r in (0, 1, 5, 10):
            np.testing.assert_allclose(logits[r][slot], ref[r][0].numpy(), rtol=0, atol=5e-5,
                                       err_msg=f"slot {slot} step {r}")
            np.testing.assert_array_equal(ids[r][slot], logits[r][slot].argmax(-1))
        for name, val in final.items():
            assert_params_close(eng.get_param(slot, name), val.numpy(), hp.lr, S, name=f"slot {slot} {name}")
    eng.close()


def _singles(eng, waves, steps, hp, record):
    out = []
    for w in waves:
        l1, _, t1 = eng.adapt(w, steps, hp, record=record)
        out.append(({r: l1[r][0] for r in record}, {n: eng.get_param(0, n) for n in eng.trainable_names()}, t1))
    return out


def test_ragged_graph_replay_equals_singles_and_eager():
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), device=0, max_batch=3, max_samples=64000)
    hp = SutaHParams()
    rec = [0, 1, 3]
    first = [synth.wave(n, 300 + i) for i, n in enumerate((32000, 17003, 24480))]
    second = [synth.wave(n, 310 + i) for i, n in enumerate((30421, 31999, 16500))]   # same 32000 layout
    eng.set_graphs(True)
    eng.adapt_varlen(first, 3, hp, record=rec, quantum=1600)
    lv, iv, tv = eng.adapt_varlen(second, 3, hp, record=rec, quantum=1600)   # every step replayed
    finals = [{n: eng.get_param(b, n) for n in eng.trainable_names()} for b in range(3)]
    eng.set_graphs(False)
    le, _, te = eng.adapt_varlen(second, 3, hp, record=rec, quantum=1600)
    assert tv == te
    for r in rec:
        for b in range(3):
            assert np.array_equal(lv[r][b], le[r][b]), (r, b)
    for b, (l1, p1, t1) in enumerate(_singles(eng, second, 3, hp, rec)):
        assert tv[b] == t1
        for r in rec:
            np.testing.assert_allclose(lv[r][b], l1[r], rtol=0, atol=logits_tol(hp.lr), err_msg=f"utt {b} step {r}")
        for n, v in p1.items():
            assert_params_close(finals[b][n], v, hp.lr, 3, name=f"utt {b} {n}")
    eng.set_graphs(True)
    eng.close()


def test_ragged_long_utterances_equal_singles():
    """T up to 749 frames (> 512): long-key attention with ragged key masks, checked against runs alone."""
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), device=0, max_batch=3, max_samples=240000)
    hp = SutaHParams()
    rec = [0, 2]
    waves = [synth.wave(n, 320 + i) for i, n in enumerate((240000, 170001, 120000))]
    lv, iv, tv = eng.adapt_varlen(waves, 2, hp, record=rec)
    assert max(tv) == 749
    finals = [{n: eng.get_param(b, n) for n in eng.trainable_names()} for b in range(3)]
    for b, (l1, p1, t1) in enumerate(_singles(eng, waves, 2, hp, rec)):
        assert tv[b] == t1
        for r in rec:
            np.testing.assert_allclose(lv[r][b], l1[r], rtol=0, atol=logits_tol(hp.lr), err_msg=f"utt {b} step {r}")
        for n, v in p1.items():
            assert_params_close(finals[b][n], v, hp.lr, 2, name=f"utt {b} {n}")
    eng.close()


def test_ragged_ted_lengths_equal_singles():
    """Config C5's longest ragged batch at logits level: T = 531 / 812 / 1874 (the 600 000-sample cap) in
    one suta_adapt_varlen call against each utterance adapted alone (reference main.py:347-348 adapts one
    utterance per call)."""
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), device=0, max_batch=3, max_samples=600000)
    hp = SutaHParams()
    rec = [0, 1, 3]
    waves = [synth.wave(n, 340 + i) for i, n in enumerate((170000, 260000, 600000))]
    lv, iv, tv = eng.adapt_varlen(waves, 3, hp, record=rec)
    assert list(tv) == [531, 812, 1874]
    finals = [{n: eng.get_param(b, n) for n in eng.trainable_names()} for b in range(3)]
    for b, (l1, p1, t1) in enumerate(_singles(eng, waves, 3, hp, rec)):
        assert tv[b] == t1
        for r in rec:
            np.testing.assert_allclose(lv[r][b], l1[r], rtol=0, atol=logits_tol(hp.lr), err_msg=f"utt {b} step {r}")
            np.testing.assert_array_equal(iv[r][b], lv[r][b].argmax(-1))
        for n, v in p1.items():
            assert_params_close(finals[b][n], v, hp.lr, 3, name=f"utt {b} {n}")
    eng.close()


def test_c4_bench_layout_bf16():
    """Config C4 exactly as bench.py --only-c4 runs it: wav2vec2-large, bench.C4_BATCH x 128 000 samples, 20 SUTA
    steps, bf16 GEMMs, greedy ids only, in the bench's timed mode (the key's third call, a graph replay), pinned
    bitwise to an eager call on the same batch (_timed_mode_equals_eager).  That call's first / middle / last slots
    against the exact-fp32 engine adapting each utterance alone (bf16 tolerance of tests/parity.py: 2.5 % of
    max|ref|, greedy ids on >= 97 % of frames) at steps 0 / 1 / 5 / 20, and slot 0 against the CPU oracle at steps 0
    and 20.  The launch census of the first (eager) call shows the schedules this layout reaches: the linears on
    the 256 x 256 bf16-plane kernel (hbx) over ceil(B x 399 / 256) row tiles, the K = 32 lm_head input gradient on
    the 128 x 128 one over ceil(B x 399 / 128), the conv stack's per-utterance (Z = B) GEMMs on bf16 planes --
    forward and input gradients (conv-A rows, per-tap weight segments) on the four-phase 256 x 256 kernel (no
    conv-seg launch left on the 128 x 128 one), weight gradients (MN-contiguous planes) on the four-phase kernel's TN
    form (round 6; formerly the 128 x 128 hbt kernel) -- and the per-utterance feature-projection weight gradient.
    Reference main.py:181,205 (forward and backward through the encoder)."""
    from oracle import w2v2_cpu as W
    import os
    from tests.parity import BF16_LOGITS_RTOL_LARGE, assert_bf16_close
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    cfg = get_config("wav2vec2-large")
    sd = synth_weights(cfg)
    B, N, S = bench.C4_BATCH, 128000, 20
    rec = bench.C4_RECORD
    eng = SutaEngine(cfg, sd, device=0, max_batch=B, max_samples=N)
    eng.set_precision("bf16")
    hp = SutaHParams()
    warm = torch.from_numpy(synth.batch(N, B, start=0)).cuda()
    x = synth.batch(N, B, start=B)
    logits, ids, T, census = _timed_mode_equals_eager(eng, warm, torch.from_numpy(x).cuda(), S, hp, rec, _slots(B))
    assert T == 399
    txt = "\n".join(f"{k}: {v}" for k, v in sorted(census.items()))
    print(txt)
    gy = _row_tiles(B, T)
    z = f" z={B} "
    # the linears on the 256 x 256 kernel: N = 1024 (out-proj, FFN2, input gradients), 3072 (QKV), 4096 (the GELU /
    # GELU' linears FFN1 and the FFN2 input gradient, through the C^T epilogue)
    for gx in (4, 12, 16):
        assert any(k.startswith("grid hbx 256x256 ") and f" gx={gx} gy={_row_tiles(B, T, 256)} z=1 " in k
                   for k in census), (gx, txt)
    # the K = 32 lm_head input gradient (below hbx's K >= 128) on the 128 x 128 kernel
    assert any(k.startswith("grid hb 128x128 ") and f" gx=8 gy={gy} z=1 " in k for k in census), (gy, txt)
    # conv dX (conv-A rows, per-tap weight segments) and the conv forward: both on the four-phase 256 x 256 kernel
    # (round 5: the conv-seg input gradients left the 128 x 128 kernel), none of them on the 128 x 128 one
    assert any(k.startswith("hbx 256x256 ") and z in k and k.endswith(" conv-seg") for k in census), txt
    assert not any(k.startswith("hb ") and z in k and k.endswith(" conv-seg") for k in census), txt
    assert any(k.startswith("hbx 256x256 ") and z in k and "conv" not in k for k in census), txt
    assert any(k.startswith("hbt4 256x256 ") and z in k for k in census), txt             # conv dW (TN form)
    assert any(z in k and k.startswith(("gbf", "x6_1plane")) for k in census), txt
    eng.set_precision("fp32")
    for slot in _slots(B):
        ref, _, _ = eng.adapt(x[slot], S, hp, record=rec)
        for r in rec:
            assert_bf16_close(logits[r][slot], ref[r][0], 0.97, f"C4 slot {slot} step {r}", rtol=BF16_LOGITS_RTOL_LARGE)
            np.testing.assert_array_equal(ids[r][slot], logits[r][slot].argmax(-1))
        if slot == 0:
            o, _ = W.run_suta({k: torch.from_numpy(v) for k, v in sd.items()}, cfg, torch.from_numpy(x[0])[None], S,
                              record=[0, 20])
            for r in (0, 20):
                np.testing.assert_allclose(ref[r][0], o[r][0].numpy(), rtol=0, atol=5e-5, err_msg=f"fp32 vs oracle {r}")
                assert_bf16_close(logits[r][0], o[r][0].numpy(), 0.97, f"C4 slot 0 step {r} vs oracle",
                                  rtol=BF16_LOGITS_RTOL_LARGE)
    eng.close()


def test_minimal_length_utterance_in_ragged_batch():
    """T = 1 (400 samples: the shortest input the conv stack accepts) beside a 2 s utterance in one ragged call,
    against each alone; 399 samples is rejected by the host (no zero-frame utterance reaches the kernels)."""
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), device=0, max_batch=2, max_samples=32000)
    hp = SutaHParams()
    rec = [0, 2]
    waves = [synth.wave(32000, 360), synth.wave(400, 361)]
    lv, iv, tv = eng.adapt_varlen(waves, 2, hp, record=rec)
    assert list(tv) == [99, 1]
    for b, (l1, p1, t1) in enumerate(_singles(eng, waves, 2, hp, rec)):
        assert tv[b] == t1
        for r in rec:
            assert np.all(np.isfinite(lv[r][b]))
            # (rtol 1e-5 beside the absolute bound: the one-frame utterance's logits (|x| up to ~5) move by fp32
            # reordering between the ragged and the single-utterance tilings -- 3.4e-5 = 7e-6 relative measured)
            np.testing.assert_allclose(lv[r][b], l1[r], rtol=1e-5, atol=logits_tol(hp.lr), err_msg=f"utt {b} step {r}")
    with pytest.raises(RuntimeError, match="too short"):
        eng.adapt_varlen([synth.wave(32000, 362), synth.wave(399, 363)], 1, hp, record=[1])
    eng.close()
