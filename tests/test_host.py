"""CPU tier: host-side drop-in pieces — CTC decode, WER, corpus loaders, sharding, gloo gather."""
import json
import os
import wave

import numpy as np
import pytest
import torch

from suta_amd import data as D
from suta_amd import dist as S
from suta_amd.config import get_config
from suta_amd.decode import batch_decode, ctc_decode, edit_distance, wer, wer_counts
from suta_amd.main import build_parser, exp_name_of

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_ctc_decode_matches_hf_tokenizer_golden():
    cases = json.load(open(os.path.join(G, "g5_ctc_decode.json")))
    for c in cases:
        assert ctc_decode(c["ids"]) == c["text"], c["ids"]


def test_batch_decode_rows():
    ids = np.array([[0, 11, 11, 5, 15, 0, 15, 8], [4, 4, 18, 0, 0, 8, 8, 4]])
    assert batch_decode(ids) == ["HELLO", "WO"]


@pytest.mark.parametrize("ref,hyp,e", [("a b c d", "a x c", 2), ("a b", "a b", 0), ("a", "", 1), ("", "a b", 2),
                                       ("the cat sat", "cat sat on the", 3)])
def test_edit_distance(ref, hyp, e):
    assert edit_distance(ref.split(), hyp.split()) == e


def test_corpus_wer_is_sum_of_edits_over_sum_of_words():
    # parity unpinned against jiwer itself (not installed); pinned by hand-counted cases
    assert wer(["hello world", "foo"], ["hello", "foo bar"]) == pytest.approx(2 / 3)
    assert wer_counts(["a  b   c"], [" a b c "]) == (0, 3)        # jiwer default transform: collapse + strip
    with pytest.raises(ValueError):
        wer([""], ["x"])


def _write_wav(path, x, sr=16000):
    with wave.open(str(path), "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(sr)
        f.writeframes((np.clip(x, -1, 1) * 32767).astype("<i2").tobytes())


def test_chime_loader_order_and_texts(tmp_path):
    apath = tmp_path / "data/audio/16kHz/enhanced"
    tpath = tmp_path / "data/transcriptions"
    rng = np.random.default_rng(0)
    texts = {}
    for sub in ("et05_bus_real", "et05_caf_simu", "et05_ped_real"):
        (apath / sub).mkdir(parents=True)
        (tpath / sub).mkdir(parents=True)
        for i in range(3):
            name = f"F0{i}_{sub[5:8].upper()}_{i}"
            _write_wav(apath / sub / f"{name}.wav", rng.standard_normal(1600 * (i + 1)) * 0.1)
            t = " ".join(["WORD"] * (i + len(sub) % 3 + 1))
            (tpath / sub / f"{name}.trn").write_text(f"{name} {t}\n")
            texts[name] = t
    ds = D.CHiMEDataset(None, 1, str(tmp_path))
    assert len(ds) == 6                                            # ped_real is not one of the 7 subsets
    lens = [len(t) for t in ds.text]
    assert lens == sorted(lens, reverse=True)
    for f, t in zip(ds.file_list, ds.text):
        assert texts[f.stem] == t


def test_chime_subsets_flag(tmp_path):
    """Config C3 'eval-real' (BASELINE.json): --chime_subsets restricts the reference's hard-coded 7 et05 subsets
    (corpus/CHiME.py:27); the default is exactly that list."""
    assert D.CHiMEDataset.SUBSETS == ["et05_bus_real", "et05_bus_simu", "et05_caf_real", "et05_caf_simu",
                                      "et05_ped_simu", "et05_str_real", "et05_str_simu"]
    assert build_parser().parse_args([]).chime_subsets is None
    apath = tmp_path / "data/audio/16kHz/enhanced"
    tpath = tmp_path / "data/transcriptions"
    rng = np.random.default_rng(5)
    for sub in D.CHiMEDataset.SUBSETS:
        (apath / sub).mkdir(parents=True)
        (tpath / sub).mkdir(parents=True)
        name = f"F01_{sub[5:8].upper()}_{sub[-4:]}"
        _write_wav(apath / sub / f"{name}.wav", rng.standard_normal(1600) * 0.1)
        (tpath / sub / f"{name}.trn").write_text(f"{name} A WORD\n")
    everything, _ = D.create_dataset(None, "chime", str(tmp_path), 1)
    assert len(everything) == 7
    real = "et05_bus_real,et05_caf_real,et05_str_real"
    a = build_parser().parse_args(["--dataset_name", "chime", "--chime_subsets", real])
    ds, _ = D.create_dataset(None, "chime", str(tmp_path), 1, a.chime_subsets.split(","))
    assert sorted(f.parent.name for f in ds.file_list) == real.split(",")
    ld = D.load_dataset(None, "chime", str(tmp_path), 1, 0.0, chime_subsets=["et05_ped_simu"])
    assert [os.path.basename(os.path.dirname(str(it[0][0]))) for it in ld.raw_batches()] == ["et05_ped_simu"]
    with pytest.raises(ValueError):
        D.create_dataset(None, "chime", str(tmp_path), 1, ["et05_ped_real"])     # not a reference subset
    with pytest.raises(ValueError):
        D.create_dataset(None, "librispeech", str(tmp_path), 1, ["et05_bus_real"])


def test_audio_reader_truncates_and_noise_is_deterministic(tmp_path):
    x = np.random.default_rng(1).standard_normal(700000) * 0.05
    _write_wav(tmp_path / "a.wav", x)
    r0 = D.AudioReader(0.0)(tmp_path / "a.wav")
    assert r0.shape == (600000,)
    a = D.AudioReader(0.01)(tmp_path / "a.wav")
    b = D.AudioReader(0.01)(tmp_path / "a.wav")
    assert np.array_equal(a, b) and not np.array_equal(a, r0)
    assert abs(np.std(a - r0) - 0.01) < 1e-3


def test_collate_sorts_bucket_by_length(tmp_path):
    for i, n in enumerate((1000, 3000, 2000)):
        _write_wav(tmp_path / f"u{i}.wav", np.zeros(n))
    items = [(str(tmp_path / f"u{i}.wav"), f"T{i}") for i in range(3)]
    lens, wavs, texts, files = D.collect_audio_batch(items, D.AudioReader())
    assert lens == (3000, 2000, 1000) and texts == ("T1", "T2", "T0")


def test_cli_flags_and_exp_name():
    a = build_parser().parse_args("--asr facebook/wav2vec2-base-960h --steps 10 --dataset_name librispeech "
                                  "--dataset_dir /d --temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir exps "
                                  "--lr 2e-5 --non_blank --train_feature --extra_noise 0.01".split())
    assert exp_name_of(a) == ("librispeech_0.3_10_2.5_wav2vec2-base-960h_non_blankTrue_noise_0.01_rew_True_div_0.0"
                              "_bias_False_feat_True_all_False_LN_True")


def test_sdpl_cli_defaults_and_exp_name():
    """main_SDPL.py:218-241 defaults and its exp_name (main_SDPL.py:266)."""
    a = build_parser(sdpl=True).parse_args("--asr facebook/wav2vec2-base-960h --dataset_name chime --episodic "
                                           "--train_feature --pl_coef 0.5".split())
    assert (a.steps, a.opt, a.em_coef, a.lr, a.pl_coef) == (10, "Adam", 1.0, 1e-4, 0.5)
    assert exp_name_of(a, sdpl=True) == ("chime_1.0_10_2.5_wav2vec2-base-960h_non_blankFalse_noise_0.0_rew_False_"
                                         "div_0.0_bias_False_feat_True_se__pl_0.5")


def test_sdpl_pseudo_label_target_rules():
    from oracle.w2v2_cpu import pseudo_label_target
    # collapse repeats, drop blanks, strip leading/trailing delimiters, keep inner ones
    assert pseudo_label_target([4, 0, 4, 5, 5, 0, 5, 4, 0, 4, 6, 4, 4]) == [5, 5, 4, 4, 6]
    assert pseudo_label_target([0, 0, 0]) == []
    with pytest.raises(KeyError):
        pseudo_label_target([5, 3, 6])


def test_lpt_shard_balances_and_covers():
    rng = np.random.default_rng(3)
    costs = list(rng.uniform(1, 30, size=101))
    for world in (1, 2, 4, 8):
        sh = S.lpt_shard(costs, world)
        assert sorted(i for s in sh for i in s) == list(range(101))
        loads = [sum(costs[i] for i in s) for s in sh]
        assert max(loads) - min(loads) <= max(costs) + 1e-9


def test_utterance_cost_monotone():
    cfg = get_config("wav2vec2-base")
    assert S.utterance_cost(32000, cfg, 10) < S.utterance_cost(128000, cfg, 10)


def test_gloo_world2_reduces_wer_counts():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    from tests._dist_worker import gloo_reduce_worker
    ps = [ctx.Process(target=gloo_reduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=90) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, red, ranks in out:
        assert red == {"0": (3, 30), "10": (1, 10)}
        assert ranks == [0, 1]


@pytest.mark.parametrize("min_fill", [0.0, 0.35])
def test_ragged_groups_partition(min_fill):
    """Driver grouping: an in-order partition of the length-sorted utterances, every group within
    gpu_batch and the padded-audio budget (a single over-long utterance stands alone); the padding-
    minimising partition pads no more than the greedy one on the bench's length mix."""
    from suta_amd.main import LAYOUT_QUANTUM as Q, ragged_groups
    rng = np.random.default_rng(20260415)
    ns = np.sort((np.clip(rng.lognormal(np.log(6.5), 0.6, 256), 1.5, 35.0) * 16000).astype(np.int64))
    budget = 512 * 16000
    groups = ragged_groups(list(ns), 64, budget, min_fill)
    assert [j for g in groups for j in g] == list(range(len(ns)))
    width = lambda g: -(-int(ns[g[-1]]) // Q) * Q  # noqa: E731
    for g in groups:
        assert len(g) <= 64
        assert len(g) == 1 or len(g) * width(g) <= budget
    padded = sum(len(g) * width(g) for g in groups)
    greedy = sum(len(g) * width(g) for g in ragged_groups(list(ns), 64, budget, 0.0))
    assert padded <= greedy
    assert ragged_groups([700000], 4, budget, min_fill) == [[0]]
    assert ragged_groups([], 4, budget, min_fill) == []


def _per_utt_lines(out):
    return [ln for ln in out.splitlines() if ln.startswith(("original WER:", "adapt-"))]


@pytest.mark.parametrize("corpus,noise", [("chime", 0.0), ("librispeech", 0.0), ("librispeech", 0.01),
                                          ("chime", 0.01), ("commonvoice", 0.01)])
def test_driver_world2_gloo_equals_world1(tmp_path, corpus, noise):
    """The real driver (suta_amd/main.py) as 2 gloo ranks with a deterministic stand-in engine whose ids
    depend on every sample it is given: LPT sharding by decoded length, the count all_reduce and the
    object gather give the world-1 counts -- with --extra_noise too, since each utterance's noise is keyed
    on its dataset index -- and rank 0 alone prints the loader / collect_params / per-utterance lines, in
    the world-1 (dataset) order."""
    from tests import corpus_fixtures as CF
    from tests.multirank import run_ranks
    if corpus == "chime":
        CF.chime(tmp_path, n=5)
        flags = f"--dataset_name chime --dataset_dir {tmp_path}"
    elif corpus == "commonvoice":
        CF.commonvoice(tmp_path)
        flags = f"--dataset_name commonvoice --dataset_dir {tmp_path}"
    else:
        CF.librispeech(tmp_path)
        flags = f"--dataset_name librispeech --dataset_dir {tmp_path}"
    argv = (f"--asr tiny-group --synthetic_weights --steps 10 {flags} --temp 2.5 --episodic --em_coef 0.3 "
            f"--reweight --log_dir {tmp_path}/exps --lr 5e-4 --non_blank --train_feature --gpu_batch 2 "
            f"--dist_backend gloo --extra_noise {noise}").split()
    (c1,), (o1,) = run_ranks(1, argv, tmp_path, fake=True)
    c2, o2 = run_ranks(2, argv, tmp_path, fake=True)
    assert c2[0] == c2[1] == c1
    assert _per_utt_lines(o2[0]) == _per_utt_lines(o1) and len(_per_utt_lines(o1)) > 0
    assert _per_utt_lines(o2[1]) == []
    assert "TTA-10 WER:" in o2[0] and "TTA-10 WER:" not in o2[1]
    for marker in ("[INFO]    There are", "wav2vec2.feature_extractor.conv_layers.0.conv", "[INFO]    optimizer:",
                   "['wav2vec2.feature_extractor.conv_layers.0.conv.weight'"):
        assert marker in o1 and marker in o2[0] and marker not in o2[1], marker


def test_noise_is_keyed_on_dataset_index(tmp_path):
    """Loading any subset of the loader batches, in any order, gives each utterance the audio a full
    pass gives it (the multi-rank invariance of --extra_noise)."""
    from tests import corpus_fixtures as CF
    CF.librispeech(tmp_path)
    full = D.load_dataset(None, "librispeech", str(tmp_path), 1, 0.01)
    ref = {i: b[1][0] for i, b in full.iter_collated(range(len(full)))}
    part = D.load_dataset(None, "librispeech", str(tmp_path), 1, 0.01)
    sub = list(range(len(part)))[::-2]
    got = {i: b[1][0] for i, b in part.iter_collated(sub, workers=3, window=2)}
    assert sub and all(np.array_equal(got[i], ref[i]) for i in sub)
    clean = D.load_dataset(None, "librispeech", str(tmp_path), 1, 0.0)
    c = {i: b[1][0] for i, b in clean.iter_collated(range(len(clean)))}
    assert all(abs(np.std(ref[i] - c[i]) - 0.01) < 2e-3 for i in ref)
    assert not np.array_equal(ref[0] - c[0], (ref[1] - c[1])[:len(c[0])])


def test_bucket_indices_follow_getitem(tmp_path):
    from tests import corpus_fixtures as CF
    CF.chime(tmp_path, n=5)
    ld = D.load_dataset(None, "chime", str(tmp_path), 2, 0.0)
    assert ld.batch_indices() == [[0, 1], [2, 3], [3, 4]]   # the last bucket moves back (CHiME.py __getitem__)
    files = [[str(f) for f, _ in b] for b in ld.raw_batches()]
    ds = D.CHiMEDataset(None, 1, str(tmp_path))
    assert files == [[str(ds.file_list[i]) for i in b] for b in ld.batch_indices()]


def test_collect_params_names_match_reference_golden():
    """suta_amd.modules restates named_modules() and the reference collect_params walk: the printed module
    names and param_names equal what the reference's own collect_params produced on transformers'
    Wav2Vec2ForCTC (golden g8), for tiny / base / large geometries and all flag pairs."""
    import json
    from suta_amd.modules import collect_params
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "g8_collect_params.json")))
    assert set(g) == {"tiny-group", "tiny-layer", "wav2vec2-base", "wav2vec2-large"}
    for name, ent in g.items():
        for key, names in ent["param_names"].items():
            printed, got = collect_params(get_config(name), "bias_only=True" in key, "train_feature=True" in key)
            assert printed == ent["printed"], name
            assert got == names, (name, key)


def test_truncation_lines_in_load_order(tmp_path, capsys):
    """data.py:19-21: the reader prints the cut message and the new shape as torch.Size, in load order."""
    x = np.random.default_rng(3).standard_normal(650000) * 0.05
    _write_wav(tmp_path / "a.wav", x)
    _write_wav(tmp_path / "b.wav", x[:1000])
    log = []
    D.collect_audio_batch([(str(tmp_path / "a.wav"), "A"), (str(tmp_path / "b.wav"), "B")], D.AudioReader(), log=log)
    assert log == [f"{tmp_path / 'a.wav'} has len torch.Size([650000]), truncate to 600000", "torch.Size([600000])"]
    D.AudioReader()(str(tmp_path / "a.wav"))
    assert capsys.readouterr().out.splitlines() == log


def test_driver_refuses_to_shard_non_episodic(tmp_path):
    from tests import corpus_fixtures as CF
    from tests.multirank import run_ranks
    CF.chime(tmp_path, n=2)
    argv = (f"--asr tiny-group --synthetic_weights --steps 2 --dataset_name chime --dataset_dir {tmp_path} "
            f"--log_dir {tmp_path}/exps --dist_backend gloo").split()
    with pytest.raises(AssertionError, match="cannot be sharded"):
        run_ranks(2, argv, tmp_path, fake=True)


def test_lpt_cost_uses_decoded_length(tmp_path):
    """FLAC files compress: the shard cost comes from STREAMINFO, not the file size."""
    from suta_amd.data import decoded_length
    from tests import corpus_fixtures as CF
    CF.librispeech(tmp_path, lengths=(6000, 9100))
    fl = sorted((tmp_path / "test-other").rglob("*.flac"))
    assert [decoded_length(str(f)) for f in fl] == [6000, 9100]
    CF.chime(tmp_path / "c", n=2)
    wv = sorted((tmp_path / "c").rglob("*.wav"))
    assert [decoded_length(str(f)) for f in wv] == [6000, 7500]


def test_legacy_weight_norm_names_in_safetensors(tmp_path):
    """Checkpoints converted from older torch name the pos-conv weight norm weight_g / weight_v; both
    checkpoint formats map them to the parametrizations names the engine expects."""
    import json
    from safetensors.numpy import save_file
    from suta_amd.weights import load_hf_checkpoint, synth_weights
    cfg = get_config("tiny-group")
    sd = synth_weights(cfg)
    pre = "wav2vec2.encoder.pos_conv_embed.conv."
    legacy = dict(sd)
    legacy[pre + "weight_g"] = legacy.pop(pre + "parametrizations.weight.original0")
    legacy[pre + "weight_v"] = legacy.pop(pre + "parametrizations.weight.original1")
    json.dump(cfg, open(tmp_path / "config.json", "w"))
    save_file(legacy, str(tmp_path / "model.safetensors"))
    got = load_hf_checkpoint(str(tmp_path))
    assert sorted(got) == sorted(sd)
    assert np.array_equal(got[pre + "parametrizations.weight.original1"], sd[pre + "parametrizations.weight.original1"])


def test_resolve_scheduler_and_optimizer_flags():
    """--scheduler resolves the reference's eval'd dotted name (main.py:20-21) to StepLR's (step_size, gamma);
    anything else is refused, as the reference's call with step_size / gamma keywords would fail for it."""
    from suta_amd import main as M
    from suta_amd.engine import SutaHParams
    assert M.resolve_scheduler(None) == (0, 0.7)
    assert M.resolve_scheduler("torch.optim.lr_scheduler.StepLR") == (1, 0.7)
    for bad in ("StepLR", "torch.optim.lr_scheduler.ExponentialLR", "os.system"):
        with pytest.raises(SystemExit):
            M.resolve_scheduler(bad)
    hp = SutaHParams(optimizer="SGD", lr_step_size=1).to_c()
    assert (hp.optimizer, hp.lr_step_size, abs(hp.lr_gamma - 0.7) < 1e-7) == (1, 1, True)
    with pytest.raises(ValueError):
        SutaHParams(optimizer="RMSprop").to_c()


def test_budget_clamped_to_free_device_memory():
    """--gpu_budget_s defaults are sized for the 288 GB MI355X; on less free memory the driver clamps them."""
    from suta_amd import main as M
    base = get_config("wav2vec2-base")
    assert M.workspace_bytes_per_audio_s(base) >= 0.36e9 / 8          # the measured 45 MB/s is covered
    assert M.clamp_budget(1312.0, base, 280e9) == 1312.0             # an MI355X keeps the default
    small = M.clamp_budget(1312.0, base, 16e9)
    assert small < 1312.0 and small * M.workspace_bytes_per_audio_s(base) <= 0.7 * 16e9 + 1
    assert M.clamp_budget(1312.0, base, None) == 1312.0


def test_engine_fixed_footprint_counts_weights_planes_and_slots():
    """The budget clamp first subtracts each engine's fixed device footprint (advisor r5): the fp32 weights, the bf16
    weight planes in bf16 mode, and per slot the trainable tensors, gradients and Adam moments."""
    from suta_amd import main as M
    from suta_amd.weights import synth_weights
    cfg = get_config("tiny-group")
    w = synth_weights(cfg)
    wb = 4.0 * sum(v.size for v in w.values())
    f1 = M.engine_fixed_bytes(cfg, w, 1)
    f8 = M.engine_fixed_bytes(cfg, w, 8)
    assert f1 > wb and f8 > f1
    slot = (f8 - f1) / 7                                      # 4 fp32 arrays per slot of the trainable tensors
    assert slot % 16 == 0 and slot > 0
    assert M.engine_fixed_bytes(cfg, w, 1, "bf16") == pytest.approx(f1 + wb)
