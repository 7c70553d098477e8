"""GPU tier: the main.py-compatible driver end to end on a synthetic CHiME-layout corpus.

Transcripts and WER are checked against the CPU oracle run on the same normalised audio.
"""
import os
import wave

import numpy as np
import pytest
import torch

from suta_amd import main as M
from suta_amd.config import get_config
from suta_amd.data import AudioReader
from suta_amd.decode import batch_decode, wer_counts
from suta_amd.synth import normalize
from suta_amd.weights import synth_weights

pytestmark = pytest.mark.gpu


def _corpus(root, n=4):
    apath = root / "data/audio/16kHz/enhanced/et05_bus_real"
    tpath = root / "data/transcriptions/et05_bus_real"
    apath.mkdir(parents=True)
    tpath.mkdir(parents=True)
    rng = np.random.default_rng(11)
    words = ["HELLO", "WORLD", "THE", "CAT", "SAT", "ON", "A", "MAT"]
    for i in range(n):
        x = rng.standard_normal(6000 + 1500 * i) * 0.1
        with wave.open(str(apath / f"U{i}.wav"), "wb") as f:
            f.setnchannels(1)
            f.setsampwidth(2)
            f.setframerate(16000)
            f.writeframes((np.clip(x, -1, 1) * 32767).astype("<i2").tobytes())
        (tpath / f"U{i}.trn").write_text(f"U{i} " + " ".join(rng.choice(words, size=3 + i)) + "\n")


@pytest.mark.parametrize("gpu_batch,engines", [(1, 1), (16, 2), (2, 2), (2, 3)])
def test_cli_end_to_end_matches_oracle(tmp_path, capsys, gpu_batch, engines):
    """gpu_batch 16: the 4 utterances (different lengths) run as one ragged batch; gpu_batch 2 with 2 / 3 engines:
    the ragged groups adapted concurrently by several engines (own streams, host threads), results by utterance."""
    from oracle import w2v2_cpu as W
    _corpus(tmp_path)
    args = (f"--asr tiny-group --synthetic_weights --steps 10 --dataset_name chime --dataset_dir {tmp_path} "
            f"--temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps --lr 5e-4 --non_blank "
            f"--train_feature --extra_noise 0 --gpu_batch {gpu_batch} --gpu_engines {engines}").split()
    counts = M.main(args)
    out = capsys.readouterr().out
    assert "original WER: " in out and "adapt-10 WER: " in out and "TTA-10 WER:" in out
    a = M.build_parser().parse_args(args)
    log = open(os.path.join(a.log_dir, M.exp_name_of(a))).read().splitlines()
    assert log[0].startswith("original WER: ") and log[4].startswith("TTA-10 WER: ")
    assert os.path.exists(os.path.join(a.log_dir, M.exp_name_of(a) + ".csv"))

    # oracle: same audio, same flags
    cfg = get_config("tiny-group")
    sd = {k: torch.from_numpy(v) for k, v in synth_weights(cfg).items()}
    from suta_amd.data import CHiMEDataset
    ds = CHiMEDataset(None, 1, str(tmp_path))
    reader = AudioReader(0.0)
    hyps = {k: [] for k in (0, 1, 3, 5, 10)}
    for f, t in zip(ds.file_list, ds.text):
        x = torch.from_numpy(normalize(reader(str(f))))[None]
        lg, _ = W.run_suta(sd, cfg, x, 10, lr=5e-4, record=[0, 1, 3, 5, 10])
        for k in hyps:
            hyps[k].append(batch_decode(lg[k].argmax(-1).numpy())[0])
    for k in hyps:
        assert tuple(counts[str(k)]) == wer_counts(list(ds.text), hyps[k]), k


def test_sdpl_cli_end_to_end(tmp_path, capsys):
    """main_SDPL.py drop-in: runs, prints the reference's lines, writes its log; the vanilla (step 0)
    WER equals the oracle's.  Adapted WERs follow pseudo-label trajectories that a single greedy flip
    can redirect (tests/parity.sdpl_logits_tol), so they are checked for presence, not equality."""
    import json
    from safetensors.numpy import save_file
    from oracle import w2v2_cpu as W
    _corpus(tmp_path)
    # a local checkpoint whose greedy path avoids <s>, </s>, <unk> (the reference raises KeyError there)
    cfg = get_config("tiny-group")
    sdn = synth_weights(cfg)
    sdn["lm_head.bias"][1:4] -= 30.0
    ck = tmp_path / "ckpt"
    ck.mkdir()
    json.dump(cfg, open(ck / "config.json", "w"))
    save_file(sdn, str(ck / "model.safetensors"))
    args = (f"--asr {ck} --steps 10 --dataset_name chime --dataset_dir {tmp_path} "
            f"--episodic --log_dir {tmp_path}/exps --train_feature --pl_coef 1").split()
    counts = M.main(args, sdpl=True)
    out = capsys.readouterr().out
    assert "'<pad>': 0" in out and "pl_coef = 1.0" in out and "adapt-10 WER: " in out and "TTA-10 WER:" in out
    a = M.build_parser(sdpl=True).parse_args(args)
    log = open(os.path.join(a.log_dir, M.exp_name_of(a, sdpl=True))).read().splitlines()
    assert log[0].startswith("original WER: ") and log[-1] == "pl_coef = 1.0"
    sd = {k: torch.from_numpy(v) for k, v in sdn.items()}
    from suta_amd.data import CHiMEDataset
    ds = CHiMEDataset(None, 1, str(tmp_path))
    reader = AudioReader(0.0)
    hyp0 = []
    for f in ds.file_list:
        x = torch.from_numpy(normalize(reader(str(f))))[None]
        hyp0.append(batch_decode(W.forward(sd, cfg, x).argmax(-1).numpy())[0])
    assert tuple(counts["0"]) == wer_counts(list(ds.text), hyp0)
    for k in (1, 3, 5, 10):
        assert counts[str(k)][1] == counts["0"][1]


def _oracle_counts(ds_files, ds_texts, cfg_name, steps, lr, extra_noise=0.0, **opt):
    from oracle import w2v2_cpu as W
    cfg = get_config(cfg_name)
    sd = {k: torch.from_numpy(v) for k, v in synth_weights(cfg).items()}
    reader = AudioReader(extra_noise)
    rec = [0] + [c for c in (1, 3, 5, 10) if c <= steps]
    hyps = {k: [] for k in rec}
    for i, f in enumerate(ds_files):   # i = dataset index = the utterance's noise key
        x = torch.from_numpy(normalize(reader(str(f), i)))[None]
        lg, _ = W.run_suta(sd, cfg, x, steps, lr=lr, record=rec, **opt)
        for k in rec:
            hyps[k].append(batch_decode(lg[k].argmax(-1).numpy())[0])
    return {k: wer_counts(list(ds_texts), hyps[k]) for k in rec}


def test_cli_world2_gloo_on_one_gpu(tmp_path):
    """Config C3's multi-rank plumbing on the one-GPU box: the real driver as 2 processes sharing
    device 0 over gloo (LPT shards by decoded length, count all_reduce, transcript gather, rank-0
    ordered print).  Counts equal the world-1 run and the CPU oracle; rank 1 prints no utterance line."""
    from tests import corpus_fixtures as CF
    from tests.multirank import run_ranks
    from suta_amd.data import CHiMEDataset
    CF.chime(tmp_path, n=5)
    argv = (f"--asr tiny-group --synthetic_weights --steps 10 --dataset_name chime --dataset_dir {tmp_path} "
            f"--temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps --lr 5e-4 --non_blank "
            f"--train_feature --extra_noise 0 --gpu_batch 2 --device 0 --dist_backend gloo").split()
    (c1,), (o1,) = run_ranks(1, argv, tmp_path, fake=False)
    c2, o2 = run_ranks(2, argv, tmp_path, fake=False)
    assert c2[0] == c2[1] == c1
    lines = lambda o: [ln for ln in o.splitlines() if ln.startswith(("original WER:", "adapt-"))]  # noqa: E731
    assert lines(o2[0]) == lines(o1) and lines(o2[1]) == []
    ds = CHiMEDataset(None, 1, str(tmp_path))
    ref = _oracle_counts(ds.file_list, ds.text, "tiny-group", 10, 5e-4)
    for k, v in ref.items():
        assert c1[str(k)] == v, k


def test_cli_librispeech_flac_ls_flags(tmp_path, capsys):
    """scripts/LS.sh (LS + 0.01 noise) flags on a LibriSpeech-layout FLAC corpus (FLAC decoded by
    libsuta_audio), w2v2-base shapes with seeded weights: the driver's corpus WER counts equal the CPU
    oracle's on the same decoded, noised, normalised audio -- run in-process (world 1) and as 2 gloo
    ranks sharing device 0 (config C2/C3's sharded path: LPT shards, per-utterance noise keyed on the
    dataset index, count all_reduce); rank 1 prints nothing of the job's log."""
    from tests import corpus_fixtures as CF
    from tests.multirank import run_ranks
    from suta_amd.data import LibriDataset
    CF.librispeech(tmp_path)
    args = (f"--asr facebook/wav2vec2-base-960h --synthetic_weights --steps 10 --dataset_name librispeech "
            f"--dataset_dir {tmp_path} --temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps "
            f"--lr 2e-5 --non_blank --train_feature --extra_noise 0.01").split()
    counts = M.main(args)
    out = capsys.readouterr().out
    assert out.count("original WER: ") >= 5 and "TTA-10 WER:" in out
    ds = LibriDataset(None, 1, str(tmp_path))
    ref = _oracle_counts(ds.file_list, ds.text, "wav2vec2-base", 10, 2e-5, extra_noise=0.01)
    for k, v in ref.items():
        assert tuple(counts[str(k)]) == v, k
    c2, o2 = run_ranks(2, args + "--gpu_batch 2 --device 0 --dist_backend gloo".split(), tmp_path, fake=False)
    assert c2[0] == c2[1] == {k: tuple(v) for k, v in counts.items()}
    per = lambda o: [ln for ln in o.splitlines() if ln.startswith(("original WER:", "adapt-"))]  # noqa: E731
    assert per(o2[0]) == per(out) and per(o2[1]) == [] and "[INFO]" not in o2[1]


def test_cli_commonvoice_mp3_cv_flags(tmp_path, capsys):
    """scripts/CV.sh flags on a CommonVoice-layout corpus (test.tsv + clips/*.mp3, MPEG-1 Layer III 44.1 kHz decoded
    by libsuta_audio's MP3 decoder and resampled to 16 kHz), w2v2-base shapes with seeded weights: corpus WER counts
    equal the CPU oracle's on the same decoded audio, in-process and as 2 gloo ranks sharing device 0."""
    from tests import corpus_fixtures as CF
    from tests.multirank import run_ranks
    from suta_amd.data import CVDataset
    CF.commonvoice(tmp_path)
    args = (f"--asr facebook/wav2vec2-base-960h --synthetic_weights --steps 10 --dataset_name commonvoice "
            f"--dataset_dir {tmp_path} --temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps "
            f"--lr 2e-5 --non_blank --train_feature --extra_noise 0").split()
    counts = M.main(args)
    out = capsys.readouterr().out
    assert out.count("original WER: ") >= 5 and "TTA-10 WER:" in out
    ds = CVDataset(None, 1, str(tmp_path))
    ref = _oracle_counts(ds.file_list, ds.text, "wav2vec2-base", 10, 2e-5)
    for k, v in ref.items():
        assert tuple(counts[str(k)]) == v, k
    c2, _ = run_ranks(2, args + "--gpu_batch 2 --device 0 --dist_backend gloo".split(), tmp_path, fake=False)
    assert c2[0] == c2[1] == {k: tuple(v) for k, v in counts.items()}


def test_cli_chime_base_world2(tmp_path, capsys):
    """Config C3 (w2v2-base on the CHiME layout, utterance-sharded): 2 gloo ranks on device 0 give the
    world-1 counts, which equal the oracle's."""
    from tests import corpus_fixtures as CF
    from tests.multirank import run_ranks
    from suta_amd.data import CHiMEDataset
    CF.chime(tmp_path, n=4)
    args = (f"--asr facebook/wav2vec2-base-960h --synthetic_weights --steps 10 --dataset_name chime "
            f"--dataset_dir {tmp_path} --temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps "
            f"--lr 2e-5 --non_blank --train_feature --extra_noise 0.005").split()
    counts = M.main(args)
    capsys.readouterr()
    c2, _ = run_ranks(2, args + "--gpu_batch 2 --device 0 --dist_backend gloo".split(), tmp_path, fake=False)
    assert c2[0] == c2[1] == {k: tuple(v) for k, v in counts.items()}
    ds = CHiMEDataset(None, 1, str(tmp_path))
    ref = _oracle_counts(ds.file_list, ds.text, "wav2vec2-base", 10, 2e-5, extra_noise=0.005)
    for k, v in ref.items():
        assert tuple(counts[str(k)]) == v, k


def test_cli_ted_long_utterances_ragged(tmp_path, capsys):
    """Config C5's path on one GPU: a TED-layout corpus of long utterances (T = 531 .. 1874 frames, one
    cut at the 600 000-sample cap) adapted by the driver as one ragged batch (--gpu_batch 64) on the
    flash attention kernels; corpus WER counts equal the CPU oracle's."""
    from tests import corpus_fixtures as CF
    from suta_amd.data import TedDataset
    CF.ted(tmp_path)
    args = (f"--asr facebook/wav2vec2-base-960h --synthetic_weights --steps 3 --dataset_name ted "
            f"--dataset_dir {tmp_path} --temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps "
            f"--lr 2e-5 --non_blank --train_feature --extra_noise 0 --gpu_batch 64").split()
    counts = M.main(args)
    out = capsys.readouterr().out
    assert out.count("original WER: ") >= 4 and out.count("adapt-3 WER:") == 4
    ds = TedDataset(None, 1, str(tmp_path))
    assert len(ds.file_list) == 4
    ref = _oracle_counts(ds.file_list, ds.text, "wav2vec2-base", 3, 2e-5)
    for k, v in ref.items():
        assert tuple(counts[str(k)]) == v, k


@pytest.mark.parametrize("opt,lr", [("AdamW", "5e-4"), ("SGD", "2e-2")])
def test_cli_scheduler_steplr(tmp_path, capsys, opt, lr):
    """--scheduler torch.optim.lr_scheduler.StepLR (main.py:20-21, 207-208; lr * 0.7^i, restored per utterance) with
    --opt AdamW / SGD through the drop-in driver, one ragged batch: corpus WER counts equal the CPU oracle's under the
    same optimizer and schedule (oracle pinned to the reference's own runs by g9); the stdout / log lines name it."""
    from tests import corpus_fixtures as CF
    from suta_amd.data import CHiMEDataset
    CF.chime(tmp_path, n=4)
    args = (f"--asr tiny-group --synthetic_weights --steps 10 --dataset_name chime --dataset_dir {tmp_path} "
            f"--temp 2.5 --episodic --em_coef 0.3 --reweight --log_dir {tmp_path}/exps --lr {lr} --non_blank "
            f"--train_feature --extra_noise 0 --gpu_batch 16 --opt {opt} "
            f"--scheduler torch.optim.lr_scheduler.StepLR").split()
    counts = M.main(args)
    out = capsys.readouterr().out
    assert "[INFO]    scheduler: torch.optim.lr_scheduler.StepLR" in out and f"optim = {opt}" in out
    a = M.build_parser().parse_args(args)
    log = open(os.path.join(a.log_dir, M.exp_name_of(a))).read().splitlines()
    assert "scheduler = <torch.optim.lr_scheduler.StepLR object>" in log
    ds = CHiMEDataset(None, 1, str(tmp_path))
    ref = _oracle_counts(ds.file_list, ds.text, "tiny-group", 10, float(lr), opt=opt, lr_step_size=1)
    for k, v in ref.items():
        assert tuple(counts[str(k)]) == v, k
    with pytest.raises(SystemExit):
        M.main(args[:-1] + ["torch.optim.lr_scheduler.ExponentialLR"])
