"""Synthetic corpora in the reference loaders' directory layouts (test infrastructure).

* chime(root): CHiME-3 enhanced 16 kHz WAVs + .trn transcripts (reference corpus/CHiME.py:9-49)
* librispeech(root): LibriSpeech test-other FLAC files + <spk>-<chapter>.trans.txt
  (reference corpus/librispeech.py:8-39), encoded by tests/flac_spec_encoder.py
* commonvoice(root): CommonVoice test.tsv + clips/*.mp3 (reference corpus/commonvoice.py:27-42), MPEG-1
  Layer III 44.1 kHz mono frames written by tests/mp3_builder.py
"""
import wave

import numpy as np

from tests import flac_spec_encoder as E
from tests import mp3_builder as M

WORDS = ["HELLO", "WORLD", "THE", "CAT", "SAT", "ON", "A", "MAT"]


def chime(root, n=4, base=6000, step=1500, seed=11):
    apath = root / "data/audio/16kHz/enhanced/et05_bus_real"
    tpath = root / "data/transcriptions/et05_bus_real"
    apath.mkdir(parents=True)
    tpath.mkdir(parents=True)
    rng = np.random.default_rng(seed)
    for i in range(n):
        x = rng.standard_normal(base + step * i) * 0.1
        with wave.open(str(apath / f"U{i}.wav"), "wb") as f:
            f.setnchannels(1)
            f.setsampwidth(2)
            f.setframerate(16000)
            f.writeframes((np.clip(x, -1, 1) * 32767).astype("<i2").tobytes())
        (tpath / f"U{i}.trn").write_text(f"U{i} " + " ".join(rng.choice(WORDS, size=3 + i)) + "\n")


def librispeech(root, lengths=(6000, 9100, 7300, 12000, 4000), seed=12):
    """test-other/<spk>/<chapter>/<spk>-<chapter>-<utt>.flac, 16-bit mono, LPC and fixed subframes."""
    rng = np.random.default_rng(seed)
    by_dir = {}
    for i, n in enumerate(lengths):
        spk, ch = 100 + i % 2, 7
        d = root / "test-other" / str(spk) / str(ch)
        d.mkdir(parents=True, exist_ok=True)
        name = f"{spk}-{ch}-{i:04d}"
        x = np.clip(rng.standard_normal(n) * 0.1, -1, 1)
        ref = np.round(x * 32767).astype(np.int64)[None]
        frames = E.simple_frames(n, 1, blocksize=4096, kind="lpc" if i % 2 == 0 else "fixed", order=8 if i % 2 == 0 else 2)
        (d / f"{name}.flac").write_bytes(E.encode(ref, 16000, 16, frames))
        by_dir.setdefault((d, f"{spk}-{ch}"), []).append(f"{name} " + " ".join(rng.choice(WORDS, size=2 + i)))
    for (d, stem), lines in by_dir.items():
        (d / f"{stem}.trans.txt").write_text("\n".join(lines) + "\n")


def ted(root, lengths=(170000, 260000, 600000, 640000), seed=13):
    """TED-LIUM 3 layout (reference corpus/ted.py:22-52): wav_segment/<id>.wav (16-bit mono 16 kHz) and
    transcription/<id>.txt; long utterances (T = 531 .. 1874 frames; the last one is cut to 600 000
    samples by the reader, reference data.py:19-22)."""
    rng = np.random.default_rng(seed)
    apath, tpath = root / "wav_segment", root / "transcription"
    apath.mkdir(parents=True)
    tpath.mkdir(parents=True)
    for i, n in enumerate(lengths):
        x = rng.standard_normal(n) * 0.1
        with wave.open(str(apath / f"talk{i}.wav"), "wb") as f:
            f.setnchannels(1)
            f.setsampwidth(2)
            f.setframerate(16000)
            f.writeframes((np.clip(x, -1, 1) * 32767).astype("<i2").tobytes())
        (tpath / f"talk{i}.txt").write_text(" ".join(rng.choice(WORDS, size=4 + 3 * i)) + "\n")


def commonvoice(root, frames=(4, 7, 5, 9, 3), seed=14):
    """test.tsv (client_id, path, sentence, ...) and clips/<name>.mp3; sentences with the punctuation and
    abbreviations preprocess_cv_text rewrites (corpus/commonvoice.py:12-24)."""
    rng = np.random.default_rng(seed)
    (root / "clips").mkdir(parents=True)
    rows = ["client_id\tpath\tsentence\tup_votes\tdown_votes"]
    for i, nf in enumerate(frames):
        data = b"".join(M.write_frame([[M.random_granule(rng, int(rng.choice([0, 0, 1, 2, 3])))] for _ in range(2)], 1)
                        for _ in range(nf))
        name = f"common_voice_en_{1000 + i}.mp3"
        (root / "clips" / name).write_bytes(data)
        words = list(rng.choice(WORDS, size=2 + i))
        words[0] = words[0].capitalize() + ","
        sentence = " ".join(words) + (" e.g. Dr. Who-ever." if i % 2 else ".")
        rows.append(f"c{i}\t{name}\t{sentence}\t2\t0")
    (root / "test.tsv").write_text("\n".join(rows) + "\n")
