"""Input pipeline and corpus loaders, drop-in for reference data.py and corpus/*.py (row f2).

Behaviour kept from the reference:
  * loaders list (wav path, transcript) pairs and sort them by TRANSCRIPT length, descending
    (TED ascending) with a stable sort (corpus/librispeech.py:22-39, CHiME.py:22-49,
    commonvoice.py:27-42, ted.py:22-52); `split` is ignored: splits are fixed per corpus
    (LS test-other; CHiME-3 et05 real+simu without ped_real, enhanced audio; CV test.tsv;
    TED wav_segment/)
  * audio_reader (data.py:13-25): decode, resample to 16 kHz, truncate at 600 000 samples,
    add extra_noise * N(0, 1) noise
  * collate (data.py:27-45): sort a bucket by audio length, descending
Deviations (documented in DESIGN.md): torchaudio/soundfile are not installed in this image, so
WAV is decoded with the standard-library `wave` module when neither is present (FLAC then needs
soundfile or torchaudio); resampling falls back to scipy's polyphase filter; the noise comes from
a torch.Generator seeded 0 in the reading process (the reference's draw depends on DataLoader
worker seeding and on transformers consuming the global RNG).
"""
from __future__ import annotations

import os
import re
import wave as _wave
from pathlib import Path
from typing import Iterator, List, Sequence, Tuple

import numpy as np

SAMPLE_RATE = 16000
MAX_LEN = 600000


# ---------------------------------------------------------------------------------------------
# corpora
# ---------------------------------------------------------------------------------------------
class _Corpus:
    file_list: Tuple
    text: Tuple

    def __init__(self, bucket_size):
        self.bucket_size = bucket_size

    def _finish(self, files, texts, ascending):
        pairs = sorted(zip(files, texts), reverse=not ascending, key=lambda x: len(x[1]))
        self.file_list, self.text = (tuple(p[0] for p in pairs), tuple(p[1] for p in pairs)) if pairs else ((), ())

    def __getitem__(self, index):
        if self.bucket_size > 1:
            index = min(len(self.file_list) - self.bucket_size, index)
            return [(f, t) for f, t in zip(self.file_list[index:index + self.bucket_size],
                                           self.text[index:index + self.bucket_size])]
        return self.file_list[index], self.text[index]

    def __len__(self):
        return len(self.file_list)


class LibriDataset(_Corpus):
    """corpus/librispeech.py:22-39 (split forced to test-other)."""

    def __init__(self, split, bucket_size, path, ascending=False):
        super().__init__(bucket_size)
        files = []
        for s in ["test-other"]:
            files += list(Path(os.path.join(path, s)).rglob("*.flac"))
        texts = [self.read_text(str(f)) for f in files]
        self._finish(files, texts, ascending)

    @staticmethod
    def read_text(file):
        src = "-".join(file.split("-")[:-1]) + ".trans.txt"
        idx = file.split("/")[-1].split(".")[0]
        with open(src) as fp:
            for line in fp:
                if idx == line.split(" ")[0]:
                    return line[:-1].split(" ", 1)[1]


class CHiMEDataset(_Corpus):
    """corpus/CHiME.py:22-49: the 7 et05 subsets, enhanced 16 kHz audio."""
    SUBSETS = ["et05_bus_real", "et05_bus_simu", "et05_caf_real", "et05_caf_simu", "et05_ped_simu",
               "et05_str_real", "et05_str_simu"]

    def __init__(self, split, bucket_size, path="", enhance=False, ascending=False, subsets: Sequence[str] = None):
        super().__init__(bucket_size)
        apath = path + "/data/audio/16kHz/enhanced"
        tpath = path + "/data/transcriptions"
        subs = list(subsets) if subsets else self.SUBSETS
        files = []
        for s in subs:
            files += list(Path(os.path.join(apath, s)).glob("*.wav"))
        texts = [self.read_text(tpath, str(f)) for f in files]
        if enhance:
            files = []
            for s in subs:
                files += list(Path(os.path.join(apath, s, "se_wav")).glob("*.wav"))
        self._finish(files, texts, ascending)

    @staticmethod
    def read_text(tpath, file):
        # CHiME.py:9-17, dots of the file name dropped exactly as the reference does
        txt = os.path.join(tpath, "".join("/".join(file.split("/")[-2:]).split(".")[:-1]) + ".trn")
        with open(txt) as fp:
            for line in fp:
                return " ".join(line.split(" ")[1:]).strip("\n")


def preprocess_cv_text(text: str) -> str:
    """corpus/commonvoice.py:12-24."""
    text = str(text)
    for a, b in (("i.e.", "that is"), ("e.g.", "for example"), ("Mr.", "Mister"), ("Mrs.", "Mistress"),
                 ("Dr.", "Doctor"), ("-", " ")):
        text = text.replace(a, b)
    text = text.upper()
    text = re.sub("[^ A-Z']", "", text)
    return " ".join(text.split())


class CVDataset(_Corpus):
    """corpus/commonvoice.py:27-42 (test.tsv)."""

    def __init__(self, split, bucket_size, path="", enhance=False, ascending=False):
        super().__init__(bucket_size)
        import pandas as pd
        df = pd.read_csv(path + "/test.tsv", sep="\t")
        texts = list(df["sentence"].apply(preprocess_cv_text).values)
        files = [os.path.join(path + "/clips", f) for f in df["path"].values]
        self._finish(files, texts, ascending)


class TedDataset(_Corpus):
    """corpus/ted.py:22-52 (ascending by default, utterances without transcript skipped)."""

    def __init__(self, split, bucket_size, path="", enhance=False, ascending=True):
        super().__init__(bucket_size)
        apath = path + "/wav_segment"
        tpath = path + "/transcription"
        cand = list(Path(os.path.join(apath, "se_wav") if enhance else apath).glob("*.wav"))
        files, texts = [], []
        for f in cand:
            t = self.read_text(tpath, str(f))
            if t is not None:
                files.append(f)
                texts.append(t)
        self._finish(files, texts, ascending)

    @staticmethod
    def read_text(tpath, file):
        name = file.split("/")[-1].replace("wav", "txt")
        p = os.path.join(tpath, name)
        if not os.path.exists(p):
            return None
        with open(p) as fp:
            for line in fp:
                return line.strip("\n")


def create_dataset(split, name, path, batch_size=1):
    """data.py:48-68."""
    n = name.lower()
    table = {"librispeech": LibriDataset, "chime": CHiMEDataset, "ted": TedDataset, "commonvoice": CVDataset}
    if n not in table:
        raise NotImplementedError(name)
    ds = table[n](split, batch_size, path)
    print(f"[INFO]    There are {len(ds)} samples.")
    return ds, batch_size


# ---------------------------------------------------------------------------------------------
# audio
# ---------------------------------------------------------------------------------------------
def _decode_audio(path: str) -> Tuple[np.ndarray, int]:
    try:
        import soundfile as sf  # noqa: F401
        x, sr = sf.read(path, dtype="float32", always_2d=True)
        return x.mean(1).astype(np.float32) if x.shape[1] > 1 else x[:, 0], sr
    except ImportError:
        pass
    try:
        import torchaudio
        w, sr = torchaudio.load(path)
        return w.reshape(-1).numpy().astype(np.float32), sr
    except ImportError:
        pass
    if not path.lower().endswith(".wav"):
        raise RuntimeError(f"cannot decode {path}: neither soundfile nor torchaudio is installed (WAV only)")
    with _wave.open(path, "rb") as f:
        sr, ch, sw, n = f.getframerate(), f.getnchannels(), f.getsampwidth(), f.getnframes()
        raw = f.readframes(n)
    if sw == 2:
        x = np.frombuffer(raw, dtype="<i2").astype(np.float32) / 32768.0
    elif sw == 4:
        x = np.frombuffer(raw, dtype="<i4").astype(np.float32) / 2147483648.0
    elif sw == 1:
        x = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise RuntimeError(f"unsupported sample width {sw} in {path}")
    if ch > 1:
        x = x.reshape(-1, ch).reshape(-1)  # the reference reshapes (C, N) to (-1): channels concatenated
    return x, sr


def resample(x: np.ndarray, sr: int, target: int = SAMPLE_RATE) -> np.ndarray:
    if sr == target:
        return x
    try:
        import torchaudio
        import torch
        return torchaudio.transforms.Resample(sr, target)(torch.from_numpy(x)[None])[0].numpy()
    except ImportError:
        from math import gcd
        from scipy.signal import resample_poly
        g = gcd(sr, target)
        return resample_poly(x, target // g, sr // g).astype(np.float32)


class AudioReader:
    """data.py:13-25 with a deterministic noise generator."""

    def __init__(self, extra_noise: float = 0.0, max_len: int = MAX_LEN, seed: int = 0):
        import torch
        self.extra_noise = extra_noise
        self.max_len = max_len
        self.gen = torch.Generator().manual_seed(seed)

    def __call__(self, path: str) -> np.ndarray:
        import torch
        x, sr = _decode_audio(str(path))
        x = resample(x, sr).reshape(-1)
        if x.shape[-1] >= self.max_len:
            print(f"{path} has len {x.shape}, truncate to {self.max_len}")
            x = x[: self.max_len]
        w = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
        if self.extra_noise:
            w = w + self.extra_noise * torch.randn(w.shape, generator=self.gen)
        return w.numpy()


def collect_audio_batch(batch, reader: AudioReader):
    """data.py:9-45: read a bucket, sort by audio length descending."""
    if type(batch[0]) is not tuple:
        batch = batch[0]
    feats = [(reader(str(b[0])), str(b[0]).split("/")[-1].split(".")[0], b[1]) for b in batch]
    feats = sorted(((len(f), n, f, t) for f, n, t in feats), reverse=True, key=lambda x: x[0])
    lens, files, wavs, texts = zip(*feats)
    return lens, wavs, texts, files


def load_dataset(split=None, name="librispeech", path=None, batch_size=1, extra_noise=0.0, num_workers=0
                 ) -> Iterator:
    """data.py:71-78 as a plain iterator (batches of `batch_size` consecutive items)."""
    ds, bs = create_dataset(split, name, path, batch_size)
    reader = AudioReader(extra_noise)

    class _Loader:
        def __len__(self):
            return (len(ds) + bs - 1) // bs

        def raw_batches(self) -> List[List[Tuple]]:
            """(path, text) items of every loader batch; audio is read only by collate()."""
            out = []
            for i in range(0, len(ds), bs):
                it = ds[i]
                out.append(list(it) if isinstance(it, list) else [it])
            return out

        def collate(self, items):
            return collect_audio_batch(items, reader)

        def __iter__(self):
            for items in self.raw_batches():
                yield self.collate(items)

    return _Loader()
