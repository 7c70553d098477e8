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
Deviations (documented in DESIGN.md): torchaudio/soundfile are not installed in this image, so FLAC
and MP3 (CommonVoice clips) are decoded by the from-spec decoders in libsuta_audio (csrc/flac.cpp,
csrc/mp3.cpp), WAV by the standard-library `wave` module, and resampling restates torchaudio's Hann-windowed sinc resampler (`resample`).  The
noise of utterance i comes from its own torch.Generator seeded `seed * 1_000_003 + i` (i = its index in
the sorted dataset), so every rank of a sharded run draws exactly the audio a single process draws
(the reference's draw depends on DataLoader worker seeding and on transformers consuming the global
RNG, SURVEY.md Appendix B.3, so noise parity with it is statistical either way).
Under torchrun only rank 0 prints the loaders' [INFO] lines.
"""
from __future__ import annotations

import os
import re
import wave as _wave
from pathlib import Path
from typing import Iterator, List, Optional, Sequence, Tuple

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
        _say(len(files), len(texts))   # commonvoice.py:40
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


def _say(*a):
    """print on rank 0 only (a sharded run is one job: its log reads like the reference's one process)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a)


def create_dataset(split, name, path, batch_size=1, chime_subsets: Optional[Sequence[str]] = None):
    """data.py:48-68.  chime_subsets: the CHiME et05 subsets to read (None = the reference's hard-coded 7,
    corpus/CHiME.py:27; config C3 "eval-real" = the three *_real ones); refused for other corpora."""
    n = name.lower()
    table = {"librispeech": LibriDataset, "chime": CHiMEDataset, "ted": TedDataset, "commonvoice": CVDataset}
    if n not in table:
        raise NotImplementedError(name)
    if chime_subsets:
        if n != "chime":
            raise ValueError(f"chime_subsets given for dataset {name!r}")
        bad = [s for s in chime_subsets if s not in CHiMEDataset.SUBSETS]
        if bad:
            raise ValueError(f"unknown CHiME subset(s) {bad}: the reference reads {CHiMEDataset.SUBSETS}")
        ds = CHiMEDataset(split, batch_size, path, subsets=list(chime_subsets))
    else:
        ds = table[n](split, batch_size, path)
    _say(f"[INFO]    There are {len(ds)} samples.")
    return ds, batch_size


# ---------------------------------------------------------------------------------------------
# audio
# ---------------------------------------------------------------------------------------------
_AUDIO_LIB = None
AUDIO_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsuta_audio.so")


def _audio_lib():
    """libsuta_audio.so (include/suta_audio.h): the from-spec FLAC and MP3 decoders, host C++."""
    global _AUDIO_LIB
    if _AUDIO_LIB is None:
        import ctypes as C
        if not os.path.exists(AUDIO_LIB_PATH):
            raise RuntimeError(f"libsuta_audio.so not found at {AUDIO_LIB_PATH}: build it with __graft_entry__.build()")
        lib = C.CDLL(AUDIO_LIB_PATH)
        u8p, i32p, i64p = C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_int64)
        lib.suta_flac_info.argtypes = [u8p, C.c_int64, i32p, i32p, i32p, i64p]
        lib.suta_flac_info.restype = C.c_int32
        lib.suta_flac_decode.argtypes = [u8p, C.c_int64, C.POINTER(C.c_float), C.c_int64, C.c_int32, i64p]
        lib.suta_flac_decode.restype = C.c_int32
        lib.suta_mp3_info.argtypes = [u8p, C.c_int64, i32p, i32p, i64p]
        lib.suta_mp3_info.restype = C.c_int32
        lib.suta_mp3_decode.argtypes = [u8p, C.c_int64, C.POINTER(C.c_float), C.c_int64, C.c_int32, i64p, i64p]
        lib.suta_mp3_decode.restype = C.c_int32
        lib.suta_audio_last_error.restype = C.c_char_p
        _AUDIO_LIB = lib
    return _AUDIO_LIB


def _as_bytes(src) -> bytes:
    if isinstance(src, (bytes, bytearray, memoryview)):
        return bytes(src)
    with open(src, "rb") as f:
        return f.read()


def flac_info(src):
    """(sample_rate, channels, bits_per_sample, total_samples) from STREAMINFO (path or bytes)."""
    import ctypes as C
    lib = _audio_lib()
    buf = np.frombuffer(_as_bytes(src), dtype=np.uint8)
    sr, ch, bps, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    st = lib.suta_flac_info(buf.ctypes.data_as(C.POINTER(C.c_uint8)), buf.size, C.byref(sr), C.byref(ch),
                            C.byref(bps), C.byref(n))
    if st:
        raise RuntimeError(f"FLAC: {lib.suta_audio_last_error().decode()}")
    return sr.value, ch.value, bps.value, n.value


def flac_decode(src, verify_crc: bool = True) -> Tuple[np.ndarray, int]:
    """torchaudio.load semantics for a FLAC file (reference data.py:15): ((C, N) float32 in [-1, 1),
    sample_rate), samples scaled by 2^-(bps-1).  Decoded by libsuta_audio (GIL released)."""
    import ctypes as C
    lib = _audio_lib()
    buf = np.frombuffer(_as_bytes(src), dtype=np.uint8)
    bp = buf.ctypes.data_as(C.POINTER(C.c_uint8))
    sr, ch, bps, total = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    st = lib.suta_flac_info(bp, buf.size, C.byref(sr), C.byref(ch), C.byref(bps), C.byref(total))
    cap = total.value if (st == 0 and total.value > 0) else max(1, buf.size * 4)
    for _ in range(2):
        out = np.empty((max(1, ch.value), cap), np.float32)
        n = C.c_int64()
        st = lib.suta_flac_decode(bp, buf.size, out.ctypes.data_as(C.POINTER(C.c_float)), cap, int(verify_crc),
                                  C.byref(n))
        if st == 4 and n.value > cap:   # SUTA_AUDIO_ERR_SPACE: retry with the stated requirement
            cap = n.value
            continue
        break
    if st:
        raise RuntimeError(f"FLAC: {lib.suta_audio_last_error().decode()}")
    return out[:, :n.value], sr.value


def mp3_info(src):
    """(sample_rate, channels, samples per channel after FFmpeg's gapless trim) by a header walk."""
    import ctypes as C
    lib = _audio_lib()
    buf = np.frombuffer(_as_bytes(src), dtype=np.uint8)
    sr, ch, n = C.c_int32(), C.c_int32(), C.c_int64()
    st = lib.suta_mp3_info(buf.ctypes.data_as(C.POINTER(C.c_uint8)), buf.size, C.byref(sr), C.byref(ch), C.byref(n))
    if st:
        raise RuntimeError(f"MP3: {lib.suta_audio_last_error().decode()}")
    return sr.value, ch.value, n.value


def mp3_decode(src, strict: bool = False, stats: bool = False):
    """torchaudio.load semantics for an MPEG audio Layer III file (reference data.py:15 on CommonVoice
    clips/*.mp3, corpus/commonvoice.py:32-38): ((C, N) float32, sample_rate), FFmpeg's decoder delay and
    gapless trimming.  strict: fail on Huffman data that runs past part2_3_length.  stats=True also returns
    [frames, granule-channels, ending exactly at part2_3_length, overrunning, without bit reservoir]."""
    import ctypes as C
    lib = _audio_lib()
    buf = np.frombuffer(_as_bytes(src), dtype=np.uint8)
    bp = buf.ctypes.data_as(C.POINTER(C.c_uint8))
    sr, ch, total = mp3_info(buf.tobytes())
    cap = max(1, total)
    out = np.empty((ch, cap), np.float32)
    n = C.c_int64()
    st_arr = np.zeros(5, np.int64)
    st = lib.suta_mp3_decode(bp, buf.size, out.ctypes.data_as(C.POINTER(C.c_float)), cap, int(strict), C.byref(n),
                             st_arr.ctypes.data_as(C.POINTER(C.c_int64)))
    if st:
        raise RuntimeError(f"MP3: {lib.suta_audio_last_error().decode()}")
    res = (out[:, :n.value], sr)
    return res + (st_arr,) if stats else res


def audio_info(path: str) -> Tuple[int, int]:
    """(samples per channel, sample rate) from the file header without decoding (WAV, FLAC, MP3), or by
    decoding for other formats.  The driver's LPT cost model uses it."""
    p = str(path)
    low = p.lower()
    if low.endswith(".mp3"):
        sr, ch, n = mp3_info(p)
        return n, sr
    if low.endswith(".flac"):
        sr, ch, bps, n = flac_info(p)
        if n > 0:
            return n, sr
    elif low.endswith(".wav"):
        try:
            with _wave.open(p, "rb") as f:
                return f.getnframes(), f.getframerate()
        except _wave.Error:
            pass
    x, sr = _decode_audio(p)
    return x.size, sr


def decoded_length(path: str, max_len: int = MAX_LEN) -> int:
    """Samples the reader will hand to the engine: channels concatenated (reference data.py:18),
    resampled to 16 kHz (torchaudio length rule ceil(n * 16000 / sr) per channel), truncated."""
    p = str(path)
    if p.lower().endswith(".flac"):
        sr, ch, bps, n = flac_info(p)
        per = n
    elif p.lower().endswith(".mp3"):
        sr, ch, per = mp3_info(p)
    elif p.lower().endswith(".wav"):
        with _wave.open(p, "rb") as f:
            sr, ch, per = f.getframerate(), f.getnchannels(), f.getnframes()
    else:
        x, sr = _decode_audio(p)
        ch, per = 1, x.size
    if sr != SAMPLE_RATE:
        from math import gcd
        g = gcd(sr, SAMPLE_RATE)
        per = -(-(SAMPLE_RATE // g) * per // (sr // g))
    return min(ch * per, max_len)


def _decode_audio(path: str) -> Tuple[np.ndarray, int]:
    """torchaudio.load(...) then .reshape(-1) (reference data.py:15-18): channels concatenated."""
    x, sr = decode_channels(path)
    return np.ascontiguousarray(x.reshape(-1)), sr


def decode_channels(path: str) -> Tuple[np.ndarray, int]:
    """torchaudio.load(path) (reference data.py:15): ((C, N) float32, sample rate).  FLAC and MP3:
    libsuta_audio; WAV: the standard library; anything else needs soundfile or torchaudio, neither of
    which is in this image."""
    path = str(path)
    low = path.lower()
    if low.endswith(".flac"):
        return flac_decode(path)
    if low.endswith(".mp3"):
        return mp3_decode(path)
    if not low.endswith(".wav"):
        try:
            import soundfile as sf
            x, sr = sf.read(path, dtype="float32", always_2d=True)      # (N, C)
            return np.ascontiguousarray(x.T), sr
        except ImportError:
            pass
        try:
            import torchaudio
            w, sr = torchaudio.load(path)
            return w.numpy().astype(np.float32), sr
        except ImportError:
            pass
        raise RuntimeError(f"cannot decode {path}: FLAC, MP3 and WAV are built in; other formats need soundfile or "
                           "torchaudio (not installed)")
    with _wave.open(path, "rb") as f:
        sr, ch, sw, n = f.getframerate(), f.getnchannels(), f.getsampwidth(), f.getnframes()
        raw = f.readframes(n)
    if sw == 2:
        x = np.frombuffer(raw, dtype="<i2").astype(np.float32) / 32768.0
    elif sw == 3:
        b = np.frombuffer(raw, dtype=np.uint8).reshape(-1, 3).astype(np.int32)
        v = (b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16))
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / 8388608.0
    elif sw == 4:
        x = np.frombuffer(raw, dtype="<i4").astype(np.float32) / 2147483648.0
    elif sw == 1:
        x = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise RuntimeError(f"unsupported sample width {sw} in {path}")
    # interleaved frames -> (C, N)
    return np.ascontiguousarray(x.reshape(-1, ch).T, dtype=np.float32), sr


def sinc_resample_kernel(orig: int, new: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """torchaudio.functional._get_sinc_resample_kernel, method "sinc_interp_hann" (torchaudio 2.x, the
    default of torchaudio.transforms.Resample used at reference data.py:16-17): the Hann-windowed sinc
    filter bank, built in float64 and cast to float32.  Returns ((new, 1, 2*width + orig) kernel, width)
    for orig/new already divided by their gcd."""
    import math
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = np.arange(-width, width + orig, dtype=np.float64)[None, None] / orig
    t = np.arange(0, -new, -1, dtype=np.float64)[:, None, None] / new + idx
    t *= base
    t = np.clip(t, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    scale = base / orig
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = k * window * scale
    return k.astype(np.float32), width


def resample(x: np.ndarray, sr: int, target: int = SAMPLE_RATE) -> np.ndarray:
    """torchaudio.transforms.Resample(sr, target)(x) restated (reference data.py:16-17): pad by the
    filter width, strided conv1d with the sinc bank, interleave the phases, keep ceil(target*n/sr)
    samples.  torchaudio is absent here, so agreement with it is "parity unpinned" beyond this
    restatement of its published algorithm (tests/test_audio.py checks band-limited behaviour)."""
    if sr == target:
        return x
    import torch
    from math import gcd
    g = gcd(int(sr), int(target))
    orig, new = int(sr) // g, int(target) // g
    kern, width = sinc_resample_kernel(orig, new)
    w = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).reshape(1, 1, -1)
    n = w.shape[-1]
    w = torch.nn.functional.pad(w, (width, width + orig))
    y = torch.nn.functional.conv1d(w, torch.from_numpy(kern), stride=orig)   # (1, new, frames)
    y = y.transpose(1, 2).reshape(-1)
    target_len = -(-new * n // orig)
    return y[:target_len].numpy()


NOISE_SEED_STRIDE = 1_000_003


class AudioReader:
    """data.py:13-25.  decode() is thread-safe (the loader runs it on worker threads) and returns the
    utterance with its decoded length; the truncation lines are printed by the caller in load order.
    noise(x, index) draws utterance `index`'s noise from its own generator (module docstring)."""

    def __init__(self, extra_noise: float = 0.0, max_len: int = MAX_LEN, seed: int = 0):
        self.extra_noise = extra_noise
        self.max_len = max_len
        self.seed = seed

    def decode(self, path: str) -> Tuple[np.ndarray, int]:
        """(waveform truncated to max_len, decoded length before truncation)."""
        x, sr = decode_channels(str(path))
        if sr != SAMPLE_RATE:  # the reference resamples the (C, N) tensor per channel, then flattens
            x = np.stack([resample(c, sr) for c in x])
        x = x.reshape(-1)
        n = int(x.shape[-1])
        if n >= self.max_len:
            x = x[: self.max_len]
        return np.ascontiguousarray(x, dtype=np.float32), n

    def truncation_lines(self, path: str, n: int) -> List[str]:
        """What the reference prints for an utterance cut at max_len (data.py:19-21: the message, then
        wav.shape, both as torch.Size)."""
        if n < self.max_len:
            return []
        return [f"{path} has len torch.Size([{n}]), truncate to {self.max_len}", f"torch.Size([{self.max_len}])"]

    def noise(self, x: np.ndarray, index: int = 0) -> np.ndarray:
        import torch
        w = torch.from_numpy(x)
        if self.extra_noise:
            g = torch.Generator().manual_seed(self.seed * NOISE_SEED_STRIDE + int(index))
            w = w + self.extra_noise * torch.randn(w.shape, generator=g)
        return w.numpy()

    def __call__(self, path: str, index: int = 0) -> np.ndarray:
        x, n = self.decode(path)
        for ln in self.truncation_lines(str(path), n):
            print(ln)
        return self.noise(x, index)


def collect_audio_batch(batch, reader: AudioReader, decoded=None, indices=None, log=None):
    """data.py:9-45: read a bucket, sort by audio length descending.  `decoded`: the bucket's
    (waveform, decoded length) pairs already decoded by loader threads; `indices`: the items' dataset
    indices (their noise seeds; default 0..len-1); `log`: a list collecting the truncation lines in load
    order (printed here when None)."""
    if type(batch[0]) is not tuple:
        batch = batch[0]
    if decoded is None:
        decoded = [reader.decode(str(b[0])) for b in batch]
    if indices is None:
        indices = range(len(batch))
    feats = []
    for (w, n), b, i in zip(decoded, batch, indices):
        for ln in reader.truncation_lines(str(b[0]), n):
            print(ln) if log is None else log.append(ln)
        feats.append((reader.noise(w, i), str(b[0]).split("/")[-1].split(".")[0], b[1]))
    feats = sorted(((len(f), n, f, t) for f, n, t in feats), reverse=True, key=lambda x: x[0])
    lens, files, wavs, texts = zip(*feats)
    return lens, wavs, texts, files


def load_dataset(split=None, name="librispeech", path=None, batch_size=1, extra_noise=0.0, num_workers=0,
                 chime_subsets: Optional[Sequence[str]] = None) -> Iterator:
    """data.py:71-78 as a plain iterator (batches of `batch_size` consecutive items)."""
    ds, bs = create_dataset(split, name, path, batch_size, chime_subsets)
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

        def batch_indices(self) -> List[List[int]]:
            """dataset index of every item of raw_batches() (a bucket starting past len - bucket_size
            is moved back, as _Corpus.__getitem__ does)."""
            out, every = [], list(range(len(ds)))
            for i in range(0, len(ds), bs):
                start = min(len(ds) - bs, i) if bs > 1 else i
                out.append(every[start:start + bs] if bs > 1 else [i])
            return out

        def collate(self, items, decoded=None, indices=None, log=None):
            return collect_audio_batch(items, reader, decoded, indices, log)

        def iter_collated(self, indices: Sequence[int], workers: int = 0, window: int = 32, log=None):
            """(index, collated batch) for the given loader batches, in order.  workers > 1 decodes
            ahead on a thread pool (the FLAC decoder and file reads release the GIL), at most
            `window` batches in flight; noise is keyed on each item's dataset index, so the result
            does not depend on which batches this process loads or in what order.  `log`: a callable
            taking (loader batch index, truncation lines) instead of printing them."""
            batches = self.raw_batches()
            didx = self.batch_indices()

            def coll(i, decoded=None):
                lines = [] if log is not None else None
                out = self.collate(batches[i], decoded, didx[i], lines)
                if log is not None:
                    log(i, lines)
                return out

            if workers <= 1:
                for i in indices:
                    yield i, coll(i)
                return
            from collections import deque
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=workers) as ex:
                pending = deque()
                it = iter(indices)
                for i in it:
                    pending.append((i, [ex.submit(reader.decode, str(f)) for f, _ in batches[i]]))
                    if len(pending) >= window:
                        break
                while pending:
                    i, futs = pending.popleft()
                    yield i, coll(i, [f.result() for f in futs])
                    nxt = next(it, None)
                    if nxt is not None:
                        pending.append((nxt, [ex.submit(reader.decode, str(f)) for f, _ in batches[nxt]]))

        def __iter__(self):
            for _, b in self.iter_collated(range(len(self)), num_workers):
                yield b

    return _Loader()
