"""CPU restatement (numpy, float64) of the ISO/IEC 11172-3 Layer III decoding arithmetic, from the quantised
spectrum to PCM — TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

It checks the MP3 decoder of libsuta_audio (csrc/mp3.cpp) on frames that tests/mp3_builder.py writes bit by bit
from a known quantised spectrum: the decoder must parse them back and produce the PCM this module computes
with the standard's formulas written out directly (no fast transforms):
  * 2.4.3.4.7 requantisation  xr = sign(is) |is|^(4/3) 2^((global_gain - 210 - 8 subblock_gain[w]) / 4)
                                     2^(-(1 + scalefac_scale) / 2 (scalefac + preflag pretab))
  * 2.4.3.4.9 mid/side stereo  L = (M + S) / sqrt 2, R = (M - S) / sqrt 2
  * 2.4.3.4.8 reordering of short windows, 2.4.3.4.10.1 alias reduction (long-block part only)
  * 2.4.3.4.10.2 IMDCT  x_i = sum_k X_k cos(pi / 2n (2i + 1 + n/2)(2k + 1)), n = 36 / 12, block windows
  * 2.4.3.4.10.3 overlap-add, frequency inversion of odd subbands
  * Annex A.2 / 2.4.3.4.10.5 polyphase synthesis with the Table B.3 window (read from csrc/mp3_tables.h)
The reference has no MP3 code of its own: it calls torchaudio.load on CommonVoice clips
(reference corpus/commonvoice.py:32-38, data.py:15).  MPEG-1, 44.1 kHz band tables only (what the builder writes).
"""
import os
import re

import numpy as np

SFB_LONG = [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576]
SFB_SHORT = [0, 4, 8, 12, 16, 22, 30, 40, 52, 66, 84, 106, 136, 192]
PRETAB = [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 2, 2, 3, 3, 3, 2, 0, 0]
ALIAS_C = np.array([-0.6, -0.535, -0.33, -0.185, -0.095, -0.041, -0.0142, -0.0037])

_TABLES_H = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "test-time-adaptation-asr-suta_amd",
                         "csrc", "mp3_tables.h")


def window_d():
    """Table B.3 D[0..511] from the 257 stored values (D[512 - i] = D[i] at multiples of 64, else -D[i])."""
    with open(_TABLES_H) as f:
        m = re.search(r"window257\[257\] = \{([^}]*)\}", f.read())
    w = np.array([int(v) for v in m.group(1).split(",")], np.float64) / 65536.0
    D = np.zeros(512)
    D[:257] = w
    for i in range(1, 257):
        D[512 - i] = w[i] if i % 64 == 0 else -w[i]
    return D


def requantize(g):
    """g: granule dict (tests/mp3_builder.py) -> xr[576] in transmitted order."""
    is_ = np.asarray(g["is"], np.float64)
    mag = np.abs(is_) ** (4.0 / 3.0) * np.sign(is_)
    mul = 0.5 * (1 + g["sf_scale"])
    xr = np.zeros(576)
    short = g["ws"] and g["block_type"] == 2
    long_end = 576 if not short else (36 if g["mixed"] else 0)
    for sfb in range(22):
        a, b = SFB_LONG[sfb], min(SFB_LONG[sfb + 1], long_end)
        if a >= long_end:
            break
        sf = g["sf_l"][sfb] if sfb < 21 else 0
        e = 0.25 * (g["gg"] - 210) - mul * (sf + (PRETAB[sfb] if g["preflag"] else 0))
        xr[a:b] = mag[a:b] * 2.0 ** e
    if short:
        for sfb in range(3 if g["mixed"] else 0, 13):
            a, width = SFB_SHORT[sfb], SFB_SHORT[sfb + 1] - SFB_SHORT[sfb]
            for w in range(3):
                sf = g["sf_s"][sfb][w] if sfb < 12 else 0
                e = 0.25 * (g["gg"] - 210 - 8 * g["subblock_gain"][w]) - mul * sf
                o = 3 * a + w * width
                xr[o:o + width] = mag[o:o + width] * 2.0 ** e
    return xr


def _imdct(X, n):
    i = np.arange(n)[:, None]
    k = np.arange(n // 2)[None, :]
    return np.cos(np.pi / (2 * n) * (2 * i + 1 + n / 2) * (2 * k + 1)) @ X


def _long_window(bt):
    i = np.arange(36)
    w = np.sin(np.pi / 36 * (i + 0.5))
    if bt == 1:
        w[18:24] = 1.0
        w[24:30] = np.sin(np.pi / 12 * (i[24:30] - 18 + 0.5))
        w[30:] = 0.0
    elif bt == 3:
        w[:6] = 0.0
        w[6:12] = np.sin(np.pi / 12 * (i[6:12] - 6 + 0.5))
        w[12:18] = 1.0
    return w


def hybrid(g, xr, overlap):
    """-> (18, 32) subband samples; overlap (32, 18) is updated in place."""
    short = g["ws"] and g["block_type"] == 2
    long_sb = 32 if not short else (2 if g["mixed"] else 0)
    x = xr.copy()
    cs = 1 / np.sqrt(1 + ALIAS_C ** 2)
    ca = ALIAS_C * cs
    for sb in range(1, long_sb):
        lo = x[18 * sb - 1 - np.arange(8)].copy()
        hi = x[18 * sb + np.arange(8)].copy()
        x[18 * sb - 1 - np.arange(8)] = lo * cs - hi * ca
        x[18 * sb + np.arange(8)] = hi * cs + lo * ca
    wins = np.zeros((3, 192))
    if short:
        for sfb in range(3 if g["mixed"] else 0, 13):
            a, width = SFB_SHORT[sfb], SFB_SHORT[sfb + 1] - SFB_SHORT[sfb]
            for w in range(3):
                wins[w, a:a + width] = xr[3 * a + w * width: 3 * a + (w + 1) * width]
    out = np.zeros((18, 32))
    win12 = np.sin(np.pi / 12 * (np.arange(12) + 0.5))
    for sb in range(32):
        if sb < long_sb:
            bt = 0 if (g["ws"] and g["mixed"] and sb < 2) else (g["block_type"] if g["ws"] else 0)
            z = _imdct(x[18 * sb:18 * sb + 18], 36) * _long_window(bt)
        else:
            z = np.zeros(36)
            for w in range(3):
                z[6 * w + 6: 6 * w + 18] += _imdct(wins[w, 6 * sb: 6 * sb + 6], 12) * win12
        v = z[:18] + overlap[sb]
        overlap[sb] = z[18:]
        if sb % 2:
            v[1::2] = -v[1::2]
        out[:, sb] = v
    return out


class Synth:
    """Polyphase synthesis by the standard's matrixing: V = N S, U gathered from V, W = U D, 32 sums of 16."""

    def __init__(self):
        self.V = np.zeros(1024)
        self.D = window_d()
        i = np.arange(64)[:, None]
        k = np.arange(32)[None, :]
        self.N = np.cos((16 + i) * (2 * k + 1) * np.pi / 64)

    def run(self, sub):
        out = []
        for S in sub:
            self.V[64:] = self.V[:-64].copy()
            self.V[:64] = self.N @ S
            U = np.zeros(512)
            for i in range(8):
                U[64 * i: 64 * i + 32] = self.V[128 * i: 128 * i + 32]
                U[64 * i + 32: 64 * i + 64] = self.V[128 * i + 96: 128 * i + 128]
            W = U * self.D
            out.append(W.reshape(16, 32).sum(axis=0))
        return np.concatenate(out)


def decode(frames, channels, ms=False):
    """frames: list of frames, each a list (granules) of per-channel granule dicts -> (channels, n) float64."""
    overlap = [np.zeros((32, 18)) for _ in range(channels)]
    synth = [Synth() for _ in range(channels)]
    pcm = [[] for _ in range(channels)]
    for fr in frames:
        for gr in fr:
            xr = [requantize(gr[ch]) for ch in range(channels)]
            if ms and channels == 2:
                m, s = xr
                xr = [(m + s) / np.sqrt(2), (m - s) / np.sqrt(2)]
            for ch in range(channels):
                pcm[ch].append(synth[ch].run(hybrid(gr[ch], xr[ch], overlap[ch])))
    return np.stack([np.concatenate(p) for p in pcm])
