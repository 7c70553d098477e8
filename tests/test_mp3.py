"""MP3 (MPEG audio Layer III) decoder of libsuta_audio (csrc/mp3.cpp) — row f2, the CommonVoice clips the reference
reads with torchaudio.load (reference corpus/commonvoice.py:32-38, data.py:15).  CPU tests.

Pins:
  * the Huffman tables (csrc/mp3_tables.h) are complete prefix codes and tables 1-7 equal the values typed from
    the standard (tools/mp3_tables.py also checks them against the copy of Annex B in FFmpeg, when present);
  * a real encoder's file (tests/golden/mp3_lavc_keypress.mp3: MathJax's a11y sound, Apache-2.0, 44.1 kHz
    stereo 64 kbit/s, written by FFmpeg's libmp3lame wrapper "Lavc56.30" with an Info frame): every one of its
    84 granule-channels' Huffman data ends exactly at part2_3_length, the frame count equals the Info frame's,
    the length follows FFmpeg's gapless rule (21 * 1152 - 576 - 529 samples), and the output is a band-limited
    signal (a wrong synthesis or frequency inversion mirrors energy into the upper half of the band);
  * frames written bit by bit from known spectra (tests/mp3_builder.py: every block type, mixed blocks,
    mid/side stereo, count1 tables A and B, all big-value tables incl. linbits) decode to the PCM that the numpy
    restatement of the standard's formulas computes (oracle/mp3_np.py) within float32 rounding.
Parity with torchaudio itself is unpinned (not installed; FFmpeg's float decoder uses other transforms, so
agreement would be to ~1e-6, not bitwise).
"""
import os
import re

import numpy as np
import pytest

import mp3_builder as B
from oracle import mp3_np as O
from suta_amd import data as D

HERE = os.path.dirname(os.path.abspath(__file__))
REAL = os.path.join(HERE, "golden", "mp3_lavc_keypress.mp3")


def test_huffman_tables_are_complete_prefix_codes():
    H = B.huff()
    for t, (lens, cods) in H.items():
        assert abs(sum(2.0 ** -l for l in lens) - 1.0) < 1e-12, t
        words = sorted(format(c, "0%db" % l) for c, l in zip(cods, lens))
        assert all(not words[i + 1].startswith(words[i]) for i in range(len(words) - 1)), t
    # tables 1 and 7 as typed from Table B.7
    assert H[1] == ([1, 3, 2, 3], [1, 1, 1, 0])
    assert H[7][0][:6] == [1, 3, 6, 8, 8, 9] and H[7][1][:6] == [1, 2, 10, 19, 16, 10]
    win = O.window_d()
    assert win[256] == 75038 / 65536 and win[1] == -1 / 65536 and win[511] == 1 / 65536


def test_real_encoder_file_parses_exactly():
    sr, ch, n = D.mp3_info(REAL)
    x, sr2, st = D.mp3_decode(REAL, strict=True, stats=True)
    assert (sr, ch, sr2) == (44100, 2, 44100)
    assert n == 21 * 1152 - 576 - 529 == x.shape[1]
    frames, granules, exact, overrun, lost = st.tolist()
    assert (frames, granules, exact, overrun, lost) == (21, 84, 84, 0, 0)
    assert np.isfinite(x).all() and 0.3 < np.abs(x).max() < 1.0
    for c in range(2):
        P = np.abs(np.fft.rfft(x[c].astype(np.float64))) ** 2
        f = np.fft.rfftfreq(x.shape[1], 1 / sr)
        assert P[f > 11025].sum() / P.sum() < 1e-6


@pytest.mark.parametrize("channels,ms,blocks", [
    (1, False, [0, 0, 0, 0]),
    (2, True, [0, 1, 2, 3]),
    (2, False, [2, 2, 0, 1]),
    (1, False, [1, 2, 2, 3]),
    (2, True, [2, 2, 2, 2]),
])
def test_built_frames_match_numpy_restatement(channels, ms, blocks):
    rng = np.random.default_rng(len(blocks) * 7 + channels * 3 + int(ms) + sum(blocks))
    frames, spec, k = [], [], 0
    for _ in range(3):
        grs = []
        for _ in range(2):
            bt = blocks[k % len(blocks)]
            k += 1
            grs.append([B.random_granule(rng, bt, mixed=int(rng.integers(0, 2))) for _ in range(channels)])
        spec.append(grs)
        frames.append(B.write_frame(grs, channels, ms))
    y, sr, st = D.mp3_decode(b"".join(frames), strict=True, stats=True)
    ref = O.decode(spec, channels, ms)
    assert sr == 44100 and y.shape == ref.shape == (channels, 3 * 1152)
    assert st.tolist() == [3, 6 * channels, 6 * channels, 0, 0]
    assert np.abs(y - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_every_big_value_table_and_count1_table():
    rng = np.random.default_rng(11)
    for t in [1, 2, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15] + list(range(16, 32)):
        g = [B.random_granule(rng, 0, nbig=100, ncount1=10) for _ in range(2)]
        for i, gg in enumerate(g):
            gg["table"] = [t, t, t]
            gg["count1_table"] = i
            mv = min(B.max_value(t), 40)
            gg["is"][:100] = rng.integers(-mv, mv + 1, 100)
        data = B.write_frame([[g[0]], [g[1]]], 1)
        y, _, st = D.mp3_decode(data, strict=True, stats=True)
        assert st.tolist() == [1, 2, 2, 0, 0], t
        ref = O.decode([[[g[0]], [g[1]]]], 1)
        assert np.abs(y - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()), t


def test_stream_edges():
    rng = np.random.default_rng(3)
    grs = [[B.random_granule(rng)] for _ in range(2)]
    frame = B.write_frame(grs, 1)
    # junk and an ID3v2 tag in front, a cut frame and an ID3v1 tag behind
    id3 = b"ID3\x04\x00\x00\x00\x00\x00\x05" + b"\x00" * 5
    data = id3 + b"\x12\x34" + frame + frame + frame[:300] + b"TAG" + b"\x00" * 125
    y, sr, st = D.mp3_decode(data, stats=True)
    assert y.shape == (1, 2 * 1152) and st.tolist()[:2] == [2, 4]
    ref = O.decode([grs, grs], 1)
    assert np.abs(y - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())
    with pytest.raises(RuntimeError, match="MP3"):
        D.mp3_decode(b"\x00" * 2000)


def test_decode_channels_dispatches_mp3(tmp_path):
    p = tmp_path / "clip.mp3"
    p.write_bytes(open(REAL, "rb").read())
    x, sr = D.decode_channels(str(p))
    assert x.shape == (2, 23087) and sr == 44100
    assert D.audio_info(str(p)) == (23087, 44100)
    # channels concatenated, resampled to 16 kHz (torchaudio length rule), as the reader hands to the engine
    assert D.decoded_length(str(p)) == 2 * -(-160 * 23087 // 441)


def _info_layout(data):
    """(x, flags, tag offset) of the real file's Info frame: x = the 'Info' marker."""
    x = data.index(b"Info")
    flags = int.from_bytes(data[x + 4:x + 8], "big")
    t = x + 8 + (4 if flags & 1 else 0) + (4 if flags & 2 else 0) + (100 if flags & 4 else 0) + (4 if flags & 8 else 0)
    assert data[t:t + 4] in (b"LAME", b"Lavc", b"Lavf")
    return x, flags, t


def _with_padding(data, pad):
    x, flags, t = _info_layout(data)
    v = int.from_bytes(data[t + 21:t + 24], "big")
    v = (v & ~4095) | pad
    return data[:t + 21] + v.to_bytes(3, "big") + data[t + 24:]


def _frame_offsets(data):
    """Audio frame offsets of the real file (44.1 kHz, constant frame length of its bitrate, padding bit aware)."""
    x, _, _ = _info_layout(data)
    o = data.rfind(b"\xff", 0, x - 4)   # the Info frame's sync
    while not (data[o] == 0xFF and data[o + 1] & 0xE0 == 0xE0):
        o -= 1
    offs = []
    rates = [0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320]
    while o + 4 <= len(data) and data[o] == 0xFF and data[o + 1] & 0xE0 == 0xE0:
        br, pad = rates[data[o + 2] >> 4], (data[o + 2] >> 1) & 1
        offs.append(o)
        o += 144000 * br // 44100 + pad
    return offs[1:]   # the Info frame carries no audio


def test_gapless_end_trim_follows_the_xing_frame_count(tmp_path):
    """FFmpeg (torchaudio's MP3 backend) trims the end only from the Xing frames field: the decoded positions
    [F * 1152 - enc_padding + 529, F * 1152) of the frames that overlap them.  Builder-made variants of the real
    file: encoder padding 1600 (F = 21: 21 * 1152 - 576 - 1600 samples), the frames field removed (flags & 1 cleared:
    no end trim, 21 * 1152 - 576 - 529), and a stream cut after 15 frames (its tail is before the window: kept)."""
    data = open(REAL, "rb").read()
    x, flags, t = _info_layout(data)
    assert flags & 1 and int.from_bytes(data[x + 8:x + 12], "big") == 21
    full, _ = D.mp3_decode(REAL)
    padded = _with_padding(data, 1600)
    p = tmp_path / "pad.mp3"
    p.write_bytes(padded)
    y, _ = D.mp3_decode(str(p))
    assert y.shape[1] == 21 * 1152 - 576 - 1600 == D.mp3_info(str(p))[2]
    np.testing.assert_array_equal(y, full[:, :y.shape[1]])
    # frames field removed: the Info frame keeps its length (4 zero bytes appended at its end)
    nofr = bytearray(padded)
    nofr[x + 4:x + 8] = (flags & ~1).to_bytes(4, "big")
    offs = _frame_offsets(data)
    info_end = offs[0]
    body = bytes(nofr[:x + 8]) + bytes(nofr[x + 12:info_end]) + b"\x00" * 4 + bytes(nofr[info_end:])
    q = tmp_path / "noframes.mp3"
    q.write_bytes(body)
    z, _ = D.mp3_decode(str(q))
    assert z.shape[1] == 21 * 1152 - 576 - 529 == D.mp3_info(str(q))[2]
    np.testing.assert_array_equal(z, full)
    # truncated after 15 audio frames (a partial 16th): no end trim, the leading skip stays
    cut = padded[:offs[15] + 100]
    r = tmp_path / "cut.mp3"
    r.write_bytes(cut)
    w, _ = D.mp3_decode(str(r))
    assert w.shape[1] == 15 * 1152 - 576 - 529
    np.testing.assert_array_equal(w, full[:, :w.shape[1]])
