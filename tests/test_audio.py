"""CPU tier: the input pipeline's audio path.

* libsuta_audio's FLAC decoder (include/suta_audio.h) against a from-spec encoder
  (tests/flac_spec_encoder.py) over every coding tool: bit-exact, i.e. decoded float32 ==
  integer samples * 2^-(bps-1), the value torchaudio.load returns (reference data.py:15).
  Files from real encoders (libFLAC, ffmpeg): none exist in this image -- parity unpinned.
* WAV decoding with the reference's channel layout ((C, N).reshape(-1), data.py:18).
* the torchaudio Resample restatement (data.py:16-17): length rule and band-limited behaviour
  (torchaudio itself is absent: parity unpinned beyond the restated algorithm).
"""
import wave

import numpy as np
import pytest

from suta_amd import data as D
from tests import flac_spec_encoder as E
from tests.flac_spec_encoder import Frame, Sub


def _signal(n, bps, channels=1, seed=0, kind="speechlike"):
    rng = np.random.default_rng(seed)
    amp = (1 << (bps - 1)) - 1
    out = []
    for c in range(channels):
        if kind == "speechlike":   # smooth (predictable) plus noise, with a clipped burst
            t = np.arange(n)
            x = 0.4 * np.sin(2 * np.pi * t * (0.01 + 0.003 * c)) + 0.05 * rng.standard_normal(n)
            x[n // 3:n // 3 + n // 10] *= 3.0
            x = np.clip(x, -1, 1)
        else:
            x = rng.uniform(-1, 1, n)
        out.append(np.round(x * amp).astype(np.int64))
    return np.stack(out)


def _check(blob, ref, bps):
    x, sr = D.flac_decode(blob)
    assert x.dtype == np.float32 and x.shape == ref.shape
    want = (ref.astype(np.float64) / float(1 << (bps - 1))).astype(np.float32)
    assert np.array_equal(x, want)
    return sr


@pytest.mark.parametrize("kind,order", [("fixed", 0), ("fixed", 1), ("fixed", 2), ("fixed", 3), ("fixed", 4),
                                        ("lpc", 1), ("lpc", 2), ("lpc", 8), ("lpc", 12), ("lpc", 32),
                                        ("verbatim", 0)])
def test_flac_subframe_types_round_trip(kind, order):
    ref = _signal(5000, 16)
    frames = E.simple_frames(5000, 1, blocksize=1152, kind=kind, order=order)
    assert _check(E.encode(ref, 16000, 16, frames), ref, 16) == 16000


def test_flac_constant_and_silent_frames():
    ref = np.zeros((1, 4096 + 1000), np.int64)
    ref[0, 4096:] = -1234
    frames = [Frame(4096, subs=[Sub("constant")]), Frame(1000, subs=[Sub("constant")])]
    _check(E.encode(ref, 16000, 16, frames), ref, 16)


@pytest.mark.parametrize("mode", ["independent", "left_side", "side_right", "mid_side"])
@pytest.mark.parametrize("bps", [16, 24])
def test_flac_stereo_decorrelation(mode, bps):
    ref = _signal(6000, bps, channels=2, seed=1)
    frames = E.simple_frames(6000, 2, blocksize=2048, kind="lpc", order=6, channel_mode=mode)
    _check(E.encode(ref, 16000, bps, frames), ref, bps)


@pytest.mark.parametrize("bps", [4, 8, 12, 16, 20, 24, 32])
def test_flac_sample_sizes(bps):
    ref = _signal(3000, bps, seed=bps, kind="noise")
    frames = E.simple_frames(3000, 1, blocksize=1024, kind="verbatim" if bps == 32 else "fixed", order=2)
    if bps not in E.BPS_CODES:   # 4 bits: only expressible as "from STREAMINFO"
        for f in frames:
            f.ss_from_streaminfo = True
    _check(E.encode(ref, 16000, bps, frames), ref, bps)


def test_flac_stereo_side_channel_of_32_bit_stream():
    """Side = L - R needs 33 bits at 32 bps: the decoder keeps it exact."""
    ref = np.array([[(1 << 31) - 1, -(1 << 31), 5, -7] * 64, [-(1 << 31), (1 << 31) - 1, -5, 7] * 64], np.int64)
    for mode in ("left_side", "side_right", "mid_side"):
        frames = [Frame(256, mode, [Sub("verbatim"), Sub("verbatim")])]
        _check(E.encode(ref, 16000, 32, frames), ref, 32)


def test_flac_residual_coding_variants():
    ref = _signal(4096 * 4, 16, seed=3)
    frames = [
        Frame(4096, subs=[Sub("fixed", 2, porder=0)]),
        Frame(4096, subs=[Sub("lpc", 8, porder=8, rice2=True)]),
        Frame(4096, subs=[Sub("fixed", 1, porder=3, escape=(0, 2, 7))]),
        Frame(4096, subs=[Sub("fixed", 2, porder=2, rice2=True, param=20)]),
    ]
    _check(E.encode(ref, 16000, 16, frames), ref, 16)
    # an escaped partition of all-zero residuals codes 0 bits per sample
    z = np.zeros((1, 1024), np.int64)
    z[0, :4] = [1, 2, 3, 4]
    _check(E.encode(z, 16000, 16, [Frame(1024, subs=[Sub("fixed", 4, porder=2, escape=(0, 1, 2, 3))])]), z, 16)


def test_flac_wasted_bits():
    ref = _signal(3000, 16, seed=4) & ~np.int64(0xF)   # 4 low zero bits in every sample
    frames = E.simple_frames(3000, 1, blocksize=1000, kind="lpc", order=4)
    blob = E.encode(ref, 16000, 16, frames)
    _check(blob, ref, 16)
    frames = [Frame(3000, subs=[Sub("fixed", 2, wasted=0)])]
    _check(E.encode(ref, 16000, 16, frames), ref, 16)


@pytest.mark.parametrize("variable", [False, True])
def test_flac_block_size_codes_and_blocking(variable):
    sizes = [192, 576, 1152, 2304, 4608, 256, 512, 1024, 2048, 4096, 8192, 100, 1000, 17, 1]
    ref = _signal(sum(sizes), 16, seed=5)
    frames = []
    for bs in sizes:
        frames.append(Frame(bs, subs=[Sub("fixed", min(2, bs - 1) if bs > 1 else 0)]))
    _check(E.encode(ref, 16000, 16, frames, variable=variable), ref, 16)


@pytest.mark.parametrize("rate,code", [(16000, None), (44100, None), (16000, 0), (16000, 12), (22050, 13),
                                       (16000, 14), (48000, 14)])
def test_flac_sample_rate_codes(rate, code):
    ref = _signal(2048, 16, seed=6)
    frames = [Frame(2048, subs=[Sub("lpc", 4)], sr_code=code)]
    assert _check(E.encode(ref, rate, 16, frames), ref, 16) == rate


def test_flac_metadata_blocks_and_id3_prefix():
    ref = _signal(4000, 16, seed=7)
    frames = E.simple_frames(4000, 1, blocksize=4096, kind="lpc", order=8)
    blob = E.encode(ref, 16000, 16, frames, extra_metadata=True, id3=True)
    _check(blob, ref, 16)
    assert D.flac_info(blob) == (16000, 1, 16, 4000)


def test_flac_many_frame_numbers():
    """Frame numbers >= 128 use multi-byte UTF-8 coding in the header."""
    ref = _signal(300 * 17, 16, seed=8)
    frames = [Frame(17, subs=[Sub("fixed", 1)]) for _ in range(300)]
    _check(E.encode(ref, 16000, 16, frames), ref, 16)


def test_flac_crc_and_truncation_errors():
    ref = _signal(4096, 16, seed=9)
    blob = bytearray(E.encode(ref, 16000, 16, E.simple_frames(4096, 1, 1024, "fixed", 2)))
    bad = bytearray(blob)
    bad[-3] ^= 0x10   # inside the last frame's body
    with pytest.raises(RuntimeError, match="CRC"):
        D.flac_decode(bytes(bad))
    with pytest.raises(RuntimeError):
        D.flac_decode(bytes(blob[:-40]))
    with pytest.raises(RuntimeError, match="fLaC"):
        D.flac_decode(b"RIFF" + bytes(100))


def test_flac_file_through_audio_reader(tmp_path):
    """A LibriSpeech-style FLAC file through the reader: same samples as the float32 reference layout,
    truncation at 600 000 samples (data.py:19-22) and the header-only length used for sharding."""
    blocks = 650000 // 5000
    ref = np.repeat(np.arange(blocks, dtype=np.int64) * 97 - 6000, 5000)[None]   # constant blocks: cheap to encode
    ref[0, :5000] = _signal(5000, 16, seed=10)[0]
    frames = [Frame(5000, subs=[Sub("lpc", 8) if i == 0 else Sub("constant")]) for i in range(blocks)]
    p = tmp_path / "1-2-0003.flac"
    p.write_bytes(E.encode(ref, 16000, 16, frames))
    x = D.AudioReader(0.0)(str(p))
    assert x.shape == (600000,)
    assert np.array_equal(x, (ref[0, :600000] / 32768.0).astype(np.float32))
    assert D.decoded_length(str(p)) == 600000
    assert D.audio_info(str(p)) == (650000, 16000)


def _write_wav(path, x_int16, rate=16000):
    C = x_int16.shape[0]
    with wave.open(str(path), "wb") as f:
        f.setnchannels(C)
        f.setsampwidth(2)
        f.setframerate(rate)
        f.writeframes(np.ascontiguousarray(x_int16.T).astype("<i2").tobytes())


def test_two_channel_wav_concatenates_channels(tmp_path):
    """torchaudio.load gives (C, N) and the reference flattens it (data.py:18): channel 0, then 1."""
    ref = _signal(1000, 16, channels=2, seed=11)
    _write_wav(tmp_path / "a.wav", ref)
    x = D.AudioReader(0.0)(str(tmp_path / "a.wav"))
    assert np.array_equal(x, (ref.reshape(-1) / 32768.0).astype(np.float32))
    ref2 = _signal(1000, 16, channels=2, seed=12)
    p = tmp_path / "b.flac"
    p.write_bytes(E.encode(ref2, 16000, 16, E.simple_frames(1000, 2, 1000, "fixed", 1, "mid_side")))
    y = D.AudioReader(0.0)(str(p))
    assert np.array_equal(y, (ref2.reshape(-1) / 32768.0).astype(np.float32))
    assert D.decoded_length(str(p)) == 2000


@pytest.mark.parametrize("sr", [8000, 22050, 44100, 48000])
def test_resample_length_rule_and_passband(sr):
    """Resample(sr, 16000): output length ceil(16000 n / sr); a 300 Hz tone survives within 1e-3
    (Hann-windowed sinc, rolloff 0.99); a tone above the new Nyquist is removed."""
    n = sr  # one second
    t = np.arange(n) / sr
    y = D.resample(np.sin(2 * np.pi * 300 * t).astype(np.float32), sr)
    assert y.shape == (-(-16000 * n // sr),)
    tt = np.arange(y.size) / 16000
    np.testing.assert_allclose(y[200:-200], np.sin(2 * np.pi * 300 * tt)[200:-200], atol=2e-3)
    if sr > 16000:
        z = D.resample(np.sin(2 * np.pi * (0.45 * sr) * t).astype(np.float32), sr)
        assert np.abs(z[200:-200]).max() < 0.02


def test_resample_kernel_is_torchaudio_shape():
    """torchaudio's bank for 48 kHz -> 16 kHz (gcd 16000: orig 3, new 1): width ceil(6*3/0.99) = 19,
    kernel length 2*19 + 3 = 41; every phase sums to ~1 (unit DC gain)."""
    k, w = D.sinc_resample_kernel(3, 1)
    assert w == 19 and k.shape == (1, 1, 41)
    k, w = D.sinc_resample_kernel(441, 160)
    assert k.shape == (160, 1, 2 * w + 441)
    np.testing.assert_allclose(k.sum(-1).reshape(-1), 1.0, atol=2e-3)


def test_threaded_loader_equals_serial(tmp_path):
    """iter_collated with a thread pool yields the serial loader's batches, noise included."""
    root = tmp_path / "test-other" / "1" / "2"
    root.mkdir(parents=True)
    lines = []
    for i in range(6):
        ref = _signal(3000 + 700 * i, 16, seed=20 + i)
        name = f"1-2-{i:04d}"
        (root / f"{name}.flac").write_bytes(E.encode(ref, 16000, 16,
                                                     E.simple_frames(ref.shape[1], 1, 1024, "lpc", 4)))
        lines.append(f"{name} WORD{i} " + "A " * i)
    (root / "1-2.trans.txt").write_text("\n".join(l.strip() for l in lines) + "\n")
    serial = D.load_dataset(None, "librispeech", str(tmp_path), 1, extra_noise=0.01)
    threaded = D.load_dataset(None, "librispeech", str(tmp_path), 1, extra_noise=0.01)
    a = list(serial.iter_collated(range(len(serial)), workers=0))
    b = list(threaded.iter_collated(range(len(threaded)), workers=4, window=2))
    assert [i for i, _ in a] == [i for i, _ in b] == list(range(6))
    for (_, x), (_, y) in zip(a, b):
        assert x[2] == y[2] and np.array_equal(x[1][0], y[1][0])


def test_flac_rfc9639_example_1_known_answer():
    """RFC 9639 Appendix D.1 (decoding example 1), the byte-exact stream of the specification: a stereo 16-bit
    44.1 kHz file of one sample per channel.  Its frame-header CRC-8 and frame CRC-16 pass, it decodes to the
    samples the RFC states (25588, 10416), and the MD5 of the decoded samples equals the one in its STREAMINFO,
    so the stream typed here is the RFC's own (a typing slip would fail a CRC or the MD5)."""
    import hashlib
    import struct
    stream = bytes.fromhex("664c6143800000221000100000000f00000f0ac442f0000000013e84b41807dc690307586a3dad1a2e0f"
                           "fff869180000bf0358fd03128baa9a")
    x, sr = D.flac_decode(stream, verify_crc=True)
    assert sr == 44100 and x.shape == (2, 1)
    ints = [int(round(v * 32768)) for v in x[:, 0]]
    assert ints == [25588, 10416]
    assert hashlib.md5(struct.pack("<2h", *ints)).digest() == stream[26:42]
