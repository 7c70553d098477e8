"""CPU tier: the C-ABI library loads and exports every entry point include/suta.h declares.

No compute calls (no GPU here).  suta_num_frames is pure host arithmetic and is exercised.
"""
import ctypes
import os
import re

import pytest

from suta_amd import engine as E
from suta_amd.config import get_config, num_frames

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "suta.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(suta_[a-z_]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(E.EXPORTS)


def test_library_exports_every_symbol():
    if not os.path.exists(E.LIB_PATH):
        pytest.fail("libsuta.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(E.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name


@pytest.mark.parametrize("n", [399, 400, 16000, 12345, 128000, 600000])
def test_num_frames_matches_conv_recursion(n):
    """399 samples: conv6's input is 1 frame, shorter than its kernel (2): no frame (torch's Conv1d raises; the
    engine rejects the utterance), where C's truncating division would have reported one."""
    lib = E.load_library()
    cfg = get_config("wav2vec2-base")
    c = E.config_to_c(cfg)
    out = ctypes.c_int64()
    assert lib.suta_num_frames(ctypes.byref(c), n, ctypes.byref(out)) == 0
    assert out.value == max(0, num_frames(cfg, n))
    assert (out.value == 0) == (n == 399)


def test_frame_counts_from_survey():
    cfg = get_config("wav2vec2-base")
    assert num_frames(cfg, 16000) == 49
    assert num_frames(cfg, 128000) == 399
    assert num_frames(cfg, 600000) == 1874


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    monkeypatch.setattr(E, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        E.load_library(str(tmp_path / "libsuta.so"))


AUDIO_HEADER = os.path.join(REPO, "include", "suta_audio.h")


def test_audio_library_exports_every_symbol():
    """libsuta_audio.so (host FLAC and MP3 decoders) exports what include/suta_audio.h declares."""
    from suta_amd import data as D
    src = re.sub(r"/\*.*?\*/", "", open(AUDIO_HEADER).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(suta_[a-z_0-9]+)\s*\(", src)))
    assert names == ["suta_audio_last_error", "suta_flac_decode", "suta_flac_info", "suta_mp3_decode",
                     "suta_mp3_info"]
    lib = ctypes.CDLL(D.AUDIO_LIB_PATH)
    for name in names:
        assert hasattr(lib, name), name
