"""suta_amd — MI355X-native SUTA (single-utterance test-time adaptation) engine.

The hot path (reference main.py:172-215 `forward_and_adapt`, run `steps` times per
utterance by main.py:347-348) executes in `libsuta.so`: hand-written gfx950 HIP kernels
behind the C ABI declared in `include/suta.h`.  This package is the Python host:
ctypes binding (`engine`), the `forward_and_adapt`-compatible drop-in (`suta`: the reference loop body of
main.py:302-348 runs on its objects), model
geometry (`config`), seeded weights (`weights`), CTC decode / WER (`decode`), and the
main.py-compatible driver (`main`).
"""
from .config import get_config, frame_lengths, num_frames, param_shapes  # noqa: F401

__version__ = "0.1.0"
