"""One rank of a multi-process driver run (tests/test_host.py, tests/test_gpu_cli.py).

usage: python tests/_cli_worker.py OUT_JSON FAKE -- <main.py flags>
The parent sets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT.  FAKE=1 replaces the
HIP engine with a deterministic stand-in (CPU tests of the sharding, gather and print order);
FAKE=0 runs the real libsuta engine.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import suta_loader  # noqa: E402

suta_loader.load()
import numpy as np  # noqa: E402


class FakeEngine:
    """ids depend only on the utterance's own samples and the step (as a real per-utterance
    adaptation would), never on the batch it was grouped into."""

    def __init__(self, cfg, weights, device=0, max_batch=1, max_samples=600000):
        from suta_amd.config import num_frames
        self.nf = lambda n: num_frames(cfg, n)

    def set_precision(self, mode):
        pass

    def _ids(self, x, r):
        T = self.nf(len(x))
        v = np.abs(np.asarray(x[: T * 320], np.float64)).reshape(T, -1).mean(1) if T else np.zeros(0)
        ids = (np.floor(v * 37.0 + r) % 9).astype(np.int32)
        return np.where(ids < 3, 0, ids + 2)

    def adapt(self, x, steps, hp, record=(), want_logits=True, **kw):
        x = np.asarray(x).reshape(-1)
        return None, {r: self._ids(x, r)[None] for r in record}, self.nf(len(x))

    def adapt_varlen(self, wavs, steps, hp, record=(), want_logits=True, **kw):
        return None, {r: [self._ids(np.asarray(w).reshape(-1), r) for w in wavs] for r in record}, \
            [self.nf(len(w)) for w in wavs]

    def close(self):
        pass


def main():
    out, fake = sys.argv[1], sys.argv[2] == "1"
    argv = sys.argv[sys.argv.index("--") + 1:]
    from suta_amd import engine as E
    from suta_amd import main as M
    if fake:
        E.SutaEngine = FakeEngine
    counts = M.main(argv)
    with open(out, "w") as f:
        json.dump({k: list(v) for k, v in counts.items()}, f)


if __name__ == "__main__":
    main()
