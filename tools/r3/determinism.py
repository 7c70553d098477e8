"""Run-to-run determinism probe (bf16 mode, wav2vec2-base, one utterance): the same adapt call repeated, with
graphs on / off and SUTA_PRE_BF16 on / off; prints, per setting, the first recorded step whose logits differ
between repeats (or 'bitwise' when all repeats agree)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import suta_loader  # noqa: E402

suta_loader.load()
import numpy as np  # noqa: E402

from suta_amd import synth  # noqa: E402
from suta_amd.config import get_config  # noqa: E402
from suta_amd.engine import SutaEngine, SutaHParams  # noqa: E402
from suta_amd.weights import synth_weights  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "wav2vec2-base"
    cfg = get_config(model)
    xs = synth.batch(32000, 2, start=40)
    rec = [0, 1, 2, 3]
    for pre in ("1", "0"):
        os.environ["SUTA_PRE_BF16"] = pre
        for graphs in (True, False):
            eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2, max_samples=32000)
            eng.set_precision("bf16")
            eng.set_graphs(graphs)
            eng.adapt(xs, 3, SutaHParams(), record=[3])
            runs = [eng.adapt(xs[1], 3, SutaHParams(), record=rec)[0] for _ in range(5)]
            eng.close()
            bad = []
            for i in range(1, len(runs)):
                for r in rec:
                    if not np.array_equal(runs[0][r][0], runs[i][r][0]):
                        d = np.abs(runs[0][r][0] - runs[i][r][0])
                        bad.append(f"run {i} step {r}: max|d| {d.max():.3g} at frame {np.unravel_index(d.argmax(), d.shape)[0]}")
                        break
            print(f"{model} pre_bf16={pre} graphs={graphs}: " + ("bitwise" if not bad else "; ".join(bad)), flush=True)


if __name__ == "__main__":
    main()
