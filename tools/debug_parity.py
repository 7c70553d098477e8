"""Debug helper: vanilla-forward error of the engine (SUTA_LIB may select a library) vs the tiny goldens,
and a ragged base batch NaN check."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import suta_loader
suta_loader.load()
from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
for preset, var in (("tiny-group", "group"), ("tiny-layer", "layer")):
    z = np.load(os.path.join(G, f"g3_tiny_{var}.npz"), allow_pickle=False)
    cfg = get_config(preset)
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=2)
    x = z["N8000/x"]
    out = eng.forward(x)[0]
    print(preset, "forward maxerr", float(np.abs(out - z["N8000/logits"][0]).max()), flush=True)
    eng.close()
if len(sys.argv) > 1:
    cfg = get_config("wav2vec2-base")
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=3)
    waves = [synth.wave(n, 50 + i) for i, n in enumerate((32000, 17003, 24480))]
    lv, iv, tv = eng.adapt_varlen(waves, 1, SutaHParams(), record=[0, 1])
    for b in range(3):
        print("varlen base utt", b, "T", tv[b], "nan step0", bool(np.isnan(lv[0][b]).any()), "nan step1",
              bool(np.isnan(lv[1][b]).any()), flush=True)
    l1, _, _ = eng.adapt(waves[0], 1, SutaHParams(), record=[0, 1])
    print("single utt0 step0 err", float(np.abs(l1[0][0] - lv[0][0]).max()))
