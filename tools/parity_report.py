"""Print max |engine - reference| per golden (GPU box).  Usage: python tools/parity_report.py"""
import ast, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import suta_loader; suta_loader.load()
from suta_amd import synth
from suta_amd.config import get_config
from suta_amd.engine import SutaEngine, SutaHParams
from suta_amd.weights import synth_weights
G = os.path.join(ROOT, "tests", "golden")
eng_cache = {}
def eng(p):
    if p not in eng_cache:
        c = get_config(p); eng_cache[p] = SutaEngine(c, synth_weights(c), max_batch=2)
    return eng_cache[p]
for v in ["group", "group_lr5e-4", "layer", "layer_lr5e-4", "group_lnonly", "group_biasonly", "group_em1"]:
    z = np.load(f"{G}/g3_tiny_{v}.npz"); h = ast.literal_eval(str(z["hp_json"]))
    e = eng("tiny-group" if v.startswith("group") else "tiny-layer")
    hp = SutaHParams(lr=h["lr"], temp=h["temp"], em_coef=h["em"], reweight=h["rw"], non_blank=h["nb"], div_coef=h["div"], train_feature=h["train_feature"], bias_only=h["bias_only"])
    for n in (8000, 12345):
        lg, _, _ = e.adapt(z[f"N{n}/x"], 10, hp, record=list(range(11)))
        d = [np.abs(lg[i][0] - z[f"N{n}/logits"][i]).max() for i in range(11)]
        pm = max(np.abs(e.get_param(0, k[len(f"N{n}/final/"):]) - z[k]).max() for k in z.files if k.startswith(f"N{n}/final/"))
        print(f"tiny {v:15s} N={n}: max|dlogits| step0 {d[0]:.2e} max {max(d):.2e}  max|dparam| {pm:.2e}")
for n in (16000, 32000):
    z = np.load(f"{G}/g4_base_{n}.npz"); e = eng("wav2vec2-base")
    steps = [int(s) for s in z["steps"]]
    lg, _, _ = e.adapt(synth.wave(n, 0 if n == 16000 else 1), 10, SutaHParams(), record=steps)
    print(f"base N={n}: " + " ".join(f"s{s}:{np.abs(lg[s][0]-z['logits'][j]).max():.2e}" for j, s in enumerate(steps)))
