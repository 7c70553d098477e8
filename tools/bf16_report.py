"""Measure the bf16 GEMM mode (SUTA_PRECISION_BF16) and the large config against the references
(GPU box).  Prints max |engine - reference| of logits, relative to max |reference logits|, and the
greedy-id agreement; the tolerances in tests/test_gpu_large_bf16.py come from these numbers.
Usage: python tools/bf16_report.py"""
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
cache = {}
def eng(p, mb=2, ms=None):
    if p not in cache:
        c = get_config(p); cache[p] = SutaEngine(c, synth_weights(c), max_batch=mb, **({"max_samples": ms} if ms else {}))
    return cache[p]
def cmp(a, r):
    d = np.abs(a - r).max(); rel = d / np.abs(r).max(); agree = float((a.argmax(-1) == r.argmax(-1)).mean())
    return f"abs {d:.2e} rel {rel:.2e} ids {agree:.3f}"
for prec in ("fp32", "bf16"):
    for v in ["group", "group_lr5e-4", "layer", "layer_lr5e-4"]:
        z = np.load(f"{G}/g3_tiny_{v}.npz"); h = ast.literal_eval(str(z["hp_json"]))
        e = eng("tiny-group" if v.startswith("group") else "tiny-layer"); e.set_precision(prec)
        hp = SutaHParams(lr=h["lr"], temp=h["temp"], em_coef=h["em"], reweight=h["rw"], non_blank=h["nb"], div_coef=h["div"], train_feature=h["train_feature"], bias_only=h["bias_only"])
        for n in (8000, 12345):
            lg, _, _ = e.adapt(z[f"N{n}/x"], 10, hp, record=list(range(11)))
            print(f"{prec} tiny {v:13s} N={n}: s0 {cmp(lg[0][0], z[f'N{n}/logits'][0])} | s10 {cmp(lg[10][0], z[f'N{n}/logits'][10])}", flush=True)
    z = np.load(f"{G}/g4_base_16000.npz"); e = eng("wav2vec2-base", ms=128000); e.set_precision(prec)
    steps = [int(s) for s in z["steps"]]
    lg, _, _ = e.adapt(synth.wave(16000, 0), 10, SutaHParams(), record=steps)
    print(f"{prec} base 16000: " + " | ".join(f"s{s} {cmp(lg[s][0], z['logits'][j])}" for j, s in enumerate(steps)), flush=True)
    z = np.load(f"{G}/g7_large_16000.npz"); e = eng("wav2vec2-large"); e.set_precision(prec)
    steps = [int(s) for s in z["steps"]]
    from tests.golden.make_golden import wave
    lg, _, _ = e.adapt(wave(16000, 7), 20, SutaHParams(), record=steps)
    print(f"{prec} large 16000: " + " | ".join(f"s{s} {cmp(lg[s][0], z['logits'][j])}" for j, s in enumerate(steps)), flush=True)
# bf16 vs exact fp32 engine at the bench length (8 s)
e = eng("wav2vec2-base", ms=128000)
x = synth.wave(128000, 4)
e.set_precision("fp32"); a, _, _ = e.adapt(x, 10, SutaHParams(), record=[0, 10])
e.set_precision("bf16"); b, _, _ = e.adapt(x, 10, SutaHParams(), record=[0, 10])
print("base 8s bf16 vs fp32: s0", cmp(b[0][0], a[0][0]), "| s10", cmp(b[10][0], a[10][0]))
