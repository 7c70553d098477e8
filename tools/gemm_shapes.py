"""Per-GEMM-shape time table of one adapt call (engine timing + launch census: HIP events around every GEMM,
eager launches).  Default: config C4 (wav2vec2-large, 64 x 128 000 samples, 20 steps, bf16).

usage: python tools/gemm_shapes.py [--model wav2vec2-large] [--batch 64] [--steps 20] [--precision bf16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import suta_loader  # noqa: E402

suta_loader.load()
import torch  # noqa: E402

from suta_amd import synth  # noqa: E402
from suta_amd.config import get_config  # noqa: E402
from suta_amd.engine import SutaEngine, SutaHParams  # noqa: E402
from suta_amd.weights import synth_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="wav2vec2-large")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--samples", type=int, default=128000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--precision", default="bf16")
    a = ap.parse_args()
    cfg = get_config(a.model)
    eng = SutaEngine(cfg, synth_weights(cfg), device=0, max_batch=a.batch, max_samples=a.samples)
    eng.set_precision(a.precision)
    hp = SutaHParams()
    x = torch.from_numpy(synth.batch(a.samples, a.batch, start=7000)).cuda()
    eng.adapt(x, a.steps, hp, want_logits=False)     # warm-up (allocations, graph capture)
    eng.sync()
    eng.set_graphs(False)
    eng.set_census(True)
    eng.set_timing(True)
    eng.adapt(x, a.steps, hp, want_logits=False)
    eng.sync()
    tex = eng.get_timing_ex()
    shapes = eng.get_gemm_shape_times()
    census = {k: v for k, v in eng.get_census().items() if not k.startswith("ms|")}
    eng.set_timing(False)
    eng.set_census(False)
    eng.close()
    tot = sum(ms for _, ms in shapes.values())
    print(f"GEMM family {tex['gemm'][0]:.1f} ms ({tex['gemm'][1]} launches); shapes below sum to {tot:.1f} ms")
    print(f"{'ms':>9s} {'%':>5s} {'n':>5s} {'us/launch':>9s} {'TF':>7s}  shape")
    for shape, (n, ms) in sorted(shapes.items(), key=lambda kv: -kv[1][1]):
        f = dict(t.split("=") for t in shape.split() if "=" in t)
        fl = 2.0 * int(f["M"]) * int(f["N"]) * int(f["K"]) * int(f["z"]) * n
        print(f"{ms:9.2f} {100 * ms / tot:5.1f} {n:5d} {1000 * ms / n:9.1f} {fl / (ms / 1e3) / 1e12:7.1f}  {shape}")
    print("census (kernel tile z split form: launches):")
    for k, v in sorted(census.items()):
        print(f"  {k}: {v}")


if __name__ == "__main__":
    main()
