"""Experiment: E engines on one GPU (each its own HIP stream, graphs and workspace), each adapting
B/E utterances per step, driven concurrently from E host threads (ctypes releases the GIL), against
one engine adapting all B.  Same synthetic workload as bench.py (8 s utterances): w2v2-base, 10 SUTA steps,
fp32 (config C2), or --c4: w2v2-large, 20 steps, bf16 GEMMs (config C4).

usage: python tools/bench_streams.py [--engines 2] [--batch 64] [--steps 3] [--c4]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import suta_loader  # noqa: E402

suta_loader.load()
import torch  # noqa: E402
from suta_amd import synth  # noqa: E402
from suta_amd.config import get_config  # noqa: E402
from suta_amd.engine import SutaEngine, SutaHParams  # noqa: E402
from suta_amd.weights import synth_weights  # noqa: E402

RECORD = [0, 1, 3, 5, 10]


def run(E, B, N, S, steps, warmup, cfg, sd, precision="fp32"):
    per = B // E
    engs = [SutaEngine(cfg, sd, device=0, max_batch=per, max_samples=N) for _ in range(E)]
    for e in engs:
        e.set_precision(precision)
    hp = SutaHParams()
    rec = [r for r in (0, 1, 5, 10, 20) if r <= S] if S == 20 else RECORD
    waves = [[torch.from_numpy(synth.batch(N, per, start=(i * E + e) * per)).to("cuda:0") for e in range(E)]
             for i in range(warmup + steps)]
    torch.cuda.synchronize()

    def step(i):
        if E == 1:
            engs[0].adapt(waves[i][0], S, hp, record=rec, want_logits=False)
            return
        th = [threading.Thread(target=engs[e].adapt, args=(waves[i][e], S, hp),
                               kwargs={"record": rec, "want_logits": False}) for e in range(E)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    for i in range(warmup):
        step(i)
    for e in engs:
        e.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    for e in engs:
        e.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for e in engs:
        e.close()
    return B * steps / el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--c4", action="store_true", help="config C4: wav2vec2-large, 20 SUTA steps, bf16 GEMMs")
    a = ap.parse_args()
    cfg = get_config("wav2vec2-large" if a.c4 else "wav2vec2-base")
    sd = synth_weights(cfg)
    N, S = 128000, (20 if a.c4 else 10)
    prec = "bf16" if a.c4 else "fp32"
    one = run(1, a.batch, N, S, a.steps, a.warmup, cfg, sd, prec)
    many = run(a.engines, a.batch, N, S, a.steps, a.warmup, cfg, sd, prec)
    print(json.dumps({"engines_1_utt_s": round(one, 3), f"engines_{a.engines}_utt_s": round(many, 3),
                      "ratio": round(many / one, 4)}), flush=True)


if __name__ == "__main__":
    main()
