"""Latency of one suta_adapt call at small batches with and without the whole-loop hipGraph.

Small batches are where the S-step loop is launch-bound (~2 000 kernels per SUTA step): this measures
batch 1 and 4 (8 s utterances, 10 steps, scripts/LS.sh flags, greedy ids recorded at 0/1/3/5/10) with
graph replay on (the driver's path) and off (eager), after a warm-up that captures the graph.
usage: python tools/bench_graphs.py [--batches 1 4] [--reps 5]
"""
import argparse
import json
import os
import sys
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n-samples", type=int, default=128000)
    ap.add_argument("--model", default="wav2vec2-base")
    a = ap.parse_args()
    cfg = get_config(a.model)
    eng = SutaEngine(cfg, synth_weights(cfg), device=0, max_batch=max(a.batches), max_samples=a.n_samples)
    hp = SutaHParams()
    rec = [0, 1, 3, 5, 10]
    out = {"model": a.model, "n_samples": a.n_samples, "suta_steps": 10, "results": []}
    for B in a.batches:
        x = torch.from_numpy(synth.batch(a.n_samples, B, start=7000)).to("cuda:0")
        for graphs in (True, False):
            eng.set_graphs(graphs)
            for _ in range(2):   # first call eager (new key), second captures the loop graph
                eng.adapt(x, 10, hp, record=rec, want_logits=False)
            eng.sync()
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                eng.adapt(x, 10, hp, record=rec, want_logits=False)
                eng.sync()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            out["results"].append({"batch": B, "graphs": graphs, "median_ms": round(1000 * ts[len(ts) // 2], 2),
                                   "min_ms": round(1000 * ts[0], 2),
                                   "utt_per_s": round(B / ts[len(ts) // 2], 3)})
            print(json.dumps(out["results"][-1]), flush=True)
    eng.set_graphs(True)
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
