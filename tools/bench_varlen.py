"""Ragged-batch throughput (SURVEY.md 8f3 / BASELINE C5-style length mix) on one GPU.

Synthetic utterances with lengths drawn from a seeded LibriSpeech-test-like distribution
(log-normal around 6.5 s, clipped to [1.5 s, 35 s]); w2v2-base shapes, 10 SUTA steps, LS.sh flags.
Compares one utterance per engine call against length-sorted ragged batches (suta_adapt_varlen,
grouped as the driver does) over the same utterances, inputs resident in HBM.  Prints one JSON line.
usage: python tools/bench_varlen.py [--n 256] [--gpu-batch 64] [--budget-s 512] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import suta_loader  # noqa: E402

suta_loader.load()
import torch  # noqa: E402

from suta_amd import synth  # noqa: E402
from suta_amd.config import get_config  # noqa: E402
from suta_amd.engine import SutaEngine, SutaHParams  # noqa: E402
from suta_amd.flops import suta_flops  # noqa: E402
from suta_amd.main import LAYOUT_QUANTUM, ragged_groups  # noqa: E402
from suta_amd.weights import synth_weights  # noqa: E402


def lengths(n, seed=20260415):
    rng = np.random.default_rng(seed)
    sec = np.clip(rng.lognormal(np.log(6.5), 0.6, n), 1.5, 35.0)
    return (sec * 16000).astype(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--gpu-batch", type=int, default=64)
    ap.add_argument("--budget-s", type=float, default=512.0, help="padded audio seconds per ragged batch")
    ap.add_argument("--min-fill", type=float, default=0.35,
                    help="0 = greedy grouping; > 0 = padding-minimising partition (suta_amd/main.py ragged_groups)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--single", type=int, default=16, help="utterances timed one per call (subset)")
    args = ap.parse_args()
    cfg = get_config("wav2vec2-base")
    ns = lengths(args.n)
    waves = [torch.from_numpy(synth.wave(int(n), 5000 + i)).cuda() for i, n in enumerate(ns)]
    eng = SutaEngine(cfg, synth_weights(cfg), max_batch=args.gpu_batch, max_samples=int(ns.max()) + 1600)
    hp = SutaHParams()
    rec = [0, 1, 3, 5, 10] if args.steps >= 10 else [0, args.steps]
    order = np.argsort(ns)
    # the driver's grouping (suta_amd/main.py ragged_groups): length-sorted, <= gpu_batch utterances and
    # <= budget seconds of padded audio per batch, layout rounded up to LAYOUT_QUANTUM
    groups = [order[g] for g in ragged_groups([int(ns[i]) for i in order], args.gpu_batch, args.budget_s * 16000,
                                                  args.min_fill)]
    q = LAYOUT_QUANTUM
    padded = [torch.zeros((len(g), -(-int(ns[g].max()) // q) * q), device="cuda") for g in groups]
    for p, g in zip(padded, groups):
        for j, i in enumerate(g):
            p[j, :ns[i]] = waves[i]
    # warm-up: one group, one single
    eng.adapt_varlen(padded[0], 1, hp, record=[1], lengths=[int(ns[i]) for i in groups[0]], want_logits=False)
    eng.adapt(waves[0][None], 1, hp, record=[1], want_logits=False)
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    for p, g in zip(padded, groups):
        eng.adapt_varlen(p, args.steps, hp, record=rec, lengths=[int(ns[i]) for i in g], want_logits=False)
    eng.sync()
    t_batch = time.perf_counter() - t0

    sub = order[np.linspace(0, len(order) - 1, args.single).astype(int)]
    t0 = time.perf_counter()
    for i in sub:
        eng.adapt(waves[i][None], args.steps, hp, record=rec, want_logits=False)
    eng.sync()
    t_single = time.perf_counter() - t0

    flops = sum(suta_flops(cfg, int(n), args.steps) for n in ns)
    pad = sum(p.shape[0] * p.shape[1] for p in padded) / float(ns.sum())
    out = {"metric": "adapted utterances/sec, ragged length mix (1.5-35 s), w2v2-base, 10 SUTA steps",
           "n_utterances": int(args.n), "mean_seconds": round(float(ns.mean()) / 16000, 2),
           "gpu_batch": args.gpu_batch, "n_batches": len(groups), "ragged_utt_per_s": round(args.n / t_batch, 3),
           "single_utt_per_s": round(len(sub) / t_single, 3),
           "ragged_speedup": round((args.n / t_batch) / (len(sub) / t_single), 2),
           "ragged_algorithmic_tflops": round(flops / t_batch / 1e12, 2),
           "padding_overhead": round(pad - 1.0, 4), "grouping": "greedy" if args.min_fill <= 0 else f"min-padding DP (min_fill {args.min_fill})",
           "single_subset": f"{len(sub)} utterances spread over the length range"}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
