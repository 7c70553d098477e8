"""Bench: adapted utterances/sec, 10-step SUTA on wav2vec2-base shapes (BASELINE.json config 2).

One bench "step" = one libsuta `suta_adapt` call over a batch of `--batch` synthetic 8 s
utterances (N = 128000 samples, T = 399 frames), each adapted for 10 SUTA steps with the
scripts/LS.sh flags (episodic reset, vanilla forward, greedy ids recorded at steps 0/1/3/5/10).
Waveforms are resident in HBM before the timed region.  Seeded random weights of the
w2v2-base architecture (no checkpoints offline).

Multi-GPU: one process per GPU (torchrun); every rank adapts its own utterances (no data-path
collective, weak scaling); a barrier + device sync brackets the timed region and the max
elapsed time over ranks is used.  value = utterances of all ranks / that time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import suta_loader  # noqa: E402

suta_loader.load()
import torch  # noqa: E402

from suta_amd import synth  # noqa: E402
from suta_amd.config import get_config, num_frames  # noqa: E402
from suta_amd.engine import SutaEngine, SutaHParams  # noqa: E402
from suta_amd.flops import reference_schedule_flops, suta_flops  # noqa: E402
from suta_amd.weights import synth_weights  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_PEAK_TFLOPS = 2500.0      # MI355X_MICROARCH.md: bf16 dense MFMA peak
BF16_SPLIT_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 6
HBM_PEAK_TBS = 8.0             # MI355X_MICROARCH.md: HBM3E peak
RECORD = [0, 1, 3, 5, 10]
# newest committed rocprofv3 PMC reduction of this workload (tools/pmc_traffic.py; profiles/<round>/README.md)
PMC_TRAFFIC = next((p for p in (os.path.join(ROOT, "profiles", r, "pmc_traffic.json") for r in ("r3", "r2", "r1"))
                    if os.path.exists(p)), None)
PMC_TRAFFIC_C4 = next((p for p in (os.path.join(ROOT, "profiles", r, f) for r, f in
                                   (("r3", "pmc_traffic_c4.json"), ("r2", "close_pmc_traffic_c4.json")))
                       if os.path.exists(p)), None)
BATCH = 164      # utterances per engine call (see --batch)
PMC_BATCH = 164    # the batch the committed headline PMC passes (profiles/r3/pmc_traffic.json) were taken at
PMC_BATCH_C4 = 164 # the batch of the committed C4 passes (profiles/r3/pmc_traffic_c4.json)
GEMM_KERNELS = ("gemm_glds_kernel", "gemm_f32_kernel", "gemm_splitk_reduce", "attn_fwd_kernel", "attn_bwd_kernel",
                "posconv_kernel", "flash_fwd_kernel", "flash_bwd_kernel", "flash_dq_reduce")
# config C4's GEMM family (bf16 mode): every kernel its "gemm" + "attention" timing families launch
GEMM_KERNELS_C4 = ("gemm_hb_kernel", "gemm_hb8_kernel", "gemm_hbt_kernel", "gemm_x6_kernel", "gemm_gbf_kernel",
                   "gemm_splitk_reduce",
                   "to_bf16_kernel", "posconv_bf16_kernel", "flash_fwd_bf16_kernel", "flash_bwd_bf16_kernel",
                   "flash_dq_reduce")
FRONT_KERNELS = ("conv0_gn_kernel", "col_stats_final", "gn_bwd_final", "conv0_dw_reduce")


def pmc(args):
    """The committed PMC reduction when this run is its workload (w2v2-base, PMC_BATCH x 8 s, 10 steps)."""
    if not (args.model == "wav2vec2-base" and args.batch == PMC_BATCH and args.n_samples == 128000 and args.suta_steps == 10
            and PMC_TRAFFIC):
        return None
    return json.load(open(PMC_TRAFFIC))


def gemm_traffic(d, kernels=GEMM_KERNELS):
    """HBM bytes per GEMM-family launch from the PMC passes."""
    n = sum(d[k]["launches"] for k in kernels if k in d)
    b = sum(d[k]["launches"] * d[k]["hbm_bytes_per_launch"] for k in kernels if k in d)
    return round(b / n) if n else None


def frontend_traffic(d):
    """HBM bytes per conv front-end call (a forward call = 2 conv0_gn passes + the statistics finaliser; a
    backward call = 2 passes + the GroupNorm-backward finaliser + the conv0 dW reduction)."""
    if "conv0_gn_kernel" not in d:
        return None
    b = sum(d[k]["launches"] * d[k]["hbm_bytes_per_launch"] for k in FRONT_KERNELS if k in d)
    return b / (d["conv0_gn_kernel"]["launches"] / 2)


def attention_flops(cfg, T, B):
    """Algorithmic FLOPs of the attention products per (forward, backward) layer call: S and PV forward,
    dP, dQ, dK, dV backward, for B utterances of T frames."""
    d = cfg["hidden_size"] // cfg["num_attention_heads"]
    unit = 2.0 * T * T * d * cfg["num_attention_heads"] * B
    return 2 * unit, 4 * unit


def cpu_baseline(cfg, n_samples, suta_steps, budget_s=25.0):
    """The oracle (PyTorch-CPU restatement of the reference loop) on host cores, bounded sample."""
    from oracle import w2v2_cpu as W
    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    sd = {k: torch.from_numpy(v) for k, v in synth_weights(cfg).items()}
    W.run_suta(sd, cfg, torch.from_numpy(synth.wave(16000, 999))[None], 1)          # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        x = torch.from_numpy(synth.wave(n_samples, 1000 + done))[None]
        W.run_suta(sd, cfg, x, suta_steps, record=[0, suta_steps])
        done += 1
        el = time.perf_counter() - t0
        if el >= budget_s or done >= 4:
            break
    return {"value": done / el, "unit": "utt/s", "cores": cores, "kind": "port",
            "sample": f"{done} utterance(s) of {n_samples} samples, {suta_steps} SUTA steps each, oracle/w2v2_cpu.py "
                      f"run_suta (torch {torch.__version__} CPU, {cores} threads), {el:.1f} s; schedule: the minimal "
                      f"one the engine runs ({suta_steps + 1} forwards + {suta_steps} backwards per utterance, "
                      f"{suta_flops(cfg, n_samples, suta_steps) / 1e9:.1f} GF), not the reference's "
                      f"{2 * suta_steps + 1} forwards ({reference_schedule_flops(cfg, n_samples, suta_steps) / 1e9:.1f} GF): "
                      f"the reference loop itself would take about "
                      f"{reference_schedule_flops(cfg, n_samples, suta_steps) / suta_flops(cfg, n_samples, suta_steps):.2f}x "
                      f"this time"}


def bench_c4(args, dev):
    """BASELINE.json config C4: wav2vec2-large-960h-lv60 shapes, 20-step SUTA, bf16 GEMMs (operands
    rounded to bf16, fp32 accumulation; norms, softmax, loss, AdamW and master tensors fp32), 1 GPU,
    8 s utterances.  A secondary line beside the C2 headline."""
    cfg = get_config("wav2vec2-large")
    B, N, S = args.c4_batch, args.n_samples, 20
    eng = SutaEngine(cfg, synth_weights(cfg), device=dev, max_batch=B, max_samples=N)
    eng.set_precision("bf16")
    hp = SutaHParams()
    rec = [0, 1, 5, 10, 20]
    steps = max(1, args.steps // 2)
    waves = [torch.from_numpy(synth.batch(N, B, start=50000 + i * B)).to(f"cuda:{dev}") for i in range(steps + 1)]
    eng.adapt(waves[0], S, hp, record=rec, want_logits=False)
    torch.cuda.synchronize()
    eng.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        eng.adapt(waves[1 + i], S, hp, record=rec, want_logits=False)
    eng.sync()
    el = time.perf_counter() - t0
    if not args.no_timing:   # roofline pass, outside the timed region
        eng.set_timing(True)
        eng.adapt(waves[1], S, hp, record=rec, want_logits=False)
        eng.sync()
        tex = eng.get_timing_ex()
    flops_utt = suta_flops(cfg, N, S)
    res = {"workload": f"wav2vec2-large SUTA {S} steps on {N}-sample (8 s) utterances, {B} utterances per step, "
                       "scripts/LS.sh flags, bf16 GEMMs", "config": "C4", "precision": "bf16", "dtype": "bf16",
           "value": round(B * steps / el, 4), "unit": "utt/s", "steps": steps,
           "ms_per_step": round(1000 * el / steps, 3), "algorithmic_tflops": round(flops_utt * B * steps / el / 1e12, 3),
           "rtf": round(el / (B * steps * N / 16000.0), 6)}
    if not args.no_timing:
        t = eng.get_timing()
        gms, gn = t["gemm"]
        ach = flops_utt * B / (gms / 1000.0) / 1e12
        res["roofline"] = {"bound": "mfma", "achieved": round(ach, 3), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ach / BF16_PEAK_TFLOPS, 4), "kernel": "bf16 GEMM family (bf16-plane linears and the layer-norm conv stack's forward / input gradients: gemm_hb_kernel; conv weight gradients: gemm_hbt_kernel; per-utterance projection GEMMs: gemm_x6_kernel one-plane form / gemm_gbf_kernel; posconv_bf16_kernel; flash attention on bf16 MFMA)",
                           "launches": int(gn), "avg_launch_ms": round(gms / max(1, gn), 5)}
        gx, ax = tex["gemm"], tex["attention"]
        talg = round((gx[2] + ax[2]) / max(1, gx[1] + ax[1]))
        d4 = json.load(open(PMC_TRAFFIC_C4)) if (PMC_TRAFFIC_C4 and B == PMC_BATCH_C4 and N == 128000) else None
        traffic = gemm_traffic(d4, GEMM_KERNELS_C4) if d4 else None
        res["roofline"].update({
            "traffic": traffic, "traffic_unit": "HBM bytes per GEMM-family launch",
            "traffic_source": f"{os.path.relpath(PMC_TRAFFIC_C4, ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE "
                              "passes of bench.py --only-c4)" if traffic else None,
            "traffic_alg": talg, "traffic_ratio": round(traffic / talg, 3) if traffic and talg else None})
        if ax[1]:
            T = num_frames(cfg, N)
            af, ab = attention_flops(cfg, T, B)
            layers = cfg["num_hidden_layers"]
            nf, nb = (S + 1) * layers, S * layers
            res["attention"] = {"launches": int(ax[1]), "ms": round(ax[0], 2),
                                "tflops": round((nf * af + nb * ab) / (ax[0] / 1000) / 1e12, 3),
                                "frac_bf16_peak": round((nf * af + nb * ab) / (ax[0] / 1000) / 1e12 / BF16_PEAK_TFLOPS, 4)}
        res["time_breakdown_ms"] = {k: round(v[0], 2) for k, v in tex.items()}
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    # 164 utterances x 399 frames = 65 436 rows = 512 row tiles of 128: every linear's grid (6 / 18 / 24 column
    # tiles on base, 8 / 24 / 32 on large) fills whole rounds of the 512 resident 128 x 128 blocks (64: 3.125 rounds of
    # the N = 1024 grids); measured 37.2 -> 38.2 utt/s (base) and 36.0 -> 38.1 (C4) on one box
    ap.add_argument("--batch", type=int, default=BATCH, help="utterances in flight per GPU (engine slots)")
    ap.add_argument("--n-samples", type=int, default=128000)
    ap.add_argument("--suta-steps", type=int, default=10)
    ap.add_argument("--model", default="wav2vec2-base")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-kernel HIP-event timing pass")
    ap.add_argument("--timing-steps", type=int, default=1,
                    help="batches of the separate, untimed roofline pass (per-launch HIP events, eager)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32-split-bf16", "bf16"],
                    help="GEMM arithmetic: exact fp32 MFMA, fp32-accurate 3-way bf16 split, or bf16 (config C4)")
    ap.add_argument("--no-c4", dest="c4", action="store_false",
                    help="skip the config-C4 line (wav2vec2-large, 20 SUTA steps, bf16 GEMMs; 1 GPU only)")
    ap.add_argument("--c4-batch", type=int, default=BATCH)
    ap.add_argument("--only-c4", action="store_true", help="print only the config-C4 line (profiling)")
    ap.add_argument("--no-split", dest="also_split", action="store_false",
                    help="do not also time the fp32-accurate split-bf16 GEMM mode")
    args = ap.parse_args()

    if args.only_c4:
        torch.cuda.set_device(0)
        print(json.dumps(bench_c4(args, 0)), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 with "
              f"`python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}`",
              file=sys.stderr)
        sys.exit(2)
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    cfg = get_config(args.model)
    B, N, S = args.batch, args.n_samples, args.suta_steps
    eng = SutaEngine(cfg, synth_weights(cfg), device=dev, max_batch=B, max_samples=N)
    eng.set_precision(args.precision)
    hp = SutaHParams()  # scripts/LS.sh flags
    nbatches = args.warmup + args.steps
    # inputs resident in HBM before timing: distinct utterances per rank and batch
    waves = [torch.from_numpy(synth.batch(N, B, start=(rank * nbatches + i) * B)).to(f"cuda:{dev}")
             for i in range(nbatches)]
    torch.cuda.synchronize()

    for i in range(args.warmup):
        eng.adapt(waves[i], S, hp, record=RECORD, want_logits=False)

    def barrier():
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        eng.adapt(waves[args.warmup + i], S, hp, record=RECORD, want_logits=False)
    eng.sync()
    barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=f"cuda:{dev}")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())
    # roofline pass (outside the timed region): per-launch HIP events on the engine stream; this runs
    # the eager path (timing disables graph replay), so its batch time is reported separately
    timing, timing_el, tsteps = None, None, max(1, min(args.timing_steps, args.steps))
    if not args.no_timing:
        eng.set_timing(True)
        barrier()
        t1 = time.perf_counter()
        for i in range(tsteps):
            eng.adapt(waves[args.warmup + i], S, hp, record=RECORD, want_logits=False)
        eng.sync()
        timing_el = time.perf_counter() - t1
        timing = eng.get_timing()
        timing_ex = eng.get_timing_ex()
        eng.set_timing(False)

    utts = B * args.steps * world
    value = utts / el
    flops_utt = suta_flops(cfg, N, S)
    out = {
        "metric": "adapted utterances/sec (whole node) at 10 SUTA steps, w2v2-base; WER parity",
        "value": round(value, 4), "unit": "utt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic", "precision": args.precision,
        "config": {"workload": f"{args.model} SUTA {S} steps on {N}-sample (8 s) utterances, {B} utterances "
                               f"per GPU per step, scripts/LS.sh flags",
                   "model": args.model, "global_batch": B * world, "seq_len": num_frames(cfg, N),
                   "n_samples": N, "suta_steps": S, "parallelism": f"utterance-sharded x{world}"},
        "algorithmic_tflops": round(flops_utt * utts / el / 1e12, 3),
    }
    if timing:
        gms, gn = timing["gemm"]
        # dominant kernel family: the fp32 MFMA GEMM (every conv/linear/attention product)
        gemm_flops = flops_utt * B * tsteps  # per-rank algorithmic GEMM-shaped FLOPs of the timing pass
        achieved = gemm_flops / (gms / 1000.0) / 1e12 if gms > 0 else None
        d = pmc(args)
        traffic = gemm_traffic(d) if d else None
        gx, ax, fx = timing_ex["gemm"], timing_ex["attention"], timing_ex["frontend"]
        traffic_alg = round((gx[2] + ax[2]) / max(1, gx[1] + ax[1]))
        out["roofline"] = {"bound": "mfma", "achieved": round(achieved, 3) if achieved else None,
                           "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4) if achieved else None,
                           "traffic": traffic,
                           "traffic_unit": "HBM bytes per GEMM launch",
                           "traffic_source": f"{os.path.relpath(PMC_TRAFFIC, ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + "
                                             "WRITE_SIZE passes of this workload)" if traffic else None,
                           "traffic_alg": traffic_alg,
                           "traffic_alg_def": "algorithmic bytes per GEMM-family launch, measured in this run: every "
                                              "operand touched once (A unique rows, B per distinct slice, C written, "
                                              "epilogue operands), no tile re-reads or split-K partials",
                           "traffic_ratio": round(traffic / traffic_alg, 3) if traffic and traffic_alg else None,
                           "kernel": "fp32 MFMA GEMM family: gemm_glds_kernel + gemm_f32_kernel + posconv_kernel + flash attention (flash_fwd_kernel, flash_bwd_kernel + flash_dq_reduce) (all launches)",
                           "launches": int(gn), "avg_launch_ms": round(gms / max(1, gn), 5),
                           "measured": f"HIP events around every GEMM-family launch on the engine stream, separate "
                                       f"pass of {tsteps} batch(es) after the timed region (eager path: "
                                       f"{round(1000 * timing_el / tsteps, 1)} ms per batch vs "
                                       f"{round(1000 * el / args.steps, 1)} ms replayed)"}
        out["time_breakdown_ms"] = {k: round(v[0], 2) for k, v in timing_ex.items()}
        # conv feature-encoder front-end (north_star: achieved HBM GB/s on the conv front-end)
        if fx[1]:
            fms = fx[0] / fx[1]
            fb = frontend_traffic(d) if d else None
            out["frontend"] = {"kernel": "conv0_gn_kernel passes (conv0 + GroupNorm + GELU, fwd and bwd) + finalisers",
                               "calls": int(fx[1]), "avg_call_ms": round(fms, 4),
                               "alg_bytes_per_call": round(fx[2] / fx[1]),
                               "alg_tbs": round(fx[2] / fx[1] / (fms / 1000) / 1e12, 3),
                               "hbm_bytes_per_call": round(fb) if fb else None,
                               "peak_tbs": HBM_PEAK_TBS}
            if fb:
                out["frontend"]["hbm_tbs"] = round(fb / (fms / 1000) / 1e12, 3)
                out["roofline"]["frontend_hbm_tbs"] = out["frontend"]["hbm_tbs"]
        # attention products alone (fused kernels): algorithmic FLOPs / their time
        if ax[1]:
            T = num_frames(cfg, N)
            af, ab = attention_flops(cfg, T, B)
            layers = cfg["num_hidden_layers"]
            nf, nb = (S + 1) * layers * tsteps, S * layers * tsteps
            out["attention"] = {"launches": int(ax[1]), "ms": round(ax[0], 2),
                                "tflops": round((nf * af + nb * ab) / (ax[0] / 1000) / 1e12, 3)}
    if args.also_split and args.precision == "fp32":
        # same workload with the fp32-accurate split-bf16 GEMMs (reported beside the headline)
        eng.set_precision("fp32-split-bf16")
        eng.adapt(waves[0], S, hp, record=RECORD, want_logits=False)
        barrier()
        t1 = time.perf_counter()
        for i in range(args.steps):
            eng.adapt(waves[args.warmup + i], S, hp, record=RECORD, want_logits=False)
        eng.sync()
        barrier()
        el2 = time.perf_counter() - t1
        if dist:
            t = torch.tensor([el2], device=f"cuda:{dev}")
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            el2 = float(t.item())
        split = {"precision": "fp32-split-bf16", "value": round(utts / el2, 4),
                 "ms_per_step": round(1000 * el2 / args.steps, 3)}
        if not args.no_timing:
            eng.set_timing(True)
            for i in range(tsteps):
                eng.adapt(waves[args.warmup + i], S, hp, record=RECORD, want_logits=False)
            t2 = eng.get_timing()
            eng.set_timing(False)
            gms2 = t2["gemm"][0]
            ach2 = flops_utt * B * tsteps / (gms2 / 1000.0) / 1e12
            split["roofline"] = {"bound": "mfma", "achieved": round(ach2, 3), "peak": BF16_SPLIT_PEAK_TFLOPS,
                                 "unit": "TFLOP/s (fp32-equivalent)", "frac": round(ach2 / BF16_SPLIT_PEAK_TFLOPS, 4),
                                 "note": "6 bf16 MFMA products per fp32 MAC: peak = 2500 TF bf16 dense / 6"}
        out["fp32_split_bf16"] = split
        eng.set_precision("fp32")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, N, S)
    eng.close()
    if world == 1 and args.c4 and args.precision == "fp32":
        out["c4"] = bench_c4(args, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
