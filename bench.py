"""Bench: adapted utterances/sec, 10-step SUTA on wav2vec2-base shapes (BASELINE.json config 2).

One bench "step" = one libsuta `suta_adapt` call over a batch of `--batch` synthetic 8 s
utterances (N = 128000 samples, T = 399 frames), each adapted for 10 SUTA steps with the
scripts/LS.sh flags (episodic reset, vanilla forward, greedy ids recorded at steps 0/1/3/5/10).
Waveforms are resident in HBM before the timed region.  Seeded random weights of the
w2v2-base architecture (no checkpoints offline).

Multi-GPU: one process per GPU -- `python bench.py --gpus N` starts the N rank processes itself (torchrun env
contract, before this process touches the GPU; `self_launch`), and the torchrun form works unchanged; every
rank adapts its own utterances (no data-path
collective, weak scaling); a barrier + device sync brackets the timed region and the max
elapsed time over ranks is used.  value = utterances of all ranks / that time.  The collectives
(barrier, max, gather of per-rank facts) go through `Comm` on `--dist-backend` (nccl = RCCL over
xGMI, the default; gloo for plumbing runs of several ranks on one device).  The rank loop is
`run()`, which takes the engine factory and the device, so tests/test_bench_dist.py drives the same
code with a stand-in engine on CPU ranks.

Beside the headline (rank 0, N = 1 only): the same workload at 64 utterances per call (`batch64`),
the fp32-accurate split-bf16 GEMM mode, config C4 (wav2vec2-large, 20 steps, bf16) and config C5
(a seeded TED-like length mix through the driver's ragged grouping).
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
from suta_amd.flops import kernel_base, reference_schedule_flops, suta_flops  # noqa: E402
from suta_amd.weights import synth_weights  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_PEAK_TFLOPS = 2500.0      # MI355X_MICROARCH.md: bf16 dense MFMA peak
BF16_SPLIT_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 6
HBM_PEAK_TBS = 8.0             # MI355X_MICROARCH.md: HBM3E peak
RECORD = [0, 1, 3, 5, 10]
C4_RECORD = [0, 1, 5, 10, 20]   # config C4 (20 steps): greedy ids recorded at these steps
# newest committed rocprofv3 PMC reduction of each workload (tools/pmc_traffic.py; profiles/<round>/README.md)
ROUNDS = ("r6", "r5", "r4", "r3", "r2", "r1")
PMC_TRAFFIC = next((p for p in (os.path.join(ROOT, "profiles", r, "pmc_traffic.json") for r in ROUNDS)
                    if os.path.exists(p)), None)
PMC_TRAFFIC_C4 = next((p for p in (os.path.join(ROOT, "profiles", r, "pmc_traffic_c4.json") for r in ROUNDS)
                       if os.path.exists(p)), None)
# 164 utterances x 399 frames = 65 436 rows = 512 row tiles of 128: every linear's grid (6 / 18 / 24 column tiles on
# base, 8 / 24 / 32 on large) fills whole rounds of the 512 resident 128 x 128 blocks.  The batch is tuned to the
# bench's fixed 8 s length (tile quantisation); the `batch64` object keeps the round-over-round comparison at 64.
BATCH = 164        # utterances per engine call (see --batch); tests/test_gpu_bench_scale.py pins this layout
C4_BATCH = BATCH   # config C4's utterances per call (see --c4-batch)
PMC_BATCH = 164    # the batch the committed headline PMC passes were taken at
PMC_BATCH_C4 = 164  # the batch of the committed C4 passes
C5_UTTERANCES = 512  # config C5: a TED-LIUM-3-test-sized seeded length mix (see --c5-n; ~30 s per pass)
GEMM_KERNELS = ("gemm_glds_kernel", "gemm_f32_kernel", "gemm_splitk_reduce", "attn_fwd_kernel", "attn_bwd_kernel",
                "posconv_kernel", "flash_fwd_kernel", "flash_bwd_kernel", "flash_dq_reduce", "flash_dq_reduce_frag")
# config C4's GEMM family (bf16 mode): every kernel its "gemm" + "attention" timing families launch.  Matched to the
# PMC table by base name (pmc_kernel_bytes: the trace may hold mangled names).
GEMM_KERNELS_C4 = ("gemm_hb_kernel", "gemm_hbx_kernel", "gemm_hbp_kernel", "gemm_hbt_kernel",
                   "gemm_x6_kernel", "gemm_gbf_kernel",
                   "gemm_splitk_reduce", "to_bf16_kernel", "posconv_bf16_kernel", "flash_fwd_bf16p_kernel",
                   "flash_bwd_bf16p_kernel", "flash_fwd_bf16_kernel", "flash_bwd_bf16_kernel", "flash_dq_reduce",
                   "flash_dq_reduce_frag")
# kernels of each family the C4 bench layout must have launched (a missing entry means a stale PMC table)
C4_REQUIRED = ("gemm_hb_kernel", "gemm_hbp_kernel", "flash_fwd_bf16p_kernel", "flash_bwd_bf16p_kernel",
               "flash_dq_reduce_frag")
FRONT_KERNELS = ("conv0_gn_kernel", "col_stats_final", "gn_bwd_final", "conv0_dw_reduce")


def pmc_kernel_bytes(d, kernels):
    """{base name: (launches, bytes per launch)} of `kernels` in the PMC table d (entries merged by base name)."""
    out = {}
    for k, v in d.items():
        b = kernel_base(k)
        if b in kernels:
            n0, by0 = out.get(b, (0, 0.0))
            n = n0 + v["launches"]
            out[b] = (n, (n0 * by0 + v["launches"] * v["hbm_bytes_per_launch"]) / n)
    return out


def pmc(args):
    """The committed PMC reduction when this run is its workload (w2v2-base, PMC_BATCH x 8 s, 10 steps)."""
    if not (args.model == "wav2vec2-base" and args.batch == PMC_BATCH and args.n_samples == 128000 and args.suta_steps == 10
            and PMC_TRAFFIC):
        return None
    return json.load(open(PMC_TRAFFIC))


def gemm_traffic(d, kernels=GEMM_KERNELS, required=()):
    """HBM bytes per GEMM-family launch from the PMC passes (None when a required kernel has no entry)."""
    kb = pmc_kernel_bytes(d, kernels)
    if any(r not in kb for r in required):
        return None
    n = sum(v[0] for v in kb.values())
    b = sum(v[0] * v[1] for v in kb.values())
    return round(b / n) if n else None


def frontend_traffic(d):
    """HBM bytes per conv front-end call (a forward call = 2 conv0_gn passes + the statistics finaliser; a
    backward call = 2 passes + the GroupNorm-backward finaliser + the conv0 dW reduction)."""
    kb = pmc_kernel_bytes(d, FRONT_KERNELS)
    if "conv0_gn_kernel" not in kb:
        return None
    b = sum(v[0] * v[1] for v in kb.values())
    return b / (kb["conv0_gn_kernel"][0] / 2)


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


# ------------------------------------------------------------------------------------------------
# the rank loop: collectives, device, timed region
# ------------------------------------------------------------------------------------------------
class Comm:
    """The bench's collectives: a barrier around the timed region, the max of the elapsed times over ranks and a
    gather of small per-rank facts.  world 1: no process group.  nccl (RCCL over xGMI) reduces device tensors,
    gloo host tensors."""

    def __init__(self, rank=0, world=1, backend="nccl", device=None):
        self.rank, self.world, self.backend, self.device = rank, world, backend, device
        if world > 1:
            import torch.distributed as tdist
            self.tdist = tdist

    def barrier(self):
        if self.world > 1:
            self.tdist.barrier()

    def world_seen(self):
        """get_world_size() of the live process group (1 without one): the ranks that actually joined."""
        import torch.distributed as tdist
        return tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1

    def max(self, x):
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        self.tdist.all_reduce(t, op=self.tdist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.tdist.all_gather_object(out, obj)
        return out


class Device:
    """Where the waveforms live and what the bench waits for: GPU `index` (torch.cuda) or, index None, the
    host (the CPU plumbing test with a stand-in engine)."""

    def __init__(self, index=None):
        self.index = index

    def put(self, a):
        t = torch.from_numpy(a)
        return t.to(f"cuda:{self.index}") if self.index is not None else t

    def sync(self):
        if self.index is not None:
            torch.cuda.synchronize(self.index)


def shard_start(rank, nbatches, batch, i):
    """First utterance index of rank `rank`'s batch i: ranks adapt disjoint utterance ranges."""
    return (rank * nbatches + i) * batch


def timed_batches(eng, waves, first, count, S, hp, record, comm, dev):
    """`count` adapt calls on waves[first:first+count], bracketed by barrier + device sync on both sides;
    returns (this rank's elapsed s, max over ranks)."""
    def fence():
        comm.barrier()
        dev.sync()
        eng.sync()
    fence()
    t0 = time.perf_counter()
    for i in range(count):
        eng.adapt(waves[first + i], S, hp, record=record, want_logits=False)
    eng.sync()
    fence()
    el = time.perf_counter() - t0
    return el, comm.max(el)


def run(args, rank, world, comm, dev, make_engine):
    """One rank of the bench; rank 0 prints the JSON line and returns it (other ranks return None)."""
    from suta_amd.engine import SutaHParams
    cfg = get_config(args.model)
    B, N, S = args.batch, args.n_samples, args.suta_steps
    eng = make_engine(cfg, B, N)
    eng.set_precision(args.precision)
    hp = SutaHParams()  # scripts/LS.sh flags
    nbatches = args.warmup + args.steps
    # inputs resident in device memory before timing: distinct utterances per rank and batch
    starts = [shard_start(rank, nbatches, B, i) for i in range(nbatches)]
    waves = [dev.put(synth.batch(N, B, start=s)) for s in starts]
    dev.sync()
    for i in range(args.warmup):
        eng.adapt(waves[i], S, hp, record=RECORD, want_logits=False)
    el_rank, el = timed_batches(eng, waves, args.warmup, args.steps, S, hp, RECORD, comm, dev)
    rank_el = comm.gather(round(el_rank, 6))
    shards = comm.gather([starts[args.warmup], starts[-1] + B])   # timed utterances [first, end) per rank
    # roofline pass (outside the timed region): per-launch HIP events on the engine stream; this runs
    # the eager path (timing disables graph replay), so its batch time is reported separately
    timing, timing_el, tsteps = None, None, max(1, min(args.timing_steps, args.steps))
    if not args.no_timing:
        eng.set_timing(True)
        comm.barrier()
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
                   "n_samples": N, "suta_steps": S, "parallelism": f"utterance-sharded x{world}",
                   "batch_note": "164 utterances x 399 frames = 512 row tiles of 128 (tuned to the bench's fixed "
                                 "length); see batch64 for the 64-per-call line"},
        "algorithmic_tflops": round(flops_utt * utts / el / 1e12, 3),
        "dist": {"backend": comm.backend if world > 1 else None, "world_seen": comm.world_seen(),
                 "rank_elapsed_s": rank_el, "utterance_shards": shards,
                 "rccl_measured": bool(world > 1 and comm.backend == "nccl")},
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
                                              "operand touched once at its stored element size (A unique rows, B per "
                                              "distinct slice, C written, epilogue operands), no tile re-reads or "
                                              "split-K partials",
                           "traffic_ratio": round(traffic / traffic_alg, 3) if traffic and traffic_alg else None,
                           "kernel": "fp32 MFMA GEMM family: gemm_glds_kernel + gemm_f32_kernel + posconv_kernel + flash attention (flash_fwd_kernel, flash_bwd_kernel + flash_dq_reduce_frag) (all launches)",
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
    if args.batch64 and B > 64 and args.steps >= 2:
        # the same workload at 64 utterances per call (the batch of rounds 1-2): round-over-round comparison
        w64 = [w[:64] for w in waves]
        eng.adapt(w64[0], S, hp, record=RECORD, want_logits=False)     # new layout: capture on the next call
        eng.adapt(w64[1], S, hp, record=RECORD, want_logits=False)
        el64_rank, el64 = timed_batches(eng, w64, args.warmup, args.steps, S, hp, RECORD, comm, dev)
        out["batch64"] = {"value": round(64 * args.steps * world / el64, 4),
                          "ms_per_step": round(1000 * el64 / args.steps, 3), "batch": 64}
    if args.also_split and args.precision == "fp32":
        # same workload with the fp32-accurate split-bf16 GEMMs (reported beside the headline)
        eng.set_precision("fp32-split-bf16")
        eng.adapt(waves[0], S, hp, record=RECORD, want_logits=False)
        el2_rank, el2 = timed_batches(eng, waves, args.warmup, args.steps, S, hp, RECORD, comm, dev)
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
    if world == 1 and args.precision == "fp32" and dev.index is not None:
        if args.c4:
            out["c4"] = bench_c4(args, dev.index)
        if args.c5:
            out["c5"] = bench_c5(args, dev.index)
    if rank == 0:
        print(json.dumps(out), flush=True)
        return out
    return None


def bench_c4(args, dev):
    """BASELINE.json config C4: wav2vec2-large-960h-lv60 shapes, 20-step SUTA, bf16 GEMMs (operands
    rounded to bf16, fp32 accumulation; norms, softmax, loss, AdamW and master tensors fp32), 1 GPU,
    8 s utterances.  A secondary line beside the C2 headline."""
    from suta_amd.engine import SutaEngine, SutaHParams
    cfg = get_config("wav2vec2-large")
    B, N, S = args.c4_batch, args.n_samples, 20
    eng = SutaEngine(cfg, synth_weights(cfg), device=dev, max_batch=B, max_samples=N)
    eng.set_precision("bf16")
    hp = SutaHParams()
    rec = C4_RECORD
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
                           "frac": round(ach / BF16_PEAK_TFLOPS, 4), "kernel": "bf16 GEMM family (bf16-plane linears: gemm_hbp_kernel (256 x 256, 16x16x32 MFMA since round 6) / gemm_hbx_kernel, gemm_hb_kernel (the K = 32 lm_head input gradient); the layer-norm conv stack's forward / input gradients: gemm_hbp_kernel (Z-batched / CONV forms); conv weight gradients: gemm_hbp_kernel TN form (round 6; gemm_hbt_kernel before); per-utterance projection GEMMs: gemm_x6_kernel one-plane form / gemm_gbf_kernel; posconv_bf16_kernel; flash attention on bf16 MFMA)",
                           "launches": int(gn), "avg_launch_ms": round(gms / max(1, gn), 5)}
        gx, ax = tex["gemm"], tex["attention"]
        talg = round((gx[2] + ax[2]) / max(1, gx[1] + ax[1]))
        d4 = json.load(open(PMC_TRAFFIC_C4)) if (PMC_TRAFFIC_C4 and B == PMC_BATCH_C4 and N == 128000) else None
        traffic = gemm_traffic(d4, GEMM_KERNELS_C4, C4_REQUIRED) if d4 else None
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


def c5_lengths(n, seed=20260416):
    """Config C5's seeded TED-like length mix: log-normal around 10 s (sigma 0.6), clipped to [2 s, 37.5 s] (the
    reference's 600 000-sample cap, data.py:19-22), in samples."""
    rng = np.random.default_rng(seed)
    sec = np.clip(rng.lognormal(np.log(10.0), 0.6, n), 2.0, 37.5)
    return np.minimum((sec * 16000).astype(np.int64), 600000)


def bench_c5(args, dev):
    """BASELINE.json config C5 on one GPU: TED-like variable-length utterances (reference corpus/ted.py sorts by
    transcript length, ascending; data.py truncates at 600 000 samples) adapted as the driver adapts them: length
    sorted, grouped by suta_amd/main.py ragged_groups with the driver's default --gpu_batch / --gpu_budget_s /
    --gpu_min_fill, each group one suta_adapt_varlen call (every utterance at its own length).  w2v2-base, 10 steps,
    LS.sh flags, fp32.  FLOPs on the true lengths; padding is reported, not credited."""
    from suta_amd.engine import SutaEngine, SutaHParams
    from suta_amd.main import LAYOUT_QUANTUM, build_parser, ragged_groups
    drv = build_parser().parse_args([])
    for k in ("gpu_batch", "gpu_budget_s", "gpu_min_fill"):   # bench overrides (A/B of the driver's defaults)
        if getattr(args, "c5_" + k, None) is not None:
            setattr(drv, k, getattr(args, "c5_" + k))
    cfg = get_config("wav2vec2-base")
    S = 10
    ns = c5_lengths(args.c5_n)
    order = np.argsort(ns, kind="stable")
    groups = [order[g] for g in ragged_groups([int(ns[i]) for i in order], drv.gpu_batch, drv.gpu_budget_s * 16000,
                                                  drv.gpu_min_fill)]
    q = LAYOUT_QUANTUM
    widths = [-(-int(ns[g].max()) // q) * q for g in groups]
    sd = synth_weights(cfg)
    E = max(1, getattr(args, "c5_engines", None) or drv.gpu_engines)   # the driver's --gpu_engines unless overridden
    engs = [SutaEngine(cfg, sd, device=dev, max_batch=max(len(g) for g in groups), max_samples=max(widths))
            for _ in range(E)]
    eng = engs[0]
    hp = SutaHParams()
    pads = []
    for g, w in zip(groups, widths):
        p = np.zeros((len(g), w), np.float32)
        for j, i in enumerate(g):
            p[j, :ns[i]] = synth.wave(int(ns[i]), 70000 + int(i))
        pads.append(torch.from_numpy(p).to(f"cuda:{dev}"))
    lens = [[int(ns[i]) for i in g] for g in groups]
    big = int(np.argmax([len(g) * w for g, w in zip(groups, widths)]))
    for e in engs:
        e.adapt_varlen(pads[big], 1, hp, record=[1], lengths=lens[big], want_logits=False)   # workspace at its max
        e.sync()
    torch.cuda.synchronize()
    # E engines (own streams, workspaces) in E host threads, the groups dealt longest-processing-time first by padded
    # samples -- as suta_amd/main.py adapt_window deals them (--gpu_engines, default 2)
    shares = [[] for _ in range(E)]
    load = [0] * E
    for j in sorted(range(len(groups)), key=lambda j: -len(groups[j]) * widths[j]):
        e = int(np.argmin(load))
        shares[e].append(j)
        load[e] += len(groups[j]) * widths[j]

    def run_share(e, js):
        for j in js:
            engs[e].adapt_varlen(pads[j], S, hp, record=RECORD, lengths=lens[j], want_logits=False)
        engs[e].sync()

    def one_pass():
        if E == 1:
            run_share(0, range(len(groups)))
            return
        import threading
        th = [threading.Thread(target=run_share, args=(e, shares[e])) for e in range(E)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    t0 = time.perf_counter()
    one_pass()
    el = time.perf_counter() - t0
    T_true = sum(num_frames(cfg, int(n)) for n in ns)
    T_pad = sum(len(g) * num_frames(cfg, w) for g, w in zip(groups, widths))
    flops = sum(suta_flops(cfg, int(n), S) for n in ns)
    res = {"workload": f"wav2vec2-base SUTA {S} steps, {len(ns)} TED-like utterances (log-normal around 10 s, "
                       "2-37.5 s, seeded), length-sorted ragged batches grouped by the driver's ragged_groups "
                       f"(--gpu_batch {drv.gpu_batch}, --gpu_budget_s {drv.gpu_budget_s:g}, --gpu_min_fill "
                       f"{drv.gpu_min_fill:g}, {E} engine(s)), scripts/LS.sh flags, fp32",
           "config": "C5", "precision": "fp32", "value": round(len(ns) / el, 4), "unit": "utt/s",
           "audio_s_per_s": round(float(ns.sum()) / 16000 / el, 2), "seconds": round(el, 3),
           "n_utterances": len(ns), "mean_seconds": round(float(ns.mean()) / 16000, 2),
           "max_seconds": round(float(ns.max()) / 16000, 2), "n_batches": len(groups),
           "batch_sizes": [len(g) for g in groups], "padded_frame_fraction": round(1.0 - T_true / T_pad, 4),
           "algorithmic_tflops": round(flops / el / 1e12, 3)}
    res["engines"] = E
    if not args.no_timing:
        eng.set_timing(True)
        run_share(0, range(len(groups)))   # (one engine: per-launch events on its stream)
        t = eng.get_timing()
        eng.set_timing(False)
        gms, gn = t["gemm"]
        ach = flops / (gms / 1000.0) / 1e12
        res["roofline"] = {"bound": "mfma", "achieved": round(ach, 3), "peak": FP32_MFMA_PEAK_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                           "kernel": "fp32 MFMA GEMM family (as the headline), FLOPs on true lengths",
                           "launches": int(gn), "avg_launch_ms": round(gms / max(1, gn), 5)}
    for e in engs:
        e.close()
    return res


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=BATCH, help="utterances in flight per GPU (engine slots)")
    ap.add_argument("--n-samples", type=int, default=128000)
    ap.add_argument("--suta-steps", type=int, default=10)
    ap.add_argument("--model", default="wav2vec2-base")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collectives under torchrun: nccl = RCCL over xGMI (one GPU per rank); gloo = host "
                         "collectives, ranks may share a device (rank r uses GPU LOCAL_RANK mod device count)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-kernel HIP-event timing pass")
    ap.add_argument("--timing-steps", type=int, default=1,
                    help="batches of the separate, untimed roofline pass (per-launch HIP events, eager)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32-split-bf16", "bf16"],
                    help="GEMM arithmetic: exact fp32 MFMA, fp32-accurate 3-way bf16 split, or bf16 (config C4)")
    ap.add_argument("--no-c4", dest="c4", action="store_false",
                    help="skip the config-C4 line (wav2vec2-large, 20 SUTA steps, bf16 GEMMs; 1 GPU only)")
    ap.add_argument("--c4-batch", type=int, default=C4_BATCH)
    ap.add_argument("--only-c4", action="store_true", help="print only the config-C4 line (profiling)")
    ap.add_argument("--no-c5", dest="c5", action="store_false",
                    help="skip the config-C5 line (TED-like length mix, driver grouping; 1 GPU only)")
    ap.add_argument("--c5-n", type=int, default=C5_UTTERANCES)
    ap.add_argument("--only-c5", action="store_true", help="print only the config-C5 line")
    ap.add_argument("--c5-gpu-batch", type=int, default=None, help="C5 grouping override (default: the driver's)")
    ap.add_argument("--c5-gpu-budget-s", type=float, default=None, help="C5 grouping override (default: the driver's)")
    ap.add_argument("--c5-gpu-min-fill", type=float, default=None, help="C5 grouping override (default: the driver's)")
    ap.add_argument("--c5-engines", type=int, default=None,
                    help="C5: engines (streams, host threads) sharing the groups (default: the driver's --gpu_engines)")
    ap.add_argument("--no-batch64", dest="batch64", action="store_false",
                    help="skip the 64-utterances-per-call line")
    ap.add_argument("--no-split", dest="also_split", action="store_false",
                    help="do not also time the fp32-accurate split-bf16 GEMM mode")
    return ap


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(n: int, argv, script: str = None, timeout_s: float = None) -> int:
    """`--gpus N` (N > 1) without a torchrun environment: start N rank processes of `script` (this file) with the
    torchrun contract -- RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1, MASTER_PORT -- and
    return the worst exit status.  This process never touches the GPU (no HIP call before or after the children
    start); rank 0's JSON line reaches stdout through the inherited descriptor.  When one rank fails, the others
    (which would wait in a barrier forever) are terminated."""
    import subprocess
    port = free_port()
    script = script or os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    t0, worst = time.time(), 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        late = timeout_s is not None and time.time() - t0 > timeout_s
        if bad or late:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(15)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            worst = bad[0] if bad else 124
            print(f"bench.py: self-launched rank failed (exit {worst}); stopped the other ranks", file=sys.stderr)
            return worst
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.2)


def main(argv=None, engine_factory=None, script=None):
    """argv: bench flags (default sys.argv[1:]).  engine_factory / script: the CPU plumbing test's stand-in engine
    (called as engine_factory(rank) -> make_engine) and the script its self-launched ranks run; None = the real
    engine on the GPU and this file."""
    argv = sys.argv[1:] if argv is None else list(argv)
    args = build_parser().parse_args(argv)
    if args.only_c4 or args.only_c5:
        torch.cuda.set_device(0)
        print(json.dumps(bench_c4(args, 0) if args.only_c4 else bench_c5(args, 0)), flush=True)
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the plain `python bench.py --gpus N` form: one rank process per GPU, launched here
        return self_launch(args.gpus, argv, script=script)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 as `python bench.py --gpus N` or "
              f"`python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}`",
              file=sys.stderr)
        return 2
    if engine_factory is not None:   # CPU plumbing test: stand-in engine, host "device", gloo only
        if world > 1:
            import torch.distributed as tdist
            tdist.init_process_group("gloo")
        comm = Comm(rank, world, "gloo", None)
        run(args, rank, world, comm, Device(None), engine_factory(rank))
        if world > 1:
            tdist.destroy_process_group()
        return 0
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a GPU (the engine has no CPU path)")
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"--dist-backend nccl: {world} ranks but {ndev} visible GPU(s); use one rank per GPU, or "
                         "--dist-backend gloo to share a device")
    gpu = local % ndev
    torch.cuda.set_device(gpu)
    if world > 1:
        import torch.distributed as tdist
        if args.dist_backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            tdist.init_process_group("gloo")
    comm = Comm(rank, world, args.dist_backend, torch.device("cuda", gpu))
    from suta_amd.engine import SutaEngine

    def make_engine(cfg, B, N):
        return SutaEngine(cfg, synth_weights(cfg), device=gpu, max_batch=B, max_samples=N)
    run(args, rank, world, comm, Device(gpu), make_engine)
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
