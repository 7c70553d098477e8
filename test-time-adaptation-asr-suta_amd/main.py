"""main.py-compatible driver (reference main.py:217-454) on the libsuta engine.

Same flags, same stdout lines ("original WER:", "adapt-k WER:", "TTA-k WER:"), same log
file `log_dir/exp_name` and CSV.  Differences, all deliberate:
  * the adapt loop runs in libsuta (HIP) with the minimal schedule: the logits recorded after
    step k equal the reference's re-inference output of step k;
  * episodic runs adapt up to --gpu_batch utterances per engine call as a ragged batch
    (suta_adapt_varlen: every utterance at its own length, results equal to running it alone;
    utterances are length-sorted inside windows of 8 batches to keep padding low, and the
    per-utterance lines are printed in dataset order).  The reference's own --batch_size > 1
    pads without a mask and breaks mcc_loss (main.py:32); it is only used for loading here;
  * under torchrun (episodic runs only), utterances are LPT-sharded over ranks by their decoded
    length (file headers), WER counts are all_reduce'd, and rank 0 prints every per-utterance line
    after the gather, in dataset order (one ordered stream, as the reference's single process);
    non-episodic adaptation carries state from one utterance to the next in dataset order
    (reference main.py:323-348), so it refuses to shard;
  * pretrained weights load from a local checkpoint directory or the local HF cache (no
    network); `--synthetic_weights` uses the seeded generator instead;
  * when --steps < 10 the CSV is written with empty WERR (the reference raises there).
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import Dict, List

import numpy as np

SAMPLE_RATE = 16000
CHECKPOINTS = (1, 3, 5, 10, 20, 40)
LAYOUT_QUANTUM = 1600  # samples: ragged-batch layout lengths are multiples of 0.1 s (5 frames)


def build_parser(sdpl: bool = False):
    """main.py:221-241 flags; sdpl: main_SDPL.py's (steps 10, opt Adam, em_coef 1, --pl_coef)."""
    p = argparse.ArgumentParser(description="TTA ASR")
    p.add_argument("--asr", type=str, default="facebook/wav2vec2-base-960h")
    p.add_argument("--steps", type=int, default=10 if sdpl else 40)
    p.add_argument("--episodic", action="store_true")
    p.add_argument("--div_coef", type=float, default=0.0)
    p.add_argument("--opt", type=str, default="Adam" if sdpl else "AdamW")
    p.add_argument("--dataset_name", type=str, default="librispeech")
    p.add_argument("--dataset_dir", type=str, default="/home/daniel094144/data/LibriSpeech")
    p.add_argument("--split", default=["test-other"])
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--em_coef", type=float, default=1.0)  # (both scripts)
    p.add_argument("--reweight", action="store_true")
    p.add_argument("--bias_only", action="store_true")
    p.add_argument("--train_feature", action="store_true")
    p.add_argument("--train_all", action="store_true")
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--temp", type=float, default=2.5)
    p.add_argument("--non_blank", action="store_true")
    p.add_argument("--log_dir", type=str, default="./exps")
    p.add_argument("--extra_noise", type=float, default=0.0)
    p.add_argument("--scheduler", default=None)
    if sdpl:
        p.add_argument("--pl_coef", type=float, default=1)
    # engine-only options
    p.add_argument("--synthetic_weights", action="store_true", help="seeded random weights (no checkpoint)")
    p.add_argument("--device", type=int, default=None)
    # defaults = the layout the headline bench measures (bench.py BATCH: 164 x 8 s = 1312 s of audio per call, about
    # 59 GB of workspace at 0.36 GB per 8 s utterance, of the 288 GB of HBM)
    p.add_argument("--gpu_batch", type=int, default=164,
                   help="max utterances adapted together as one ragged batch (episodic runs; 1 = one per call)")
    p.add_argument("--gpu_budget_s", type=float, default=1312.0,
                   help="max padded audio seconds per ragged batch (utterances x longest)")
    p.add_argument("--gpu_min_fill", type=float, default=0.3,
                   help="ragged grouping: 0 = greedy; > 0 = padding-minimising partition charging a batch at least "
                        "this fraction of --gpu_budget_s (bench.py c5, TED-like mix of 512 utterances at --gpu_batch 164 "
                        "/ --gpu_budget_s 1312: 0.2 / 0.3 / 0.4 / 0.5 / 0.7 -> 20.8 / 21.6 / 21.5-21.6 / 20.9 / 20.8 "
                        "utt/s, profiles/r5/c5_mf*.json; on round 4's 96-utterance mix 0.15-0.25 was the optimum)")
    p.add_argument("--gpu_engines", type=int, default=2,
                   help="episodic runs: engines per GPU (own HIP stream, workspace and host thread) adapting ragged "
                        "groups concurrently; the padded-audio budget is per engine (bench.py c5, 512 TED-like "
                        "utterances: 1 / 2 engines 21.60 / 22.93 utt/s, profiles/r5/c5_e*.json)")
    p.add_argument("--dist_backend", default="auto", choices=["auto", "nccl", "gloo"],
                   help="torch.distributed backend under torchrun (auto: nccl = RCCL when a GPU is visible)")
    p.add_argument("--num_workers", type=int, default=4,
                   help="audio decode threads (FLAC/WAV decode + resample ahead of the engine)")
    p.add_argument("--chime_subsets", default=None,
                   help="--dataset_name chime: comma-separated et05 subsets (default: the reference's 7 of "
                        "corpus/CHiME.py:27, real and simu); config C3 'eval-real' = "
                        "et05_bus_real,et05_caf_real,et05_str_real")
    p.add_argument("--precision", default="fp32", choices=["fp32", "fp32-split-bf16", "bf16"],
                   help="GEMM arithmetic (fp32 = the reference's; bf16 = BASELINE config C4)")
    return p


def ragged_groups(sorted_lengths, max_batch: int, budget_samples: float, min_fill: float = 0.0):
    """Consecutive groups of length-sorted utterances: at most max_batch utterances and at most
    budget_samples of padded audio (count x longest, layout rounded up to LAYOUT_QUANTUM).

    min_fill = 0: greedy (fill each group up to a limit).  min_fill > 0: the partition minimising the
    total padded audio, a group being charged at least min_fill * budget_samples (a group with less
    audio under-fills the GPU) -- dynamic programming over the sorted order."""
    w = [-(-int(n) // LAYOUT_QUANTUM) * LAYOUT_QUANTUM for n in sorted_lengths]
    if min_fill <= 0:
        groups, cur = [], []
        for j, width in enumerate(w):
            if cur and (len(cur) >= max_batch or (len(cur) + 1) * width > budget_samples):
                groups.append(cur)
                cur = []
            cur.append(j)
        if cur:
            groups.append(cur)
        return groups
    n, floor = len(w), min_fill * budget_samples
    best, arg = [0.0] + [float("inf")] * n, [0] * (n + 1)
    for j in range(1, n + 1):
        for i in range(max(0, j - max_batch), j):
            area = (j - i) * w[j - 1]
            if area > budget_samples and j - i > 1:
                continue
            v = best[i] + max(area, floor)
            if v < best[j]:
                best[j], arg[j] = v, i
    groups, j = [], n
    while j > 0:
        groups.append(list(range(arg[j], j)))
        j = arg[j]
    return groups[::-1]


def resolve_scheduler(name):
    """--scheduler: the reference eval()s the string in main.py's namespace and calls the result with
    (optimizer, step_size=1, gamma=0.7) (main.py:20-21); of torch's schedulers only StepLR takes those keywords, so
    the engine implements StepLR (lr * 0.7^i on optimizer step i, restored per utterance when episodic).  The name
    is resolved as a dotted path from `torch` (no eval); None = no scheduler.  Returns (lr_step_size, gamma)."""
    if name is None:
        return 0, 0.7
    import torch
    obj = None
    parts = str(name).split(".")
    if parts[0] == "torch":
        obj = torch
        for q in parts[1:]:
            obj = getattr(obj, q, None)
    if obj is not torch.optim.lr_scheduler.StepLR:
        raise SystemExit(f"--scheduler {name}: the engine implements torch.optim.lr_scheduler.StepLR (the one torch "
                         "scheduler the reference's eval(scheduler)(optimizer, step_size=1, gamma=0.7) constructs)")
    return 1, 0.7


def workspace_bytes_per_audio_s(cfg) -> float:
    """Upper estimate of the engine's device workspace per second of padded audio in a batch (DESIGN.md section 2:
    measured 0.36 GB per 8 s base utterance = 45 MB/s): 50 frames/s x 4 B x layers x 14 H saved per frame in the
    encoder, plus ~3 fp32 buffers of the conv stack's 512 channels over its ~6350 frames per second."""
    return 50 * 4 * cfg["num_hidden_layers"] * 14 * cfg["hidden_size"] + 6350 * 512 * 4 * 3


def engine_fixed_bytes(cfg, weights, max_batch: int, precision: str = "fp32") -> float:
    """Device bytes an engine holds whatever its batch layout (advisor r5): its fp32 copy of the weights, the bf16
    planes of the frozen linear weights in bf16 mode (W and W^T: one fp32 copy's worth), and per utterance slot the
    trainable tensors, their gradients and both Adam moments (plus the pristine copy)."""
    from .config import param_shapes
    from .modules import collect_params
    wbytes = 4.0 * sum(int(np.asarray(v).size) for v in weights.values())
    shapes = dict(param_shapes(cfg))
    _, names = collect_params(cfg, bias_only=False, train_feature=True)
    pn = sum(int(np.prod(shapes[n])) for n in dict.fromkeys(names) if n in shapes)
    return wbytes * (2.0 if precision == "bf16" else 1.0) + 4.0 * pn * (4 * max_batch + 1)


def clamp_budget(budget_s: float, cfg, free_bytes, frac: float = 0.7) -> float:
    """The ragged-batch audio budget limited to `frac` of the device's free memory (the defaults are sized for the
    288 GB of an MI355X; a smaller GPU would otherwise fail its first allocation)."""
    if not free_bytes:
        return budget_s
    return max(1.0, min(budget_s, frac * free_bytes / workspace_bytes_per_audio_s(cfg)))


def exp_name_of(a, sdpl: bool = False) -> str:
    """main.py:267 (main_SDPL.py:266 when sdpl)."""
    base = (a.dataset_name + "_" + str(a.em_coef) + "_" + str(a.steps) + "_" + str(a.temp) + "_" +
            a.asr.split("/")[-1] + "_" + "non_blank" + str(a.non_blank) + "_noise_" + str(a.extra_noise) + "_rew_" +
            str(a.reweight) + "_div_" + str(a.div_coef) + "_bias_" + str(a.bias_only) + "_feat_" +
            str(a.train_feature))
    if sdpl:
        return base + "_se_" + "_pl_" + str(a.pl_coef)
    return base + "_all_" + str(a.train_all) + "_LN_" + str(True)


def load_model(asr: str, synthetic: bool):
    from .config import get_config
    from .weights import load_hf_checkpoint, synth_weights
    if os.path.isdir(asr):
        return get_config(asr), load_hf_checkpoint(asr)
    try:
        from huggingface_hub import snapshot_download
        d = snapshot_download(asr, local_files_only=True)
        return get_config(d), load_hf_checkpoint(d)
    except Exception:
        if not synthetic:
            raise RuntimeError(f"no local checkpoint for '{asr}' (offline); pass a checkpoint directory or "
                               "--synthetic_weights")
    cfg = get_config(asr)
    return cfg, synth_weights(cfg)


def main(argv=None, sdpl: bool = False):
    """sdpl: the main_SDPL.py driver (pseudo-label CTC objective, main_SDPL.py:143-209).  As there, the
    adaptation loss uses pl_coef = 1 whatever --pl_coef says (main_SDPL.py:345-346 passes `pl_coef=1.`);
    --pl_coef only enters the experiment name and log."""
    a = build_parser(sdpl).parse_args(argv)
    if sdpl:
        a.train_all = False
    if a.opt not in ("AdamW", "Adam", "SGD"):
        raise SystemExit(f"--opt {a.opt}: the engine implements AdamW, Adam (== AdamW at the reference's weight "
                         "decay 0) and SGD")
    lr_step_size, lr_gamma = resolve_scheduler(a.scheduler)
    if a.train_all:
        raise SystemExit("--train_all: full-model adaptation is outside the engine's scope")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not a.episodic:
        raise SystemExit("non-episodic SUTA adapts utterances sequentially (state carries over, reference "
                         "main.py:323-348): it cannot be sharded over ranks; run it with one process")
    import torch
    device = a.device if a.device is not None else local
    backend = a.dist_backend
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    count_device = None
    if world > 1:
        import torch.distributed as tdist
        if backend == "nccl":
            torch.cuda.set_device(device)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", device))
            count_device = torch.device("cuda", device)   # RCCL reduces device tensors only
        else:
            tdist.init_process_group("gloo")
    say = print if rank == 0 else (lambda *x, **k: None)

    from .data import load_dataset
    from .decode import batch_decode, wer, wer_counts
    from .dist import gather_objects, lpt_shard, reduce_counts, utterance_cost
    from .engine import SutaEngine, SutaHParams
    from .synth import normalize

    exp_name = exp_name_of(a, sdpl)
    if sdpl:
        from .decode import VOCAB
        say({t: i for i, t in enumerate(VOCAB)})  # main_SDPL.py:269-271 prints vocab.json
    subsets = [x for x in a.chime_subsets.split(",") if x] if a.chime_subsets else None
    dataset = load_dataset(a.split, a.dataset_name, a.dataset_dir, a.batch_size, a.extra_noise,
                           chime_subsets=subsets)
    say("------------------------------------")
    say(f"exp: {exp_name}")
    tail = ((f"pl_coef = {a.pl_coef}",) if sdpl else (f"train_all = {a.train_all}", f"train_LN = {True}"))
    for line in (f"eposidic? {a.episodic}", f"lr = {a.lr}", f"optim = {a.opt}", f"step = {a.steps}",
                 f"em_coef = {a.em_coef}", f"reweight = {a.reweight}", f"batch size = {a.batch_size}",
                 f"temperature = {a.temp}", f"non_blank = {str(a.non_blank)}", f"extra_noise = {a.extra_noise}",
                 f"scheduler = {str(a.scheduler)}", f"div_coef = {str(a.div_coef)}", f"bias_only = {a.bias_only}",
                 f"train_feature = {a.train_feature}") + tail:
        say(line)

    cfg, weights = load_model(a.asr, a.synthetic_weights)
    # collect_params (main.py:79-80 prints every module name; main_SDPL.py's copy does not), setup_optimizer
    # (main.py:19-20), then print(param_names) (main.py:314, main_SDPL.py:321)
    from .modules import collect_params
    printed, param_names = collect_params(cfg, a.bias_only, a.train_feature)
    if not sdpl:
        for nm in printed:
            say(nm)
    say(f"[INFO]    optimizer: {getattr(torch.optim, a.opt)}")
    say(f"[INFO]    scheduler: {a.scheduler}")
    say(param_names)
    gb = max(1, a.gpu_batch) if a.episodic else 1  # non-episodic adaptation is sequential
    # non-episodic adaptation carries state across utterances in one engine's slot: one engine
    n_eng = max(1, a.gpu_engines) if (a.episodic and gb > 1) else 1
    if torch.cuda.is_available():
        # the engines' fixed footprint (weights, bf16 weight planes, per-slot state) comes off the free memory first
        free = torch.cuda.mem_get_info(device)[0] - n_eng * engine_fixed_bytes(cfg, weights, gb, a.precision)
        budget = clamp_budget(a.gpu_budget_s, cfg, max(1.0, free), frac=0.7 / n_eng)
        if budget < a.gpu_budget_s:
            say(f"[suta_amd] --gpu_budget_s {a.gpu_budget_s} x {n_eng} engine(s) exceeds 70 % of the free device "
                f"memory; using {budget:.0f} s")
            a.gpu_budget_s = budget
    engines = [SutaEngine(cfg, weights, device=device, max_batch=gb) for _ in range(n_eng)]
    for e in engines:
        e.set_precision(a.precision)
    engine = engines[0]
    hp = SutaHParams(lr=a.lr, temp=a.temp, em_coef=a.em_coef, div_coef=0.0 if sdpl else a.div_coef,
                     reweight=a.reweight, non_blank=a.non_blank, train_feature=a.train_feature,
                     bias_only=a.bias_only, episodic=a.episodic, pl_coef=1.0 if sdpl else 0.0, optimizer=a.opt,
                     lr_step_size=lr_step_size, lr_gamma=lr_gamma)
    record = [0] + ([c for c in CHECKPOINTS if c <= a.steps] if a.episodic else [])
    if not a.episodic:
        record = sorted(set([0, a.steps]))

    # shard batches over ranks by estimated cost (decoded length from the file headers)
    batches = dataset.raw_batches()
    if world > 1:
        from .data import decoded_length
        costs = [sum(utterance_cost(max(1, decoded_length(str(f))), cfg, a.steps) for f, _ in b)
                 for b in batches]
        mine = lpt_shard(costs, world)[rank]
    else:
        mine = list(range(len(batches)))

    def adapt_window(items):
        """ids {record step: (T,)} per item, adapting length-sorted groups of gb as ragged batches.  With several
        engines the groups are dealt longest-first to the least-loaded engine (padded samples) and each engine's
        share runs in its own host thread on its own stream; every utterance's result is the same whichever engine
        adapts it (episodic: the slot starts from the pristine tensors)."""
        order = sorted(range(len(items)), key=lambda i: len(items[i][1])) if gb > 1 else list(range(len(items)))
        out = [None] * len(items)
        groups = [[order[j] for j in grp] for grp in ragged_groups([len(items[i][1]) for i in order], gb,
                                                                   a.gpu_budget_s * SAMPLE_RATE, a.gpu_min_fill)]

        def run(eng, grps):
            for grp in grps:
                if gb == 1:
                    _, ids, _ = eng.adapt(items[grp[0]][1], a.steps, hp, record=record, want_logits=False)
                    out[grp[0]] = {r: ids[r][0] for r in record}
                else:  # layout rounded up to LAYOUT_QUANTUM: equal layouts replay one captured step
                    _, ids, _ = eng.adapt_varlen([items[i][1] for i in grp], a.steps, hp, record=record,
                                                 want_logits=False, quantum=LAYOUT_QUANTUM)
                    for j, i in enumerate(grp):
                        out[i] = {r: ids[r][j] for r in record}
        if n_eng == 1 or len(groups) == 1:
            run(engine, groups)
            return out
        import threading
        shares, load = [[] for _ in range(n_eng)], [0] * n_eng
        for grp in sorted(groups, key=lambda g: -len(g) * max(len(items[i][1]) for i in g)):
            e = load.index(min(load))
            shares[e].append(grp)
            load[e] += len(grp) * max(len(items[i][1]) for i in grp)
        errs = []

        def guarded(eng, grps):
            try:
                run(eng, grps)
            except BaseException as exc:   # re-raised in the calling thread
                errs.append(exc)
        th = [threading.Thread(target=guarded, args=(engines[e], shares[e])) for e in range(n_eng) if shares[e]]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return out

    results = []
    start = time.time()
    window: List = []

    def emit(rec):
        for ln in rec["lines"]:
            print(*ln)

    def flush():
        for (bi, x, text, pre), ids in zip(window, adapt_window(window)):
            rec = {"idx": bi, "text": text, "duration": len(x) / SAMPLE_RATE, "hyp": {},
                   "lines": [(ln,) for ln in pre]}
            ori = batch_decode(ids[0][None])
            rec["hyp"][0] = ori[0]
            ori_wer = wer([text], ori)
            rec["lines"].append(("original WER: ", ori_wer))
            if a.episodic:
                for c in CHECKPOINTS:
                    if c <= a.steps:
                        h = batch_decode(ids[c][None])
                        rec["hyp"][c] = h[0]
                        ada = wer([text], h)
                        rec["lines"].append((f"adapt-{c} WER: " + (" " if c < 10 else ""), ada))
                        if c == 10:
                            rec["werr"] = ori_wer - ada
            if world == 1:
                emit(rec)   # one process: stream the lines as the reference does
            results.append(rec)
        window.clear()

    truncated = {}   # loader batch -> the reader's truncation lines (data.py:19-21), printed before its WER lines
    for bi, (lens, wavs, texts, files) in dataset.iter_collated(mine, a.num_workers,
                                                                log=lambda i, lines: truncated.__setitem__(i, lines)):
        for j, (wav, text) in enumerate(zip(wavs, texts)):
            window.append((bi, normalize(wav), text, truncated.pop(bi, []) if j == 0 else []))
        if len(window) >= 8 * gb:
            flush()
    flush()
    elapsed = time.time() - start

    allres = [r for part in gather_objects(results) for r in part]
    allres.sort(key=lambda r: r["idx"])   # stable: utterances of one loader batch keep their order
    if world > 1 and rank == 0:
        for rec in allres:   # one ordered stream of per-utterance lines, in dataset order
            emit(rec)
    # corpus WER counts, reduced over ranks (the one data collective)
    local_counts = {}
    for key in [0] + list(CHECKPOINTS):
        sel = [r for r in results if key in r["hyp"]]
        local_counts[str(key)] = wer_counts([r["text"] for r in sel], [r["hyp"][key] for r in sel]) if sel else (0, 0)
    counts = reduce_counts(local_counts, device=count_device)
    if rank == 0:
        def cw(k):
            e, w = counts[str(k)]
            return e / w if w else float("nan")
        lines = [f"original WER: {cw(0)}"]
        if a.steps >= 10:
            lines += [f"TTA-{k} WER: {cw(k)}" for k in (1, 3, 5, 10)]
        if a.steps >= 20:
            lines.append(f"TTA-20 WER: {cw(20)}")
        if a.steps >= 40:
            lines.append(f"TTA-40 WER: {cw(40)}")
        print("asr:", a.asr)
        if not sdpl:  # main_SDPL.py:395-407 prints neither line and writes no CSV
            print("non-adapted count = 0")
            print(f"dataset num = {len(batches)}")
        for ln in lines:
            print(ln)
        print("------------------------------------")
        print(f"[suta_amd] adapted {len(allres)} utterances in {elapsed:.1f} s on rank 0's shard, {world} rank(s)")
        os.makedirs(a.log_dir, exist_ok=True)
        # the log is written after setup_optimizer rebound `scheduler` to the scheduler object (main.py:308, 445)
        sched_obj = "None" if a.scheduler is None else "<torch.optim.lr_scheduler.StepLR object>"
        tail = ((f"pl_coef = {a.pl_coef}",) if sdpl else (f"train_all = {str(a.train_all)}", f"train_LN = {str(True)}"))
        with open(os.path.join(a.log_dir, exp_name), "w") as f:
            for ln in lines:
                f.write(ln + "\n")
            for ln in (f"eposidic? {a.episodic}", f"lr = {a.lr}", f"optim = {a.opt}", f"step = {a.steps}",
                       f"em_coef = {a.em_coef}", f"reweight = {a.reweight}", f"batch size = {a.batch_size}",
                       f"temperature = {a.temp}", f"non_blank = {str(a.non_blank)}", f"extra_noise = {a.extra_noise}",
                       f"scheduler = {sched_obj}", f"div_coef = {str(a.div_coef)}",
                       f"bias_only = {str(a.bias_only)}", f"train_feature = {str(a.train_feature)}") + tail:
                f.write(ln + "\n")
        if not sdpl:
            import pandas as pd
            durations = [r["duration"] for r in allres]
            werrs = [r.get("werr", np.nan) for r in allres]
            pd.DataFrame({"duration": durations, "WERR": werrs}).to_csv(os.path.join(a.log_dir, exp_name + ".csv"))
    for e in engines:
        e.close()
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()
    return counts


if __name__ == "__main__":
    main()
