"""GPU tier: `bench.py --gpus 2 --dist-backend gloo` as two rank processes sharing device 0, the real engine.

The same code path the driver's N-GPU scaling run takes (torchrun env contract, one engine per rank, per-rank
utterance shards, barrier-bracketed timed region, max over ranks, rank-0-only JSON), with gloo collectives so two
ranks fit one GPU; the RCCL (nccl) backend itself is exercised only by the driver's 8-GPU run.  CPU form with a
stand-in engine: tests/test_bench_dist.py."""
import json
import os
import subprocess
import sys

import pytest

from tests.multirank import REPO, free_port

pytestmark = pytest.mark.gpu


def test_bench_two_gloo_ranks_on_one_gpu():
    world, port = 2, free_port()
    B, steps, warmup = 4, 2, 1
    argv = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
            "--batch", str(B), "--n-samples", "32000", "--steps", str(steps), "--warmup", str(warmup),
            "--no-cpu-baseline", "--no-c4", "--no-c5", "--no-split", "--no-batch64"]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
        procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=300))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, f"rank failed ({p.returncode}):\n{o[-2000:]}\n{e[-3000:]}"
    json_lines = [[ln for ln in o.splitlines() if ln.startswith("{")] for o, _ in outs]
    assert len(json_lines[0]) == 1 and json_lines[1] == [], json_lines
    out = json.loads(json_lines[0][0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 * B and out["dist"]["backend"] == "gloo"
    el = out["dist"]["rank_elapsed_s"]
    assert out["value"] == pytest.approx(B * steps * world / max(el), rel=1e-3)
    nb = steps + warmup
    assert out["dist"]["utterance_shards"] == [[(r * nb + warmup) * B, (r * nb + nb) * B] for r in range(world)]
    assert out["roofline"]["frac"] > 0 and out["attention"]["tflops"] > 0


def test_bench_self_launch_two_gloo_ranks_on_one_gpu():
    """The plain `python bench.py --gpus 2` form with no torchrun environment: bench.py starts the two rank
    processes itself (bench.self_launch) before touching the GPU; rank 0 prints the one JSON line with the live
    process group's size."""
    B, steps, warmup = 4, 2, 1
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    argv = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
            "--batch", str(B), "--n-samples", "32000", "--steps", str(steps), "--warmup", str(warmup),
            "--no-cpu-baseline", "--no-c4", "--no-c5", "--no-split", "--no-batch64", "--no-timing"]
    p = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, f"{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dist"]["world_seen"] == 2 and out["dist"]["backend"] == "gloo"
    el = out["dist"]["rank_elapsed_s"]
    assert out["value"] == pytest.approx(B * steps * 2 / max(el), rel=1e-3)
