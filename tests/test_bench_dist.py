"""CPU tier: bench.py's multi-rank path (bench.run under world size 2, gloo) with a stand-in engine.

What `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` relies on: each rank adapts its own
utterance range (no overlap), the timed region is bracketed by barriers, `value` = utterances of all ranks / the
max elapsed time over ranks, and only rank 0 prints the JSON line.  The GPU form of the same check (two gloo ranks
sharing device 0, the real engine) is tests/test_gpu_bench_dist.py.  Reference: main.py:303,323 runs one device;
the sharding is the build's own."""
import json
import multiprocessing as mp
import os

import numpy as np
import pytest

from tests.multirank import free_port

ARGV = ["--gpus", "2", "--dist-backend", "gloo", "--model", "tiny-group", "--batch", "3", "--n-samples", "4000",
        "--suta-steps", "2", "--steps", "3", "--warmup", "1", "--no-timing", "--no-cpu-baseline", "--no-c4",
        "--no-c5", "--no-batch64", "--no-split"]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_two_ranks_shard_time_and_print(tmp_path, world):
    """World sizes 2, 4 and 8 (the driver's SCALE run launches 1 / 2 / 4 / 8 ranks)."""
    from tests import _bench_dist_worker as W
    from suta_amd import synth
    port = free_port()
    argv = list(ARGV)
    argv[argv.index("--gpus") + 1] = str(world)
    ctx = mp.get_context("spawn")
    outs = [str(tmp_path / f"rank{r}.json") for r in range(world)]
    procs = [ctx.Process(target=W.bench_rank, args=(r, world, port, outs[r], argv)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0, p.exitcode
    res = [json.load(open(o)) for o in outs]
    # rank 0 alone prints, one JSON line
    for r in range(1, world):
        assert res[r]["stdout"] == "" and res[r]["ret"] is None
    lines = [ln for ln in res[0]["stdout"].splitlines() if ln.strip()]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out == res[0]["ret"]
    B, steps, warmup = 3, 3, 1
    nb = steps + warmup
    assert out["n_gpus"] == world and out["scaling"] == "weak" and out["dist"]["backend"] == "gloo"
    assert out["dist"]["world_seen"] == world and out["dist"]["rccl_measured"] is False
    # value = utterances of all ranks / max elapsed over ranks
    el = out["dist"]["rank_elapsed_s"]
    # the closing barrier holds every rank until the slowest has finished: rank 1's stand-in sleeps 0.1 s per call
    assert len(el) == world and min(el) >= steps * 0.1
    assert out["value"] == pytest.approx(B * steps * world / max(el), rel=1e-3)
    assert out["ms_per_step"] == pytest.approx(1000 * max(el) / steps, rel=1e-3)
    # disjoint utterance ranges, and each rank adapted exactly its own utterances
    shards = out["dist"]["utterance_shards"]
    assert shards == [[(r * nb + warmup) * B, (r * nb + nb) * B] for r in range(world)]
    for r in range(world):
        want = [float(synth.wave(4000, i)[0]) for i in range(r * nb * B, (r + 1) * nb * B)]
        np.testing.assert_array_equal(np.array(res[r]["seen"], np.float32), np.array(want, np.float32))
    for r in range(1, world):
        assert not set(res[0]["seen"]) & set(res[r]["seen"])


def _selflaunch(tmp_path, world, extra_env=None):
    import subprocess
    import sys
    from tests.multirank import REPO
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(BENCH_SEEN_DIR=str(tmp_path), **(extra_env or {}))
    argv = list(ARGV)
    argv[argv.index("--gpus") + 1] = str(world)
    return subprocess.run([sys.executable, os.path.join(REPO, "tests", "_bench_selflaunch_worker.py")] + argv,
                          env=env, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launches_ranks_without_torchrun_env(tmp_path, world):
    """`python bench.py --gpus N` with no torchrun environment (the plain form of the driver's BENCH command) starts
    the N ranks itself (bench.self_launch): one JSON line from rank 0 with n_gpus = world_seen = N, every rank
    adapting its own shard."""
    from suta_amd import synth
    p = _selflaunch(tmp_path, world)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["dist"]["world_seen"] == world and out["dist"]["backend"] == "gloo"
    B, nb = 3, 4
    for r in range(world):
        seen = json.load(open(tmp_path / f"seen{r}.json"))
        want = [float(synth.wave(4000, i)[0]) for i in range(r * nb * B, (r + 1) * nb * B)]
        np.testing.assert_array_equal(np.array(seen, np.float32), np.array(want, np.float32))


def test_bench_self_launch_stops_ranks_when_one_fails(tmp_path):
    """A rank that dies leaves the others waiting for it in the rendezvous / a barrier: the launcher terminates them
    and returns the failing rank's status."""
    p = _selflaunch(tmp_path, 2, {"BENCH_FAIL_RANK": "1"})
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_driver_defaults_run_the_bench_layout():
    """suta_amd/main.py's --gpu_batch / --gpu_budget_s defaults admit the headline's layout (bench.BATCH 8 s
    utterances in one call), so the drop-in driver runs what bench.py measures."""
    import bench
    from suta_amd.main import build_parser, ragged_groups
    a = build_parser().parse_args([])
    assert a.gpu_batch == bench.BATCH
    assert a.gpu_budget_s >= bench.BATCH * 128000 / 16000
    groups = ragged_groups([128000] * bench.BATCH, a.gpu_batch, a.gpu_budget_s * 16000, a.gpu_min_fill)
    assert [len(g) for g in groups] == [bench.BATCH]
