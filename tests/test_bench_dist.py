"""CPU tier: bench.py's multi-rank path (bench.run under world size 2, gloo) with a stand-in engine.

What `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` relies on: each rank adapts its own
utterance range (no overlap), the timed region is bracketed by barriers, `value` = utterances of all ranks / the
max elapsed time over ranks, and only rank 0 prints the JSON line.  The GPU form of the same check (two gloo ranks
sharing device 0, the real engine) is tests/test_gpu_bench_dist.py.  Reference: main.py:303,323 runs one device;
the sharding is the build's own."""
import json
import multiprocessing as mp

import numpy as np
import pytest

from tests.multirank import free_port

ARGV = ["--gpus", "2", "--dist-backend", "gloo", "--model", "tiny-group", "--batch", "3", "--n-samples", "4000",
        "--suta-steps", "2", "--steps", "3", "--warmup", "1", "--no-timing", "--no-cpu-baseline", "--no-c4",
        "--no-c5", "--no-batch64", "--no-split"]


@pytest.mark.parametrize("world", [2, 4])
def test_bench_two_ranks_shard_time_and_print(tmp_path, world):
    """World sizes 2 and 4 (the driver's SCALE run launches 1 / 2 / 4 / 8 ranks; 8 processes are not started here)."""
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
