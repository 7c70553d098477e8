"""Spawned CPU rank of bench.run() with a stand-in engine (tests/test_bench_dist.py): the bench's multi-rank
plumbing -- per-rank utterance shards, barrier + max-over-ranks timing, gather of per-rank facts, rank-0-only
output -- over gloo, without a GPU."""
import contextlib
import io
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


class StandInEngine:
    """Records the utterances it is given (first sample of each row: synth waves are seeded per utterance index)
    and sleeps a rank-dependent time per call, so the ranks' elapsed times differ."""

    def __init__(self, rank):
        self.rank = rank
        self.seen = []

    def set_precision(self, mode):
        pass

    def adapt(self, wav, steps, hp, record=(), want_logits=True):
        self.seen += [float(v) for v in wav[:, 0]]
        time.sleep(0.05 * (self.rank + 1))
        return None, {}, 0

    def sync(self):
        pass

    def close(self):
        pass


def bench_rank(rank, world, port, out_path, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import bench
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    args = bench.build_parser().parse_args(argv)
    eng = StandInEngine(rank)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        ret = bench.run(args, rank, world, bench.Comm(rank, world, "gloo"), bench.Device(None),
                        lambda cfg, B, N: eng)
    torch.distributed.destroy_process_group()
    json.dump({"stdout": buf.getvalue(), "ret": ret, "seen": eng.seen}, open(out_path, "w"))
