"""Spawned world_size>1 gloo workers (importable without conftest: registers suta_amd itself)."""
import os

import suta_loader

suta_loader.load()
import torch  # noqa: E402

from suta_amd import dist as S  # noqa: E402


def gloo_reduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    counts = {"0": (rank + 1, 10 * (rank + 1)), "10": (rank, 5)}
    red = S.reduce_counts(counts)
    objs = S.gather_objects({"rank": rank})
    q.put((rank, red, [o["rank"] for o in objs]))
    torch.distributed.destroy_process_group()
