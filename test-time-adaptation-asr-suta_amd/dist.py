"""Utterance sharding across the GPUs of one node.

Episodic SUTA resets every utterance (main.py:327-328), so utterances are independent:
they are assigned to ranks by LPT (longest processing time first, greedy to the least-loaded
rank) on an estimated cost, each rank adapts its shard with its own engine, and the only
collective is the final reduction of WER counts (plus an object gather of the transcripts
for the logs).  With backend "nccl" the all_reduce runs on RCCL over xGMI; the CPU tests use
"gloo".
"""
from __future__ import annotations

import heapq
from typing import Dict, List, Sequence, Tuple


def lpt_shard(costs: Sequence[float], world: int) -> List[List[int]]:
    """Indices per rank; ties broken by index so every rank computes the same plan."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap = [(0.0, r) for r in range(world)]
    heapq.heapify(heap)
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    for s in shards:
        s.sort()
    return shards


def utterance_cost(n_samples: int, cfg: dict, steps: int) -> float:
    from .flops import suta_flops
    return suta_flops(cfg, max(int(n_samples), 400), steps)


def reduce_counts(counts: Dict[str, Tuple[int, int]], device=None) -> Dict[str, Tuple[int, int]]:
    """Sum {checkpoint: (edits, ref_words)} over ranks with one all_reduce of an int64 tensor."""
    import torch
    import torch.distributed as dist
    keys = sorted(counts)
    t = torch.tensor([v for k in keys for v in counts[k]], dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    vals = t.cpu().tolist()
    return {k: (vals[2 * i], vals[2 * i + 1]) for i, k in enumerate(keys)}


def gather_objects(obj):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
