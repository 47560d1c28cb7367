"""Per-file sharding of a TFRecord directory across GPUs.

Files are independent units with their own offset space, so the multi-GPU path needs no data
exchange: rank k decodes its own files on its own device. Files are assigned longest-first to the
least-loaded rank (LPT on file bytes) — deterministic, so every rank computes the same partition
without communicating. torch.distributed (RCCL on ROCm, gloo on CPU) is used only for the barrier
and the max-over-ranks timing around a step.
"""

from __future__ import annotations

import heapq
import os
from collections.abc import Sequence


def lpt_partition(sizes: Sequence[int], world: int) -> list[list[int]]:
    """Indices of `sizes` per rank; each rank's list is in ascending index order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0, r) for r in range(world)]
    parts: list[list[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda j: (-int(sizes[j]), j)):
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return [sorted(p) for p in parts]


def shard_paths(paths: Sequence[str], rank: int, world: int) -> list[str]:
    """This rank's files (sorted names, as the reference sorts its index: reader.py:158)."""
    paths = sorted(paths)
    sizes = [os.path.getsize(p) for p in paths]
    return [paths[i] for i in lpt_partition(sizes, world)[rank]]


def max_over_ranks(value: float) -> float:
    """Max of a per-rank float over the process group (identity without one)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return value
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
