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

import numpy as np


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


class ShardBatch:
    """The files of one rank's shard as one device batch: their images concatenated (each file's
    absolute offsets shifted by its base), the framing index of every file (native, bit-exact with
    indexer.pyx:212-252), and per record the file it came from. Records are in (file name, start)
    order, the reference's index order (reader.py:158)."""

    def __init__(self, names: list[str], images: list[np.ndarray]) -> None:
        from tfr_reader.cython import indexer

        order = sorted(range(len(names)), key=lambda i: names[i])
        self.names = [names[i] for i in order]
        images = [images[i] for i in order]
        ptrs = [indexer.index_buffer(img) for img in images]
        sizes = np.array([img.size for img in images], np.uint64)
        self.file_base = np.zeros(len(images) + 1, np.uint64)
        np.cumsum(sizes, out=self.file_base[1:])
        counts = np.array([p.shape[0] for p in ptrs], np.int64)
        self.file_first = np.zeros(len(images) + 1, np.int64)
        np.cumsum(counts, out=self.file_first[1:])
        self.buf = np.concatenate(images) if images else np.zeros(0, np.uint8)
        shift = np.repeat(self.file_base[:-1], counts)
        allp = np.concatenate(ptrs) if ptrs else np.zeros((0, 3), np.uint64)
        self.file_starts = allp[:, 0].copy()  # offsets inside each file (the index's tfrecord_start)
        self.file_ends = allp[:, 1].copy()
        self.starts = self.file_starts + shift
        self.ends = self.file_ends + shift
        self.file_of = np.repeat(np.arange(len(images)), counts)

    def __len__(self) -> int:
        return int(self.starts.shape[0])

    @property
    def nbytes(self) -> int:
        return int(self.buf.size)

    def index_rows(self) -> list[tuple[str, int, int]]:
        """(tfrecord_filename, tfrecord_start, tfrecord_end) per record, as the dataset index holds."""
        return [(self.names[f], int(s), int(e)) for f, s, e in
                zip(self.file_of.tolist(), self.file_starts.tolist(), self.file_ends.tolist())]


def read_shard(paths: Sequence[str]) -> ShardBatch:
    """Load and index the given TFRecord files (their basenames name them)."""
    from tfr_reader import _io

    imgs = [_io.file_image(p) for p in paths]  # (decompressed streams of ZLIB / GZIP files)
    return ShardBatch([os.path.basename(p) for p in paths], imgs)


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
