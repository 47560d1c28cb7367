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


def resolve_devices(devices) -> list[int]:
    """Device list of the multi-device host paths: None -> [0]; "all" -> every visible device; an
    int -> [it]; a sequence -> as given (repeats are separate lanes on one device)."""
    if devices is None:
        return [0]
    if isinstance(devices, str):
        if devices != "all":
            raise ValueError(f"devices must be 'all', an int or a list of ints, not {devices!r}")
        from tfr_reader import _native as N

        n = int(N.lib().tfrg_device_count())
        if n < 1:
            raise RuntimeError("no HIP device visible")
        return list(range(n))
    if isinstance(devices, (int, np.integer)):
        return [int(devices)]
    out = [int(d) for d in devices]
    if not out:
        raise ValueError("devices is empty")
    return out


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


#: one decode call covers < 4 GiB of input (u32 byte views); a shard is decoded as record-range
#: batches of at most this many bytes, each into its own context's result columns
DEFAULT_BATCH_BYTES = 1 << 30


def plan_batches(starts: np.ndarray, ends: np.ndarray, batch_bytes: int = DEFAULT_BATCH_BYTES,
                 nbytes: int | None = None, balanced: bool = True) -> np.ndarray:
    """Cut records (non-decreasing starts: one shard image in file order) into contiguous runs
    whose byte span is at most ``batch_bytes`` (``balanced``: the fewest such runs, of nearly equal
    spans). Returns rows (r0, r1, lo, hi): records [r0, r1)
    read bytes [lo, hi), lo aligned down to 16 so a batch's base keeps the 16-byte alignment of the
    image. ``nbytes`` (the image size) clamps a last record that runs past EOF (indexer.pyx:225-249
    indexes it; it decodes as truncated)."""
    st = np.ascontiguousarray(starts, np.uint64)
    en = np.ascontiguousarray(ends, np.uint64)
    n = int(st.shape[0])
    if batch_bytes < 32 or batch_bytes >= 1 << 32:
        raise ValueError("batch_bytes must be in [32, 2^32)")
    if n and (np.diff(st.astype(np.int64)) < 0).any():
        raise ValueError("plan_batches needs non-decreasing starts (one image in file order)")
    top = np.maximum.accumulate(np.maximum(en, st)) if n else en
    if nbytes is not None:
        top = np.minimum(top, np.uint64(nbytes))
    if not n:
        return np.zeros((0, 4), np.int64)
    balanced = balanced and os.environ.get("TFRG_PLAN_BALANCED", "1") != "0"  # (A/B measurements)
    if balanced:
        rows = _balanced_rows(st, top, batch_bytes)
        if rows is not None:
            return rows
    return _greedy_rows(st, top, batch_bytes)


def _rows_from_cuts(st: np.ndarray, top: np.ndarray, cuts: np.ndarray) -> np.ndarray:
    """Rows (r0, r1, lo, hi) of the record runs between consecutive cut indices (0 and n included)."""
    r0, r1 = cuts[:-1], cuts[1:]
    lo = (st[r0].astype(np.int64)) & ~15
    hi = np.maximum(top[r1 - 1].astype(np.int64), lo)
    return np.stack([r0, r1, lo, hi], axis=1).astype(np.int64)


def _balanced_rows(st: np.ndarray, top: np.ndarray, cap: int) -> np.ndarray | None:
    """The fewest batches the cap allows, k = ceil(span / cap), of nearly equal spans: batch i starts
    at the record boundary nearest lo0 + i * span / k, so each batch is within one record of span / k
    and there is never a (k+1)-th sliver. k + 1 (then k + 2 …) only when such a cut would leave a
    batch over the cap (records larger than the slack); None when no balanced plan fits (records
    wider than the cap: the greedy plan puts them alone)."""
    n = int(st.shape[0])
    lo0 = int(st[0]) & ~15
    span = int(top[-1]) - lo0
    k0 = max(1, -(-span // cap))
    sti = st.astype(np.int64)
    for k in range(k0, min(n, k0 + 8) + 1):
        if k == 1:
            cuts = np.array([0, n], np.int64)
        else:
            t = lo0 + (np.arange(1, k, dtype=np.int64) * span) // k
            c = np.searchsorted(sti, t, side="left")  # first record starting at or after t
            c = np.clip(c, 1, n - 1)
            prev = np.clip(c - 1, 1, n - 1)
            c = np.where(np.abs(sti[prev] - t) < np.abs(sti[c] - t), prev, c)  # the nearer boundary
            cuts = np.concatenate([[0], c, [n]]).astype(np.int64)
            if (np.diff(cuts) <= 0).any():
                continue
        rows = _rows_from_cuts(st, top, cuts)
        if ((rows[:, 3] - rows[:, 2]) <= cap).all() and ((rows[:, 1] - rows[:, 0]) <= 1 << 30).all():
            return rows
    return None


def _greedy_rows(st: np.ndarray, top: np.ndarray, cap: int) -> np.ndarray:
    """Each batch as wide as the cap allows (the last one takes what is left)."""
    n = int(st.shape[0])
    rows = []
    r0 = 0
    while r0 < n:
        lo = int(st[r0]) & ~15
        r1 = int(np.searchsorted(top, np.uint64(lo + cap), side="right"))
        if r1 <= r0:
            r1 = r0 + 1  # one record wider than a batch: alone (the device rejects it if >= 4 GiB)
        r1 = min(r1, r0 + (1 << 30))
        rows.append((r0, r1, lo, max(int(top[r1 - 1]), lo)))
        r0 = r1
    return np.array(rows, np.int64).reshape(-1, 4)


class ShardResult:
    """Results of a shard decoded as several batches: ``parts[k] = (r0, r1, BatchResult)``, record
    r of the shard being record r - r0 of its batch. Records stay in shard order, i.e. (file name,
    start) order for a ``ShardBatch`` (reader.py:158)."""

    def __init__(self, parts: list) -> None:
        self.parts = parts
        self._first = np.array([p[0] for p in parts] + [parts[-1][1] if parts else 0], np.int64)

    def __len__(self) -> int:
        return int(self._first[-1])

    def locate(self, i: int):
        """(BatchResult, index inside it) of shard record i."""
        if i < 0 or i >= len(self):
            raise IndexError(i)
        k = int(np.searchsorted(self._first, i, side="right")) - 1
        return self.parts[k][2], i - self.parts[k][0]

    @property
    def status(self) -> np.ndarray:
        return np.concatenate([p[2].status for p in self.parts]) if self.parts else np.zeros(0, np.int32)

    @property
    def verdict(self) -> np.ndarray:
        return np.concatenate([p[2].verdict for p in self.parts]) if self.parts else np.zeros(0, np.uint8)

    def feature(self, i: int):
        r, j = self.locate(i)
        return r.feature(j)

    def features(self) -> list:
        """Every record as a ``Feature``; raises the first failing record's exception, in order."""
        out: list = []
        for _, _, r in self.parts:
            out += r.features()
        return out


class ShardDecoder:
    """Decodes one rank's shard on one device as record-range batches (``plan_batches``) of at most
    ``batch_bytes`` each: one decode context per batch, so every batch's result columns stay valid
    together, and the batches spread over ``n_streams`` streams so one batch's kernel tails overlap
    the next batch's work. All contexts share one key table. This is the per-device unit of the
    file-sharded directory decode: the reference reads a directory through a process
    pool over files (indexer.py:121-134) and a thread pool over records (reader.py:212-247)."""

    def __init__(self, device: int = 0, batch_bytes: int = DEFAULT_BATCH_BYTES, n_streams: int = 2,
                 spec_varint: bool = False, keys=None, value_caps: bool = True, balanced: bool = True) -> None:
        from tfr_reader import hip

        self.device = device
        self.value_caps = value_caps  # learn(): size the value columns from the sample
        self.batch_bytes = int(batch_bytes)
        self.balanced = balanced  # plan_batches: k equal batches (False: each as wide as the cap)
        self.n_streams = max(1, int(n_streams))
        self.spec_varint = spec_varint
        self.keys = keys or hip.KeyTable()
        self.decs: list = []

    def close(self) -> None:
        for d in self.decs:
            d.close()
        self.decs = []

    def _decoders(self, k: int) -> list:
        from tfr_reader import hip

        while len(self.decs) < k:
            self.decs.append(hip.HipDecoder(self.device, self.spec_varint, keys=self.keys))
        return self.decs[:k]

    def plan(self, starts, ends, nbytes: int | None = None) -> np.ndarray:
        return plan_batches(starts, ends, self.batch_bytes, nbytes, self.balanced)

    # ------------------------------------------------------------------ host input
    def decode(self, buf: np.ndarray, starts, ends, **kw) -> ShardResult:
        """Decode records [starts[i], ends[i]) of one host image (non-decreasing starts), batch k on
        context k; the streams' host threads run concurrently (ctypes releases the GIL). Keyword
        arguments as ``HipDecoder.decode``."""
        from concurrent.futures import ThreadPoolExecutor

        buf = np.asarray(buf).reshape(-1).view(np.uint8)
        st = np.ascontiguousarray(starts, np.uint64)
        en = np.ascontiguousarray(ends, np.uint64)
        plan = self.plan(st, en, buf.size)
        decs = self._decoders(len(plan))
        out: list = [None] * len(plan)

        def one(k: int) -> None:
            r0, r1, lo, hi = (int(x) for x in plan[k])
            res = decs[k].decode(buf[lo:hi], st[r0:r1] - np.uint64(lo), en[r0:r1] - np.uint64(lo), **kw)
            out[k] = (r0, r1, res)

        if len(plan):  # the first batch learns the key set (and the record-shape templates) alone
            one(0)

        def run(t: int) -> None:
            for k in range(1 + t, len(plan), self.n_streams):
                one(k)

        with ThreadPoolExecutor(self.n_streams) as ex:
            list(ex.map(run, range(min(self.n_streams, max(1, len(plan))))))
        return ShardResult(out)

    # ------------------------------------------------------------------ device-resident input
    @staticmethod
    def rebase(plan: np.ndarray, starts, ends) -> tuple[np.ndarray, np.ndarray]:
        """Per-batch offsets: record r of batch k as offsets from the batch base plan[k, 2]."""
        st = np.ascontiguousarray(starts, np.uint64)
        en = np.ascontiguousarray(ends, np.uint64)
        base = np.repeat(plan[:, 2].astype(np.uint64), (plan[:, 1] - plan[:, 0]).astype(np.int64))
        return st - base, en - base

    @classmethod
    def rebase32(cls, plan: np.ndarray, starts, ends) -> tuple[np.ndarray | None, np.ndarray, np.ndarray]:
        """u32 per-batch offsets for ``decode_device32``: (starts32 or None, ends32, first start of
        each batch). starts32 is None when the records of every batch lie back to back (record r
        starts where record r - 1 ends), as the framing index of files without trailing bytes
        gives them: only the 4-byte ends are then uploaded and read."""
        st, en = cls.rebase(plan, starts, ends)
        if st.size and max(int(st.max()), int(en.max())) >= 1 << 32:
            raise ValueError("a batch spans 4 GiB or more: plan smaller batches")
        first = st[plan[:, 0].astype(np.int64)] if len(plan) else np.zeros(0, np.uint64)
        back_to_back = np.ones(st.shape[0], bool)
        if st.size > 1:
            back_to_back[1:] = st[1:] == en[:-1]
        back_to_back[plan[:, 0].astype(np.int64)] = True  # (a batch's first record: first_start)
        st32 = None if back_to_back.all() else st.astype(np.uint32)
        return st32, en.astype(np.uint32), first.astype(np.uint32)

    def learn(self, plan: np.ndarray, buf: np.ndarray, starts, ends, sample: int = 4096) -> None:
        """Key table and record-shape templates of every batch context from a host sample of the
        first records (device-only callers; the host path learns them itself)."""
        buf = np.asarray(buf).reshape(-1).view(np.uint8)
        st = np.ascontiguousarray(starts, np.uint64)
        en = np.ascontiguousarray(ends, np.uint64)
        decs = self._decoders(len(plan))
        if not decs or not st.size:
            return
        # records spread over the whole shard (its first ones may have shapes the rest has not),
        # gathered back to back
        idx = np.unique(np.linspace(0, st.size - 1, min(st.size, sample)).astype(np.int64))
        s, e = st[idx].astype(np.int64), np.minimum(en[idx], np.uint64(buf.size)).astype(np.int64)
        e = np.maximum(e, s)
        part = np.concatenate([buf[a:b] for a, b in zip(s.tolist(), e.tolist())]) if idx.size else buf[:0]
        pe = np.cumsum(e - s).astype(np.uint64)
        ps = pe - (e - s).astype(np.uint64)
        r = decs[0].decode(part, ps, pe)
        # value capacities from the sample's values per input byte (x 1.25 + 64 Ki): the batches'
        # value columns sized to their data instead of the worst case (one int64 per byte: ~13x the
        # input); a batch that exceeds them is re-decoded with the worst case (HipDecoder.info)
        kt = [int(x) for x in r.info.kind_totals]
        per = max(int(part.size), 1)
        for k, d in enumerate(decs):
            d.push_schema()
            d.learn_templates(part, ps, pe)
            if self.value_caps and k < len(plan):
                nb = int(plan[k, 3] - plan[k, 2])
                caps = [int(kt[j] * nb / per * 1.25) + 65536 for j in (3, 2, 1)]
                d.set_value_caps(*caps)

    def decode_device(self, plan: np.ndarray, d_bytes: int, d_start: int, d_end: int, streams=None,
                      max_record: int | None = None, **kw) -> None:
        """Enqueue every batch of a device-resident shard: image at d_bytes (readable to its 16-byte
        round-up), d_start / d_end the ``rebase``d offsets (u64 device arrays). Batch k runs on
        ``streams[k % len(streams)]`` (HIP stream handles; default: each context's own stream).
        ``max_record``: an upper bound on end - start (HipDecoder.set_record_bound), if known."""
        decs = self._decoders(len(plan))
        if max_record is not None:
            for d in decs:
                d.set_record_bound(max_record)
        for k, (r0, r1, lo, hi) in enumerate(plan.tolist()):
            s = streams[k % len(streams)] if streams else None
            decs[k].decode_device(d_bytes + lo, hi - lo, d_start + 8 * r0, d_end + 8 * r0, r1 - r0, stream=s, **kw)

    def decode_device32(self, plan: np.ndarray, d_bytes: int, d_start32: int | None, d_end32: int, firsts,
                        streams=None, max_record: int | None = None, **kw) -> None:
        """``decode_device`` with the u32 offsets of ``rebase32`` (device arrays; ``d_start32`` None
        for back-to-back records, ``firsts`` the first start of every batch)."""
        decs = self._decoders(len(plan))
        if max_record is not None:
            for d in decs:
                d.set_record_bound(max_record)
        for k, (r0, r1, lo, hi) in enumerate(plan.tolist()):
            s = streams[k % len(streams)] if streams else None
            decs[k].decode_device32(d_bytes + lo, hi - lo, d_start32 + 4 * r0 if d_start32 else None, d_end32 + 4 * r0,
                                    int(firsts[k]), r1 - r0, stream=s, **kw)

    def device_bytes(self) -> tuple[int, int]:
        """(device memory of every batch context, decodes re-run so far: a value hint too small or
        an optimistic decode that left records, tfrg_ctx_device_bytes)."""
        b = r = 0
        for d in self.decs:
            x, y = d.device_bytes()
            b, r = b + x, r + y
        return b, r

    def infos(self, plan: np.ndarray) -> list:
        """Decode summaries of the last ``decode_device`` (waits for it)."""
        return [d.info() for d in self.decs[: len(plan)]]

    def fetch(self, plan: np.ndarray, buf: np.ndarray, starts, ends) -> ShardResult:
        """Host copies of the last ``decode_device``'s results (``buf``: the host image; bytes views
        index it from each batch's base)."""
        buf = np.asarray(buf).reshape(-1).view(np.uint8)
        rs, re = self.rebase(plan, starts, ends)
        parts = []
        for k, (r0, r1, lo, _) in enumerate(plan.tolist()):
            d = self.decs[k]
            parts.append((r0, r1, d._fetch(buf[lo:], rs[r0:r1], re[r0:r1], d.info(), False)))
        return ShardResult(parts)


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
