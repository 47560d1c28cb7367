"""Whole-dataset streaming decode: file images -> pinned staging -> HBM -> decode -> host columns.

The batched replacement of the reference's read loops (``load_records``' per-record ThreadPool,
reader.py:212-247, and the per-file process pool of indexer.py:121-134) for reading whole files:
``StreamDecoder.batches(paths)`` packs the files (their images: mmap, or the decompressed stream of
a ZLIB / GZIP file) into batches of up to ``batch_bytes`` (record-aligned cuts for larger files) and
runs them through libtfrg's double-buffered ``tfrg_stream``: while batch k decodes on one slot's
stream, batch k+1 is copied into the other slot's pinned buffer by native threads, indexed and sent
H2D. Each yielded ``StreamBatch`` carries every value already in host memory (bytes_list payloads
gathered on the device into a byte column by default, so nothing refers back to the staging).
"""

from __future__ import annotations

import ctypes as C
import os
from collections import deque
from collections.abc import Iterable, Iterator
from dataclasses import dataclass

import numpy as np

from tfr_reader import _io, hip
from tfr_reader import _native as N
from tfr_reader.cython import indexer as native


@dataclass
class StreamBatch:
    """One decoded batch: ``result`` (a BatchResult) over the records of ``pieces``, each piece
    (file name, first record of the piece in that file) holding ``piece_records[i]`` records in
    file order."""

    pieces: list[tuple[str, int]]
    piece_records: list[int]
    result: hip.BatchResult
    stage_ms: list[float]  # read/copy, index, H2D + decode, D2H (ms, the slot's worker)


class StreamDecoder:
    """``devices``: decode on several devices (a list of device indices, repeats allowed: two
    entries of one device are two independent lanes on it; "all": every visible device). Batch k
    goes to lane k % len(devices); batches are still yielded in plan order (file order, then record
    order), so the output is the same whatever the lane count."""

    def __init__(self, device: int = 0, batch_bytes: int = 256 << 20, copy_threads: int = 8,
                 spec_varint: bool = False, materialize_bytes: bool = True, crc: bool = True,
                 copy_results: bool = True, devices=None) -> None:
        from tfr_reader import shard

        self._lib = N.lib()
        devs = shard.resolve_devices(devices) if devices is not None else [device]
        self.keys = hip.KeyTable()
        self._lanes = []  # (tfrg_stream handle, [decoder of slot 0, slot 1])
        for d in devs:
            h = C.c_void_p()
            N.check(self._lib.tfrg_stream_create(d, batch_bytes, copy_threads, C.byref(h)), "tfrg_stream_create")
            decs = [hip.HipDecoder.wrap(self._lib.tfrg_stream_ctx(h, k), d, self.keys, spec_varint) for k in (0, 1)]
            self._lanes.append((h, decs))
        self.devices = devs
        self._s = self._lanes[0][0]
        self.dec = self._lanes[0][1]
        self.batch_bytes = batch_bytes
        self.materialize_bytes = materialize_bytes
        self.crc = crc
        self.copy_results = copy_results
        self.timing = {"wait": 0.0, "device": 0.0, "fetch": 0.0}  # s spent in _finish: staging, GPU, D2H

    def close(self) -> None:
        """Frees the pinned buffers: results wrapped without ``copy_results`` are invalid after this."""
        for h, _ in getattr(self, "_lanes", []):
            if h:
                self._lib.tfrg_stream_destroy(h)
        self._lanes = []
        self._s = None

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------------ planning
    def _plan(self, paths: Iterable[str]) -> Iterator[list[tuple]]:
        """Batches of pieces of at most batch_bytes each. A piece is (name, first record, path,
        offset, size, image): a plain file is read by the stream's threads with pread (no mmap page
        faults; image None), a compressed one passes its decompressed stream (image). Files larger
        than a batch are cut at record boundaries."""
        cur, size = [], 0
        for p in paths:
            name = p.rsplit("/", 1)[-1]
            fsize = os.path.getsize(p)
            comp = fsize > 0 and _io.is_compressed(p)
            img = _io.file_image(p) if comp else None
            total = img.size if comp else fsize
            if total <= self.batch_bytes:
                parts = [(name, 0, None if comp else p, 0, total, img)]
            else:  # record-aligned cuts of a large file
                whole = img if comp else _io.file_image(p)
                ptr = native.index_buffer(whole)
                parts, r0 = [], 0
                while r0 < ptr.shape[0]:
                    lo = int(ptr[r0, 0])
                    r1 = int(np.searchsorted(ptr[:, 1], lo + self.batch_bytes, side="right"))
                    if r1 <= r0:
                        raise ValueError(f"a record of {p} is larger than batch_bytes")
                    hi = int(ptr[r1 - 1, 1])
                    parts.append((name, r0, None if comp else p, lo, hi - lo, whole[lo:hi] if comp else None))
                    r0 = r1
            for part in parts:
                if size + part[4] > self.batch_bytes and cur:
                    yield cur
                    cur, size = [], 0
                cur.append(part)
                size += part[4]
        if cur:
            yield cur

    # ------------------------------------------------------------------ run
    def _submit(self, lane: int, slot: int, pieces) -> None:
        h, decs = self._lanes[lane]
        decs[slot].push_schema()
        k = len(pieces)
        ptrs = (C.c_void_p * k)(*[pc[5].ctypes.data if pc[5] is not None else None for pc in pieces])
        names = (C.c_char_p * k)(*[pc[2].encode() if pc[2] is not None else None for pc in pieces])
        offs = np.array([pc[3] for pc in pieces], np.uint64)
        sizes = np.array([pc[4] for pc in pieces], np.uint64)
        flags = decs[slot]._flags(False, self.crc, False, self.materialize_bytes)
        N.check(self._lib.tfrg_stream_submit(h, slot, ptrs, names, N.ptr(offs, N.u64p), N.ptr(sizes, N.u64p), k,
                                             flags), "tfrg_stream_submit")

    def _finish(self, lane: int, slot: int, pieces) -> StreamBatch:
        import time

        t0 = time.perf_counter()
        n = C.c_uint64()
        nb = C.c_uint64()
        pr = np.zeros(len(pieces), np.uint64)  # (the pieces' images stay referenced until here)
        ms = (C.c_double * 4)()
        h, decs = self._lanes[lane]
        N.check(self._lib.tfrg_stream_wait(h, slot, C.byref(n), C.byref(nb), N.ptr(pr, N.u64p), len(pieces),
                                           ms), "tfrg_stream_wait")
        d = decs[slot]
        n_rec, nbytes = int(n.value), int(nb.value)
        d.push_schema()  # (keys learned from the other slot's batch)
        hb = self._lib.tfrg_stream_host_buffer(h, slot)
        buf = np.ctypeslib.as_array(C.cast(hb, C.POINTER(C.c_uint8)), shape=(max(nbytes, 1),))[:nbytes]
        sp, ep = N.u64p(), N.u64p()
        self._lib.tfrg_stream_host_ranges(h, slot, C.byref(sp), C.byref(ep))
        st = np.ctypeslib.as_array(sp, shape=(max(n_rec, 1),))[:n_rec].copy()
        en = np.ctypeslib.as_array(ep, shape=(max(n_rec, 1),))[:n_rec].copy()
        t1 = time.perf_counter()
        info = N.TfrgInfo()
        cols = N.TfrgColumns()
        N.check(self._lib.tfrg_stream_result(h, slot, C.byref(info), C.byref(cols)), "tfrg_stream_result")
        t2 = time.perf_counter()
        if info.n_miss_records:  # new keys (usually the first batch only): learn them, decode again
            res = d.decode(buf.copy(), st, en, crc=self.crc, materialize_bytes=self.materialize_bytes)
        else:
            res = self._wrap(d, cols, info, buf, st, en)
        t3 = time.perf_counter()
        self.timing["wait"] += t1 - t0
        self.timing["device"] += t2 - t1
        self.timing["fetch"] += t3 - t2
        return StreamBatch([(pc[0], pc[1]) for pc in pieces], pr.astype(int).tolist(), res, list(ms))

    def _wrap(self, d, cols, info, buf, st, en) -> hip.BatchResult:
        """A BatchResult over the slot's pinned result columns, copied into numpy arrays when
        ``copy_results`` (the default). Without it the arrays are views of the slot's pinned buffers,
        valid only until the caller asks for the next batch: the slot is then handed its next batch
        (and may reallocate its buffers)."""
        n, ns = info.n_records, info.n_slots
        kt = info.kind_totals

        def arr(ptr, dtype, shape):
            count = int(np.prod(shape)) if shape else 0
            if not ptr or count == 0:
                return np.zeros(shape, dtype)
            a = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(count,))
            a = a.reshape(shape)
            return a.copy() if self.copy_results else a

        r = hip.BatchResult()
        r.starts, r.ends, r.payload_only = st, en, False
        r.status = arr(cols.status, np.int32, (n,))
        r.aux = arr(cols.aux, np.int64, (n,))
        r.verdict = arr(cols.verdict, np.uint8, (n,))
        r.order = arr(cols.order, np.uint16, (ns, n))
        r.row_splits = arr(cols.row_splits, np.uint32, (ns, n + 1))
        r.slot_base = arr(cols.slot_base, np.uint64, (max(ns, 1),))
        r.i64 = arr(cols.i64, np.int64, (kt[3],))
        r.f32 = arr(cols.f32, np.uint32, (kt[2],))
        r.bytes_len = arr(cols.bytes_len, np.uint32, (kt[1],))
        if self.materialize_bytes:
            r.bytes_data = arr(cols.bytes_data, np.uint8, (info.bytes_data_len,))
            r.bytes_offsets = arr(cols.bytes_offsets, np.uint64, (kt[1] + 1,))
            r.bytes_off = np.zeros(0, np.uint32)
            r.buf = buf.copy() if info.n_errors else None  # (only the key-UTF-8 error message reads it)
        else:
            r.bytes_off = arr(cols.bytes_off, np.uint32, (kt[1],))
            r.buf = buf.copy()  # the views index the staging copy, which the slot's next batch overwrites
        r.slot_key = [self.keys.key_str[k] for k in self.keys.slot_key[:ns]]
        r.slot_kind = list(self.keys.slot_kind[:ns])
        r.info = info
        return r

    def batches(self, paths: Iterable[str]) -> Iterator[StreamBatch]:
        """Decoded batches in plan order. Up to two batches per lane are in flight (one staging
        while the other decodes); batch k runs on lane k % lanes, slot (k // lanes) % 2."""
        pending: deque = deque()
        L = len(self._lanes)
        for k, pieces in enumerate(self._plan(paths)):
            if len(pending) == 2 * L:
                yield self._finish(*pending.popleft())
            lane, slot = k % L, (k // L) % 2
            self._submit(lane, slot, pieces)
            pending.append((lane, slot, pieces))
        while pending:
            yield self._finish(*pending.popleft())
