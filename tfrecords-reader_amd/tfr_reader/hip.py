"""HIP decode engine: batches of TFRecord byte ranges -> columnar device decode -> Feature objects.

This is the batched replacement of the reference's per-record ``decoder.example_from_bytes``
(src/tfr_reader/cython/decoder.pyx:107) behind the ``Feature`` API (example/feature.py:51-151).
The host side owns the key table ("schema"): keys are discovered by the device (schema misses),
interned here (UTF-8 validity decided by CPython's own decoder, as decoder.pyx:164 does) and the
batch is decoded again. A dataset's key set is small and stable, so this converges in one extra
pass on the first batch and costs nothing afterwards.
"""

from __future__ import annotations

import contextlib
import ctypes as C
import gc
import threading
from collections.abc import Sequence

import numpy as np

from tfr_reader import _native as N
from tfr_reader import _status as S

try:  # C bases of the Feature objects over a batch's columns (csrc/tfrg_py.cpp, built with libtfrg)
    from tfr_reader import _tfrg_py as _PY
except ImportError:
    _PY = None

KIND_NAMES = {1: "bytes_list", 2: "float_list", 3: "int64_list"}


_GC_LOCK = threading.Lock()
_GC_DEPTH = 0       # batches being built right now, over all threads
_GC_RESTORE = False  # the collector was enabled when the outermost of them began


@contextlib.contextmanager
def _no_gc():
    """Cyclic GC paused while a batch's Python objects are built: creating millions of lists and
    tuples otherwise triggers generation scans over all of them (4-5x the construction time).
    Reference-counted over threads: the collector is re-enabled only when the last concurrent build
    ends, and only if it was enabled when the first one began (a caller's own gc.disable() holds)."""
    global _GC_DEPTH, _GC_RESTORE
    with _GC_LOCK:
        if _GC_DEPTH == 0:
            _GC_RESTORE = gc.isenabled()
            gc.disable()
        _GC_DEPTH += 1
    try:
        yield
    finally:
        with _GC_LOCK:
            _GC_DEPTH -= 1
            if _GC_DEPTH == 0 and _GC_RESTORE:
                gc.enable()

#: records larger than this (framed bytes) are decoded one wavefront per record (libtfrg default)
DEFAULT_LANE_MAX = 2048
KIND_IDS = {v: k for k, v in KIND_NAMES.items()}


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return buf.reshape(-1).view(np.uint8)
    return np.frombuffer(buf, dtype=np.uint8)


class KeyTable:
    """Interned keys and (key, kind) slots, mirrored to the device by ``HipDecoder``."""

    def __init__(self) -> None:
        self.key_ids: dict[bytes, int] = {}
        self.keys: list[bytes] = []
        self.key_str: list[str | None] = []
        self.slots: dict[tuple[int, int], int] = {}
        self.slot_key: list[int] = []
        self.slot_kind: list[int] = []
        self.version = 0
        self.lock = threading.RLock()  # (decoders of several host threads may share one table)

    def intern(self, key: bytes, kind: int) -> bool:
        """Add key (and its (key, kind) slot when kind != 0 and the key is valid UTF-8).
        Returns True if anything new was added."""
        with self.lock:
            return self._intern(key, kind)

    def _intern(self, key: bytes, kind: int) -> bool:
        new = False
        kid = self.key_ids.get(key)
        if kid is None:
            kid = len(self.keys)
            self.key_ids[key] = kid
            self.keys.append(key)
            try:
                self.key_str.append(key.decode("utf-8"))
            except UnicodeDecodeError:
                self.key_str.append(None)
            new = True
        if kind and self.key_str[kid] is not None and (kid, kind) not in self.slots:
            self.slots[(kid, kind)] = len(self.slot_key)
            self.slot_key.append(kid)
            self.slot_kind.append(kind)
            new = True
        if new:
            self.version += 1
        return new


class HipDecoder:
    """One device context (one HIP device, one host thread at a time)."""

    def __init__(self, device: int = 0, spec_varint: bool = False, keys: KeyTable | None = None) -> None:
        self._lib = N.lib()
        self.device = device
        self.spec_varint = spec_varint
        self.keys = keys or KeyTable()
        self._pushed = -1
        self._lock = threading.Lock()
        h = C.c_void_p()
        N.check(self._lib.tfrg_ctx_create(device, C.byref(h)), "tfrg_ctx_create")
        self._ctx = h

    @classmethod
    def wrap(cls, ctx: int, device: int, keys: KeyTable, spec_varint: bool = False) -> HipDecoder:
        """A decoder over a context owned elsewhere (a tfrg_stream slot): shares ``keys``, never
        destroys the context."""
        d = cls.__new__(cls)
        d._lib = N.lib()
        d.device = device
        d.spec_varint = spec_varint
        d.keys = keys
        d._pushed = -1
        d._lock = threading.Lock()
        d._ctx = C.c_void_p(ctx)
        d._owned = False
        return d

    def close(self) -> None:
        if self._ctx and getattr(self, "_owned", True):
            self._lib.tfrg_ctx_destroy(self._ctx)
        self._ctx = None

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def set_lane_max(self, nbytes: int) -> None:
        N.check(self._lib.tfrg_ctx_set_lane_max(self._ctx, nbytes), "tfrg_ctx_set_lane_max")

    def set_templates(self, on: bool) -> None:
        """Record-shape templates (tfrg_learn_templates): on by default."""
        N.check(self._lib.tfrg_ctx_set_templates(self._ctx, int(bool(on))), "tfrg_ctx_set_templates")

    def template_count(self) -> int:
        return int(self._lib.tfrg_template_count(self._ctx))

    def learn_templates(self, buf: np.ndarray, starts: np.ndarray, ends: np.ndarray, payload_only: bool = False) -> int:
        """Learn record shapes from a host sample (device-only callers; tfrg_decode_host does it itself)."""
        b = np.ascontiguousarray(buf, np.uint8)
        st = np.ascontiguousarray(starts, np.uint64)
        en = np.ascontiguousarray(ends, np.uint64)
        k = self._lib.tfrg_learn_templates(self._ctx, N.ptr(b), b.size, N.ptr(st), N.ptr(en), st.size,
                                           N.FLAG_PAYLOAD_ONLY if payload_only else 0)
        N.check(min(k, 0), "tfrg_learn_templates")
        return int(k)


    def set_record_bound(self, nbytes: int) -> None:
        """Upper bound on (end - start) of the records of later ``decode_device`` calls (0 = unknown):
        a bound <= lane_max skips the large-record count launch (tfrg_ctx_set_record_bound)."""
        N.check(self._lib.tfrg_ctx_set_record_bound(self._ctx, int(nbytes)), "tfrg_ctx_set_record_bound")

    def set_wave_stage(self, nbytes: int) -> None:
        """Records above lane_max spanning <= nbytes go to the LDS-staged wavefront kernels."""
        N.check(self._lib.tfrg_ctx_set_wave_stage(self._ctx, nbytes), "tfrg_ctx_set_wave_stage")

    def set_profiling(self, on: bool) -> None:
        N.check(self._lib.tfrg_ctx_set_profiling(self._ctx, int(on)), "tfrg_ctx_set_profiling")

    def profile_last(self) -> dict[str, float]:
        """Per-kernel durations (ms) of the last decode (needs set_profiling(True) before it)."""
        ms = (C.c_float * 16)()
        names = (C.c_char_p * 16)()
        k = self._lib.tfrg_profile_last(self._ctx, ms, names, 16)
        if k < 0:
            N.check(k, "tfrg_profile_last")
        return {names[i].decode(): float(ms[i]) for i in range(k)}

    # ------------------------------------------------------------------ schema
    def push_schema(self) -> None:
        kt = self.keys
        if self._pushed == kt.version:
            return
        with kt.lock:
            self._push_schema(kt)

    def _push_schema(self, kt: KeyTable) -> None:
        blob = b"".join(kt.keys)
        offs = np.zeros(len(kt.keys) + 1, np.uint64)
        if kt.keys:
            offs[1:] = np.cumsum([len(k) for k in kt.keys])
        flags = np.array([0 if s is not None else 1 for s in kt.key_str] or [0], np.uint32)
        blob_arr = np.frombuffer(blob or b"\0", np.uint8)
        sk = np.array(kt.slot_key or [0], np.uint32)
        sd = np.array(kt.slot_kind or [1], np.uint8)
        N.check(
            self._lib.tfrg_set_schema(
                self._ctx, len(kt.keys), N.ptr(blob_arr), N.ptr(offs, N.u64p), N.ptr(flags, N.u32p),
                len(kt.slot_key), N.ptr(sk, N.u32p), N.ptr(sd, N.u8p),
            ),
            "tfrg_set_schema",
        )
        self._pushed = kt.version

    # ------------------------------------------------------------------ decode
    def _flags(self, payload_only: bool, crc: bool, strict_crc: bool = False, materialize_bytes: bool = False) -> int:
        f = 0
        if payload_only:
            f |= N.FLAG_PAYLOAD_ONLY
        if self.spec_varint:
            f |= N.FLAG_SPEC_VARINT
        if not crc:
            f |= N.FLAG_NO_CRC
        if strict_crc:
            f |= N.FLAG_STRICT_CRC
        if materialize_bytes:
            f |= N.FLAG_MATERIALIZE_BYTES
        return f

    def info(self) -> N.TfrgInfo:
        info = N.TfrgInfo()
        N.check(self._lib.tfrg_result_info(self._ctx, C.byref(info)), "tfrg_result_info")
        return info

    def set_value_caps(self, int64_values: int = 0, float_values: int = 0, bytes_values: int = 0) -> None:
        """Capacity hints for the values of the following decodes (0: the worst case, ~13x the
        batch bytes of device memory); a decode that exceeds one is re-run with the worst case inside
        ``info()`` (tfrg_ctx_set_value_caps)."""
        N.check(self._lib.tfrg_ctx_set_value_caps(self._ctx, int(int64_values), int(float_values), int(bytes_values)),
                "tfrg_ctx_set_value_caps")

    def device_bytes(self) -> tuple[int, int]:
        """(device memory held by this decoder's context, decodes re-run: a value-capacity hint too
        small, or an optimistic decode that left records no template took)."""
        b, r = C.c_uint64(), C.c_uint64()
        N.check(self._lib.tfrg_ctx_device_bytes(self._ctx, C.byref(b), C.byref(r)), "tfrg_ctx_device_bytes")
        return int(b.value), int(r.value)

    def device_columns(self) -> N.TfrgColumns:
        """Device pointers of the last result (tfrg_result_device): valid until the next decode on
        this decoder; the placed slots' identity row splits are written into them on the decode's
        stream first."""
        cols = N.TfrgColumns()
        N.check(self._lib.tfrg_result_device(self._ctx, C.byref(cols)), "tfrg_result_device")
        return cols

    def _learn_misses(self, buf: np.ndarray, info: N.TfrgInfo) -> bool:
        m = min(info.n_miss_entries, 1 << 16)
        miss = np.zeros((max(m, 1), 4), np.uint32)
        cols = N.TfrgColumns()
        cols.miss = N.ptr(miss, N.u32p)
        N.check(self._lib.tfrg_result_fetch(self._ctx, C.byref(cols)), "tfrg_result_fetch")
        new = False
        seen = set()
        for _rec, kind, off, ln in miss[:m].tolist():
            k = (off, ln, kind)
            if k in seen:
                continue
            seen.add(k)
            new |= self.keys.intern(bytes(buf[off : off + ln]), kind)
        return new

    SEED_SAMPLE = 64  # records per host decode whose keys seed the key table (tfrg_scan_keys)

    def _seed_keys(self, buf: np.ndarray, st: np.ndarray, en: np.ndarray, flags: int) -> None:
        """Intern the keys of a sample of the batch's records before the device sees them, so a first
        decode of a new schema does not send every record through the exact walker's miss pass."""
        n = int(st.shape[0])
        if n == 0 or buf.size == 0:
            return
        if n > self.SEED_SAMPLE:
            pick = np.linspace(0, n - 1, self.SEED_SAMPLE).astype(np.int64)
            st, en = np.ascontiguousarray(st[pick]), np.ascontiguousarray(en[pick])
        cap = 256
        out = np.zeros((cap, 3), np.uint64)
        k = int(self._lib.tfrg_scan_keys(N.ptr(buf), buf.size, N.ptr(st, N.u64p), N.ptr(en, N.u64p), st.size,
                                         flags & N.FLAG_PAYLOAD_ONLY, N.ptr(out, N.u64p), cap))
        for off, ln, kind in out[:k].tolist():
            self.keys.intern(bytes(buf[off : off + ln]), kind)

    def decode(
        self,
        buf,
        starts: Sequence[int] | np.ndarray,
        ends: Sequence[int] | np.ndarray,
        *,
        payload_only: bool = False,
        crc: bool = True,
        strict_crc: bool = False,
        materialize_bytes: bool = False,
    ) -> BatchResult:
        """Decode records [starts[i], ends[i]) of a host buffer (framed unless payload_only).

        ``strict_crc``: records whose length field or masked CRC-32C does not match fail with
        ``DataLossError`` (TFRG_FLAG_STRICT_CRC) instead of only clearing their verdict bits.
        ``materialize_bytes``: bytes_list payloads are gathered on the device into one byte column
        (``BatchResult.bytes_data`` / ``bytes_offsets``) and fetched, instead of being sliced from
        the host copy of the input."""
        buf = _as_u8(buf)
        st = np.ascontiguousarray(starts, dtype=np.uint64)
        en = np.ascontiguousarray(ends, dtype=np.uint64)
        if st.shape != en.shape:
            raise ValueError("starts and ends differ in length")
        n = int(st.shape[0])
        flags = self._flags(payload_only, crc, strict_crc, materialize_bytes)
        with self._lock:
            self._seed_keys(buf, st, en, flags)
            # every round interns at least one new key (else it raises), and at most 65,536 miss
            # entries are reported per round, so high-cardinality key sets take several rounds
            while True:
                self.push_schema()
                N.check(
                    self._lib.tfrg_decode_host(
                        self._ctx, N.ptr(buf) if buf.size else None, buf.size, N.ptr(st, N.u64p),
                        N.ptr(en, N.u64p), n, flags, None,
                    ),
                    "tfrg_decode_host",
                )
                info = self.info()
                if info.scan_timeout:
                    raise N.NativeError("row-split scan look-back timed out")
                if info.n_miss_records == 0:
                    break
                # (another decoder sharing the key table may have interned the keys first)
                if not self._learn_misses(buf, info) and self._pushed == self.keys.version:
                    raise N.NativeError("schema misses reported but no new key learned")
            return self._fetch(buf, st, en, info, payload_only, materialize_bytes)

    def decode_device(self, d_bytes: int, nbytes: int, d_start: int, d_end: int, n: int, *,
                      payload_only: bool = False, crc: bool = True, stream: int | None = None,
                      strict_crc: bool = False, materialize_bytes: bool = False) -> None:
        """Asynchronous decode of a device-resident batch (raw device pointers; bench path)."""
        self.push_schema()
        N.check(
            self._lib.tfrg_decode_device(
                self._ctx, C.c_void_p(d_bytes), nbytes, C.c_void_p(d_start), C.c_void_p(d_end), n,
                self._flags(payload_only, crc, strict_crc, materialize_bytes), C.c_void_p(stream) if stream else None,
            ),
            "tfrg_decode_device",
        )

    def decode_device32(self, d_bytes: int, nbytes: int, d_start32: int | None, d_end32: int, first_start: int,
                        n: int, *, payload_only: bool = False, crc: bool = True, stream: int | None = None,
                        strict_crc: bool = False, materialize_bytes: bool = False) -> None:
        """``decode_device`` with u32 offsets; ``d_start32`` None: back-to-back records, record 0 at
        ``first_start`` and record i > 0 where record i - 1 ends (only the u32 ends are read)."""
        self.push_schema()
        N.check(
            self._lib.tfrg_decode_device32(
                self._ctx, C.c_void_p(d_bytes), nbytes, C.c_void_p(d_start32) if d_start32 else None,
                C.c_void_p(d_end32), first_start, n,
                self._flags(payload_only, crc, strict_crc, materialize_bytes), C.c_void_p(stream) if stream else None,
            ),
            "tfrg_decode_device32",
        )

    def _fetch(self, buf, st, en, info: N.TfrgInfo, payload_only: bool, materialize: bool = False) -> BatchResult:
        n, ns = info.n_records, info.n_slots
        kt = info.kind_totals
        r = BatchResult()
        r.buf, r.starts, r.ends, r.payload_only = buf, st, en, payload_only
        r.status = np.empty(n, np.int32)
        r.aux = np.empty(n, np.int64)
        r.verdict = np.empty(n, np.uint8)
        r.order = np.empty((ns, n), np.uint16)
        r.row_splits = np.empty((ns, n + 1), np.uint32)
        r.slot_base = np.empty(max(ns, 1), np.uint64)
        r.i64 = np.empty(kt[3], np.int64)
        r.f32 = np.empty(kt[2], np.uint32)
        r.bytes_off = np.empty(kt[1], np.uint32)
        r.bytes_len = np.empty(kt[1], np.uint32)
        names = ["status", "aux", "verdict", "order", "row_splits", "slot_base", "i64", "f32", "bytes_off",
                 "bytes_len"]
        if materialize:
            r.bytes_data = np.empty(info.bytes_data_len, np.uint8)
            r.bytes_offsets = np.empty(kt[1] + 1, np.uint64)
            names += ["bytes_data", "bytes_offsets"]
        cols = N.TfrgColumns()
        for name in names:
            arr = getattr(r, name)
            setattr(cols, name, N.ptr(arr, dict(N.TfrgColumns._fields_)[name]))
        N.check(self._lib.tfrg_result_fetch(self._ctx, C.byref(cols)), "tfrg_result_fetch")
        r.slot_key = [self.keys.key_str[k] for k in self.keys.slot_key[:ns]]
        r.slot_kind = list(self.keys.slot_kind[:ns])
        r.info = info
        return r


class BatchResult:
    """Columnar result of one batch; ``feature(i)`` builds the reference ``Feature`` view."""

    buf: np.ndarray
    starts: np.ndarray
    ends: np.ndarray
    payload_only: bool
    status: np.ndarray
    aux: np.ndarray
    verdict: np.ndarray
    order: np.ndarray
    row_splits: np.ndarray
    slot_base: np.ndarray
    i64: np.ndarray
    f32: np.ndarray
    bytes_off: np.ndarray
    bytes_len: np.ndarray
    slot_key: list[str]
    slot_kind: list[int]
    bytes_data: np.ndarray | None = None  # materialize_bytes: the device-gathered byte column
    bytes_offsets: np.ndarray | None = None  # its u64 offsets (one per bytes element, + 1)
    _lay = None  # (record -> layout index, layouts), built on first use
    _py = None  # per slot: (values as Python objects, rebased row splits), built on first use

    def _bytes_elems(self, lo: int, hi: int) -> list[bytes]:
        """bytes elements [lo, hi) of the bytes value array, as ``bytes``."""
        if hi <= lo:
            return []
        if _PY is not None:  # (copied in C straight from the buffer)
            if self.bytes_data is not None:
                o = self.bytes_offsets[lo : hi + 1].astype(np.int64)
                return _PY.split_bytes(self.bytes_data, o[:-1], np.diff(o))
            return _PY.split_bytes(self.buf, self.bytes_off[lo:hi].astype(np.int64), self.bytes_len[lo:hi].astype(np.int64))
        if self.bytes_data is not None:
            o = self.bytes_offsets[lo : hi + 1].tolist()
            d = self.bytes_data
            return [d[o[j] : o[j + 1]].tobytes() for j in range(hi - lo)]
        b = self.buf
        return [b[o : o + ln].tobytes() for o, ln in zip(self.bytes_off[lo:hi].tolist(),
                                                           self.bytes_len[lo:hi].tolist())]

    def __len__(self) -> int:
        return int(self.status.shape[0])

    def payload_start(self, i: int) -> int:
        return int(self.starts[i]) + (0 if self.payload_only else 12)

    def error(self, i: int) -> BaseException | None:
        st = int(self.status[i])
        if st == S.OK:
            return None
        key = None
        if st == S.ERR_KEY_UTF8:
            aux = int(self.aux[i]) & 0xFFFFFFFFFFFFFFFF
            off, ln = aux >> 32, aux & 0xFFFFFFFF
            p = self.payload_start(i) + off
            key = bytes(self.buf[p : p + ln])
        return S.exception_for(st, int(self.aux[i]), key)

    def raise_for(self, i: int) -> None:
        e = self.error(i)
        if e is not None:
            raise e

    def slot_values(self, s: int, i: int) -> list:
        lo = int(self.slot_base[s]) + int(self.row_splits[s, i])
        hi = int(self.slot_base[s]) + int(self.row_splits[s, i + 1])
        kind = self.slot_kind[s]
        if kind == 3:
            return self.i64[lo:hi].tolist()
        if kind == 2:
            return self.f32[lo:hi].view(np.float32).tolist()
        return self._bytes_elems(lo, hi)

    def record_dict(self, i: int) -> dict:
        """key -> raw feature (reference dict order). Raises the record's exception."""
        self.raise_for(i)
        col = self.order[:, i]
        present = np.flatnonzero(col)
        present = present[np.argsort(col[present], kind="stable")]
        return {self.slot_key[s]: ColumnFeature(self, int(s), i) for s in present.tolist()}

    def feature(self, i: int):
        """Record i as a ``Feature`` (raises the record's exception)."""
        self.raise_for(i)
        if self._lay is None:
            self._lay = self._layouts()
        inv, layouts = self._lay
        if self._py is None:
            self._py = [None] * len(self.slot_kind)
        if _PY is not None:
            return _PY.make_records(_record_class(), self, self._py, i, inv[i : i + 1], layouts)[0]
        return _record_class()((self, i, layouts[int(inv[i])]))

    def _pycol(self, s: int):
        """Slot s over the whole batch as Python objects, converted once and cached: (the values of
        the slot's column as a list, its row splits rebased to that list). A record's ``.value`` is
        then one list slice (the fresh list the reference returns per access)."""
        py = self._py
        if py is None:
            py = self._py = [None] * len(self.slot_kind)
        c = py[s]
        if c is None:
            with _no_gc():
                c = py[s] = self._pycol_build(s)
        return c

    def _pycol_build(self, s: int):
        base = int(self.slot_base[s])
        rs = self.row_splits[s]
        r0 = int(rs[0])
        lo, hi = base + r0, base + int(rs[-1])
        kind = self.slot_kind[s]
        if kind == 3:
            vals = self.i64[lo:hi].tolist()
        elif kind == 2:
            vals = self.f32[lo:hi].view(np.float32).tolist()
        else:
            vals = self._bytes_list(lo, hi)
        return vals, ((rs - np.uint32(r0)).tolist() if r0 else rs.tolist())

    def _bytes_list(self, lo: int, hi: int) -> list[bytes]:
        """bytes elements [lo, hi) as ``bytes``, sliced from one bytes copy of the region they span."""
        if hi <= lo:
            return []
        if _PY is not None:
            return self._bytes_elems(lo, hi)
        if self.bytes_data is not None:
            o = self.bytes_offsets[lo : hi + 1]
            a = int(o[0])
            blob = self.bytes_data[a : int(o[-1])].tobytes()
            ol = (o - np.uint64(a)).tolist()
            return [blob[ol[j] : ol[j + 1]] for j in range(hi - lo)]
        off = self.bytes_off[lo:hi]
        ln = self.bytes_len[lo:hi]
        a = int(off.min())
        b = int((off.astype(np.uint64) + ln).max())
        if b - a > 4 * (int(ln.sum()) + 64 * (hi - lo)):  # (scattered views: per-element copies)
            return self._bytes_elems(lo, hi)
        blob = self.buf[a:b].tobytes()
        ol = (off - np.uint32(a)).tolist()
        return [blob[x : x + n] for x, n in zip(ol, ln.tolist())]

    def _layouts(self) -> tuple[np.ndarray, list[_Layout]]:
        """Per record, the index of its key layout (present slots in dict order); records of a
        dataset share a handful of layouts, so the per-record work is one array lookup."""
        ns, n = self.order.shape
        if ns == 0:
            return np.zeros(n, np.int64), [_Layout((), self.slot_key, self.slot_kind)]
        if ns <= 4:
            sig = np.zeros(n, np.uint64)
            for s in range(ns):
                sig |= self.order[s].astype(np.uint64) << np.uint64(16 * s)
            uniq, inv = np.unique(sig, return_inverse=True)
            cols = [[(int(u) >> (16 * s)) & 0xFFFF for s in range(ns)] for u in uniq.tolist()]
        else:
            uniq, inv = np.unique(np.ascontiguousarray(self.order.T), axis=0, return_inverse=True)
            cols = uniq.tolist()
        layouts = []
        for col in cols:
            present = sorted((rk, s) for s, rk in enumerate(col) if rk)
            layouts.append(_Layout(tuple(s for _, s in present), self.slot_key, self.slot_kind))
        return inv.reshape(-1), layouts

    def features(self, start: int = 0, stop: int | None = None) -> list:
        """Records [start, stop) as ``Feature`` objects (views over the batch's columns: a slot's
        values become Python objects once per batch, on first access). Raises the first failing
        record's exception, in record order, like decoding them one by one."""
        stop = len(self) if stop is None else min(stop, len(self))
        bad = np.flatnonzero(self.status[start:stop])
        if bad.size:
            self.raise_for(start + int(bad[0]))
        if self._lay is None:
            self._lay = self._layouts()
        inv, layouts = self._lay
        if self._py is None:
            self._py = [None] * len(self.slot_kind)
        rec = _record_class()
        with _no_gc():
            if _PY is not None:  # records made in C
                return _PY.make_records(rec, self, self._py, start, inv[start:stop], layouts)
            # one (batch, record, layout) tuple per record (built by tuple.__new__: no Python __init__)
            return [rec((self, i, layouts[j])) for i, j in zip(range(start, stop), inv[start:stop].tolist())]

    def column(self, key: str, kind: str | None = None) -> tuple[np.ndarray, np.ndarray]:
        """Ragged column of one key over the batch: (values, offsets) with record i's values at
        ``values[offsets[i]:offsets[i + 1]]`` (numpy views of the fetched columns; floats as
        float32, bytes as an object array of ``bytes``). Records without the key contribute none."""
        slots = [s for s, k in enumerate(self.slot_key) if k == key and (kind is None or
                                                                      KIND_NAMES[self.slot_kind[s]] == kind)]
        if not slots:
            raise KeyError(key)
        if len(slots) > 1:  # (the key table outlives batches: only the kinds present here count)
            slots = [s for s in slots if self.order[s].any()] or slots[:1]
        if len(slots) > 1:
            raise ValueError(f"key {key!r} has several kinds in this batch; pass kind=")
        s = slots[0]
        base = int(self.slot_base[s])
        rs = self.row_splits[s].astype(np.int64)
        lo, hi = base + int(rs[0]), base + int(rs[-1])
        k = self.slot_kind[s]
        if k == 3:
            vals = self.i64[lo:hi]
        elif k == 2:
            vals = self.f32[lo:hi].view(np.float32)
        else:
            vals = np.array(self._bytes_elems(lo, hi), dtype=object)
        return vals, rs - rs[0]

    def crc_ok(self) -> np.ndarray:
        return (self.verdict & 6) == 6


class _Layout:
    """Present slots of a record in dict order, with the key -> slot map they imply."""

    __slots__ = ("slots", "keys", "index", "acc")

    def __init__(self, slots: tuple[int, ...], slot_key: list[str], slot_kind: list[int] | None = None) -> None:
        self.slots = slots
        self.keys = [slot_key[s] for s in slots]
        self.index = dict(zip(self.keys, slots))
        # key -> (slot, accessor class) for the Feature fast path (_HipRecord.__getitem__)
        self.acc = {k: (s, _accessor_classes()[slot_kind[s]]) for k, s in self.index.items()} if slot_kind else {}


class _RecordView:
    """Read-only ``key -> ColumnFeature`` mapping of one record (what ``Feature`` wraps); the
    column views are built on access."""

    __slots__ = ("_r", "_i", "_l")

    def __init__(self, r: BatchResult, i: int, layout: _Layout) -> None:
        self._r, self._i, self._l = r, i, layout

    def __len__(self) -> int:
        return len(self._l.slots)

    def __iter__(self):
        return iter(self._l.keys)

    def __contains__(self, key) -> bool:
        return key in self._l.index

    def keys(self):
        return list(self._l.keys)

    def __getitem__(self, key: str) -> ColumnFeature:
        return ColumnFeature(self._r, self._l.index[key], self._i)

    def items(self):
        return [(k, ColumnFeature(self._r, s, self._i)) for k, s in zip(self._l.keys, self._l.slots)]

    def values(self):
        return [ColumnFeature(self._r, s, self._i) for s in self._l.slots]


class _ValueList:
    """A decoded value list with the reference list-object surface (decoder.pyx:352-376)."""

    __slots__ = ("_r", "_s", "_i", "_bytes")

    def __init__(self, r: BatchResult, s: int, i: int, is_bytes: bool) -> None:
        self._r, self._s, self._i, self._bytes = r, s, i, is_bytes

    @property
    def value(self) -> list:
        return self._r.slot_values(self._s, self._i)  # a fresh list per access, as the reference

    def __getitem__(self, item: int):
        return self.value[item]

    def __len__(self) -> int:
        if not self._bytes:  # only BytesList defines __len__ in the reference (decoder.pyx:359)
            raise TypeError(f"object of type '{type(self).__name__}' has no len()")
        return len(self.value)


class ColumnFeature:
    """One key's value in a decoded record: the reference cython ``Feature`` surface
    (decoder.pyx:314-349): ``WhichOneof`` and kind-checked list properties."""

    __slots__ = ("_r", "_s", "_i")

    def __init__(self, r: BatchResult, s: int, i: int) -> None:
        self._r, self._s, self._i = r, s, i

    @property
    def kind(self) -> str:
        return KIND_NAMES[self._r.slot_kind[self._s]]

    def WhichOneof(self, _kind: str) -> str:  # noqa: N802 (protobuf API name)
        return self.kind

    def _list(self, want: str, article: str) -> _ValueList:
        if self.kind != want:
            raise Exception(f"Feature is not {article} {want}")  # noqa: TRY002
        return _ValueList(self._r, self._s, self._i, want == "bytes_list")

    @property
    def float_list(self) -> _ValueList:
        return self._list("float_list", "a")

    @property
    def int64_list(self) -> _ValueList:
        return self._list("int64_list", "an")

    @property
    def bytes_list(self) -> _ValueList:
        return self._list("bytes_list", "a")


# ---------------------------------------------------------------------- Feature fast path
_RECORD_CLASS = None
_ACC_CLASSES = None


class _ListRaw:
    """A raw feature over one decoded list (``Feature.feature[key]`` of the fast path)."""

    __slots__ = ("kind", "_v")

    def __init__(self, kind: str, v: list) -> None:
        self.kind, self._v = kind, v

    def WhichOneof(self, _kind: str) -> str:  # noqa: N802 (protobuf API name)
        return self.kind

    def _list(self, want: str, article: str):
        if self.kind != want:
            raise Exception(f"Feature is not {article} {want}")  # noqa: TRY002
        return _Values(self._v)

    @property
    def float_list(self):
        return self._list("float_list", "a")

    @property
    def int64_list(self):
        return self._list("int64_list", "an")

    @property
    def bytes_list(self):
        return self._list("bytes_list", "a")


class _Values:
    __slots__ = ("_v",)

    def __init__(self, v: list) -> None:
        self._v = v

    @property
    def value(self) -> list:
        return list(self._v)

    def __getitem__(self, item):
        return self._v[item]


def _accessor_classes() -> dict:
    """kind -> accessor class: ``Int64List`` / ``FloatList`` / ``BytesList`` subclasses over a slice
    of a slot's cached Python list (``.value`` returns a fresh list, as the reference's does)."""
    global _ACC_CLASSES
    if _ACC_CLASSES is None:
        from tfr_reader.example import feature as F  # noqa: PLC0415

        def make(base, kind):
            if _PY is not None:
                # C base (csrc/tfrg_py.cpp ColAcc): made and read without bytecode, no __dict__ and
                # no GC tracking per object; an instance of ``base`` by ABC registration
                ns = {"__slots__": (), "feature": property(lambda self: _ListRaw(kind, self.value))}
                if base is F.BytesList:
                    ns["bytes_io"] = F.BytesList.bytes_io
                CAcc = type(base.__name__, (_PY.ColAcc,), ns)
                CAcc.__qualname__ = base.__name__
                base.register(CAcc)
                return CAcc

            # a (values, lo, hi) tuple: created by tuple.__new__ alone (no Python __init__ per access)
            class Acc(tuple, base):
                __slots__ = ()
                __init__ = tuple.__init__

                @property
                def value(self):
                    return self[0][self[1] : self[2]]

                @property
                def feature(self):
                    return _ListRaw(kind, self[0][self[1] : self[2]])

            Acc.__name__ = Acc.__qualname__ = base.__name__
            return Acc

        _ACC_CLASSES = {3: make(F.Int64List, "int64_list"), 2: make(F.FloatList, "float_list"),
                        1: make(F.BytesList, "bytes_list")}
    return _ACC_CLASSES


def _record_class():
    """The device path's ``Feature``: a (BatchResult, record, layout) tuple (one C-level allocation
    per record). ``f[key]`` builds the accessor (``Int64List`` / ``FloatList`` / ``BytesList`` over
    a slice of the batch's cached per-slot Python list) and ``.value`` is one list slice; a missing
    key raises the reference's KeyError (feature.py:88-92). ``.feature`` is the reference's
    key -> raw feature mapping."""
    global _RECORD_CLASS
    if _RECORD_CLASS is None:
        from tfr_reader.example.feature import Feature  # noqa: PLC0415

        if _PY is not None:
            # C base (csrc/tfrg_py.cpp ColRec): f[key], len(f), f.fields_names in C, no __dict__ and
            # no GC tracking per record; Feature's own methods, and an instance of Feature by ABC
            # registration
            class CFeature(_PY.ColRec):
                __slots__ = ()
                __eq__ = Feature.__eq__
                __ne__ = lambda self, other: not self == other  # noqa: E731
                __hash__ = None
                __repr__ = Feature.__repr__
                as_dict = Feature.as_dict
                fields = Feature.fields

                @property
                def feature(self):  # the reference's key -> raw feature mapping
                    return _RecordView(self._batch, self._i, self._lay)

                def __iter__(self):  # (the reference's Feature has no iteration of its own)
                    raise TypeError("'Feature' object is not iterable")

                def __reduce__(self):  # a plain Feature of the record's values (no batch reference)
                    r, i, lay = self._batch, self._i, self._lay
                    raw = {k: _ListRaw(KIND_NAMES[r.slot_kind[s]], r.slot_values(s, i)) for k, s in zip(lay.keys, lay.slots)}
                    return (Feature, (raw,))

            CFeature.__name__ = CFeature.__qualname__ = "Feature"
            Feature.register(CFeature)
            _RECORD_CLASS = CFeature
            return _RECORD_CLASS

        fields = tuple.__iter__  # (C-level unpacking: __getitem__ is the feature lookup here)

        class HipFeature(tuple, Feature):
            __slots__ = ()
            __init__ = tuple.__init__
            __eq__ = Feature.__eq__
            __ne__ = lambda self, other: not self == other  # noqa: E731
            __hash__ = None
            __repr__ = Feature.__repr__

            @property
            def feature(self):  # the reference's key -> raw feature mapping
                r, i, lay = fields(self)
                return _RecordView(r, i, lay)

            def __len__(self) -> int:
                return len(tuple.__getitem__(self, 2).slots)

            def __iter__(self):  # (the reference's Feature has no iteration of its own)
                raise TypeError("'Feature' object is not iterable")

            @property
            def fields_names(self) -> list[str]:
                return list(tuple.__getitem__(self, 2).keys)

            def __reduce__(self):  # a plain Feature of the record's values (no batch reference)
                r, i, lay = fields(self)
                raw = {k: _ListRaw(KIND_NAMES[r.slot_kind[s]], r.slot_values(s, i)) for k, s in zip(lay.keys, lay.slots)}
                return (Feature, (raw,))

            def __getitem__(self, key: str):
                r, i, lay = fields(self)
                ent = lay.acc.get(key)
                if ent is None:
                    raise KeyError(f"Feature '{key}' not found in the example, expected one of {lay.keys}")
                s, cls = ent
                c = r._py[s]
                if c is None:
                    c = r._pycol(s)
                rs = c[1]
                return cls((c[0], rs[i], rs[i + 1]))

        HipFeature.__name__ = HipFeature.__qualname__ = "Feature"
        _RECORD_CLASS = HipFeature
    return _RECORD_CLASS


# ---------------------------------------------------------------------- module-level default engine
_DEFAULT: dict[int, HipDecoder] = {}
_DEFAULT_LOCK = threading.Lock()


def default_decoder(device: int = 0) -> HipDecoder:
    with _DEFAULT_LOCK:
        d = _DEFAULT.get(device)
        if d is None:
            d = _DEFAULT[device] = HipDecoder(device)
        return d


def decode_payloads(payloads: Sequence[bytes], device: int = 0) -> BatchResult:
    """Decode bare Example payloads (decode(raw) semantics) in one device batch."""
    lens = np.fromiter((len(p) for p in payloads), dtype=np.uint64, count=len(payloads))
    ends = np.cumsum(lens, dtype=np.uint64)
    starts = ends - lens
    buf = b"".join(payloads)
    return default_decoder(device).decode(buf, starts, ends, payload_only=True)
