"""Dataset-level readers (reference: src/tfr_reader/reader.py).

``TFRecordFileReader.get_example`` (reader.py:36-56) and ``TFRecordDatasetReader.__getitem__`` /
``load_records`` / ``select`` (reader.py:168-247) keep their signatures and exceptions, but the
records are decoded in device batches: ``load_records`` groups the selection by file, stages the
needed byte ranges in one host buffer and decodes them in one libtfrg call instead of one
open/seek/read/decode per record on a thread pool (reader.py:242-247).
"""

from __future__ import annotations

import fnmatch
import hashlib
import os
import struct
import threading
from collections.abc import Iterable, Sequence
from pathlib import Path

import numpy as np

from tfr_reader import _frame as F
from tfr_reader import _io, example, hip, host, indexer, logging

LOGGER = logging.Logger(__name__)

#: host batches are split below the device limit of 4 GiB per decode call
MAX_BATCH_BYTES = 1 << 30
#: per-slot columns cost ~18 B per (slot, record) (order, count, loc, row splits): batches of
#: high-cardinality (sparse) key sets are split by records so that slots x records stays bounded
SLOT_BUDGET_BYTES = 4 << 30
SLOT_COLUMN_BYTES = 18


def _decode_bounded(dec, buf: np.ndarray, st: np.ndarray, en: np.ndarray, **kw):
    """dec.decode over record chunks of at most SLOT_BUDGET_BYTES / (18 x slots) records (the slot
    count known before each chunk; a chunk that learns many new keys only shrinks the next ones)
    and at most MAX_BATCH_BYTES of input each. Each chunk passes only its own byte span (16-byte
    aligned base, offsets rebased), so the host->HBM copy per call is the chunk, not the buffer.
    Yields (first record index, BatchResult)."""
    n = st.size
    at = 0
    top = np.maximum.accumulate(np.maximum(en, st)) if n else en
    while at < n:
        slots = max(1, len(dec.keys.slot_key))
        k = max(1024, SLOT_BUDGET_BYTES // (SLOT_COLUMN_BYTES * slots))
        if slots < 64:  # (a schema still being learned: a first chunk of bounded size)
            k = min(k, 1 << 16)
        s, e = st[at : at + k], en[at : at + k]
        lo = int(s.min()) & ~15
        if (np.diff(s.astype(np.int64)) >= 0).all():  # (sorted ranges: cut where the span ends)
            cut = int(np.searchsorted(top[at : at + k], np.uint64(lo + MAX_BATCH_BYTES), side="right"))
            k = max(1, cut)
            s, e = s[:k], e[:k]
        hi = min(int(e.max()), buf.size)
        base = np.uint64(lo)
        yield at, dec.decode(buf[lo:max(hi, lo)], s - base, e - base, **kw)
        at += k


def _check_path(path) -> None:
    p = str(path)
    if p.startswith("gs://"):
        raise ImportError("Google storage paths are not supported by this build (local files only).")
    if not os.path.exists(p):
        raise FileNotFoundError(f"Path {p} does not exist.")


def _decode_framed_bytes(data: bytes, start: int, end: int, dec=None) -> example.Feature:
    """Decode the framed record held in ``data`` (the bytes read for [start, end))."""
    imp = example.feature.TFRECORD_READER_DECODER_IMP
    if imp == "protobuf" or (dec is None and (imp == "cython" or len(data) <= host.HOST_MAX_BYTES)):
        # one record: the host decode (reader.py:55 slices the framing off, no CRC check)
        return example.decode(data[12:-4])
    r = (dec or hip.default_decoder()).decode(data, [0], [end - start])
    return r.feature(0)


class TFRecordFileReader:
    """Reads single framed records of one TFRecord file by byte offsets (reader.py:18-76). A
    ZLIB / GZIP compressed file is read through its decompressed stream (tfr_reader/_io.py)."""

    def __init__(self, filepath: str):
        _check_path(filepath)
        self.tfrecord_filepath = filepath
        self._file = None  # the open file's image (mmap / decompressed stream), as reader.py:18-76's handle

    def get_example(self, start: int, end: int) -> example.Feature:
        if self._file is None:
            raise OSError("File is not open. Use context manager!")
        data = self._file[start:end].tobytes() if start < self._file.size else b""
        if not data:
            raise OSError(f"Failed to read data from {(start, end)}!")
        return _decode_framed_bytes(data, start, end)

    def _open(self):
        if self._file is None:
            self._file = _io.file_image(self.tfrecord_filepath)

    def _close(self):
        self._file = None

    def __enter__(self):
        self._open()
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self._close()
        return False


#: device list used when a caller passes devices=None (tfr_reader.set_devices)
_DEFAULT_DEVICES = None
_LANE_DECODERS: dict = {}


def set_devices(devices) -> None:
    """Default devices of ``load_ranges`` / ``load_records`` / ``__getitem__(Iterable)``: None (device
    0), "all", an int or a list of device indices (tfr_reader.shard.resolve_devices). Each (lane,
    device) pair used keeps one decode context (its batch-sized device arenas) for the life of the
    process, so the next call reuses it; ``release_lane_decoders()`` frees the extra ones."""
    global _DEFAULT_DEVICES
    from tfr_reader import shard

    _DEFAULT_DEVICES = None if devices is None else shard.resolve_devices(devices)


def release_lane_decoders() -> None:
    """Close the decode contexts of lanes > 0 (load_ranges with several lanes per device) and free
    their device memory; the next call creates them again."""
    for d in _LANE_DECODERS.values():
        d.close()
    _LANE_DECODERS.clear()


def _lane_decoder(lane: int, device: int):
    """The decode context of lane `lane` on `device` (lane 0: the module default of the device)."""
    if lane == 0:
        return hip.default_decoder(device)
    d = _LANE_DECODERS.get((lane, device))
    if d is None:
        d = _LANE_DECODERS[(lane, device)] = hip.HipDecoder(device)
    return d


def load_ranges(paths: Sequence[str], starts: Sequence[int], ends: Sequence[int],
                devices=None) -> list[example.Feature]:
    """Decode framed records given as (file, start, end), in order, in device batches.

    Records are grouped by file. A file whose selected bytes are a large part of it is decoded
    straight from its image (mmap / decompressed stream: no host copy, the ranges index into it);
    sparser selections are staged back to back by the native gather (tfrg_gather_ranges) into
    batches of up to MAX_BATCH_BYTES. Raises the exception of the first failing record in order,
    like the reference's ordered ``ThreadPoolExecutor.map`` (reader.py:246-247).

    ``devices`` (default: ``set_devices``, else device 0): with several, the files are spread over
    them by LPT on their selected bytes, one host thread and decode context per entry (the
    reference's thread pool over records, reader.py:242-247, and process pool over files,
    indexer.py:121-134); results are merged back into selection order.
    """
    from tfr_reader import shard

    n = len(paths)
    out: list = [None] * n
    errors: list[BaseException | None] = [None] * n
    if example.feature.TFRECORD_READER_DECODER_IMP in ("protobuf", "cython"):  # record by record on the host
        imgs: dict = {}
        for i in range(n):
            img = imgs.get(paths[i])
            if img is None:
                _check_path(paths[i])
                img = imgs[paths[i]] = _io.file_image(paths[i])
            s, e = int(starts[i]), int(ends[i])
            data = img[s:e].tobytes() if s < img.size else b""
            if not data:
                raise OSError(f"Failed to read data from {(s, e)}!")
            out[i] = _decode_framed_bytes(data, s, e)
        return out
    starts = np.asarray(starts, np.uint64).reshape(-1)
    ends = np.asarray(ends, np.uint64).reshape(-1)
    by_file: dict[str, list[int]] = {}
    for i, p in enumerate(paths):
        by_file.setdefault(p, []).append(i)
    items = [(p, np.asarray(ii, np.int64)) for p, ii in by_file.items()]
    devs = shard.resolve_devices(devices if devices is not None else _DEFAULT_DEVICES)
    if len(devs) == 1 or len(items) == 1:
        _load_files(_lane_decoder(0, devs[0]), items, starts, ends, out, errors)
    else:
        from concurrent.futures import ThreadPoolExecutor

        sel = [int((ends[ii] - starts[ii]).sum()) for _, ii in items]
        parts = shard.lpt_partition(sel, len(devs))

        def lane(k: int) -> None:
            if parts[k]:
                _load_files(_lane_decoder(k, devs[k]), [items[j] for j in parts[k]], starts, ends, out, errors)

        with ThreadPoolExecutor(len(devs)) as ex:
            list(ex.map(lane, range(len(devs))))
    for i in range(n):
        if errors[i] is not None:
            raise errors[i]
    return out


def _load_files(dec, items, starts: np.ndarray, ends: np.ndarray, out: list, errors: list) -> None:
    """load_ranges' work for the (path, selection indices) items of one decode context."""
    from tfr_reader import _native as N

    def take(res, idx: np.ndarray) -> None:
        il = idx.tolist()
        if not res.status.any():  # (the usual case: every record decoded, one layout pass)
            for i, f in zip(il, res.features()):
                out[i] = f
            return
        for j, i in enumerate(il):
            e = res.error(j)
            if e is not None:
                errors[i] = e
            else:
                out[i] = res.feature(j)

    pend_img: list[np.ndarray] = []
    pend_idx: list[np.ndarray] = []
    pend_bytes = 0

    def flush() -> None:
        nonlocal pend_img, pend_idx, pend_bytes
        if not pend_idx:
            return
        idx = np.concatenate(pend_idx)
        buf = np.empty(pend_bytes, np.uint8)
        at = 0
        for img, ii in zip(pend_img, pend_idx):
            st, en = starts[ii], ends[ii]
            at += N.lib().tfrg_gather_ranges(N.ptr(img), N.ptr(st, N.u64p), N.ptr(en, N.u64p), st.size,
                                             N.ptr(buf[at:]) if buf.size else None)
        lens = (ends[idx] - starts[idx]).astype(np.uint64)
        b_en = np.cumsum(lens, dtype=np.uint64)
        for at, res in _decode_bounded(dec, buf, b_en - lens, b_en):
            take(res, idx[at : at + res.status.size])
        pend_img, pend_idx, pend_bytes = [], [], 0

    for path, ii in items:
        _check_path(path)
        img = _io.file_image(path)  # (mmap, or the decompressed stream of a ZLIB / GZIP file)
        fsize = int(img.size)
        s, e = starts[ii], ends[ii]
        bad = (s >= fsize) | (e <= s)
        for i in ii[bad].tolist():
            errors[i] = OSError(f"Failed to read data from {(int(starts[i]), int(ends[i]))}!")
        short = ~bad & (e > fsize)
        for i in ii[short].tolist():  # short read: decode alone so its buffer ends where the file does
            try:
                out[i] = _decode_framed_bytes(img[int(starts[i]) : fsize].tobytes(), int(starts[i]), int(ends[i]),
                                              dec)
            except Exception as exc:  # noqa: BLE001 — re-raised in selection order
                errors[i] = exc
        ok = ii[~bad & ~short]
        if not ok.size:
            continue
        sel = int((ends[ok] - starts[ok]).sum())
        if sel * 4 >= fsize and fsize <= MAX_BATCH_BYTES:  # dense selection: the image itself
            # bytes values gathered on the device (materialize_bytes): the Features own copies, as the
            # reference's bytes objects do, instead of views into a mapping the file may change under
            for at, res in _decode_bounded(dec, img, starts[ok], ends[ok], materialize_bytes=True):
                take(res, ok[at : at + res.status.size])
            continue
        for lo in range(0, ok.size, 1 << 20):  # sparse selection: staged back to back
            part = ok[lo : lo + (1 << 20)]
            nb = int((ends[part] - starts[part]).sum())
            if pend_bytes + nb > MAX_BATCH_BYTES:
                flush()
            pend_img.append(img)
            pend_idx.append(part)
            pend_bytes += nb
    flush()


class _OpenSource:
    __slots__ = ("kind", "value", "refs", "evicted")

    def __init__(self, kind: str, value) -> None:
        self.kind, self.value, self.refs, self.evicted = kind, value, 0, False


def _open_record_source(path: str) -> _OpenSource:
    _check_path(path)
    if _io.is_compressed(path):
        return _OpenSource("img", _io.file_image(path))
    return _OpenSource("fd", os.open(path, os.O_RDONLY))


class _OpenFiles:
    """What ds[i] keeps open per file: a descriptor (plain files, one pread per record) or the
    decompressed image (ZLIB / GZIP). Thread-safe: lookups, eviction of the oldest beyond ``cap``
    and reference counts are under one lock, and an evicted descriptor is closed by its last reader,
    so a pread never runs on a closed (or reused) descriptor. The reference opens the file per call
    (reader.py:168-184) and shares nothing between threads."""

    def __init__(self, cap: int) -> None:
        self.cap = cap
        self.lock = threading.Lock()
        self.items: dict[str, _OpenSource] = {}

    def acquire(self, path: str, opener=None):
        with self.lock:
            h = self.items.get(path)
            if h is None:
                if opener is None:
                    return None
                h = opener(path)
                if len(self.items) >= self.cap:
                    self._evict(self.items.pop(next(iter(self.items))))
                self.items[path] = h
            h.refs += 1
            return h

    def release(self, h: _OpenSource) -> None:
        with self.lock:
            h.refs -= 1
            if h.evicted and h.refs == 0:
                self._close(h)

    def _evict(self, h: _OpenSource) -> None:
        h.evicted = True
        if h.refs == 0:
            self._close(h)

    @staticmethod
    def _close(h: _OpenSource) -> None:
        if h.kind == "fd" and h.value is not None:
            os.close(h.value)
        h.value = None

    def close_all(self) -> None:
        with self.lock:
            items, self.items = self.items, {}
            for h in items.values():
                self._evict(h)


class TFRecordDatasetReader:
    """Indexed TFRecord dataset (reader.py:79-290)."""

    def __init__(
        self,
        dataset_dir: str | Path,
        index_df=None,
        verbose: bool = True,
        index_cache_dir: str | Path | None = None,
    ):
        _check_path(dataset_dir)
        self.dataset_dir = str(dataset_dir)
        self.verbose = verbose
        self.logger = logging.Logger(self.__class__.__name__, verbose)
        self.index_cache_dir = Path(index_cache_dir) if index_cache_dir is not None else None
        if index_df is None:
            index_path = join_path(dataset_dir, indexer.INDEX_FILENAME)
            index_df = self._load_or_cache_index(index_path)
        self.index_df = F.with_row_index(index_df, "_row_id")
        self._sql = None
        self._cols = None  # (paths, file index per row, starts, ends), built on first access
        self._files = _OpenFiles(self.MAX_OPEN_FILES)  # ds[i]: descriptors / decompressed images
        self.logger.info(f"Loaded dataset index with N={F.height(self.index_df)} records ...")

    @property
    def ctx(self):
        if self._sql is None:
            self._sql = F.SQL(self.index_df)
        return self._sql

    def __len__(self) -> int:
        return self.size

    @property
    def size(self) -> int:
        return F.height(self.index_df)

    @classmethod
    def build_index_from_dataset_dir(
        cls,
        dataset_dir: str | Path,
        index_fn: example.IndexFunc | None = None,
        filepattern: str = "*.tfrecord",
        processes: int = 1,
        index_cache_dir: str | Path | None = None,
    ) -> TFRecordDatasetReader:
        _check_path(dataset_dir)
        data = indexer.create_index_for_directory(
            dataset_dir, index_fn=index_fn, filepattern=filepattern, processes=processes
        )
        ds = F.sort_frame(F.make_frame(data), ["tfrecord_filename", "tfrecord_start"])
        F.write_parquet(ds, Path(dataset_dir) / indexer.INDEX_FILENAME)
        return cls(str(dataset_dir), index_df=ds, index_cache_dir=index_cache_dir)

    def _rows(self, idxs: list[int]) -> tuple[list[str], np.ndarray, np.ndarray]:
        """(path, start, end) of index rows, from column arrays taken once (no per-row frame access)."""
        if self._cols is None:
            c = F.columns(self.index_df, ["tfrecord_filename", "tfrecord_start", "tfrecord_end"])
            names = np.asarray(c["tfrecord_filename"], dtype=object)
            uniq, inv = np.unique(names, return_inverse=True)
            self._cols = ([join_path(self.dataset_dir, u) for u in uniq.tolist()], inv,
                          np.asarray(c["tfrecord_start"], np.uint64), np.asarray(c["tfrecord_end"], np.uint64))
        files, inv, st, en = self._cols
        ii = np.asarray(idxs, np.int64)
        return [files[k] for k in inv[ii].tolist()], st[ii], en[ii]

    def __getitem__(self, idx):
        if type(idx) is int and self._cols is not None:  # (one record: no ABC check, no frame access)
            files, inv, st, en = self._cols
            if idx < 0 or idx >= st.shape[0]:
                raise IndexError(f"Index {idx=} out of bounds, dataset size={self.size}")
            start, end = int(st[idx]), int(en[idx])
            path = files[inv[idx]]
            if end - start > 16 and end - start - 16 <= host.HOST_MAX_BYTES \
                    and example.feature.TFRECORD_READER_DECODER_IMP != "protobuf":
                h = self._files.acquire(path)
                if h is not None:
                    try:
                        data = os.pread(h.value, end - start, start) if h.kind == "fd" else None
                    finally:
                        self._files.release(h)
                    if data is not None and len(data) == end - start:  # (else the general path reports it)
                        return host.decode(data[12:-4])
        if isinstance(idx, Iterable):
            idxs = [int(i) for i in idx]
            for i in idxs:
                if i < 0 or i >= self.size:
                    raise IndexError(f"Index idx={i} out of bounds, dataset size={self.size}")
            if not idxs:
                return []
            return load_ranges(*self._rows(idxs))
        if idx < 0 or idx >= self.size:
            raise IndexError(f"Index {idx=} out of bounds, dataset size={self.size}")
        if self._cols is None:
            self._rows([])
        files, inv, st, en = self._cols
        i = int(idx)
        path, start, end = files[inv[i]], int(st[i]), int(en[i])
        data = self._record_bytes(path, start, end)
        if not data:
            raise OSError(f"Failed to read data from {(start, end)}!")
        return _decode_framed_bytes(data, start, end)

    #: files kept open for ds[i] (the least recently opened are closed beyond this)
    MAX_OPEN_FILES = 64

    def _record_bytes(self, path: str, start: int, end: int) -> bytes:
        """Bytes [start, end) of one file (reader.py:36-56 reads them with seek + read per call): a
        plain file is read with one pread on a descriptor kept open by this dataset, a ZLIB / GZIP
        file is sliced from its decompressed image (tfr_reader/_io.py)."""
        h = self._files.acquire(path, opener=_open_record_source)
        try:
            if h.kind == "fd":
                return os.pread(h.value, max(end - start, 0), start) if end > start else b""
            img = h.value
            return img[start:end].tobytes() if start < img.size else b""
        finally:
            self._files.release(h)

    def close(self) -> None:
        """Close the file descriptors ds[i] keeps open (one still being read is closed by its reader)."""
        self._files.close_all()

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def select(self, sql_query: str):
        selection = self.ctx.execute(sql_query)
        self.logger.info(f"Selected N={F.height(selection)} records ...")
        return selection, self.load_records(selection)

    def query(self, sql_query: str):
        return self.ctx.execute(sql_query)

    def load_records(self, selection, max_workers: int | None = None, devices=None) -> list[example.Feature]:
        """Decode the records of an index selection, in selection order (one device batch per
        <= 1 GiB of record bytes; ``max_workers`` is accepted for API compatibility). ``devices``:
        spread the selection's files over several GPUs (``load_ranges``)."""
        cols = F.columns(selection, ["tfrecord_filename", "tfrecord_start", "tfrecord_end"])
        paths = [join_path(self.dataset_dir, f) for f in cols["tfrecord_filename"]]
        return load_ranges(paths, cols["tfrecord_start"], cols["tfrecord_end"], devices)

    def _load_or_cache_index(self, index_path: str):
        if self.index_cache_dir is None:
            if not os.path.exists(index_path):
                raise FileNotFoundError(
                    f"Index file {index_path} does not exist. Please create the index first.",
                )
            self.logger.info("Loading dataset index from %s ...", index_path)
            return F.read_parquet(Path(index_path).read_bytes())
        self.index_cache_dir.mkdir(parents=True, exist_ok=True)
        path_hash = hashlib.sha256(index_path.encode("utf-8")).hexdigest()
        cached = self.index_cache_dir / f"{path_hash}_{indexer.INDEX_FILENAME}"
        if cached.exists():
            self.logger.info("Loading dataset index from cache %s ...", cached)
            return F.read_parquet(cached.read_bytes())
        if not os.path.exists(index_path):
            raise FileNotFoundError(
                f"Index file {index_path} does not exist. Please create the index first.",
            )
        raw = Path(index_path).read_bytes()
        cached.write_bytes(raw)
        return F.read_parquet(raw)


def inspect_dataset_example(dataset_dir: str, filepattern: str = "*.tfrecord"):
    """First example of the first matching file plus its key/kind/length table (reader.py:293-324)."""
    _check_path(dataset_dir)
    paths = [os.path.join(dataset_dir, p) for p in os.listdir(dataset_dir)]
    paths = sorted(p for p in paths if fnmatch.fnmatch(p, filepattern))
    LOGGER.info("Found N=%s TFRecord files ...", len(paths))
    img = _io.file_image(paths[0])  # (the decompressed stream of a ZLIB / GZIP file)
    length_bytes = img[:8].tobytes()
    if not length_bytes:
        raise IndexError("Failed to read length bytes")
    length = struct.unpack("<Q", length_bytes)[0]
    data = img[12 : 12 + length].tobytes()
    if not data or len(data) < length:
        raise OSError("Failed to read data!")
    feature = example.decode(data)
    info = [
        {"key": k, "type": feature.feature[k].WhichOneof("kind"), "length": len(feature[k].value)}
        for k in list(feature.feature)
    ]
    return feature, info


def load_from_directory(
    dataset_dir: str | Path,
    *,
    filepattern: str = "*.tfrecord",
    index_fn: example.IndexFunc | None = None,
    processes: int = 1,
    override: bool = False,
    index_cache_dir: str | Path | None = None,
) -> TFRecordDatasetReader:
    if (Path(dataset_dir) / indexer.INDEX_FILENAME).exists() and not override:
        LOGGER.info("Index file already exists. Loading the dataset from the index ...")
        return TFRecordDatasetReader(dataset_dir, index_cache_dir=index_cache_dir)
    return TFRecordDatasetReader.build_index_from_dataset_dir(
        dataset_dir, index_fn, filepattern, processes, index_cache_dir=index_cache_dir
    )


def join_path(base_path: str | Path, suffix: str) -> str:
    base = str(base_path)
    return base + suffix if base.endswith("/") else base + "/" + suffix
